// Independent H.264 decoder -- see h264_decoder.h.  Clause numbers refer to
// ITU-T H.264 (04/2017).
#include "h264_decoder.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>

#include "../common/h264_mb.h"
#include "../common/h264_tables.h"

namespace mivc {
namespace h264 {

std::vector<uint8_t> DecodedPicture::cropped_i420() const {
  std::vector<uint8_t> o(static_cast<size_t>(width) * height * 3 / 2);
  uint8_t* dst = o.data();
  for (int yy = 0; yy < height; ++yy)
    std::memcpy(dst + static_cast<size_t>(yy) * width, y.data() + static_cast<size_t>(yy + crop_y) * coded_width + crop_x,
                width);
  dst += static_cast<size_t>(width) * height;
  int cw = coded_width / 2, w2 = width / 2, h2 = height / 2;
  for (int yy = 0; yy < h2; ++yy)
    std::memcpy(dst + static_cast<size_t>(yy) * w2, u.data() + static_cast<size_t>(yy + crop_y / 2) * cw + crop_x / 2, w2);
  dst += static_cast<size_t>(w2) * h2;
  for (int yy = 0; yy < h2; ++yy)
    std::memcpy(dst + static_cast<size_t>(yy) * w2, v.data() + static_cast<size_t>(yy + crop_y / 2) * cw + crop_x / 2, w2);
  return o;
}

namespace {

struct Pic {
  int wmb = 0, hmb = 0, W = 0, H = 0;
  int frame_num = 0, idr = 0, slice_type = 0, id = 0;
  std::vector<uint8_t> Y, U, V;
  std::vector<int> slice;       // per MB slice index, -1 = not decoded
  std::vector<int8_t> kind;     // MbKind
  std::vector<int8_t> qp;       // QP_Y
  std::vector<int8_t> qp_dbk;   // QP used by the deblocking filter (0 for I_PCM)
  std::vector<uint8_t> tc;      // [mb][24] TotalCoeff (luma 16 in blkIdx order, Cb 4, Cr 4)
  std::vector<uint8_t> nz;      // [mb][16] luma blk (raster) has non-zero levels
  std::vector<uint8_t> i4;      // [mb][16] Intra4x4PredMode (raster)
  std::vector<int16_t> mv;      // [mb][16][2] raster
  std::vector<int8_t> ref;      // [mb][16] raster (ref idx, -1 intra)
  std::vector<int> refpic;      // [mb][16] raster (ref picture id, -1 intra)
  std::vector<uint8_t> rec_hdr; // parse-only: [mb][64] MbHeader
  std::vector<int16_t> rec_coef;// parse-only: non-zero 16-level blocks, packed
  std::vector<uint32_t> rec_mask, rec_off;  // parse-only: [mb] block mask / first block
  bool gpu_ok = true;
  int nslices = 0;
  void init(int w, int h, bool planes = true) {
    wmb = w;
    hmb = h;
    W = w * 16;
    H = h * 16;
    size_t n = static_cast<size_t>(w) * h;
    if (planes) {
      Y.assign(static_cast<size_t>(W) * H, 0);
      U.assign(static_cast<size_t>(W / 2) * (H / 2), 0);
      V.assign(U.size(), 0);
    }
    slice.assign(n, -1);
    kind.assign(n, 0);
    qp.assign(n, 0);
    qp_dbk.assign(n, 0);
    tc.assign(n * 24, 0);
    nz.assign(n * 16, 0);
    i4.assign(n * 16, 2);
    mv.assign(n * 32, 0);
    ref.assign(n * 16, -1);
    refpic.assign(n * 16, -1);
  }
  void init_records() {
    size_t n = static_cast<size_t>(wmb) * hmb;
    rec_hdr.assign(n * sizeof(MbHeader), 0);
    rec_mask.assign(n, 0);
    rec_off.assign(n, 0);
    rec_coef.clear();
    rec_coef.reserve(n * 64);
  }
  int px(int x, int y) const { return Y[static_cast<size_t>(y) * W + x]; }
};

struct SliceParams {
  int disable_idc = 0, alpha_off = 0, beta_off = 0;
  int cb_off = 0, cr_off = 0;
};

inline int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
inline int clip_px(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }
inline int med3(int a, int b, int c) { return std::max(std::min(a, b), std::min(std::max(a, b), c)); }

// --- independent implementations of the normative arithmetic ------------------
// 8.5.12.2 (rows, then columns, then +32 >> 6)
void idct4(int* b) {
  int t[16];
  for (int r = 0; r < 4; ++r) {
    const int* s = b + 4 * r;
    int a0 = s[0] + s[2];
    int a1 = s[0] - s[2];
    int a2 = (s[1] >> 1) - s[3];
    int a3 = s[1] + (s[3] >> 1);
    t[4 * r + 0] = a0 + a3;
    t[4 * r + 1] = a1 + a2;
    t[4 * r + 2] = a1 - a2;
    t[4 * r + 3] = a0 - a3;
  }
  for (int c = 0; c < 4; ++c) {
    int a0 = t[c] + t[8 + c];
    int a1 = t[c] - t[8 + c];
    int a2 = (t[4 + c] >> 1) - t[12 + c];
    int a3 = t[4 + c] + (t[12 + c] >> 1);
    b[c] = (a0 + a3 + 32) >> 6;
    b[4 + c] = (a1 + a2 + 32) >> 6;
    b[8 + c] = (a1 - a2 + 32) >> 6;
    b[12 + c] = (a0 - a3 + 32) >> 6;
  }
}
// LevelScale4x4 with flat weights: 16 * normAdjust (8.5.9)
int level_scale(int qp_mod6, int x, int y) {
  static const int v[6][3] = {{10, 16, 13}, {11, 18, 14}, {13, 20, 16}, {14, 23, 18}, {16, 25, 20}, {18, 29, 23}};
  int cls = ((x & 1) == 0 && (y & 1) == 0) ? 0 : (((x & 1) == 1 && (y & 1) == 1) ? 1 : 2);
  return 16 * v[qp_mod6][cls];
}
// 8.5.12.1 scaling of one AC/4x4 coefficient
int scale4(int c, int qp, int x, int y) {
  int ls = level_scale(qp % 6, x, y);
  if (qp >= 24) return (c * ls) << (qp / 6 - 4);
  return (c * ls + (1 << (3 - qp / 6))) >> (4 - qp / 6);
}

// CAVLC VLC lookup by peeking
int read_vlc(BitReader& br, const uint8_t* lens, const uint8_t* bits, int n) {
  uint32_t pk = br.peek(16);
  for (int i = 0; i < n; ++i) {
    int l = lens[i];
    if (!l) continue;
    if ((pk >> (16 - l)) == bits[i]) {
      br.skip(l);
      return i;
    }
  }
  throw std::runtime_error("invalid VLC code");
}

}  // namespace

struct Decoder::Impl {
  SPS sps[32];
  PPS pps[256];
  bool have_sps[32] = {}, have_pps[256] = {};
  std::shared_ptr<Pic> cur;
  int cur_frame_num = -1;
  int cur_nal_ref = 0;
  std::vector<SliceParams> slices;
  std::vector<std::shared_ptr<Pic>> dpb;  // short-term references
  int next_pic_id = 1;
  int crop[4] = {0, 0, 0, 0};
  int max_frame_num = 16;
  int max_refs = 1;
  bool skip_deblock = false;
  bool parse_only = false;

  // per-slice state
  SliceHeader sh;
  const PPS* pp = nullptr;
  const SPS* sp = nullptr;
  int slice_idx = 0;
  std::vector<std::shared_ptr<Pic>> ref_list;

  // per-MB scratch
  int blk_done[16];  // current MB: 4x4 block (raster) available (decoded / MV assigned)

  // ------------------------------------------------------------ neighbours (6.4.11/6.4.12)
  bool mb_ok(int addr) const { return addr >= 0 && cur->slice[addr] == slice_idx; }
  // luma location (xN,yN) relative to the current MB -> (mbaddr, raster 4x4 index); -1 if unavailable.
  int nb_loc(int addr, int xN, int yN, int* blk) const {
    int mx = addr % cur->wmb, my = addr / cur->wmb;
    int n;
    if (yN < 0) {
      if (my == 0) return -1;
      if (xN < 0) n = mx > 0 ? addr - cur->wmb - 1 : -1;
      else if (xN < 16) n = addr - cur->wmb;
      else n = mx < cur->wmb - 1 ? addr - cur->wmb + 1 : -1;
    } else if (yN < 16) {
      if (xN < 0) n = mx > 0 ? addr - 1 : -1;
      else if (xN < 16) n = addr;
      else return -1;
    } else {
      return -1;
    }
    if (n < 0) return -1;
    int xW = (xN + 16) & 15, yW = (yN + 16) & 15;
    *blk = (xW >> 2) + 4 * (yW >> 2);
    if (n == addr) return blk_done[*blk] ? n : -1;
    return mb_ok(n) ? n : -1;
  }

  // ------------------------------------------------------------ picture management
  void finish_picture(std::vector<DecodedPicture>& out) {
    if (!cur) return;
    if (!skip_deblock && !parse_only) deblock_picture();
    DecodedPicture d;
    d.coded_width = cur->W;
    d.coded_height = cur->H;
    d.crop_x = crop[0] * 2;
    d.crop_y = crop[2] * 2;
    d.width = cur->W - 2 * (crop[0] + crop[1]);
    d.height = cur->H - 2 * (crop[2] + crop[3]);
    d.frame_num = cur->frame_num;
    d.idr = cur->idr;
    d.slice_type = cur->slice_type;
    d.y = cur->Y;
    d.u = cur->U;
    d.v = cur->V;
    size_t n = cur->kind.size();
    d.mb_kind = cur->kind;
    d.mb_qp = cur->qp;
    d.mv = cur->mv;
    d.ref = cur->ref;
    d.nz = cur->nz;
    if (parse_only) {
      d.hdr = std::move(cur->rec_hdr);
      d.coef = std::move(cur->rec_coef);
      d.blk_mask = std::move(cur->rec_mask);
      d.blk_off = std::move(cur->rec_off);
      d.slice_qp = pic_slice_qp;
      d.pic_id = cur->id;
      d.ref_id = pic_ref_id;
      d.nal_ref = cur_nal_ref != 0;
      d.alpha_off = slices.empty() ? 0 : slices[0].alpha_off;
      d.beta_off = slices.empty() ? 0 : slices[0].beta_off;
      d.chroma_qp_offset = slices.empty() ? 0 : slices[0].cb_off;
      d.deblock = slices.empty() ? 1 : (slices[0].disable_idc != 1);
      bool ok = cur->gpu_ok && cur->nslices == 1;
      for (const SliceParams& sp2 : slices) ok = ok && sp2.cb_off == sp2.cr_off && sp2.disable_idc != 2;
      d.gpu_ok = ok;
    }
    (void)n;
    out.push_back(std::move(d));
    if (cur_nal_ref) {
      if (cur->idr) dpb.clear();
      dpb.push_back(cur);
      while (static_cast<int>(dpb.size()) > std::max(1, max_refs)) dpb.erase(dpb.begin());
    }
    cur.reset();
  }

  int pic_slice_qp = 0, pic_ref_id = -1;
  void start_picture(const SliceHeader& h) {
    cur = std::make_shared<Pic>();
    cur->init(sp->width_mbs, sp->height_mbs, !parse_only);
    if (parse_only) cur->init_records();
    pic_slice_qp = h.qp;
    pic_ref_id = -1;
    cur->frame_num = h.frame_num;
    cur->idr = h.nal_unit_type == NAL_IDR;
    cur->slice_type = h.slice_type;
    cur->id = next_pic_id++;
    cur_frame_num = h.frame_num;
    cur_nal_ref = h.nal_ref_idc;
    slices.clear();
    crop[0] = sp->crop_left;
    crop[1] = sp->crop_right;
    crop[2] = sp->crop_top;
    crop[3] = sp->crop_bottom;
    max_frame_num = 1 << sp->log2_max_frame_num;
    max_refs = sp->max_num_ref_frames;
  }

  void build_ref_list() {
    ref_list.clear();
    if (sh.slice_type != SLICE_P) return;
    std::vector<std::shared_ptr<Pic>> v = dpb;
    auto wrap = [&](int fn) { return fn > sh.frame_num ? fn - max_frame_num : fn; };
    std::sort(v.begin(), v.end(), [&](const std::shared_ptr<Pic>& a, const std::shared_ptr<Pic>& b) {
      return wrap(a->frame_num) > wrap(b->frame_num);
    });
    if (v.empty()) throw std::runtime_error("P slice without reference picture");
    for (int i = 0; i < sh.num_ref_idx_l0_active; ++i) ref_list.push_back(v[std::min<size_t>(i, v.size() - 1)]);
  }

  // ------------------------------------------------------------ slice data
  void decode_slice(const NalUnit& nal, std::vector<DecodedPicture>& out) {
    BitReader br(nal.rbsp.data(), nal.rbsp.size());
    SliceHeader h = parse_slice_header(br, nal.nal_unit_type, nal.nal_ref_idc, sps, pps);
    if (!have_pps[h.pps_id]) throw std::runtime_error("slice references missing PPS");
    const PPS* p = &pps[h.pps_id];
    if (!have_sps[p->sps_id]) throw std::runtime_error("PPS references missing SPS");
    if (p->entropy_coding_mode) throw std::runtime_error("CABAC decoding not supported by the CPU oracle");
    if (p->transform_8x8_mode) throw std::runtime_error("8x8 transform not supported by the CPU oracle");
    bool new_pic = !cur || h.first_mb == 0 || h.frame_num != cur_frame_num ||
                   (h.nal_unit_type == NAL_IDR) != (cur && cur->idr);
    if (new_pic) {
      finish_picture(out);
      sh = h;
      pp = p;
      sp = &sps[p->sps_id];
      start_picture(h);
    }
    sh = h;
    pp = p;
    sp = &sps[p->sps_id];
    SliceParams spar;
    spar.disable_idc = h.disable_deblocking_filter_idc;
    spar.alpha_off = h.alpha_offset_div2 * 2;
    spar.beta_off = h.beta_offset_div2 * 2;
    spar.cb_off = p->chroma_qp_index_offset;
    spar.cr_off = p->second_chroma_qp_index_offset;
    slices.push_back(spar);
    slice_idx = static_cast<int>(slices.size()) - 1;
    cur->nslices = static_cast<int>(slices.size());
    if (h.num_ref_idx_l0_active > 1 || p->constrained_intra_pred) cur->gpu_ok = false;
    build_ref_list();
    if (!ref_list.empty()) {
      if (pic_ref_id >= 0 && pic_ref_id != ref_list[0]->id) cur->gpu_ok = false;
      pic_ref_id = ref_list[0]->id;
    }

    int nmb = cur->wmb * cur->hmb;
    int addr = h.first_mb;
    int qp = h.qp;
    bool more = true;
    while (more) {
      if (addr >= nmb) throw std::runtime_error("slice runs past the picture");
      if (sh.slice_type == SLICE_P) {
        int run = br.get_ue();
        for (int i = 0; i < run; ++i) {
          if (addr >= nmb) throw std::runtime_error("skip run past the picture");
          decode_skip(addr, qp);
          ++addr;
        }
        if (run > 0) {
          more = br.more_rbsp_data();
          if (!more) break;
        }
      }
      decode_mb(br, addr, qp);
      ++addr;
      more = br.more_rbsp_data();
    }
  }

  void begin_mb(int addr) {
    cur->slice[addr] = slice_idx;
    for (int i = 0; i < 16; ++i) blk_done[i] = 0;
    for (int i = 0; i < 16; ++i) {
      cur->ref[addr * 16 + i] = -1;
      cur->refpic[addr * 16 + i] = -1;
      cur->mv[addr * 32 + 2 * i] = cur->mv[addr * 32 + 2 * i + 1] = 0;
      cur->nz[addr * 16 + i] = 0;
      cur->i4[addr * 16 + i] = 2;
    }
    for (int i = 0; i < 24; ++i) cur->tc[addr * 24 + i] = 0;
  }

  // ------------------------------------------------------------ motion vector prediction (8.4.1.3)
  struct NbMv {
    bool avail;
    int ref;
    int mv[2];
  };
  NbMv nb_mv(int addr, int xN, int yN) {
    NbMv r{false, -1, {0, 0}};
    int blk;
    int n = nb_loc(addr, xN, yN, &blk);
    if (n < 0) return r;
    r.avail = true;
    if (mbk_is_intra(cur->kind[n]) && n != addr) return r;
    r.ref = cur->ref[n * 16 + blk];
    r.mv[0] = cur->mv[n * 32 + 2 * blk];
    r.mv[1] = cur->mv[n * 32 + 2 * blk + 1];
    return r;
  }
  void pred_mv(int addr, int x, int y, int w, int h, int shape, int part, int ref, int out[2]) {
    NbMv A = nb_mv(addr, x - 1, y);
    NbMv B = nb_mv(addr, x, y - 1);
    NbMv C = nb_mv(addr, x + w, y - 1);
    if (!C.avail) C = nb_mv(addr, x - 1, y - 1);
    (void)h;
    if (shape == 1) {  // 16x8
      if (part == 0 && B.ref == ref) { out[0] = B.mv[0]; out[1] = B.mv[1]; return; }
      if (part == 1 && A.ref == ref) { out[0] = A.mv[0]; out[1] = A.mv[1]; return; }
    } else if (shape == 2) {  // 8x16
      if (part == 0 && A.ref == ref) { out[0] = A.mv[0]; out[1] = A.mv[1]; return; }
      if (part == 1 && C.ref == ref) { out[0] = C.mv[0]; out[1] = C.mv[1]; return; }
    }
    if (!B.avail && !C.avail && A.avail) {
      B = A;
      C = A;
    }
    int match = (A.ref == ref) + (B.ref == ref) + (C.ref == ref);
    if (match == 1) {
      const NbMv& m = A.ref == ref ? A : (B.ref == ref ? B : C);
      out[0] = m.mv[0];
      out[1] = m.mv[1];
      return;
    }
    out[0] = med3(A.mv[0], B.mv[0], C.mv[0]);
    out[1] = med3(A.mv[1], B.mv[1], C.mv[1]);
  }
  void assign_part(int addr, int bx, int by, int w4, int h4, int ref, int mvx, int mvy) {
    for (int y = by; y < by + h4; ++y)
      for (int x = bx; x < bx + w4; ++x) {
        int r = x + 4 * y;
        cur->ref[addr * 16 + r] = static_cast<int8_t>(ref);
        cur->refpic[addr * 16 + r] = ref_list[ref]->id;
        cur->mv[addr * 32 + 2 * r] = static_cast<int16_t>(mvx);
        cur->mv[addr * 32 + 2 * r + 1] = static_cast<int16_t>(mvy);
        blk_done[r] = 1;
      }
  }

  void decode_skip(int addr, int qp) {
    begin_mb(addr);
    cur->kind[addr] = MBK_PSKIP;
    cur->qp[addr] = static_cast<int8_t>(qp);
    cur->qp_dbk[addr] = static_cast<int8_t>(qp);
    int mv[2] = {0, 0};
    NbMv A = nb_mv(addr, -1, 0);
    NbMv B = nb_mv(addr, 0, -1);
    bool zero = !A.avail || !B.avail || (A.ref == 0 && A.mv[0] == 0 && A.mv[1] == 0) ||
                (B.ref == 0 && B.mv[0] == 0 && B.mv[1] == 0);
    if (!zero) pred_mv(addr, 0, 0, 16, 16, 0, 0, 0, mv);
    assign_part(addr, 0, 0, 4, 4, 0, mv[0], mv[1]);
    if (parse_only) {
      cur->rec_off[addr] = static_cast<uint32_t>(cur->rec_coef.size() / 16);
      store_record(addr, MBK_PSKIP, 0, qp, 0, 0, nullptr);
      return;
    }
    inter_pred(addr);
  }

  // parse-only: MbHeader + levels of MB addr (lum/lumdc/cdc/cac already in the records)
  void store_record(int addr, int kind, int cbp, int qp, int i16_mode, int chroma_mode, const int* i4modes) {
    MbHeader h{};
    h.kind = static_cast<uint8_t>(kind);
    h.cbp = static_cast<uint8_t>(cbp);
    h.qp = static_cast<int8_t>(qp);
    h.i16_mode = static_cast<uint8_t>(i16_mode);
    h.chroma_mode = static_cast<uint8_t>(chroma_mode);
    for (int q = 0; q < 4; ++q) {
      int r0 = (q & 1) * 2 + (q >> 1) * 8;  // top-left 4x4 block of quadrant q
      h.mv[0][q][0] = cur->mv[addr * 32 + 2 * r0];
      h.mv[0][q][1] = cur->mv[addr * 32 + 2 * r0 + 1];
      h.ref[0][q] = cur->ref[addr * 16 + r0];
      h.ref[1][q] = -1;
      for (int k = 0; k < 4; ++k) {  // the quadrant must carry one vector (no sub-8x8 split)
        int r = r0 + (k & 1) + (k >> 1) * 4;
        if (cur->mv[addr * 32 + 2 * r] != h.mv[0][q][0] || cur->mv[addr * 32 + 2 * r + 1] != h.mv[0][q][1])
          cur->gpu_ok = false;
      }
    }
    for (int b = 0; b < 16; ++b) h.i4_modes[b] = static_cast<uint8_t>(i4modes ? i4modes[b] : 2);
    std::memcpy(cur->rec_hdr.data() + static_cast<size_t>(addr) * sizeof(MbHeader), &h, sizeof(MbHeader));
  }

  // ------------------------------------------------------------ inter prediction (8.4.2.2)
  static int ref_y(const Pic& r, int x, int y) {
    return r.Y[static_cast<size_t>(clampi(y, 0, r.H - 1)) * r.W + clampi(x, 0, r.W - 1)];
  }
  static int half_h1(const Pic& r, int x, int y) {  // intermediate b1 at (x+1/2, y)
    return tap6(ref_y(r, x - 2, y), ref_y(r, x - 1, y), ref_y(r, x, y), ref_y(r, x + 1, y), ref_y(r, x + 2, y),
                ref_y(r, x + 3, y));
  }
  static int half_v1(const Pic& r, int x, int y) {  // intermediate h1 at (x, y+1/2)
    return tap6(ref_y(r, x, y - 2), ref_y(r, x, y - 1), ref_y(r, x, y), ref_y(r, x, y + 1), ref_y(r, x, y + 2),
                ref_y(r, x, y + 3));
  }
  static int luma_sample(const Pic& r, int xi, int yi, int xf, int yf) {
    auto b = [&](int x, int y) { return clip_px((half_h1(r, x, y) + 16) >> 5); };
    auto h = [&](int x, int y) { return clip_px((half_v1(r, x, y) + 16) >> 5); };
    auto j = [&](int x, int y) {
      int j1 = tap6(half_h1(r, x, y - 2), half_h1(r, x, y - 1), half_h1(r, x, y), half_h1(r, x, y + 1),
                    half_h1(r, x, y + 2), half_h1(r, x, y + 3));
      return clip_px((j1 + 512) >> 10);
    };
    int G = ref_y(r, xi, yi);
    switch (yf * 4 + xf) {
      case 0: return G;
      case 1: return (G + b(xi, yi) + 1) >> 1;                    // a
      case 2: return b(xi, yi);                                   // b
      case 3: return (ref_y(r, xi + 1, yi) + b(xi, yi) + 1) >> 1; // c
      case 4: return (G + h(xi, yi) + 1) >> 1;                    // d
      case 5: return (b(xi, yi) + h(xi, yi) + 1) >> 1;            // e
      case 6: return (b(xi, yi) + j(xi, yi) + 1) >> 1;            // f
      case 7: return (b(xi, yi) + h(xi + 1, yi) + 1) >> 1;        // g
      case 8: return h(xi, yi);                                   // h
      case 9: return (h(xi, yi) + j(xi, yi) + 1) >> 1;            // i
      case 10: return j(xi, yi);                                  // j
      case 11: return (j(xi, yi) + h(xi + 1, yi) + 1) >> 1;       // k
      case 12: return (ref_y(r, xi, yi + 1) + h(xi, yi) + 1) >> 1; // n
      case 13: return (h(xi, yi) + b(xi, yi + 1) + 1) >> 1;       // p
      case 14: return (j(xi, yi) + b(xi, yi + 1) + 1) >> 1;       // q
      case 15: return (h(xi + 1, yi) + b(xi, yi + 1) + 1) >> 1;   // r
    }
    return 0;
  }
  static int chroma_sample(const std::vector<uint8_t>& plane, int cw, int ch, int xi, int yi, int xf, int yf) {
    auto P = [&](int x, int y) {
      return static_cast<int>(plane[static_cast<size_t>(clampi(y, 0, ch - 1)) * cw + clampi(x, 0, cw - 1)]);
    };
    return ((8 - xf) * (8 - yf) * P(xi, yi) + xf * (8 - yf) * P(xi + 1, yi) + (8 - xf) * yf * P(xi, yi + 1) +
            xf * yf * P(xi + 1, yi + 1) + 32) >>
           6;
  }
  // predict the whole MB into the picture buffers from per-4x4 MVs
  void inter_pred(int addr) {
    int mx = addr % cur->wmb, my = addr / cur->wmb;
    int cw = cur->W / 2, ch = cur->H / 2;
    for (int r = 0; r < 16; ++r) {
      int bx = r & 3, by = r >> 2;
      const Pic& ref = *ref_list[cur->ref[addr * 16 + r]];
      int mvx = cur->mv[addr * 32 + 2 * r], mvy = cur->mv[addr * 32 + 2 * r + 1];
      for (int y = 0; y < 4; ++y)
        for (int x = 0; x < 4; ++x) {
          int px = mx * 16 + bx * 4 + x, py = my * 16 + by * 4 + y;
          int xi = px + (mvx >> 2), yi = py + (mvy >> 2);
          cur->Y[static_cast<size_t>(py) * cur->W + px] = static_cast<uint8_t>(luma_sample(ref, xi, yi, mvx & 3, mvy & 3));
        }
      for (int y = 0; y < 2; ++y)
        for (int x = 0; x < 2; ++x) {
          int px = mx * 8 + bx * 2 + x, py = my * 8 + by * 2 + y;
          int xi = px + (mvx >> 3), yi = py + (mvy >> 3);
          cur->U[static_cast<size_t>(py) * cw + px] =
              static_cast<uint8_t>(chroma_sample(ref.U, cw, ch, xi, yi, mvx & 7, mvy & 7));
          cur->V[static_cast<size_t>(py) * cw + px] =
              static_cast<uint8_t>(chroma_sample(ref.V, cw, ch, xi, yi, mvx & 7, mvy & 7));
        }
    }
  }

  // ------------------------------------------------------------ CAVLC residual (9.2)
  int total_coeff_of(int n, int idx) const { return cur->tc[n * 24 + idx]; }
  int nc_luma(int addr, int blkidx) {
    int bx = kBlkX[blkidx], by = kBlkY[blkidx];
    int ba, bb;
    // neighbour blocks are looked up without the "decoded" restriction on the current MB
    // (left/top blocks of the current MB always precede it in decoding order)
    for (int i = 0; i < 16; ++i) blk_tmp[i] = blk_done[i];
    for (int i = 0; i < 16; ++i) blk_done[i] = 1;
    int na = nb_loc(addr, bx * 4 - 1, by * 4, &ba);
    int nbk = nb_loc(addr, bx * 4, by * 4 - 1, &bb);
    for (int i = 0; i < 16; ++i) blk_done[i] = blk_tmp[i];
    int nA = na >= 0 ? (cur->kind[na] == MBK_PSKIP ? 0 : total_coeff_of(na, kRasterToBlk[ba])) : 0;
    int nB = nbk >= 0 ? (cur->kind[nbk] == MBK_PSKIP ? 0 : total_coeff_of(nbk, kRasterToBlk[bb])) : 0;
    if (na >= 0 && nbk >= 0) return (nA + nB + 1) >> 1;
    if (na >= 0) return nA;
    if (nbk >= 0) return nB;
    return 0;
  }
  int nc_chroma(int addr, int comp, int blk) {
    int cx = blk & 1, cy = blk >> 1;
    int mx = addr % cur->wmb, my = addr / cur->wmb;
    int a = cx > 0 ? addr : (mx > 0 && mb_ok(addr - 1) ? addr - 1 : -1);
    int b = cy > 0 ? addr : (my > 0 && mb_ok(addr - cur->wmb) ? addr - cur->wmb : -1);
    int ia = 16 + comp * 4 + cy * 2 + (cx > 0 ? cx - 1 : 1);
    int ib = 16 + comp * 4 + (cy > 0 ? cy - 1 : 1) * 2 + cx;
    int nA = a >= 0 ? (cur->kind[a] == MBK_PSKIP ? 0 : total_coeff_of(a, ia)) : 0;
    int nB = b >= 0 ? (cur->kind[b] == MBK_PSKIP ? 0 : total_coeff_of(b, ib)) : 0;
    if (a >= 0 && b >= 0) return (nA + nB + 1) >> 1;
    if (a >= 0) return nA;
    if (b >= 0) return nB;
    return 0;
  }
  int blk_tmp[16];

  // residual_block_cavlc (7.3.5.3.2); writes coefficient levels into lv[start..end]
  int read_block(BitReader& br, int* lv, int start, int end, int max_num, int nc) {
    for (int i = 0; i < max_num; ++i) lv[i] = 0;
    int tc, t1;
    if (nc == -1) {
      int k = read_vlc(br, kChromaDcCoeffTokenLen, kChromaDcCoeffTokenBits, 20);
      tc = k >> 2;
      t1 = k & 3;
    } else if (nc >= 8) {
      int code = br.get(6);
      if (code == 3) {
        tc = 0;
        t1 = 0;
      } else {
        tc = (code >> 2) + 1;
        t1 = code & 3;
        if (t1 > tc) throw std::runtime_error("bad FLC coeff_token");
      }
    } else {
      int t = nc < 2 ? 0 : (nc < 4 ? 1 : 2);
      int k = read_vlc(br, kCoeffTokenLen[t], kCoeffTokenBits[t], 68);
      tc = k >> 2;
      t1 = k & 3;
    }
    if (tc == 0) return 0;
    if (tc > end - start + 1) throw std::runtime_error("TotalCoeff exceeds block size");
    int level[16], run[16];
    int suffix_len = (tc > 10 && t1 < 3) ? 1 : 0;
    for (int i = 0; i < tc; ++i) {
      if (i < t1) {
        level[i] = br.get_bit() ? -1 : 1;
        continue;
      }
      int prefix = 0;
      while (br.get_bit() == 0) {
        if (++prefix > 32) throw std::runtime_error("bad level_prefix");
      }
      int code = (std::min(15, prefix) << suffix_len);
      int ssize = suffix_len;
      if (prefix == 14 && suffix_len == 0) ssize = 4;
      if (prefix >= 15) ssize = prefix - 3;
      if (suffix_len > 0 || prefix >= 14) {
        if (ssize > 0) code += static_cast<int>(br.get(ssize));
      }
      if (prefix >= 15 && suffix_len == 0) code += 15;
      if (prefix >= 16) code += (1 << (prefix - 3)) - 4096;
      if (i == t1 && t1 < 3) code += 2;
      level[i] = (code % 2 == 0) ? (code + 2) >> 1 : (-code - 1) >> 1;
      if (suffix_len == 0) suffix_len = 1;
      if (std::abs(level[i]) > (3 << (suffix_len - 1)) && suffix_len < 6) ++suffix_len;
    }
    int zeros_left = 0;
    if (tc < end - start + 1) {
      if (max_num == 4) {
        zeros_left = read_vlc(br, kChromaDcTotalZerosLen[tc - 1], kChromaDcTotalZerosBits[tc - 1], 4);
      } else {
        zeros_left = read_vlc(br, kTotalZerosLen[tc - 1], kTotalZerosBits[tc - 1], 16);
      }
    }
    for (int i = 0; i < tc - 1; ++i) {
      if (zeros_left > 0) {
        int t = std::min(zeros_left, 7) - 1;
        run[i] = read_vlc(br, kRunBeforeLen[t], kRunBeforeBits[t], 15);
        if (run[i] > zeros_left) throw std::runtime_error("run_before exceeds zerosLeft");
      } else {
        run[i] = 0;
      }
      zeros_left -= run[i];
    }
    run[tc - 1] = zeros_left;
    int pos = -1;
    for (int i = tc - 1; i >= 0; --i) {
      pos += run[i] + 1;
      if (start + pos > end) throw std::runtime_error("coefficient index out of range");
      lv[start + pos] = level[i];
    }
    return tc;
  }

  // ------------------------------------------------------------ intra prediction (8.3)
  // fetch neighbour sample of the current picture at MB-relative luma position; -1 if unavailable
  int intra_avail(int addr, int xN, int yN) {
    int blk;
    int n = nb_loc(addr, xN, yN, &blk);
    if (n < 0) return 0;
    if (n != addr && pp->constrained_intra_pred && !mbk_is_intra(cur->kind[n])) return 0;
    return 1;
  }

  void pred4x4(int addr, int blkidx, int mode, uint8_t* pred) {
    int mx = addr % cur->wmb, my = addr / cur->wmb;
    int bx = kBlkX[blkidx] * 4, by = kBlkY[blkidx] * 4;
    int X0 = mx * 16 + bx, Y0 = my * 16 + by;
    int top[8], left[4], tl = 0;
    bool has_top = intra_avail(addr, bx, by - 1);
    bool has_left = intra_avail(addr, bx - 1, by);
    bool has_tl = intra_avail(addr, bx - 1, by - 1);
    bool has_tr = intra_avail(addr, bx + 4, by - 1);
    if (has_top)
      for (int x = 0; x < 4; ++x) top[x] = cur->px(X0 + x, Y0 - 1);
    if (has_top) {
      if (has_tr)
        for (int x = 4; x < 8; ++x) top[x] = cur->px(X0 + x, Y0 - 1);
      else
        for (int x = 4; x < 8; ++x) top[x] = top[3];
    }
    if (has_left)
      for (int y = 0; y < 4; ++y) left[y] = cur->px(X0 - 1, Y0 + y);
    if (has_tl) tl = cur->px(X0 - 1, Y0 - 1);
    auto P = [&](int x, int y) -> int {  // p[x,y] with x,y in -1..7
      if (y == -1 && x == -1) return tl;
      if (y == -1) return top[x];
      return left[y];
    };
    auto need = [&](bool c) {
      if (!c) throw std::runtime_error("intra 4x4 mode uses unavailable samples");
    };
    for (int y = 0; y < 4; ++y)
      for (int x = 0; x < 4; ++x) {
        int v = 0;
        switch (mode) {
          case 0: need(has_top); v = P(x, -1); break;
          case 1: need(has_left); v = P(-1, y); break;
          case 2: {
            if (has_top && has_left) v = (top[0] + top[1] + top[2] + top[3] + left[0] + left[1] + left[2] + left[3] + 4) >> 3;
            else if (has_left) v = (left[0] + left[1] + left[2] + left[3] + 2) >> 2;
            else if (has_top) v = (top[0] + top[1] + top[2] + top[3] + 2) >> 2;
            else v = 128;
            break;
          }
          case 3:
            need(has_top);
            if (x == 3 && y == 3) v = (P(6, -1) + 3 * P(7, -1) + 2) >> 2;
            else v = (P(x + y, -1) + 2 * P(x + y + 1, -1) + P(x + y + 2, -1) + 2) >> 2;
            break;
          case 4:
            need(has_top && has_left && has_tl);
            if (x > y) v = (P(x - y - 2, -1) + 2 * P(x - y - 1, -1) + P(x - y, -1) + 2) >> 2;
            else if (x < y) v = (P(-1, y - x - 2) + 2 * P(-1, y - x - 1) + P(-1, y - x) + 2) >> 2;
            else v = (P(0, -1) + 2 * P(-1, -1) + P(-1, 0) + 2) >> 2;
            break;
          case 5: {
            need(has_top && has_left && has_tl);
            int z = 2 * x - y;
            if (z >= 0 && (z & 1) == 0) v = (P(x - (y >> 1) - 1, -1) + P(x - (y >> 1), -1) + 1) >> 1;
            else if (z >= 0) v = (P(x - (y >> 1) - 2, -1) + 2 * P(x - (y >> 1) - 1, -1) + P(x - (y >> 1), -1) + 2) >> 2;
            else if (z == -1) v = (P(-1, 0) + 2 * P(-1, -1) + P(0, -1) + 2) >> 2;
            else v = (P(-1, y - 1) + 2 * P(-1, y - 2) + P(-1, y - 3) + 2) >> 2;
            break;
          }
          case 6: {
            need(has_top && has_left && has_tl);
            int z = 2 * y - x;
            if (z >= 0 && (z & 1) == 0) v = (P(-1, y - (x >> 1) - 1) + P(-1, y - (x >> 1)) + 1) >> 1;
            else if (z >= 0) v = (P(-1, y - (x >> 1) - 2) + 2 * P(-1, y - (x >> 1) - 1) + P(-1, y - (x >> 1)) + 2) >> 2;
            else if (z == -1) v = (P(-1, 0) + 2 * P(-1, -1) + P(0, -1) + 2) >> 2;
            else v = (P(x - 1, -1) + 2 * P(x - 2, -1) + P(x - 3, -1) + 2) >> 2;
            break;
          }
          case 7:
            need(has_top);
            if ((y & 1) == 0) v = (P(x + (y >> 1), -1) + P(x + (y >> 1) + 1, -1) + 1) >> 1;
            else v = (P(x + (y >> 1), -1) + 2 * P(x + (y >> 1) + 1, -1) + P(x + (y >> 1) + 2, -1) + 2) >> 2;
            break;
          case 8: {
            need(has_left);
            int z = x + 2 * y;
            if (z < 5 && (z & 1) == 0) v = (P(-1, y + (x >> 1)) + P(-1, y + (x >> 1) + 1) + 1) >> 1;
            else if (z < 5) v = (P(-1, y + (x >> 1)) + 2 * P(-1, y + (x >> 1) + 1) + P(-1, y + (x >> 1) + 2) + 2) >> 2;
            else if (z == 5) v = (P(-1, 2) + 3 * P(-1, 3) + 2) >> 2;
            else v = P(-1, 3);
            break;
          }
          default: throw std::runtime_error("bad intra4x4 mode");
        }
        pred[y * 4 + x] = static_cast<uint8_t>(v);
      }
  }

  void pred16x16(int addr, int mode, uint8_t* pred) {
    int mx = addr % cur->wmb, my = addr / cur->wmb;
    int X0 = mx * 16, Y0 = my * 16;
    bool has_top = intra_avail(addr, 0, -1), has_left = intra_avail(addr, -1, 0), has_tl = intra_avail(addr, -1, -1);
    int top[16], left[16], tl = has_tl ? cur->px(X0 - 1, Y0 - 1) : 0;
    for (int i = 0; i < 16; ++i) {
      top[i] = has_top ? cur->px(X0 + i, Y0 - 1) : 0;
      left[i] = has_left ? cur->px(X0 - 1, Y0 + i) : 0;
    }
    if (mode == 0 && !has_top) throw std::runtime_error("I16 V without top");
    if (mode == 1 && !has_left) throw std::runtime_error("I16 H without left");
    if (mode == 3 && !(has_top && has_left && has_tl)) throw std::runtime_error("I16 plane without neighbours");
    int dc = 128;
    if (mode == 2) {
      int st = 0, sl = 0;
      for (int i = 0; i < 16; ++i) {
        st += top[i];
        sl += left[i];
      }
      if (has_top && has_left) dc = (st + sl + 16) >> 5;
      else if (has_left) dc = (sl + 8) >> 4;
      else if (has_top) dc = (st + 8) >> 4;
    }
    int a = 0, b = 0, c = 0;
    if (mode == 3) {
      int H = 0, V = 0;
      for (int i = 0; i < 8; ++i) {
        H += (i + 1) * (top[8 + i] - (6 - i >= 0 ? top[6 - i] : tl));
        V += (i + 1) * (left[8 + i] - (6 - i >= 0 ? left[6 - i] : tl));
      }
      a = 16 * (left[15] + top[15]);
      b = (5 * H + 32) >> 6;
      c = (5 * V + 32) >> 6;
    }
    for (int y = 0; y < 16; ++y)
      for (int x = 0; x < 16; ++x) {
        int v;
        switch (mode) {
          case 0: v = top[x]; break;
          case 1: v = left[y]; break;
          case 2: v = dc; break;
          default: v = clip_px((a + b * (x - 7) + c * (y - 7) + 16) >> 5); break;
        }
        pred[y * 16 + x] = static_cast<uint8_t>(v);
      }
  }

  void pred_chroma(int addr, int mode, const std::vector<uint8_t>& plane, uint8_t* pred) {
    int mx = addr % cur->wmb, my = addr / cur->wmb;
    int cw = cur->W / 2;
    int X0 = mx * 8, Y0 = my * 8;
    bool has_top = intra_avail(addr, 0, -1), has_left = intra_avail(addr, -1, 0), has_tl = intra_avail(addr, -1, -1);
    auto C = [&](int x, int y) { return static_cast<int>(plane[static_cast<size_t>(y) * cw + x]); };
    int top[8], left[8], tl = has_tl ? C(X0 - 1, Y0 - 1) : 0;
    for (int i = 0; i < 8; ++i) {
      top[i] = has_top ? C(X0 + i, Y0 - 1) : 0;
      left[i] = has_left ? C(X0 - 1, Y0 + i) : 0;
    }
    if (mode == 0) {
      for (int blk = 0; blk < 4; ++blk) {
        int xo = (blk & 1) * 4, yo = (blk >> 1) * 4;
        int st = 0, sl = 0;
        for (int i = 0; i < 4; ++i) {
          st += top[xo + i];
          sl += left[yo + i];
        }
        int dc;
        if ((xo == 0 && yo == 0) || (xo > 0 && yo > 0)) {
          if (has_top && has_left) dc = (st + sl + 4) >> 3;
          else if (has_left) dc = (sl + 2) >> 2;
          else if (has_top) dc = (st + 2) >> 2;
          else dc = 128;
        } else if (xo > 0 && yo == 0) {
          if (has_top) dc = (st + 2) >> 2;
          else if (has_left) dc = (sl + 2) >> 2;
          else dc = 128;
        } else {
          if (has_left) dc = (sl + 2) >> 2;
          else if (has_top) dc = (st + 2) >> 2;
          else dc = 128;
        }
        for (int y = 0; y < 4; ++y)
          for (int x = 0; x < 4; ++x) pred[(yo + y) * 8 + xo + x] = static_cast<uint8_t>(dc);
      }
      return;
    }
    if (mode == 1 && !has_left) throw std::runtime_error("chroma H without left");
    if (mode == 2 && !has_top) throw std::runtime_error("chroma V without top");
    if (mode == 3 && !(has_top && has_left && has_tl)) throw std::runtime_error("chroma plane without neighbours");
    int a = 0, b = 0, c = 0;
    if (mode == 3) {
      int H = 0, V = 0;
      for (int i = 0; i < 4; ++i) {
        H += (i + 1) * (top[4 + i] - (2 - i >= 0 ? top[2 - i] : tl));
        V += (i + 1) * (left[4 + i] - (2 - i >= 0 ? left[2 - i] : tl));
      }
      a = 16 * (left[7] + top[7]);
      b = (34 * H + 32) >> 6;
      c = (34 * V + 32) >> 6;
    }
    for (int y = 0; y < 8; ++y)
      for (int x = 0; x < 8; ++x) {
        int v;
        if (mode == 1) v = left[y];
        else if (mode == 2) v = top[x];
        else v = clip_px((a + b * (x - 3) + c * (y - 3) + 16) >> 5);
        pred[y * 8 + x] = static_cast<uint8_t>(v);
      }
  }

  // ------------------------------------------------------------ macroblock layer (7.3.5)
  void decode_mb(BitReader& br, int addr, int& qp) {
    begin_mb(addr);
    int mb_type = br.get_ue();
    bool pslice = sh.slice_type == SLICE_P;
    int kind;
    int i16_mode = 0, cbp_luma = 0, cbp_chroma = 0, cbp = 0;
    int ptype = -1;  // P partitioning 0..4
    if (pslice && mb_type < 5) {
      ptype = mb_type;
      kind = mb_type == 0 ? MBK_P16x16 : mb_type == 1 ? MBK_P16x8 : mb_type == 2 ? MBK_P8x16 : MBK_P8x8;
    } else {
      int it = pslice ? mb_type - 5 : mb_type;
      if (it == 0) kind = MBK_I4x4;
      else if (it <= 24) {
        kind = MBK_I16x16;
        i16_mode = (it - 1) % 4;
        cbp_chroma = ((it - 1) / 4) % 3;
        cbp_luma = (it >= 13) ? 15 : 0;
      } else if (it == 25) kind = MBK_IPCM;
      else throw std::runtime_error("bad mb_type " + std::to_string(mb_type));
    }
    cur->kind[addr] = static_cast<int8_t>(kind);
    int mx = addr % cur->wmb, my = addr / cur->wmb;
    int cw = cur->W / 2;
    if (kind == MBK_IPCM) {
      while (!br.byte_aligned()) {
        if (br.get_bit()) throw std::runtime_error("pcm_alignment_zero_bit is 1");
      }
      for (int y = 0; y < 16; ++y)
        for (int x = 0; x < 16; ++x) cur->Y[static_cast<size_t>(my * 16 + y) * cur->W + mx * 16 + x] = br.get(8);
      for (int y = 0; y < 8; ++y)
        for (int x = 0; x < 8; ++x) cur->U[static_cast<size_t>(my * 8 + y) * cw + mx * 8 + x] = br.get(8);
      for (int y = 0; y < 8; ++y)
        for (int x = 0; x < 8; ++x) cur->V[static_cast<size_t>(my * 8 + y) * cw + mx * 8 + x] = br.get(8);
      for (int i = 0; i < 24; ++i) cur->tc[addr * 24 + i] = 16;
      for (int i = 0; i < 16; ++i) cur->nz[addr * 16 + i] = 1;
      cur->qp[addr] = static_cast<int8_t>(qp);
      cur->qp_dbk[addr] = 0;
      for (int i = 0; i < 16; ++i) blk_done[i] = 1;
      cur->gpu_ok = false;
      return;
    }
    // ---- prediction syntax
    int i4modes[16];
    int chroma_mode = 0;
    if (kind == MBK_I4x4) {
      for (int blk = 0; blk < 16; ++blk) {
        int flag = br.get_bit();
        int rem = flag ? 0 : br.get(3);
        // predIntra4x4PredMode (8.3.1.1)
        int bx = kBlkX[blk] * 4, by = kBlkY[blk] * 4;
        for (int i = 0; i < 16; ++i) blk_tmp[i] = blk_done[i];
        for (int i = 0; i < 16; ++i) blk_done[i] = 1;
        int ba, bb;
        int na = nb_loc(addr, bx - 1, by, &ba);
        int nb = nb_loc(addr, bx, by - 1, &bb);
        for (int i = 0; i < 16; ++i) blk_done[i] = blk_tmp[i];
        bool dcpred = na < 0 || nb < 0 ||
                      (na != addr && pp->constrained_intra_pred && !mbk_is_intra(cur->kind[na])) ||
                      (nb != addr && pp->constrained_intra_pred && !mbk_is_intra(cur->kind[nb]));
        int pred;
        if (dcpred) {
          pred = 2;
        } else {
          int ma = (na == addr) ? i4modes[kRasterToBlk[ba]] : (cur->kind[na] == MBK_I4x4 ? cur->i4[na * 16 + ba] : 2);
          int mb = (nb == addr) ? i4modes[kRasterToBlk[bb]] : (cur->kind[nb] == MBK_I4x4 ? cur->i4[nb * 16 + bb] : 2);
          pred = std::min(ma, mb);
        }
        i4modes[blk] = flag ? pred : (rem < pred ? rem : rem + 1);
        cur->i4[addr * 16 + kBlkX[blk] + 4 * kBlkY[blk]] = static_cast<uint8_t>(i4modes[blk]);
      }
    }
    if (kind == MBK_I4x4 || kind == MBK_I16x16) {
      chroma_mode = br.get_ue();
      if (chroma_mode > 3) throw std::runtime_error("bad intra_chroma_pred_mode");
    }
    if (!mbk_is_intra(kind)) {
      int nref = sh.num_ref_idx_l0_active;
      if (ptype == 0 || ptype == 1 || ptype == 2) {
        int nparts = ptype == 0 ? 1 : 2;
        int refs[2] = {0, 0};
        for (int p = 0; p < nparts; ++p) refs[p] = nref > 1 ? br.get_te(nref - 1) : 0;
        for (int p = 0; p < nparts; ++p) {
          if (refs[p] >= nref) throw std::runtime_error("ref_idx out of range");
          int bx = 0, by = 0, w4 = 4, h4 = 4;
          if (ptype == 1) { by = p * 2; h4 = 2; }
          if (ptype == 2) { bx = p * 2; w4 = 2; }
          int mvd0 = br.get_se(), mvd1 = br.get_se();
          int pmv[2];
          pred_mv(addr, bx * 4, by * 4, w4 * 4, h4 * 4, ptype, p, refs[p], pmv);
          assign_part(addr, bx, by, w4, h4, refs[p], pmv[0] + mvd0, pmv[1] + mvd1);
        }
      } else {
        int sub[4], refs[4] = {0, 0, 0, 0};
        for (int s = 0; s < 4; ++s) {
          sub[s] = br.get_ue();
          if (sub[s] > 3) throw std::runtime_error("bad sub_mb_type");
        }
        if (ptype == 3 && nref > 1)
          for (int s = 0; s < 4; ++s) refs[s] = br.get_te(nref - 1);
        for (int s = 0; s < 4; ++s) {
          int sx = (s & 1) * 2, sy = (s >> 1) * 2;
          int nsp = sub[s] == 0 ? 1 : (sub[s] == 3 ? 4 : 2);
          int w4 = (sub[s] == 0 || sub[s] == 1) ? 2 : 1;
          int h4 = (sub[s] == 0 || sub[s] == 2) ? 2 : 1;
          for (int k = 0; k < nsp; ++k) {
            int bx = sx, by = sy;
            if (sub[s] == 1) by += k;
            else if (sub[s] == 2) bx += k;
            else if (sub[s] == 3) { bx += k & 1; by += k >> 1; }
            int mvd0 = br.get_se(), mvd1 = br.get_se();
            int pmv[2];
            pred_mv(addr, bx * 4, by * 4, w4 * 4, h4 * 4, 0, 0, refs[s], pmv);
            assign_part(addr, bx, by, w4, h4, refs[s], pmv[0] + mvd0, pmv[1] + mvd1);
          }
        }
      }
    }
    if (kind != MBK_I16x16) {
      int code = br.get_ue();
      if (code > 47) throw std::runtime_error("bad coded_block_pattern");
      cbp = mbk_is_intra(kind) ? kGolombToIntraCbp[code] : kGolombToInterCbp[code];
      cbp_luma = cbp & 15;
      cbp_chroma = cbp >> 4;
    }
    if (cbp_luma || cbp_chroma || kind == MBK_I16x16) {
      int d = br.get_se();
      if (d < -26 || d > 25) throw std::runtime_error("mb_qp_delta out of range");
      qp = ((qp + d + 52) % 52);
    }
    cur->qp[addr] = static_cast<int8_t>(qp);
    cur->qp_dbk[addr] = static_cast<int8_t>(qp);
    // ---- residual syntax
    int lum[16][16] = {};  // per blkIdx, scan order
    int lumdc[16] = {};
    int cdc[2][4] = {};
    int cac[2][4][16] = {};
    for (int i = 0; i < 16; ++i) blk_done[i] = 1;  // for nC lookups inside the MB
    if (kind == MBK_I16x16) read_block(br, lumdc, 0, 15, 16, nc_luma(addr, 0));
    for (int b8 = 0; b8 < 4; ++b8)
      for (int b4 = 0; b4 < 4; ++b4) {
        int blk = b8 * 4 + b4;
        if (!(cbp_luma & (1 << b8))) continue;
        int nc = nc_luma(addr, blk);
        int t = kind == MBK_I16x16 ? read_block(br, lum[blk], 1, 15, 15, nc) : read_block(br, lum[blk], 0, 15, 16, nc);
        cur->tc[addr * 24 + blk] = static_cast<uint8_t>(t);
      }
    if (cbp_chroma)
      for (int c = 0; c < 2; ++c) read_block(br, cdc[c], 0, 3, 4, -1);
    if (cbp_chroma & 2)
      for (int c = 0; c < 2; ++c)
        for (int b = 0; b < 4; ++b) {
          int t = read_block(br, cac[c][b], 1, 15, 15, nc_chroma(addr, c, b));
          cur->tc[addr * 24 + 16 + c * 4 + b] = static_cast<uint8_t>(t);
        }
    for (int blk = 0; blk < 16; ++blk) {
      bool any = false;
      for (int i = 0; i < 16; ++i) any |= lum[blk][i] != 0;
      if (kind == MBK_I16x16) any |= lumdc[blk] != 0;  // not used for bS (intra), informative
      cur->nz[addr * 16 + kBlkX[blk] + 4 * kBlkY[blk]] = any;
    }
    if (parse_only) {
      // packed levels: one 16-entry block per non-zero block, in mask-bit order
      // (bits 0-15 luma blkIdx, 16 luma DC, 17 chroma DC Cb|Cr, 18-25 chroma AC comp*4+b)
      uint32_t mask = 0;
      cur->rec_off[addr] = static_cast<uint32_t>(cur->rec_coef.size() / 16);
      auto put = [&](int bit, const int* v, int n, const int* v2) {
        bool any = false;
        for (int i = 0; i < n; ++i) any |= v[i] != 0 || (v2 && v2[i] != 0);
        if (!any) return;
        mask |= 1u << bit;
        size_t b = cur->rec_coef.size();
        cur->rec_coef.resize(b + 16, 0);
        for (int i = 0; i < n; ++i) cur->rec_coef[b + i] = static_cast<int16_t>(v[i]);
        if (v2)
          for (int i = 0; i < n; ++i) cur->rec_coef[b + n + i] = static_cast<int16_t>(v2[i]);
      };
      for (int blk = 0; blk < 16; ++blk) put(blk, lum[blk], 16, nullptr);
      if (kind == MBK_I16x16) put(16, lumdc, 16, nullptr);
      put(17, cdc[0], 4, cdc[1]);
      for (int cc = 0; cc < 2; ++cc)
        for (int b = 0; b < 4; ++b) put(18 + cc * 4 + b, cac[cc][b], 16, nullptr);
      cur->rec_mask[addr] = mask;
      if (kind != MBK_I4x4 && kind != MBK_I16x16 && kind != MBK_P16x16 && kind != MBK_P16x8 &&
          kind != MBK_P8x16 && kind != MBK_P8x8)
        cur->gpu_ok = false;
      store_record(addr, kind, cbp_luma | (cbp_chroma << 4), qp, i16_mode, chroma_mode,
                   kind == MBK_I4x4 ? i4modes : nullptr);
      for (int i = 0; i < 16; ++i) blk_done[i] = 1;
      return;
    }
    for (int i = 0; i < 16; ++i) blk_done[i] = 0;
    // ---- reconstruction
    int X0 = mx * 16, Y0 = my * 16;
    if (kind == MBK_I4x4) {
      for (int blk = 0; blk < 16; ++blk) {
        uint8_t pred[16];
        pred4x4(addr, blk, i4modes[blk], pred);
        int d[16];
        for (int i = 0; i < 16; ++i) d[i] = 0;
        for (int i = 0; i < 16; ++i) {
          int r = kZigzag4x4[i];
          d[r] = scale4(lum[blk][i], qp, r & 3, r >> 2);
        }
        idct4(d);
        int bx = kBlkX[blk] * 4, by = kBlkY[blk] * 4;
        for (int y = 0; y < 4; ++y)
          for (int x = 0; x < 4; ++x)
            cur->Y[static_cast<size_t>(Y0 + by + y) * cur->W + X0 + bx + x] = static_cast<uint8_t>(clip_px(pred[y * 4 + x] + d[y * 4 + x]));
        blk_done[kBlkX[blk] + 4 * kBlkY[blk]] = 1;
      }
    } else if (kind == MBK_I16x16) {
      uint8_t pred[256];
      pred16x16(addr, i16_mode, pred);
      // luma DC: inverse scan into 4x4 (block geometry), Hadamard, scale (8.5.10)
      int c[16], f[16], tmp[16];
      for (int i = 0; i < 16; ++i) c[kZigzag4x4[i]] = lumdc[i];
      for (int y = 0; y < 4; ++y) {  // rows
        int* s = c + 4 * y;
        tmp[4 * y + 0] = s[0] + s[1] + s[2] + s[3];
        tmp[4 * y + 1] = s[0] + s[1] - s[2] - s[3];
        tmp[4 * y + 2] = s[0] - s[1] - s[2] + s[3];
        tmp[4 * y + 3] = s[0] - s[1] + s[2] - s[3];
      }
      for (int x = 0; x < 4; ++x) {
        int s0 = tmp[x], s1 = tmp[4 + x], s2 = tmp[8 + x], s3 = tmp[12 + x];
        f[x] = s0 + s1 + s2 + s3;
        f[4 + x] = s0 + s1 - s2 - s3;
        f[8 + x] = s0 - s1 - s2 + s3;
        f[12 + x] = s0 - s1 + s2 - s3;
      }
      int ls = level_scale(qp % 6, 0, 0);
      for (int blk = 0; blk < 16; ++blk) {
        int bx = kBlkX[blk], by = kBlkY[blk];
        int fv = f[bx + 4 * by];
        int dcv = qp >= 36 ? (fv * ls) << (qp / 6 - 6) : (fv * ls + (1 << (5 - qp / 6))) >> (6 - qp / 6);
        int d[16];
        for (int i = 0; i < 16; ++i) d[i] = 0;
        for (int i = 1; i < 16; ++i) {
          int r = kZigzag4x4[i];
          d[r] = scale4(lum[blk][i], qp, r & 3, r >> 2);
        }
        d[0] = dcv;
        idct4(d);
        for (int y = 0; y < 4; ++y)
          for (int x = 0; x < 4; ++x) {
            int px = bx * 4 + x, py = by * 4 + y;
            cur->Y[static_cast<size_t>(Y0 + py) * cur->W + X0 + px] = static_cast<uint8_t>(clip_px(pred[py * 16 + px] + d[y * 4 + x]));
          }
      }
    } else {
      inter_pred(addr);
      for (int blk = 0; blk < 16; ++blk) {
        if (!(cbp_luma & (1 << (blk >> 2)))) continue;
        int d[16];
        for (int i = 0; i < 16; ++i) d[i] = 0;
        for (int i = 0; i < 16; ++i) {
          int r = kZigzag4x4[i];
          d[r] = scale4(lum[blk][i], qp, r & 3, r >> 2);
        }
        idct4(d);
        int bx = kBlkX[blk] * 4, by = kBlkY[blk] * 4;
        for (int y = 0; y < 4; ++y)
          for (int x = 0; x < 4; ++x) {
            uint8_t& o = cur->Y[static_cast<size_t>(Y0 + by + y) * cur->W + X0 + bx + x];
            o = static_cast<uint8_t>(clip_px(o + d[y * 4 + x]));
          }
      }
    }
    // chroma
    for (int comp = 0; comp < 2; ++comp) {
      std::vector<uint8_t>& plane = comp == 0 ? cur->U : cur->V;
      uint8_t pred[64];
      if (mbk_is_intra(kind)) {
        pred_chroma(addr, chroma_mode, plane, pred);
      } else {
        for (int y = 0; y < 8; ++y)
          for (int x = 0; x < 8; ++x) pred[y * 8 + x] = plane[static_cast<size_t>(my * 8 + y) * cw + mx * 8 + x];
      }
      int qpc = chroma_qp(qp, comp == 0 ? pp->chroma_qp_index_offset : pp->second_chroma_qp_index_offset);
      int c0 = cdc[comp][0], c1 = cdc[comp][1], c2 = cdc[comp][2], c3 = cdc[comp][3];
      int f[4] = {c0 + c1 + c2 + c3, c0 - c1 + c2 - c3, c0 + c1 - c2 - c3, c0 - c1 - c2 + c3};
      int ls = level_scale(qpc % 6, 0, 0);
      for (int b = 0; b < 4; ++b) {
        int d[16];
        for (int i = 0; i < 16; ++i) d[i] = 0;
        if (cbp_chroma & 2)
          for (int i = 1; i < 16; ++i) {
            int r = kZigzag4x4[i];
            d[r] = scale4(cac[comp][b][i], qpc, r & 3, r >> 2);
          }
        d[0] = ((f[b] * ls) << (qpc / 6)) >> 5;
        bool any = cbp_chroma != 0;
        if (any) idct4(d);
        int xo = (b & 1) * 4, yo = (b >> 1) * 4;
        for (int y = 0; y < 4; ++y)
          for (int x = 0; x < 4; ++x) {
            int v = pred[(yo + y) * 8 + xo + x] + (any ? d[y * 4 + x] : 0);
            plane[static_cast<size_t>(my * 8 + yo + y) * cw + mx * 8 + xo + x] = static_cast<uint8_t>(clip_px(v));
          }
      }
    }
    for (int i = 0; i < 16; ++i) blk_done[i] = 1;
  }

  // ------------------------------------------------------------ deblocking (8.7)
  int bs_of(int mbp, int blkp, int mbq, int blkq, bool mb_edge) {
    bool ip = mbk_is_intra(cur->kind[mbp]), iq = mbk_is_intra(cur->kind[mbq]);
    if (mb_edge && (ip || iq)) return 4;
    if (ip || iq) return 3;
    if (cur->nz[mbp * 16 + blkp] || cur->nz[mbq * 16 + blkq]) return 2;
    if (cur->refpic[mbp * 16 + blkp] != cur->refpic[mbq * 16 + blkq]) return 1;
    int dx = cur->mv[mbp * 32 + 2 * blkp] - cur->mv[mbq * 32 + 2 * blkq];
    int dy = cur->mv[mbp * 32 + 2 * blkp + 1] - cur->mv[mbq * 32 + 2 * blkq + 1];
    if (std::abs(dx) >= 4 || std::abs(dy) >= 4) return 1;
    return 0;
  }

  // filter one line of samples across an edge. s points to q0; step = distance between p0 and q0 neighbours
  static void filter_line(uint8_t* q0p, int step, int bs, int alpha, int beta, int tc0, bool chroma) {
    int p0 = q0p[-step], p1 = q0p[-2 * step], q0 = q0p[0], q1 = q0p[step];
    if (!(std::abs(p0 - q0) < alpha && std::abs(p1 - p0) < beta && std::abs(q1 - q0) < beta)) return;
    int p2 = chroma ? 0 : q0p[-3 * step], q2 = chroma ? 0 : q0p[2 * step];
    int ap = std::abs(p2 - p0), aq = std::abs(q2 - q0);
    if (bs < 4) {
      int tc = chroma ? tc0 + 1 : tc0 + (ap < beta) + (aq < beta);
      int delta = clampi((((q0 - p0) << 2) + (p1 - q1) + 4) >> 3, -tc, tc);
      q0p[-step] = static_cast<uint8_t>(clip_px(p0 + delta));
      q0p[0] = static_cast<uint8_t>(clip_px(q0 - delta));
      if (!chroma) {
        if (ap < beta) q0p[-2 * step] = static_cast<uint8_t>(p1 + clampi((p2 + ((p0 + q0 + 1) >> 1) - (p1 << 1)) >> 1, -tc0, tc0));
        if (aq < beta) q0p[step] = static_cast<uint8_t>(q1 + clampi((q2 + ((p0 + q0 + 1) >> 1) - (q1 << 1)) >> 1, -tc0, tc0));
      }
    } else {
      if (!chroma && ap < beta && std::abs(p0 - q0) < ((alpha >> 2) + 2)) {
        int p3 = q0p[-4 * step];
        q0p[-step] = static_cast<uint8_t>((p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3);
        q0p[-2 * step] = static_cast<uint8_t>((p2 + p1 + p0 + q0 + 2) >> 2);
        q0p[-3 * step] = static_cast<uint8_t>((2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3);
      } else {
        q0p[-step] = static_cast<uint8_t>((2 * p1 + p0 + q1 + 2) >> 2);
      }
      if (!chroma && aq < beta && std::abs(p0 - q0) < ((alpha >> 2) + 2)) {
        int q3 = q0p[3 * step];
        q0p[0] = static_cast<uint8_t>((p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3);
        q0p[step] = static_cast<uint8_t>((p0 + q0 + q1 + q2 + 2) >> 2);
        q0p[2 * step] = static_cast<uint8_t>((2 * q3 + 3 * q2 + q1 + q0 + p0 + 4) >> 3);
      } else {
        q0p[0] = static_cast<uint8_t>((2 * q1 + q0 + p1 + 2) >> 2);
      }
    }
  }

  void deblock_picture() {
    int W = cur->W, cw = W / 2;
    int nmb = cur->wmb * cur->hmb;
    for (int addr = 0; addr < nmb; ++addr) {
      if (cur->slice[addr] < 0) continue;
      const SliceParams& spar = slices[cur->slice[addr]];
      if (spar.disable_idc == 1) continue;
      int mx = addr % cur->wmb, my = addr / cur->wmb;
      bool left = mx > 0 && !(spar.disable_idc == 2 && cur->slice[addr - 1] != cur->slice[addr]);
      bool top = my > 0 && !(spar.disable_idc == 2 && cur->slice[addr - cur->wmb] != cur->slice[addr]);
      for (int dir = 0; dir < 2; ++dir) {  // 0: vertical edges, 1: horizontal edges
        for (int e = 0; e < 4; ++e) {
          if (e == 0 && !(dir == 0 ? left : top)) continue;
          int mbp = e == 0 ? (dir == 0 ? addr - 1 : addr - cur->wmb) : addr;
          int bS[4];
          for (int k = 0; k < 4; ++k) {
            int blkq = dir == 0 ? (e + 4 * k) : (k + 4 * e);
            int blkp = dir == 0 ? (e == 0 ? 3 + 4 * k : e - 1 + 4 * k) : (e == 0 ? k + 12 : k + 4 * (e - 1));
            bS[k] = bs_of(mbp, blkp, addr, blkq, e == 0);
          }
          // luma
          int qpav = (cur->qp_dbk[mbp] + cur->qp_dbk[addr] + 1) >> 1;
          int ia = clampi(qpav + spar.alpha_off, 0, 51), ib = clampi(qpav + spar.beta_off, 0, 51);
          int alpha = kAlpha[ia], beta = kBeta[ib];
          for (int i = 0; i < 16; ++i) {
            int bs = bS[i >> 2];
            if (!bs) continue;
            int tc0 = bs < 4 ? kTc0[ia][bs - 1] : 0;
            uint8_t* q0;
            int step;
            if (dir == 0) {
              q0 = &cur->Y[static_cast<size_t>(my * 16 + i) * W + mx * 16 + e * 4];
              step = 1;
            } else {
              q0 = &cur->Y[static_cast<size_t>(my * 16 + e * 4) * W + mx * 16 + i];
              step = W;
            }
            filter_line(q0, step, bs, alpha, beta, tc0, false);
          }
          // chroma: edges 0 and 2 (luma) map to chroma edges 0 and 4
          if (e == 0 || e == 2) {
            int ce = e / 2;  // 0 or 1 -> chroma offset 0 or 4
            for (int comp = 0; comp < 2; ++comp) {
              int off = comp == 0 ? spar.cb_off : spar.cr_off;
              int qpp = cur->kind[mbp] == MBK_IPCM ? chroma_qp(0, off) : chroma_qp(cur->qp_dbk[mbp], off);
              int qpq = cur->kind[addr] == MBK_IPCM ? chroma_qp(0, off) : chroma_qp(cur->qp_dbk[addr], off);
              int qa = (qpp + qpq + 1) >> 1;
              int iac = clampi(qa + spar.alpha_off, 0, 51), ibc = clampi(qa + spar.beta_off, 0, 51);
              int ac = kAlpha[iac], bc = kBeta[ibc];
              std::vector<uint8_t>& pl = comp == 0 ? cur->U : cur->V;
              for (int i = 0; i < 8; ++i) {
                int bs = bS[i >> 1];
                if (!bs) continue;
                int tc0 = bs < 4 ? kTc0[iac][bs - 1] : 0;
                uint8_t* q0;
                int step;
                if (dir == 0) {
                  q0 = &pl[static_cast<size_t>(my * 8 + i) * cw + mx * 8 + ce * 4];
                  step = 1;
                } else {
                  q0 = &pl[static_cast<size_t>(my * 8 + ce * 4) * cw + mx * 8 + i];
                  step = cw;
                }
                filter_line(q0, step, bs, ac, bc, tc0, true);
              }
            }
          }
        }
      }
    }
  }
};

Decoder::Decoder() : impl_(new Impl) {}
Decoder::~Decoder() = default;

void Decoder::decode(const uint8_t* data, size_t n) {
  impl_->skip_deblock = skip_deblock_;
  std::vector<NalUnit> nals = parse_annexb(data, n);
  for (NalUnit& u : nals) {
    switch (u.nal_unit_type) {
      case NAL_SPS: {
        BitReader br(u.rbsp.data(), u.rbsp.size());
        SPS s = parse_sps(br);
        impl_->sps[s.sps_id] = s;
        impl_->have_sps[s.sps_id] = true;
        break;
      }
      case NAL_PPS: {
        BitReader br(u.rbsp.data(), u.rbsp.size());
        PPS p = parse_pps(br, impl_->sps);
        impl_->pps[p.pps_id] = p;
        impl_->have_pps[p.pps_id] = true;
        break;
      }
      case NAL_SLICE:
      case NAL_IDR:
        impl_->decode_slice(u, out_);
        break;
      case NAL_AUD:
        impl_->finish_picture(out_);
        break;
      default:
        break;
    }
  }
}

void Decoder::flush() { impl_->finish_picture(out_); }

void Decoder::set_parse_only(bool v) { impl_->parse_only = v; }

}  // namespace h264
}  // namespace mivc
