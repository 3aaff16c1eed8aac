// HEVC syntax exerciser: random but conformant Main / Main 10 bitstreams that use every
// coding tool the general decoder (hevc_dec.cc) supports and the production encoder does
// not emit -- B slices (TMVP, combined merge candidates, mvd_l1_zero), every PartMode incl.
// AMP, CTB 16 / 32 / 64, the full transform tree, transform_skip, cu_transquant_bypass,
// PCM, scaling lists, long-term references, list modification, weighted prediction,
// several slices and dependent slice segments, tiles, WPP, deblocking overrides, SAO.
//
// Every decision is random; the writer only tracks what syntax parsing depends on
// (context selection, MPM candidates for the scan order, the transform tree rules), so the
// decoded pictures are noise -- the point is a stream the CPU decoder and the gfx950
// reconstruction (hevc_decode.hip) must reproduce bit-exactly (tests/test_gpu_hevc_decode.py).
// No external HEVC encoder or decoder exists in this image to produce such streams.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <random>
#include <stdexcept>
#include <vector>

#include "bitstream.h"
#include "hevc_cabac.h"
#include "hevc_codec.h"
#include "hevc_ctx_tables.h"
#include "hevc_dec_ps.h"

namespace mivc {
namespace hevc {

using dec::kNumDCtx;
using namespace dec;

namespace {

void put_nal(std::vector<uint8_t>& out, int type, const std::vector<uint8_t>& rbsp) {
  static const uint8_t sc[4] = {0, 0, 0, 1};
  out.insert(out.end(), sc, sc + 4);
  out.push_back(static_cast<uint8_t>(type << 1));
  out.push_back(1);  // nuh_layer_id 0, nuh_temporal_id_plus1 1
  int zeros = 0;
  for (uint8_t b : rbsp) {
    if (zeros >= 2 && b <= 3) {
      out.push_back(3);
      zeros = 0;
    }
    out.push_back(b);
    zeros = b == 0 ? zeros + 1 : 0;
  }
}

int count_epb(const std::vector<uint8_t>& b) {
  int zeros = 0, n = 0;
  for (uint8_t c : b) {
    if (zeros >= 2 && c <= 3) {
      ++n;
      zeros = 0;
    }
    zeros = c == 0 ? zeros + 1 : 0;
  }
  return n;
}

void init_states(CtxState* c, int init_type, int qp) {
  CtxS t[kNumDCtx];
  init_ctx(t, init_type, qp);
  for (int i = 0; i < kNumDCtx; ++i) {
    c[i].state = t[i].state;
    c[i].mps = t[i].mps;
  }
}

int ceil_log2(int v) {
  int n = 0;
  while ((1 << n) < v) ++n;
  return n;
}

uint32_t zorder(int bx, int by) {
  uint32_t z = 0;
  for (int i = 0; i < 4; ++i) z |= static_cast<uint32_t>(((bx >> i) & 1) << (2 * i)) | static_cast<uint32_t>(((by >> i) & 1) << (2 * i + 1));
  return z;
}

struct Rng {
  std::mt19937 g;
  explicit Rng(uint32_t s) : g(s) {}
  int r(int lo, int hi) { return std::uniform_int_distribution<int>(lo, hi)(g); }  // inclusive
  bool p(double prob) { return std::uniform_real_distribution<double>(0.0, 1.0)(g) < prob; }
};

struct Cfg {
  int bd = 8, W = 64, H = 64, conf[4] = {0, 0, 0, 0};
  int log2_ctb = 5, log2_min_cb = 3, log2_max_tb = 5, depth_inter = 1, depth_intra = 1;
  bool amp = true, sao = true, pcm = false, scaling = false, sps_lists = false, pps_lists = false, strong = true,
       tmvp = true, long_term = false;
  int pcm_bd = 8, pcm_bd_c = 8, log2_min_pcm = 3, log2_max_pcm = 3;
  bool pcm_lf_disabled = false;
  // PPS
  bool dep_slices = false, output_flag = false, sdh = false, cabac_init_present = false, cip = false, tskip = false,
       cu_qp_delta = false, slice_chroma = false, wp = false, wbp = false, bypass = false, tiles = false, wpp = false,
       lf_tiles = true, lf_slices = false, dbk_ctrl = false, dbk_override = false, dbk_disabled = false, lists_mod = false;
  int extra_bits = 0, num_ref_l0 = 1, num_ref_l1 = 1, init_qp = 30, qp_depth = 0, cb_off = 0, cr_off = 0;
  int beta = 0, tc = 0, par_mrg = 2;
  int tile_cols = 1, tile_rows = 1;
  bool uniform = true;
  std::vector<int> col_w, row_h;
  int log2_poc = 8;
};

// one scaling_list_data() with random lists (some predicted / default)
void write_scaling(BitWriter& bw, Rng& R) {
  for (int sid = 0; sid < 4; ++sid) {
    const int coefs = std::min(64, 1 << (4 + (sid << 1)));
    for (int m = 0; m < 6; m += sid == 3 ? 3 : 1) {
      if (R.p(0.3)) {
        bw.put_bit(0);
        const int maxd = sid == 3 ? m / 3 : m;
        bw.put_ue(static_cast<uint32_t>(R.r(0, maxd)));
        continue;
      }
      bw.put_bit(1);
      int next = 8;
      if (sid > 1) {
        const int dc = R.r(4, 60);
        bw.put_se(dc - 8);
        next = dc;
      }
      for (int i = 0; i < coefs; ++i) {
        const int want = R.r(4, 64);
        int d = want - next;
        if (d > 127) d -= 256;
        if (d < -128) d += 256;
        bw.put_se(d);
        next = (next + d + 256) % 256;
      }
    }
  }
}

struct Pic {
  int poc = 0;
  bool lt = false;
};

class Exerciser {
 public:
  explicit Exerciser(uint32_t seed) : R(seed ^ 0x9E3779B9u) {}

  std::vector<uint8_t> run() {
    choose_config();
    write_parameter_sets();
    const int npics = R.r(3, 7);
    // decoding order of POCs: anchors every 2..4 with the pictures between them afterwards
    std::vector<int> order = {0};
    int anchor = 0;
    while (static_cast<int>(order.size()) < npics) {
      const int step = R.r(1, 4);
      const int next = anchor + step;
      order.push_back(next);
      for (int p = anchor + 1; p < next && static_cast<int>(order.size()) < npics; ++p) order.push_back(p);
      anchor = next;
    }
    for (size_t i = 0; i < order.size(); ++i) write_picture(static_cast<int>(i), order[i]);
    return out;
  }

 private:
  Rng R;
  Cfg c;
  std::vector<uint8_t> out;
  std::vector<Pic> dpb;
  // picture geometry
  int wctb = 0, hctb = 0, nctb = 0, w4 = 0, h4 = 0, ctb = 32, l4 = 3;
  std::vector<int> rs2ts, ts2rs, tile_id, col_bd, row_bd;
  // per 4x4 state of the current picture
  std::vector<uint8_t> depth, skip, intra, pcm, mode, done;
  std::vector<int> ctb_slice;  // SliceAddrRs of each CTB (-1: not coded yet)
  // slice
  int slice_type = 2, slice_addr = 0, max_merge = 5, num_ref[2] = {0, 0}, slice_qp = 30, init_type = 0;
  bool sao_y = false, sao_c = false, mvd_l1_zero = false;
  CtxState ctx[kNumDCtx], wpp_ctx[kNumDCtx], ds_ctx[kNumDCtx];
  bool wpp_saved = false;
  CabacEncoder* enc = nullptr;
  BitWriter* bwp = nullptr;
  int qp_cur = 30, qg_log2 = 6;
  bool qp_coded = false;
  int cu_log2 = 3, cu_part = 0, chroma_mode = 0;
  bool cu_intra = false, cu_bypass = false;
  int pu_modes[4] = {1, 1, 1, 1};

  // ------------------------------------------------------------------ configuration
  void choose_config() {
    c.bd = R.p(0.4) ? 10 : 8;
    c.log2_ctb = R.r(4, 6);
    c.log2_min_cb = R.r(3, std::min(c.log2_ctb, 4));
    c.log2_max_tb = R.r(3, std::min(c.log2_ctb, 5));
    c.depth_inter = R.r(0, std::min(2, c.log2_ctb - 2));
    c.depth_intra = R.r(0, std::min(2, c.log2_ctb - 2));
    const int mcb = 1 << c.log2_min_cb;
    c.W = mcb * R.r(std::max(2, 24 / mcb), 176 / mcb);
    c.H = mcb * R.r(std::max(2, 16 / mcb), 120 / mcb);
    if (R.p(0.3)) {
      c.conf[1] = R.r(0, 3);
      c.conf[3] = R.r(0, 3);
    }
    c.amp = R.p(0.7);
    c.sao = R.p(0.7);
    c.pcm = R.p(0.3);
    c.log2_min_pcm = R.r(3, std::min(c.log2_ctb, 5));
    c.log2_max_pcm = R.r(c.log2_min_pcm, std::min(c.log2_ctb, 5));
    c.pcm_bd = R.r(4, c.bd);
    c.pcm_bd_c = R.r(4, c.bd);
    c.pcm_lf_disabled = R.p(0.5);
    c.scaling = R.p(0.35);
    c.sps_lists = c.scaling && R.p(0.5);
    c.pps_lists = c.scaling && R.p(0.5);
    c.strong = R.p(0.6);
    c.tmvp = R.p(0.7);
    c.long_term = R.p(0.4);
    c.log2_poc = R.r(4, 8);
    c.dep_slices = R.p(0.4);
    c.output_flag = R.p(0.3);
    c.extra_bits = R.r(0, 2);
    c.sdh = R.p(0.5);
    c.cabac_init_present = R.p(0.5);
    c.num_ref_l0 = R.r(1, 3);
    c.num_ref_l1 = R.r(1, 3);
    c.init_qp = R.r(22, 38);
    c.cip = R.p(0.25);
    c.tskip = R.p(0.5);
    c.cu_qp_delta = R.p(0.5);
    c.qp_depth = R.r(0, c.log2_ctb - c.log2_min_cb);
    c.cb_off = R.r(-4, 4);
    c.cr_off = R.r(-4, 4);
    c.slice_chroma = R.p(0.4);
    c.wp = R.p(0.4);
    c.wbp = R.p(0.4);
    c.bypass = R.p(0.3);
    const int ctbs = 1 << c.log2_ctb;
    const int wc = (c.W + ctbs - 1) / ctbs, hc = (c.H + ctbs - 1) / ctbs;
    c.tiles = (wc > 1 || hc > 1) && R.p(0.4);
    if (c.tiles) {
      c.tile_cols = R.r(1, std::min(wc, 3));
      c.tile_rows = R.r(1, std::min(hc, 3));
      if (c.tile_cols * c.tile_rows == 1) c.tiles = false;
      c.uniform = R.p(0.5);
      if (!c.uniform) {
        int left = wc;
        for (int i = 0; i < c.tile_cols - 1; ++i) {
          const int w = R.r(1, left - (c.tile_cols - 1 - i));
          c.col_w.push_back(w);
          left -= w;
        }
        left = hc;
        for (int j = 0; j < c.tile_rows - 1; ++j) {
          const int h = R.r(1, left - (c.tile_rows - 1 - j));
          c.row_h.push_back(h);
          left -= h;
        }
      }
      c.lf_tiles = R.p(0.5);
    }
    c.wpp = !c.tiles && R.p(0.4);
    c.lf_slices = R.p(0.5);
    c.dbk_ctrl = R.p(0.6);
    c.dbk_override = c.dbk_ctrl && R.p(0.5);
    c.dbk_disabled = c.dbk_ctrl && R.p(0.2);
    c.beta = R.r(-6, 6);
    c.tc = R.r(-6, 6);
    c.lists_mod = R.p(0.5);
    c.par_mrg = R.r(2, c.log2_ctb);
  }

  void write_ptl(BitWriter& bw) {
    bw.put(0, 2);
    bw.put(0, 1);
    const int prof = c.bd > 8 ? 2 : 1;
    bw.put(prof, 5);
    for (int j = 0; j < 32; ++j) bw.put_bit(j == prof || (prof == 1 && j == 2));
    bw.put_bit(1);
    bw.put_bit(0);
    bw.put_bit(0);
    bw.put_bit(1);
    bw.put(0, 32);
    bw.put(0, 12);
    bw.put(186, 8);
  }

  void write_parameter_sets() {
    {  // VPS
      BitWriter bw;
      bw.put(0, 4);
      bw.put(1, 1);
      bw.put(1, 1);
      bw.put(0, 6);
      bw.put(0, 3);
      bw.put(1, 1);
      bw.put(0xFFFF, 16);
      write_ptl(bw);
      bw.put_bit(1);
      bw.put_ue(5);
      bw.put_ue(4);
      bw.put_ue(0);
      bw.put(0, 6);
      bw.put_ue(0);
      bw.put_bit(0);
      bw.put_bit(0);
      bw.trailing();
      put_nal(out, VPS_NUT, bw.bytes());
    }
    {  // SPS
      BitWriter bw;
      bw.put(0, 4);
      bw.put(0, 3);
      bw.put(1, 1);
      write_ptl(bw);
      bw.put_ue(0);
      bw.put_ue(1);
      bw.put_ue(static_cast<uint32_t>(c.W));
      bw.put_ue(static_cast<uint32_t>(c.H));
      const bool conf = c.conf[1] || c.conf[3];
      bw.put_bit(conf);
      if (conf) {
        bw.put_ue(0);
        bw.put_ue(static_cast<uint32_t>(c.conf[1]));
        bw.put_ue(0);
        bw.put_ue(static_cast<uint32_t>(c.conf[3]));
      }
      bw.put_ue(static_cast<uint32_t>(c.bd - 8));
      bw.put_ue(static_cast<uint32_t>(c.bd - 8));
      bw.put_ue(static_cast<uint32_t>(c.log2_poc - 4));
      bw.put_bit(1);
      bw.put_ue(5);
      bw.put_ue(4);
      bw.put_ue(0);
      bw.put_ue(static_cast<uint32_t>(c.log2_min_cb - 3));
      bw.put_ue(static_cast<uint32_t>(c.log2_ctb - c.log2_min_cb));
      bw.put_ue(0);  // log2_min_luma_transform_block_size_minus2 (4x4)
      bw.put_ue(static_cast<uint32_t>(c.log2_max_tb - 2));
      bw.put_ue(static_cast<uint32_t>(c.depth_inter));
      bw.put_ue(static_cast<uint32_t>(c.depth_intra));
      bw.put_bit(c.scaling);
      if (c.scaling) {
        bw.put_bit(c.sps_lists);
        if (c.sps_lists) write_scaling(bw, R);
      }
      bw.put_bit(c.amp);
      bw.put_bit(c.sao);
      bw.put_bit(c.pcm);
      if (c.pcm) {
        bw.put(static_cast<uint32_t>(c.pcm_bd - 1), 4);
        bw.put(static_cast<uint32_t>(c.pcm_bd_c - 1), 4);
        bw.put_ue(static_cast<uint32_t>(c.log2_min_pcm - 3));
        bw.put_ue(static_cast<uint32_t>(c.log2_max_pcm - c.log2_min_pcm));
        bw.put_bit(c.pcm_lf_disabled);
      }
      // short-term RPS candidates (parsed, incl. inter-RPS prediction; slices code their own)
      const int nst = R.r(0, 3);
      num_sps_st_ = nst;
      bw.put_ue(static_cast<uint32_t>(nst));
      std::vector<int> prev;  // deltas of the previous set (inter prediction refers to it)
      for (int i = 0; i < nst; ++i) {
        const bool inter = i > 0 && R.p(0.5) && prev.size() < 8;
        if (i > 0) bw.put_bit(inter);
        std::vector<int> cur;
        if (inter) {
          const int sign = R.p(0.5), mag = R.r(1, 3), drps = sign ? -mag : mag;
          bw.put_bit(sign);
          bw.put_ue(static_cast<uint32_t>(mag - 1));
          for (size_t j = 0; j <= prev.size(); ++j) {
            const bool used = R.p(0.5);
            bw.put_bit(used);
            bool use_delta = true;
            if (!used) {
              use_delta = R.p(0.5);
              bw.put_bit(use_delta);
            }
            const int dp = j < prev.size() ? prev[j] + drps : drps;
            if (use_delta && dp != 0) cur.push_back(dp);
          }
        } else {
          const int nn = R.r(0, 3), np = R.r(0, 2);
          bw.put_ue(static_cast<uint32_t>(nn));
          bw.put_ue(static_cast<uint32_t>(np));
          int acc = 0;
          for (int k = 0; k < nn; ++k) {
            const int d = R.r(0, 2);
            bw.put_ue(static_cast<uint32_t>(d));
            bw.put_bit(R.p(0.5));
            acc -= d + 1;
            cur.push_back(acc);
          }
          acc = 0;
          for (int k = 0; k < np; ++k) {
            const int d = R.r(0, 2);
            bw.put_ue(static_cast<uint32_t>(d));
            bw.put_bit(R.p(0.5));
            acc += d + 1;
            cur.push_back(acc);
          }
        }
        prev = cur;
      }
      bw.put_bit(c.long_term);
      if (c.long_term) {
        const int n = R.r(0, 2);
        num_sps_lt_ = n;
        bw.put_ue(static_cast<uint32_t>(n));
        for (int i = 0; i < n; ++i) {
          bw.put(static_cast<uint32_t>(R.r(0, (1 << c.log2_poc) - 1)), c.log2_poc);
          bw.put_bit(R.p(0.5));
        }
      }
      bw.put_bit(c.tmvp);
      bw.put_bit(c.strong);
      bw.put_bit(0);  // vui
      bw.put_bit(0);  // extensions
      bw.trailing();
      put_nal(out, SPS_NUT, bw.bytes());
    }
    {  // PPS
      BitWriter bw;
      bw.put_ue(0);
      bw.put_ue(0);
      bw.put_bit(c.dep_slices);
      bw.put_bit(c.output_flag);
      bw.put(static_cast<uint32_t>(c.extra_bits), 3);
      bw.put_bit(c.sdh);
      bw.put_bit(c.cabac_init_present);
      bw.put_ue(static_cast<uint32_t>(c.num_ref_l0 - 1));
      bw.put_ue(static_cast<uint32_t>(c.num_ref_l1 - 1));
      bw.put_se(c.init_qp - 26);
      bw.put_bit(c.cip);
      bw.put_bit(c.tskip);
      bw.put_bit(c.cu_qp_delta);
      if (c.cu_qp_delta) bw.put_ue(static_cast<uint32_t>(c.qp_depth));
      bw.put_se(c.cb_off);
      bw.put_se(c.cr_off);
      bw.put_bit(c.slice_chroma);
      bw.put_bit(c.wp);
      bw.put_bit(c.wbp);
      bw.put_bit(c.bypass);
      bw.put_bit(c.tiles);
      bw.put_bit(c.wpp);
      if (c.tiles) {
        bw.put_ue(static_cast<uint32_t>(c.tile_cols - 1));
        bw.put_ue(static_cast<uint32_t>(c.tile_rows - 1));
        bw.put_bit(c.uniform);
        if (!c.uniform) {
          for (int w : c.col_w) bw.put_ue(static_cast<uint32_t>(w - 1));
          for (int h : c.row_h) bw.put_ue(static_cast<uint32_t>(h - 1));
        }
        bw.put_bit(c.lf_tiles);
      }
      bw.put_bit(c.lf_slices);
      bw.put_bit(c.dbk_ctrl);
      if (c.dbk_ctrl) {
        bw.put_bit(c.dbk_override);
        bw.put_bit(c.dbk_disabled);
        if (!c.dbk_disabled) {
          bw.put_se(c.beta);
          bw.put_se(c.tc);
        }
      }
      bw.put_bit(c.pps_lists);
      if (c.pps_lists) write_scaling(bw, R);
      bw.put_bit(c.lists_mod);
      bw.put_ue(static_cast<uint32_t>(c.par_mrg - 2));
      bw.put_bit(0);  // slice_segment_header_extension_present_flag
      bw.put_bit(0);  // pps_extension_present_flag
      bw.trailing();
      put_nal(out, PPS_NUT, bw.bytes());
    }
    // geometry + tile scan (6.5.1)
    ctb = 1 << c.log2_ctb;
    l4 = c.log2_ctb - 2;
    wctb = (c.W + ctb - 1) / ctb;
    hctb = (c.H + ctb - 1) / ctb;
    nctb = wctb * hctb;
    w4 = c.W / 4;
    h4 = c.H / 4;
    const int cols = c.tiles ? c.tile_cols : 1, rows = c.tiles ? c.tile_rows : 1;
    std::vector<int> cw(cols), rh(rows);
    if (!c.tiles || c.uniform) {
      for (int i = 0; i < cols; ++i) cw[i] = ((i + 1) * wctb) / cols - (i * wctb) / cols;
      for (int j = 0; j < rows; ++j) rh[j] = ((j + 1) * hctb) / rows - (j * hctb) / rows;
    } else {
      int acc = 0;
      for (int i = 0; i < cols - 1; ++i) acc += (cw[i] = c.col_w[i]);
      cw[cols - 1] = wctb - acc;
      acc = 0;
      for (int j = 0; j < rows - 1; ++j) acc += (rh[j] = c.row_h[j]);
      rh[rows - 1] = hctb - acc;
    }
    col_bd.assign(cols + 1, 0);
    row_bd.assign(rows + 1, 0);
    for (int i = 0; i < cols; ++i) col_bd[i + 1] = col_bd[i] + cw[i];
    for (int j = 0; j < rows; ++j) row_bd[j + 1] = row_bd[j] + rh[j];
    rs2ts.assign(nctb, 0);
    ts2rs.assign(nctb, 0);
    tile_id.assign(nctb, 0);
    for (int rs = 0; rs < nctb; ++rs) {
      const int tbx = rs % wctb, tby = rs / wctb;
      int tx = 0, ty = 0;
      for (int i = 0; i < cols; ++i)
        if (tbx >= col_bd[i]) tx = i;
      for (int j = 0; j < rows; ++j)
        if (tby >= row_bd[j]) ty = j;
      int v = 0;
      for (int i = 0; i < tx; ++i) v += rh[ty] * cw[i];
      for (int j = 0; j < ty; ++j) v += wctb * rh[j];
      v += (tby - row_bd[ty]) * cw[tx] + tbx - col_bd[tx];
      rs2ts[rs] = v;
      ts2rs[v] = rs;
      tile_id[v] = ty * cols + tx;
    }
  }

  int tile_col_start(int x) const {
    int s = 0;
    for (size_t i = 0; i + 1 < col_bd.size(); ++i)
      if (x >= col_bd[i]) s = col_bd[i];
    return s;
  }

  // ------------------------------------------------------------------ picture
  void write_picture(int idx, int poc) {
    const bool idr = idx == 0;
    const size_t n4 = static_cast<size_t>(w4) * h4;
    depth.assign(n4, 0);
    skip.assign(n4, 0);
    intra.assign(n4, 0);
    pcm.assign(n4, 0);
    mode.assign(n4, 1);
    done.assign(n4, 0);
    ctb_slice.assign(nctb, -1);
    // reference picture set: every picture kept, some used; one may turn long-term
    std::vector<Pic> rps = dpb;
    if (idr) rps.clear();
    if (rps.size() > 4) {
      std::sort(rps.begin(), rps.end(), [](const Pic& a, const Pic& b) { return a.poc < b.poc; });
      rps.erase(rps.begin(), rps.begin() + static_cast<long>(rps.size() - 4));
    }
    if (c.long_term && rps.size() >= 2 && R.p(0.4)) {
      int oldest = 0;
      for (size_t i = 1; i < rps.size(); ++i)
        if (rps[i].poc < rps[oldest].poc) oldest = static_cast<int>(i);
      rps[oldest].lt = true;
    }
    std::vector<uint8_t> used(rps.size(), 0);
    int npc = 0;
    for (size_t i = 0; i < rps.size(); ++i) {
      used[i] = R.p(0.7);
      npc += used[i];
    }
    if (!rps.empty() && npc == 0) {
      used[0] = 1;
      npc = 1;
    }
    const int pic_type = idr ? 2 : (npc == 0 ? 2 : (R.p(0.5) ? 0 : 1));  // slice type of this picture's slices
    const bool pic_tmvp = c.tmvp && !idr && R.p(0.8);
    pic_output = R.p(0.8);
    // slice segments: boundaries in tile-scan order
    std::vector<int> starts = {0};
    std::vector<bool> dep = {false};
    for (int ts = 1; ts < nctb; ++ts) {
      const int rs = ts2rs[ts];
      bool allowed;
      if (c.tiles) allowed = tile_id[ts] != tile_id[ts - 1];  // slices hold whole tiles
      else if (c.wpp) allowed = (rs % wctb) == 0;           // WPP: segments start at row starts
      else allowed = true;
      if (allowed && R.p(c.tiles ? 0.5 : 0.12)) {
        starts.push_back(ts);
        dep.push_back(c.dep_slices && R.p(0.5));
      }
    }
    starts.push_back(nctb);
    int col_ref_poc = -1;
    SliceState indep;
    for (size_t s = 0; s + 1 < starts.size(); ++s)
      write_slice(idx, poc, idr, rps, used, npc, pic_type, pic_tmvp, starts[s], starts[s + 1], dep[s], s == 0, indep,
                  col_ref_poc);
    // the picture joins the DPB; pictures not in this RPS are gone
    dpb = rps;
    dpb.push_back(Pic{poc, false});
  }

  struct SliceState {
    int type = 2, num_ref[2] = {0, 0}, max_merge = 5, qp = 30, cb = 0, cr = 0;
    bool sao_y = false, sao_c = false, mvd_l1_zero = false, cabac_init = false, dbk_off = false, lf = false;
    int beta = 0, tc = 0;
    int addr = 0;
  };

  void write_slice(int idx, int poc, bool idr, const std::vector<Pic>& rps, const std::vector<uint8_t>& used, int npc,
                   int pic_type, bool tmvp, int ts0, int ts1, bool dependent, bool first, SliceState& st,
                   int& col_ref_poc) {
    BitWriter bw;
    bw.put_bit(first);
    if (idr) bw.put_bit(0);  // no_output_of_prior_pics_flag
    bw.put_ue(0);
    if (!first) {
      if (c.dep_slices) bw.put_bit(dependent);
      bw.put(static_cast<uint32_t>(ts2rs[ts0]), ceil_log2(nctb));
    }
    if (!dependent) {
      st = SliceState();
      st.addr = ts2rs[ts0];
      for (int i = 0; i < c.extra_bits; ++i) bw.put_bit(R.p(0.5));
      st.type = pic_type;
      bw.put_ue(static_cast<uint32_t>(st.type));
      if (c.output_flag) bw.put_bit(pic_output);
      if (!idr) {
        bw.put(static_cast<uint32_t>(poc & ((1 << c.log2_poc) - 1)), c.log2_poc);
        bw.put_bit(0);  // short_term_ref_pic_set_sps_flag: explicit set
        // st_ref_pic_set(num_short_term_ref_pic_sets): never inter-predicted here
        std::vector<std::pair<int, int>> neg, pos;  // (delta, used)
        for (size_t i = 0; i < rps.size(); ++i) {
          if (rps[i].lt) continue;
          const int d = rps[i].poc - poc;
          (d < 0 ? neg : pos).push_back({d, used[i]});
        }
        std::sort(neg.begin(), neg.end(), [](auto& a, auto& b) { return a.first > b.first; });
        std::sort(pos.begin(), pos.end(), [](auto& a, auto& b) { return a.first < b.first; });
        if (num_sps_st() > 0) bw.put_bit(0);  // inter_ref_pic_set_prediction_flag
        bw.put_ue(static_cast<uint32_t>(neg.size()));
        bw.put_ue(static_cast<uint32_t>(pos.size()));
        int prev = 0;
        for (auto& e : neg) {
          bw.put_ue(static_cast<uint32_t>(prev - e.first - 1));
          bw.put_bit(e.second);
          prev = e.first;
        }
        prev = 0;
        for (auto& e : pos) {
          bw.put_ue(static_cast<uint32_t>(e.first - prev - 1));
          bw.put_bit(e.second);
          prev = e.first;
        }
        if (c.long_term) {
          if (num_sps_lt() > 0) bw.put_ue(0);  // num_long_term_sps
          std::vector<std::pair<int, int>> lts;
          for (size_t i = 0; i < rps.size(); ++i)
            if (rps[i].lt) lts.push_back({rps[i].poc, used[i]});
          // decreasing POC: the MSB cycles are non-decreasing, so their differences are >= 0
          std::sort(lts.begin(), lts.end(), [](auto& a, auto& b) { return a.first > b.first; });
          bw.put_ue(static_cast<uint32_t>(lts.size()));
          const int maxlsb = 1 << c.log2_poc;
          int prev_cycle = 0;
          for (size_t i = 0; i < lts.size(); ++i) {
            bw.put(static_cast<uint32_t>(lts[i].first & (maxlsb - 1)), c.log2_poc);
            bw.put_bit(lts[i].second);
            bw.put_bit(1);  // delta_poc_msb_present_flag
            // DeltaPocMsbCycleLt = (POCcur msb - POClt msb) / MaxLsb, coded differentially
            const int cyc = ((poc - (poc & (maxlsb - 1))) - (lts[i].first - (lts[i].first & (maxlsb - 1)))) / maxlsb;
            bw.put_ue(static_cast<uint32_t>(i == 0 ? cyc : cyc - prev_cycle));
            prev_cycle = cyc;
          }
        }
        if (c.tmvp) bw.put_bit(tmvp);
      }
      if (c.sao) {
        st.sao_y = R.p(0.7);
        st.sao_c = R.p(0.7);
        bw.put_bit(st.sao_y);
        bw.put_bit(st.sao_c);
      }
      if (st.type != 2) {
        st.num_ref[0] = c.num_ref_l0;
        st.num_ref[1] = st.type == 0 ? c.num_ref_l1 : 0;
        // with TMVP every slice must reach the picture's collocated picture: L0 then holds
        // every used picture (num_ref_idx_l0 >= NumPicTotalCurr, no modification of L0)
        const bool ovr = tmvp || R.p(0.5);
        bw.put_bit(ovr);
        if (ovr) {
          st.num_ref[0] = R.r(1, std::min(4, 2 * npc));
          if (tmvp) st.num_ref[0] = std::max(st.num_ref[0], npc);
          bw.put_ue(static_cast<uint32_t>(st.num_ref[0] - 1));
          if (st.type == 0) {
            st.num_ref[1] = R.r(1, std::min(4, 2 * npc));
            bw.put_ue(static_cast<uint32_t>(st.num_ref[1] - 1));
          }
        }
        // reference lists (8.3.4) as POCs, for the collocated picture constraint
        std::vector<int> before, after, lt;
        for (size_t i = 0; i < rps.size(); ++i) {
          if (!used[i]) continue;
          if (rps[i].lt) lt.push_back(rps[i].poc);
          else (rps[i].poc < poc ? before : after).push_back(rps[i].poc);
        }
        std::sort(before.begin(), before.end(), [](int a, int b) { return a > b; });
        std::sort(after.begin(), after.end());
        // LT order follows the slice header order (decreasing POC)
        std::sort(lt.begin(), lt.end(), [](int a, int b) { return a > b; });
        std::vector<int> lists[2];
        for (int l = 0; l < (st.type == 0 ? 2 : 1); ++l) {
          std::vector<int> tmp;
          const int n = std::max(st.num_ref[l], npc);
          while (static_cast<int>(tmp.size()) < n) {
            auto& a = l == 0 ? before : after;
            auto& b = l == 0 ? after : before;
            for (int v : a)
              if (static_cast<int>(tmp.size()) < n) tmp.push_back(v);
            for (int v : b)
              if (static_cast<int>(tmp.size()) < n) tmp.push_back(v);
            for (int v : lt)
              if (static_cast<int>(tmp.size()) < n) tmp.push_back(v);
          }
          std::vector<int> entry(st.num_ref[l]);
          bool mod = false;
          if (c.lists_mod && npc > 1) {
            mod = !(tmvp && l == 0) && R.p(0.5);
            bw.put_bit(mod);
          }
          for (int i = 0; i < st.num_ref[l]; ++i) {
            entry[i] = mod ? R.r(0, npc - 1) : i;
            if (mod) bw.put(static_cast<uint32_t>(entry[i]), ceil_log2(npc));
            lists[l].push_back(tmp[entry[i]]);
          }
        }
        if (st.type == 0) {
          st.mvd_l1_zero = R.p(0.3);
          bw.put_bit(st.mvd_l1_zero);
        }
        if (c.cabac_init_present) {
          st.cabac_init = R.p(0.5);
          bw.put_bit(st.cabac_init);
        }
        if (tmvp) {
          // every slice of the picture collocates with the same picture
          int from_l0 = 1, ref_idx = 0;
          bool found = false;
          for (int tries = 0; tries < 8 && !found; ++tries) {
            from_l0 = st.type == 0 ? R.r(0, 1) : 1;
            const auto& L = lists[from_l0 ? 0 : 1];
            ref_idx = R.r(0, static_cast<int>(L.size()) - 1);
            if (col_ref_poc < 0 || L[ref_idx] == col_ref_poc) found = true;
          }
          if (!found) {
            for (int l = 0; l < (st.type == 0 ? 2 : 1) && !found; ++l)
              for (size_t i = 0; i < lists[l].size() && !found; ++i)
                if (lists[l][i] == col_ref_poc) {
                  from_l0 = l == 0;
                  ref_idx = static_cast<int>(i);
                  found = true;
                }
          }
          if (!found) throw std::runtime_error("exerciser: collocated picture not in this slice's lists");
          col_ref_poc = lists[from_l0 ? 0 : 1][ref_idx];
          if (st.type == 0) bw.put_bit(from_l0);
          if (st.num_ref[from_l0 ? 0 : 1] > 1) bw.put_ue(static_cast<uint32_t>(ref_idx));
        }
        if ((c.wp && st.type == 1) || (c.wbp && st.type == 0)) {
          const int dy = R.r(0, 7);
          bw.put_ue(static_cast<uint32_t>(dy));
          const int dc = R.r(0, 7) - dy;
          bw.put_se(dc);
          for (int l = 0; l < (st.type == 0 ? 2 : 1); ++l) {
            std::vector<int> lf(st.num_ref[l]), cf(st.num_ref[l]);
            for (int i = 0; i < st.num_ref[l]; ++i) bw.put_bit(lf[i] = R.p(0.6));
            for (int i = 0; i < st.num_ref[l]; ++i) bw.put_bit(cf[i] = R.p(0.6));
            for (int i = 0; i < st.num_ref[l]; ++i) {
              if (lf[i]) {
                bw.put_se(R.r(-40, 40));
                bw.put_se(R.r(-60, 60));
              }
              if (cf[i])
                for (int j = 0; j < 2; ++j) {
                  bw.put_se(R.r(-40, 40));
                  bw.put_se(R.r(-100, 100));
                }
            }
          }
        }
        st.max_merge = R.r(1, 5);
        bw.put_ue(static_cast<uint32_t>(5 - st.max_merge));
      }
      const int qd = R.r(-4, 4);
      st.qp = c.init_qp + qd;
      bw.put_se(qd);
      if (c.slice_chroma) {
        st.cb = R.r(-3, 3);
        st.cr = R.r(-3, 3);
        bw.put_se(st.cb);
        bw.put_se(st.cr);
      }
      st.dbk_off = c.dbk_disabled;
      if (c.dbk_override) {
        const bool ov = R.p(0.5);
        bw.put_bit(ov);
        if (ov) {
          st.dbk_off = R.p(0.3);
          bw.put_bit(st.dbk_off);
          if (!st.dbk_off) {
            bw.put_se(R.r(-6, 6));
            bw.put_se(R.r(-6, 6));
          }
        }
      }
      st.lf = c.lf_slices;
      if (c.lf_slices && (st.sao_y || st.sao_c || !st.dbk_off)) {
        st.lf = R.p(0.5);
        bw.put_bit(st.lf);
      }
    }
    // slice data into substreams
    slice_type = st.type;
    slice_addr = st.addr;
    num_ref[0] = st.num_ref[0];
    num_ref[1] = st.num_ref[1];
    max_merge = st.max_merge;
    slice_qp = st.qp;
    sao_y = st.sao_y;
    sao_c = st.sao_c;
    mvd_l1_zero = st.mvd_l1_zero;
    init_type = st.type == 2 ? 0 : (st.type == 1 ? (st.cabac_init ? 2 : 1) : (st.cabac_init ? 1 : 2));
    std::vector<std::vector<uint8_t>> subs;
    write_slice_data(ts0, ts1, dependent, subs);
    if (c.tiles || c.wpp) {
      bw.put_ue(static_cast<uint32_t>(subs.size() - 1));
      if (subs.size() > 1) {
        uint32_t mx = 1;
        for (size_t i = 0; i + 1 < subs.size(); ++i)
          mx = std::max<uint32_t>(mx, static_cast<uint32_t>(subs[i].size() + count_epb(subs[i])));
        const int len = std::max(1, ceil_log2(static_cast<int>(mx)));
        bw.put_ue(static_cast<uint32_t>(len - 1));
        for (size_t i = 0; i + 1 < subs.size(); ++i)
          bw.put(static_cast<uint32_t>(subs[i].size() + count_epb(subs[i]) - 1), len);
      }
    }
    // byte_alignment()
    bw.put_bit(1);
    bw.align_zero();
    std::vector<uint8_t> rbsp = bw.bytes();
    for (auto& s : subs) rbsp.insert(rbsp.end(), s.begin(), s.end());
    const int type = idr ? IDR_W_RADL : TRAIL_R;
    put_nal(out, type, rbsp);
    (void)idx;
  }

  int num_sps_st_ = -1;
  int num_sps_st() {
    // the SPS written above: recover the count from the stream is overkill; track it instead
    return num_sps_st_;
  }
  int num_sps_lt() { return num_sps_lt_; }
  int num_sps_lt_ = 0;

  // ------------------------------------------------------------------ slice data
  void write_slice_data(int ts0, int ts1, bool dependent, std::vector<std::vector<uint8_t>>& subs) {
    BitWriter* bw = new BitWriter();
    CabacEncoder* ce = new CabacEncoder(*bw);
    bwp = bw;
    enc = ce;
    enc->start();
    start_contexts(ts0, true, dependent);
    for (int ts = ts0; ts < ts1; ++ts) {
      const int rs = ts2rs[ts];
      ctb_slice[rs] = slice_addr;
      write_ctu(rs, ts);
      const int rx = rs % wctb;
      if (c.wpp && rx == tile_col_start(rx) + 1) {
        std::copy(ctx, ctx + kNumDCtx, wpp_ctx);
        wpp_saved = true;
      }
      const bool last = ts + 1 == ts1;
      enc->terminate(last ? 1 : 0);
      if (last) {
        if (c.dep_slices) std::copy(ctx, ctx + kNumDCtx, ds_ctx);
        enc->finish();
        bw->put_bit(1);
        bw->align_zero();
        subs.push_back(bw->bytes());
        break;
      }
      const int nrs = ts2rs[ts + 1];
      const bool new_tile = c.tiles && tile_id[ts + 1] != tile_id[ts];
      const bool new_row = c.wpp && (nrs % wctb) == tile_col_start(nrs % wctb);
      if (new_tile || new_row) {
        enc->terminate(1);  // end_of_subset_one_bit
        enc->finish();
        bw->put_bit(1);
        bw->align_zero();
        subs.push_back(bw->bytes());
        delete ce;
        delete bw;
        bw = new BitWriter();
        ce = new CabacEncoder(*bw);
        bwp = bw;
        enc = ce;
        enc->start();
        start_contexts(ts + 1, false, false);
      }
    }
    delete ce;
    delete bw;
    enc = nullptr;
    bwp = nullptr;
  }

  void start_contexts(int ts, bool slice_start, bool dependent) {
    const int rs = ts2rs[ts];
    const int rx = rs % wctb, ry = rs / wctb;
    const bool first_in_tile = ts == 0 || tile_id[ts] != tile_id[ts - 1];
    const bool row_start = rx == tile_col_start(rx);
    if (first_in_tile && (slice_start || c.tiles)) {
      init_states(ctx, init_type, slice_qp);
    } else if (c.wpp && row_start) {
      bool avail = false;
      if (ry > 0 && (rx + 1) * ctb < c.W) {
        const int nrs = (ry - 1) * wctb + rx + 1;
        avail = ctb_slice[nrs] == slice_addr;
      }
      if (avail && wpp_saved) std::copy(wpp_ctx, wpp_ctx + kNumDCtx, ctx);
      else init_states(ctx, init_type, slice_qp);
    } else if (slice_start && dependent) {
      std::copy(ds_ctx, ds_ctx + kNumDCtx, ctx);
    } else {
      init_states(ctx, init_type, slice_qp);
    }
    if ((slice_start && !dependent) || first_in_tile || (c.wpp && row_start)) qp_prev = slice_qp;
  }
  int qp_prev = 30;
  bool pic_output = true;

  // availability (6.4.1) for the context / MPM derivations
  size_t g4(int x, int y) const { return static_cast<size_t>(y >> 2) * w4 + (x >> 2); }
  uint32_t zaddr(int x, int y) const {
    const int rs = (y >> c.log2_ctb) * wctb + (x >> c.log2_ctb);
    const int m = (1 << l4) - 1;
    return (static_cast<uint32_t>(rs2ts[rs]) << (2 * l4)) | zorder((x >> 2) & m, (y >> 2) & m);
  }
  bool avail(int xc, int yc, int xn, int yn) const {
    if (xn < 0 || yn < 0 || xn >= c.W || yn >= c.H) return false;
    const int rsn = (yn >> c.log2_ctb) * wctb + (xn >> c.log2_ctb), rsc = (yc >> c.log2_ctb) * wctb + (xc >> c.log2_ctb);
    if (ctb_slice[rsn] < 0 || ctb_slice[rsn] != ctb_slice[rsc]) return false;
    if (tile_id[rs2ts[rsn]] != tile_id[rs2ts[rsc]]) return false;
    return zaddr(xn, yn) <= zaddr(xc, yc) && done[g4(xn, yn)];
  }

  // ------------------------------------------------------------------ CTU
  void bin(int b, int ci) { enc->encode(b, ctx[ci]); }
  void byp(int b) { enc->bypass(b); }
  void bypn(uint32_t v, int n) {
    for (int i = n - 1; i >= 0; --i) byp((v >> i) & 1);
  }

  std::vector<int8_t> sao_type_y, sao_type_c;
  void write_ctu(int rs, int ts) {
    const int rx = rs % wctb, ry = rs / wctb;
    (void)ts;
    if (sao_y || sao_c) write_sao(rs, rx, ry);
    coding_quadtree(rx * ctb, ry * ctb, c.log2_ctb, 0);
  }

  void write_sao(int rs, int rx, int ry) {
    const int ts = rs2ts[rs];
    if (rx > 0 && rs > slice_addr && tile_id[ts] == tile_id[rs2ts[rs - 1]]) {
      const bool m = R.p(0.3);
      bin(m, C_SAO_MERGE);
      if (m) return;
    }
    if (ry > 0 && rs - wctb >= slice_addr && tile_id[ts] == tile_id[rs2ts[rs - wctb]]) {
      const bool m = R.p(0.3);
      bin(m, C_SAO_MERGE);
      if (m) return;
    }
    int type_c = 0;
    for (int ci = 0; ci < 3; ++ci) {
      if ((ci == 0 && !sao_y) || (ci > 0 && !sao_c)) continue;
      int type = type_c;
      if (ci < 2) {
        type = R.r(0, 2);
        bin(type != 0, C_SAO_TYPE);
        if (type) byp(type == 2);
        if (ci == 1) type_c = type;
      }
      if (!type) continue;
      const int cmax = (1 << (std::min(c.bd, 10) - 5)) - 1;
      int a[4];
      for (int i = 0; i < 4; ++i) {
        a[i] = R.r(0, cmax);
        for (int k = 0; k < a[i]; ++k) byp(1);
        if (a[i] < cmax) byp(0);
      }
      if (type == 1) {
        for (int i = 0; i < 4; ++i)
          if (a[i]) byp(R.p(0.5));
        bypn(static_cast<uint32_t>(R.r(0, 31)), 5);
      } else if (ci < 2) {
        bypn(static_cast<uint32_t>(R.r(0, 3)), 2);
      }
    }
  }

  void coding_quadtree(int x0, int y0, int log2, int d) {
    const int n = 1 << log2;
    bool split;
    if (x0 + n <= c.W && y0 + n <= c.H && log2 > c.log2_min_cb) {
      int cnt = 0;
      if (avail(x0, y0, x0 - 1, y0) && depth[g4(x0 - 1, y0)] > d) ++cnt;
      if (avail(x0, y0, x0, y0 - 1) && depth[g4(x0, y0 - 1)] > d) ++cnt;
      split = R.p(log2 > 4 ? 0.6 : 0.35);
      bin(split, C_SPLIT_CU + cnt);
    } else {
      split = log2 > c.log2_min_cb;
    }
    if (c.cu_qp_delta && log2 >= c.log2_ctb - c.qp_depth) qp_coded = false;
    if (split) {
      const int h = n / 2;
      for (int q = 0; q < 4; ++q) {
        const int x1 = x0 + (q & 1) * h, y1 = y0 + (q >> 1) * h;
        if (x1 < c.W && y1 < c.H) coding_quadtree(x1, y1, log2 - 1, d + 1);
      }
      return;
    }
    coding_unit(x0, y0, log2, d);
  }

  void mark(int x0, int y0, int n, int d, bool sk, bool in, bool pc) {
    for (int y = y0; y < y0 + n && y < c.H; y += 4)
      for (int x = x0; x < x0 + n && x < c.W; x += 4) {
        const size_t k = g4(x, y);
        depth[k] = static_cast<uint8_t>(d);
        skip[k] = sk;
        intra[k] = in;
        pcm[k] = pc;
      }
  }
  void mark_done(int x0, int y0, int n) {
    for (int y = y0; y < y0 + n && y < c.H; y += 4)
      for (int x = x0; x < x0 + n && x < c.W; x += 4) done[g4(x, y)] = 1;
  }

  void coding_unit(int x0, int y0, int log2, int d) {
    const int n = 1 << log2;
    cu_log2 = log2;
    cu_bypass = false;
    if (c.bypass) {
      cu_bypass = R.p(0.2);
      bin(cu_bypass, C_TQ_BYPASS);
    }
    bool sk = false;
    if (slice_type != 2) {
      int cnt = 0;
      if (avail(x0, y0, x0 - 1, y0) && skip[g4(x0 - 1, y0)]) ++cnt;
      if (avail(x0, y0, x0, y0 - 1) && skip[g4(x0, y0 - 1)]) ++cnt;
      sk = R.p(0.25);
      bin(sk, C_SKIP + cnt);
    }
    if (sk) {
      mark(x0, y0, n, d, true, false, false);
      cu_intra = false;
      cu_part = 0;
      prediction_unit(x0, y0, n, n, true);
      mark_done(x0, y0, n);
      return;
    }
    cu_intra = slice_type == 2 || R.p(0.3);
    if (slice_type != 2) bin(cu_intra, C_PRED_MODE);
    cu_part = 0;  // PartMode as in hevc_dec.cc: 0 2Nx2N 1 2NxN 2 Nx2N 3 NxN 4 2NxnU 5 2NxnD 6 nLx2N 7 nRx2N
    if (cu_intra) {
      if (log2 == c.log2_min_cb) {
        cu_part = R.p(0.4) ? 3 : 0;
        bin(cu_part == 0, C_PART_MODE);
      }
    } else {
      std::vector<int> opts = {0, 1, 2};
      if (log2 == c.log2_min_cb && log2 > 3) opts.push_back(3);
      if (c.amp && log2 > c.log2_min_cb) {
        opts.push_back(4);
        opts.push_back(5);
        opts.push_back(6);
        opts.push_back(7);
      }
      cu_part = opts[R.r(0, static_cast<int>(opts.size()) - 1)];
      write_part_mode(cu_part, log2);
    }
    mark(x0, y0, n, d, false, cu_intra, false);
    bool is_pcm = false;
    if (cu_intra) {
      if (cu_part == 0 && c.pcm && log2 >= c.log2_min_pcm && log2 <= c.log2_max_pcm) {
        is_pcm = R.p(0.25);
        enc->terminate(is_pcm);
      }
      if (is_pcm) {
        mark(x0, y0, n, d, false, true, true);
        write_pcm(log2);
        mark_done(x0, y0, n);
        return;
      }
      write_intra_modes(x0, y0, log2);
    } else {
      const int h = n / 2, q = n / 4;
      switch (cu_part) {
        case 0: prediction_unit(x0, y0, n, n, false); break;
        case 1: prediction_unit(x0, y0, n, h, false); prediction_unit(x0, y0 + h, n, h, false); break;
        case 2: prediction_unit(x0, y0, h, n, false); prediction_unit(x0 + h, y0, h, n, false); break;
        case 4: prediction_unit(x0, y0, n, q, false); prediction_unit(x0, y0 + q, n, n - q, false); break;
        case 5: prediction_unit(x0, y0, n, n - q, false); prediction_unit(x0, y0 + n - q, n, q, false); break;
        case 6: prediction_unit(x0, y0, q, n, false); prediction_unit(x0 + q, y0, n - q, n, false); break;
        case 7: prediction_unit(x0, y0, n - q, n, false); prediction_unit(x0 + n - q, y0, q, n, false); break;
        default:
          prediction_unit(x0, y0, h, h, false);
          prediction_unit(x0 + h, y0, h, h, false);
          prediction_unit(x0, y0 + h, h, h, false);
          prediction_unit(x0 + h, y0 + h, h, h, false);
      }
    }
    bool root = true;
    if (!cu_intra && !(cu_part == 0 && last_merge)) {
      root = R.p(0.7);
      bin(root, C_ROOT_CBF);
    }
    if (root) {
      const int isplit = cu_intra && cu_part == 3;
      const int maxd = cu_intra ? c.depth_intra + isplit : c.depth_inter;
      transform_tree(x0, y0, x0, y0, log2, 0, 0, maxd, isplit, 1, 1);
    }
    mark_done(x0, y0, n);
  }

  void write_part_mode(int pm, int log2) {
    if (pm == 0) {
      bin(1, C_PART_MODE);
      return;
    }
    bin(0, C_PART_MODE);
    if (log2 == c.log2_min_cb) {
      if (pm == 1) {
        bin(1, C_PART_MODE + 1);
        return;
      }
      bin(0, C_PART_MODE + 1);
      if (log2 == 3) return;  // Nx2N
      bin(pm == 2, C_PART_MODE + 2);
      return;
    }
    if (!c.amp) {
      bin(pm == 1, C_PART_MODE + 1);
      return;
    }
    const bool hor = pm == 1 || pm == 4 || pm == 5;
    bin(hor, C_PART_MODE + 1);
    if (hor) {
      bin(pm == 1, C_PART_MODE + 3);
      if (pm != 1) byp(pm == 5);
    } else {
      bin(pm == 2, C_PART_MODE + 3);
      if (pm != 2) byp(pm == 7);
    }
  }

  void write_pcm(int log2) {
    enc->finish();
    bwp->put_bit(1);
    bwp->align_zero();
    const int n = 1 << log2, nc = n / 2;
    for (int i = 0; i < n * n; ++i) bwp->put(static_cast<uint32_t>(R.r(0, (1 << c.pcm_bd) - 1)), c.pcm_bd);
    for (int i = 0; i < 2 * nc * nc; ++i) bwp->put(static_cast<uint32_t>(R.r(0, (1 << c.pcm_bd_c) - 1)), c.pcm_bd_c);
    enc->start();
  }

  int mpm_cand(int xp, int yp, int xn, int yn, bool above) {
    if (!avail(xp, yp, xn, yn)) return 1;
    const size_t k = g4(xn, yn);
    if (!intra[k] || pcm[k]) return 1;
    if (above && yn < ((yp >> c.log2_ctb) << c.log2_ctb)) return 1;
    return mode[k];
  }
  void write_intra_modes(int x0, int y0, int log2) {
    const int n = 1 << log2;
    const int npu = cu_part == 3 ? 4 : 1, h = cu_part == 3 ? n / 2 : n;
    int prev[4], mi[4], rem[4];
    for (int k = 0; k < npu; ++k) {
      const int xp = x0 + (k & 1) * h, yp = y0 + (k >> 1) * h;
      const int a = mpm_cand(xp, yp, xp - 1, yp, false), b = mpm_cand(xp, yp, xp, yp - 1, true);
      int cl[3];
      if (a == b) {
        if (a < 2) {
          cl[0] = 0;
          cl[1] = 1;
          cl[2] = 26;
        } else {
          cl[0] = a;
          cl[1] = 2 + ((a + 29) % 32);
          cl[2] = 2 + ((a - 2 + 1) % 32);
        }
      } else {
        cl[0] = a;
        cl[1] = b;
        cl[2] = (a != 0 && b != 0) ? 0 : ((a != 1 && b != 1) ? 1 : 26);
      }
      const int m = R.r(0, 34);
      pu_modes[k] = m;
      prev[k] = 0;
      for (int i = 0; i < 3; ++i)
        if (cl[i] == m) {
          prev[k] = 1;
          mi[k] = i;
        }
      if (!prev[k]) {
        int s[3] = {cl[0], cl[1], cl[2]};
        std::sort(s, s + 3);
        int r = m;
        for (int i = 2; i >= 0; --i)
          if (m > s[i]) --r;
        rem[k] = r;
      }
      // the PU's mode is visible to the next PU's candidate derivation (and to later CUs)
      for (int y = yp; y < yp + h; y += 4)
        for (int x = xp; x < xp + h; x += 4) mode[g4(x, y)] = static_cast<uint8_t>(m);
      mark_done(xp, yp, h);  // later PUs of an NxN CU see this one
    }
    // undo the early done marks of the CU (the CU completes after its transform tree)
    for (int y = y0; y < y0 + n && y < c.H; y += 4)
      for (int x = x0; x < x0 + n && x < c.W; x += 4) done[g4(x, y)] = 0;
    for (int k = 0; k < npu; ++k) bin(prev[k], C_PREV_INTRA);
    for (int k = 0; k < npu; ++k) {
      if (prev[k]) {
        byp(mi[k] > 0);
        if (mi[k] > 0) byp(mi[k] > 1);
      } else {
        bypn(static_cast<uint32_t>(rem[k]), 5);
      }
    }
    const int cm = R.r(0, 4);
    bin(cm != 4, C_CHROMA_MODE);
    if (cm != 4) bypn(static_cast<uint32_t>(cm), 2);
    if (cm == 4) {
      chroma_mode = pu_modes[0];
    } else {
      const int tab[4] = {0, 26, 10, 1};
      chroma_mode = tab[cm] == pu_modes[0] ? 34 : tab[cm];
    }
  }

  bool last_merge = false;
  void prediction_unit(int xp, int yp, int w, int h, bool sk) {
    (void)xp;
    (void)yp;
    bool merge = sk;
    if (!sk) {
      merge = R.p(0.4);
      bin(merge, C_MERGE_FLAG);
    }
    if (w == (1 << cu_log2) && h == (1 << cu_log2)) last_merge = merge;
    if (merge) {
      if (max_merge > 1) {
        const int idx = R.r(0, max_merge - 1);
        bin(idx > 0, C_MERGE_IDX);
        for (int i = 1; i < idx; ++i) byp(1);
        if (idx > 0 && idx < max_merge - 1) byp(0);
      }
      return;
    }
    int idc = 0;
    if (slice_type == 0) {
      if (w + h != 12) {
        idc = R.r(0, 2);
        const int dd = depth[g4(xp, yp)];
        bin(idc == 2, C_INTER_PRED + dd);
        if (idc != 2) bin(idc, C_INTER_PRED + 4);
      } else {
        idc = R.r(0, 1);
        bin(idc, C_INTER_PRED + 4);
      }
    }
    for (int l = 0; l < 2; ++l) {
      if ((l == 0 && idc == 1) || (l == 1 && idc == 0)) continue;
      if (num_ref[l] > 1) {
        const int r = R.r(0, num_ref[l] - 1), cmax = num_ref[l] - 1;
        for (int i = 0; i < r; ++i) {
          if (i < 2) bin(1, C_REF_IDX + i);
          else byp(1);
        }
        if (r < cmax) {
          if (r < 2) bin(0, C_REF_IDX + r);
          else byp(0);
        }
      }
      if (!(l == 1 && mvd_l1_zero && idc == 2)) write_mvd();
      bin(R.p(0.5), C_MVP);
    }
  }
  void write_mvd() {
    int v[2];
    for (int k = 0; k < 2; ++k) v[k] = R.p(0.2) ? 0 : (R.p(0.1) ? R.r(-600, 600) : R.r(-24, 24));
    const int a0 = std::abs(v[0]), a1 = std::abs(v[1]);
    bin(a0 > 0, C_MVD_G0);
    bin(a1 > 0, C_MVD_G0);
    if (a0) bin(a0 > 1, C_MVD_G1);
    if (a1) bin(a1 > 1, C_MVD_G1);
    for (int k = 0; k < 2; ++k) {
      const int a = std::abs(v[k]);
      if (!a) continue;
      if (a > 1) write_egk(static_cast<uint32_t>(a - 2), 1);
      byp(v[k] < 0);
    }
  }
  void write_egk(uint32_t v, int k) {
    while (v >= (1u << k)) {
      byp(1);
      v -= 1u << k;
      ++k;
    }
    byp(0);
    bypn(v, k);
  }

  // ------------------------------------------------------------------ transform tree
  void transform_tree(int x0, int y0, int xb, int yb, int log2, int dd, int blk, int maxd, int isplit, int pcb, int pcr) {
    int split;
    if (log2 <= c.log2_max_tb && log2 > 2 && dd < maxd && !(isplit && dd == 0)) {
      split = R.p(0.4);
      bin(split, C_SPLIT_TF + 5 - log2);
    } else {
      const bool inter_split = c.depth_inter == 0 && !cu_intra && cu_part != 0 && dd == 0;
      split = log2 > c.log2_max_tb || (isplit && dd == 0) || inter_split;
    }
    int cb = 0, cr = 0;
    if (log2 > 2) {
      if (dd == 0 || pcb) bin(cb = R.p(0.5), C_CBF_CHROMA + dd);
      if (dd == 0 || pcr) bin(cr = R.p(0.5), C_CBF_CHROMA + dd);
    } else {
      cb = pcb;
      cr = pcr;
    }
    if (split) {
      const int h = 1 << (log2 - 1);
      for (int k = 0; k < 4; ++k)
        transform_tree(x0 + (k & 1) * h, y0 + (k >> 1) * h, x0, y0, log2 - 1, dd + 1, k, maxd, isplit, cb, cr);
      return;
    }
    int cy = 1;
    if (cu_intra || dd != 0 || cb || cr) bin(cy = R.p(0.6), C_CBF_LUMA + (dd == 0 ? 1 : 0));
    if ((cy || cb || cr) && c.cu_qp_delta && !qp_coded) write_qp_delta();
    const int my = cu_intra ? static_cast<int>(mode[g4(x0, y0)]) : -1;
    const int mc = cu_intra ? chroma_mode : -1;
    if (cy) residual(log2, 0, my);
    if (log2 > 2) {
      if (cb) residual(log2 - 1, 1, mc);
      if (cr) residual(log2 - 1, 2, mc);
    } else if (blk == 3) {
      if (cb) residual(2, 1, mc);
      if (cr) residual(2, 2, mc);
    }
    (void)xb;
    (void)yb;
  }

  void write_qp_delta() {
    const int off = 6 * (c.bd - 8);
    int d = R.p(0.3) ? 0 : R.r(-8, 8);
    // keep QpY in range from the worst-case prediction
    d = std::max(-(26 + off / 2), std::min(25 + off / 2, d));
    const int a = std::abs(d);
    const int pre = std::min(a, 5);
    for (int i = 0; i < pre; ++i) bin(1, C_QP_DELTA + (i > 0));
    if (pre < 5) bin(0, C_QP_DELTA + (pre > 0));
    else write_egk(static_cast<uint32_t>(a - 5), 0);
    if (a) byp(d < 0);
    qp_coded = true;
  }

  // residual_coding() of a random sparse block
  void residual(int log2, int cidx, int intra_mode) {
    const int n = 1 << log2;
    if (c.tskip && !cu_bypass && log2 <= 2) bin(R.p(0.4), C_TSKIP + (cidx ? 1 : 0));
    int scan = 0;
    if (intra_mode >= 0 && (log2 == 2 || (log2 == 3 && cidx == 0))) {
      if (intra_mode >= 6 && intra_mode <= 14) scan = 2;
      else if (intra_mode >= 22 && intra_mode <= 30) scan = 1;
    }
    const int log2sb = log2 - 2, nsb = 1 << log2sb;
    int sbx[64], sby[64], px[16], py[16];
    for (int i = 0; i < nsb * nsb; ++i) {
      const int p = scan_pos(scan, log2sb, i);
      sbx[i] = p & 255;
      sby[i] = p >> 8;
    }
    for (int i = 0; i < 16; ++i) {
      const int p = scan_pos(scan, 2, i);
      px[i] = p & 255;
      py[i] = p >> 8;
    }
    // levels by (subblock, position) in scan order
    const int total = nsb * nsb * 16;
    std::vector<int> lev(total, 0);
    const int last = R.r(0, std::min(total - 1, R.p(0.5) ? 15 : total - 1));
    lev[last] = R.p(0.5) ? 1 : R.r(1, R.p(0.1) ? 3000 : 6);
    const double dens = R.p(0.5) ? 0.15 : 0.5;
    for (int i = 0; i < last; ++i)
      if (R.p(dens)) lev[i] = R.p(0.7) ? 1 : R.r(1, R.p(0.05) ? 2000 : 5);
    for (int i = 0; i <= last; ++i)
      if (lev[i] && R.p(0.5)) lev[i] = -lev[i];
    const int lsb = last / 16, lpos = last % 16;
    int lx = sbx[lsb] * 4 + px[lpos], ly = sby[lsb] * 4 + py[lpos];
    if (scan == 2) std::swap(lx, ly);
    write_last(lx, log2, cidx, C_LAST_X);
    write_last(ly, log2, cidx, C_LAST_Y);
    write_last_suffix(lx);
    write_last_suffix(ly);
    uint8_t csbf[8][8] = {};
    int g1ctx_prev = 1;
    bool first_sb = true;
    const bool sdh = c.sdh && !cu_bypass;
    for (int i = lsb; i >= 0; --i) {
      const int xs = sbx[i], ys = sby[i];
      const int* L = &lev[i * 16];
      bool any = false;
      for (int p = 0; p < 16; ++p) any |= L[p] != 0;
      bool infer_dc = false;
      if (i < lsb && i > 0) {
        int cs = 0;
        if (xs < nsb - 1) cs += csbf[xs + 1][ys];
        if (ys < nsb - 1) cs += csbf[xs][ys + 1];
        csbf[xs][ys] = any;
        bin(any, C_CSBF + std::min(cs, 1) + (cidx ? 2 : 0));
        infer_dc = true;
      } else {
        csbf[xs][ys] = 1;
      }
      int prev_csbf = 0;
      if (xs < nsb - 1) prev_csbf += csbf[xs + 1][ys];
      if (ys < nsb - 1) prev_csbf += csbf[xs][ys + 1] << 1;
      if (!csbf[xs][ys]) continue;
      // sig flags; a coded-csbf subblock whose only level is at position 0 has it inferred
      bool infer = infer_dc;
      for (int p = (i == lsb ? lpos - 1 : 15); p >= 0; --p) {
        if (p == 0 && infer) break;
        const int xc = xs * 4 + px[p], yc = ys * 4 + py[p];
        bin(L[p] != 0, C_SIG + sig_ctx(xc, yc, log2, cidx, scan, prev_csbf, xs, ys));
        if (L[p]) infer = false;
      }
      bool any_sig = false;
      for (int p = 0; p < 16; ++p) any_sig |= L[p] != 0;
      int ctx_set = (i == 0 || cidx > 0) ? 0 : 2;
      if (!first_sb && g1ctx_prev == 0) ++ctx_set;
      int g1ctx = 1, ng1 = 0, last_g1 = -1;
      int g1[16] = {}, g2[16] = {};
      for (int p = 15; p >= 0; --p) {
        if (!L[p]) continue;
        if (ng1 < 8) {
          g1[p] = std::abs(L[p]) > 1;
          bin(g1[p], C_GT1 + (cidx ? 16 : 0) + ctx_set * 4 + g1ctx);
          ++ng1;
          if (g1[p]) {
            g1ctx = 0;
            if (last_g1 < 0) last_g1 = p;
          } else if (g1ctx > 0 && g1ctx < 3) {
            ++g1ctx;
          }
        }
      }
      if (any_sig) {
        first_sb = false;
        g1ctx_prev = g1ctx;
      }
      if (last_g1 >= 0) {
        g2[last_g1] = std::abs(L[last_g1]) > 2;
        bin(g2[last_g1], C_GT2 + (cidx ? 4 : 0) + ctx_set);
      }
      int first_sig = -1, last_sig = -1;
      for (int p = 0; p < 16; ++p)
        if (L[p]) {
          if (first_sig < 0) first_sig = p;
          last_sig = p;
        }
      const bool hidden = sdh && last_sig - first_sig > 3;
      for (int p = 15; p >= 0; --p)
        if (L[p] && !(hidden && p == first_sig)) byp(L[p] < 0);
      int nsig = 0, rice = 0;
      for (int p = 15; p >= 0; --p) {
        if (!L[p]) continue;
        const int a = std::abs(L[p]);
        const int base = 1 + g1[p] + g2[p];
        const int thr = nsig < 8 ? (p == last_g1 ? 3 : 2) : 1;
        if (base == thr) {
          write_remaining(a - base, rice);
          if (a > 3 * (1 << rice)) rice = std::min(rice + 1, 4);
        }
        ++nsig;
      }
    }
    (void)n;
  }
  void write_last(int v, int log2, int cidx, int base) {
    int off, shift;
    if (cidx == 0) {
      off = 3 * (log2 - 2) + ((log2 - 1) >> 2);
      shift = (log2 + 1) >> 2;
    } else {
      off = 15;
      shift = log2 - 2;
    }
    const int pre = last_prefix_of(v), cmax = (log2 << 1) - 1;
    for (int i = 0; i < pre; ++i) bin(1, base + off + (i >> shift));
    if (pre < cmax) bin(0, base + off + (pre >> shift));
  }
  static int last_prefix_of(int v) {
    if (v < 4) return v;
    int p = 4;
    while (true) {
      const int nb = (p >> 1) - 1;
      const int lo = (1 << nb) * (2 + (p & 1));
      if (v < lo + (1 << nb)) return p;
      ++p;
    }
  }
  void write_last_suffix(int v) {
    const int p = last_prefix_of(v);
    if (p <= 3) return;
    const int nb = (p >> 1) - 1;
    bypn(static_cast<uint32_t>(v - (1 << nb) * (2 + (p & 1))), nb);
  }
  void write_remaining(int v, int rice) {
    if (v < (4 << rice)) {
      const int pre = v >> rice;
      for (int i = 0; i < pre; ++i) byp(1);
      byp(0);
      bypn(static_cast<uint32_t>(v & ((1 << rice) - 1)), rice);
      return;
    }
    // prefix > 3: value ((1 << (prefix - 3)) + 2) << rice + suffix of (prefix - 3 + rice) bits
    int prefix = 4;
    while (v >= (((1 << (prefix - 2)) + 2) << rice)) ++prefix;
    for (int i = 0; i < prefix; ++i) byp(1);
    byp(0);
    const int k = prefix - 3 + rice;
    bypn(static_cast<uint32_t>(v - (((1 << (prefix - 3)) + 2) << rice)), k);
  }
  static int sig_ctx(int xc, int yc, int log2, int cidx, int scan, int prev_csbf, int xs, int ys) {
    static const int map4[15] = {0, 1, 4, 5, 2, 3, 4, 5, 6, 6, 8, 8, 7, 7, 8};
    int s;
    if (log2 == 2) {
      s = map4[(yc << 2) + xc];
    } else if (xc + yc == 0) {
      s = 0;
    } else {
      const int xp = xc & 3, yp = yc & 3;
      switch (prev_csbf) {
        case 0: s = (xp + yp == 0) ? 2 : (xp + yp < 3) ? 1 : 0; break;
        case 1: s = yp == 0 ? 2 : (yp == 1 ? 1 : 0); break;
        case 2: s = xp == 0 ? 2 : (xp == 1 ? 1 : 0); break;
        default: s = 2;
      }
      if (cidx == 0) {
        if (xs > 0 || ys > 0) s += 3;
        if (log2 == 3) s += scan == 0 ? 9 : 15;
        else s += 21;
      } else {
        s += log2 == 3 ? 9 : 12;
      }
    }
    return cidx == 0 ? s : 27 + s;
  }

 public:
  void set_sps_counts(int st, int lt) {
    num_sps_st_ = st;
    num_sps_lt_ = lt;
  }
};

}  // namespace

std::vector<uint8_t> hevc_exercise(uint32_t seed) {
  Exerciser e(seed);
  return e.run();
}

}  // namespace hevc
}  // namespace mivc
