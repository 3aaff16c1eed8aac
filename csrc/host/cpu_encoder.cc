#include "cpu_encoder.h"
#include "cabac_writer.h"

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstring>
#include <stdexcept>

#include "../common/h264_enc_math.h"
#include "../common/h264_pred.h"
#include "cavlc_writer.h"
#include "h264_decoder.h"

namespace mivc {
namespace h264 {

SPS make_sps(const EncoderConfig& cfg) {
  SPS s;
  s.width_mbs = (cfg.width + 15) / 16;
  s.height_mbs = (cfg.height + 15) / 16;
  s.crop_right = (s.width_mbs * 16 - cfg.width) / 2;
  s.crop_bottom = (s.height_mbs * 16 - cfg.height) / 2;
  if (cfg.bit_depth > 8) {
    s.profile_idc = 110;  // High 10 (A.2.5; bit depths up to 10 -- deeper ones are written as such)
    s.constraint_flags = 0;
    s.bit_depth_luma = s.bit_depth_chroma = cfg.bit_depth;
    if (cfg.bit_depth_chroma > 0) s.bit_depth_chroma = cfg.bit_depth_chroma;
  } else if (cfg.t8x8) {
    s.profile_idc = 100;  // High
    s.constraint_flags = 0;
  } else if (cfg.cabac || cfg.bframes > 0) {
    s.profile_idc = 77;   // Main
    s.constraint_flags = 0x40;  // constraint_set1 (Main-compatible)
  } else {
    s.profile_idc = 66;
    s.constraint_flags = 0xC0;  // Constrained Baseline
  }
  s.level_idc = choose_level(s.width_mbs, s.height_mbs, cfg.fps);
  if (cfg.level_idc > 0) {
    // -level: the requested level must admit the picture size and rate (Table A-1)
    if (cfg.level_idc < s.level_idc)
      throw std::runtime_error("H.264: picture size / frame rate exceed the requested level " +
                               std::to_string(cfg.level_idc / 10) + "." + std::to_string(cfg.level_idc % 10));
    s.level_idc = cfg.level_idc;
  }
  s.log2_max_frame_num = 16;
  if (cfg.bframes > 0) {
    s.poc_type = 0;
    s.log2_max_poc_lsb = 16;
    // B pictures are output one behind their future anchor; with a reference B in between
    // (b-pyramid) the non-reference ones wait behind two pictures
    s.max_num_reorder = cfg.pyramid ? 2 : 1;
  } else {
    s.poc_type = 2;
  }
  // must equal models/gop.py dpb_frames(): the active references plus one with B pictures; a
  // pyramid needs >= 4 (see dpb_frames)
  s.max_num_ref_frames = std::max(1, cfg.refs) + (cfg.bframes > 0 ? 1 : 0);
  if (cfg.pyramid && cfg.bframes >= 2) s.max_num_ref_frames = std::max(s.max_num_ref_frames, 4);
  s.vui_present = cfg.vui;
  if (cfg.cqm && !cfg.t8x8) throw std::runtime_error("H.264: scaling matrices need the High profile (t8x8)");
  if (cfg.cqm == 3) s.scaling_present = 1;  // the default matrices, overridden by the PPS lists (rule B)
  if (cfg.cqm == 1 || cfg.cqm == 2) {
    s.scaling_present = 1;
    for (int i = 0; i < 8; ++i) s.sl_coded[i] = cfg.cqm == 2 && ((cfg.cqm_coded >> i) & 1);
    std::memcpy(s.sl4, cfg.cqm4, sizeof(s.sl4));
    std::memcpy(s.sl8, cfg.cqm8, sizeof(s.sl8));
  }
  // time_scale / (2 * num_units_in_tick) = fps
  s.num_units_in_tick = 1000;
  s.time_scale = static_cast<uint32_t>(std::lround(cfg.fps * 2000.0));
  return s;
}

PPS make_pps(const EncoderConfig& cfg) {
  PPS p;
  p.pic_init_qp = 26;
  p.entropy_coding_mode = cfg.cabac ? 1 : 0;
  p.transform_8x8_mode = cfg.t8x8 ? 1 : 0;
  p.num_ref_idx_l0_default = std::max(1, cfg.refs);
  p.weighted_bipred_idc = cfg.bframes > 0 ? cfg.weighted_bipred : 0;
  p.weighted_pred = cfg.weightp ? 1 : 0;
  p.constrained_intra_pred = cfg.constrained_intra ? 1 : 0;
  p.chroma_qp_index_offset = cfg.chroma_qp_offset;
  p.second_chroma_qp_index_offset = cfg.chroma_qp_offset;
  p.deblocking_filter_control_present = 1;
  if (cfg.cqm == 3) {
    p.scaling_present = 1;
    for (int i = 0; i < 8; ++i) p.sl_coded[i] = (cfg.cqm_coded >> i) & 1;
    std::memcpy(p.sl4, cfg.cqm4, sizeof(p.sl4));
    std::memcpy(p.sl8, cfg.cqm8, sizeof(p.sl8));
  }
  return p;
}

namespace {

struct Planes {
  int W = 0, H = 0;
  std::vector<uint8_t> y, u, v;
  void alloc(int w, int h) {
    W = w;
    H = h;
    y.assign(static_cast<size_t>(w) * h, 0);
    u.assign(static_cast<size_t>(w / 2) * (h / 2), 0);
    v.assign(u.size(), 0);
  }
};

struct ClampRef {
  const uint8_t* p;
  int w, h;
  int operator()(int x, int y) const {
    x = x < 0 ? 0 : (x >= w ? w - 1 : x);
    y = y < 0 ? 0 : (y >= h ? h - 1 : y);
    return p[static_cast<size_t>(y) * w + x];
  }
};

class FrameEncoder {
 public:
  FrameEncoder(const EncoderConfig& cfg, int wmb, int hmb) : cfg_(cfg), wmb_(wmb), hmb_(hmb) {
    rec_.alloc(wmb * 16, hmb * 16);
    mbs_.resize(static_cast<size_t>(wmb) * hmb);
    coef_.resize(static_cast<size_t>(wmb) * hmb * kCoefPerMb);
    mvs_.resize(static_cast<size_t>(wmb) * hmb * 2);
  }

  void encode(const Planes& src, const Planes* ref, bool islice, int qp) {
    std::memset(mbs_.data(), 0, mbs_.size() * sizeof(MbHeader));
    for (MbHeader& h : mbs_) std::memset(h.ref, 0xFF, sizeof(h.ref));  // no list used until inter
    std::fill(coef_.begin(), coef_.end(), 0);
    src_ = &src;
    ref_ = ref;
    islice_ = islice;
    qp_ = qp;
    lambda_ = kLambda[qp];
    for (int my = 0; my < hmb_; ++my)
      for (int mx = 0; mx < wmb_; ++mx) encode_mb(mx, my);
  }

  std::vector<MbHeader> mbs_;
  std::vector<int16_t> coef_;
  Planes rec_;
  // the effective scaling lists of the picture (raster; the decoder's derivation of the
  // parameter sets this encoder wrote): [0..5] intra Y / Cb / Cr, inter Y / Cb / Cr
  uint8_t sl4_[6][16];

 private:
  int sy(int x, int y) const { return src_->y[static_cast<size_t>(y) * src_->W + x]; }

  // ---------------------------------------------------------------- transform helpers
  // residual 4x4 (raster) -> quantised levels in scan order; returns reconstructed residual in res (raster)
  // weighted LevelScale4x4 dequantisation (8.5.12.1) with scaling list wl (raster)
  static int dequant_w(int c, int qp, int r, const uint8_t* wl) {
    const int ls = wl[r] * kDequantV[qp % 6][kPosClass[r]];
    if (qp >= 24) return (c * ls) << (qp / 6 - 4);
    return (c * ls + (1 << (3 - qp / 6))) >> (4 - qp / 6);
  }
  // list: scaling list index (0..5: intra Y / Cb / Cr, inter Y / Cb / Cr)
  void tq4x4(int* res, int qp, bool intra, int16_t* out_scan, bool skip_dc, int list) {
    int w[16];
    for (int i = 0; i < 16; ++i) w[i] = res[i];
    forward_core4x4(w);
    int qbits = 15 + qp / 6;
    int bias = intra ? 21 : 11;
    const uint8_t* wl = sl4_[list];
    int lv[16];
    // the quantiser divides by the weight (x264-style MF * 16 / w); only the dequantisation
    // has to match the decoder
    for (int r = 0; r < 16; ++r) lv[r] = quant_coef(w[r], kQuantMF[qp % 6][kPosClass[r]] * 16 / wl[r], qbits, bias);
    if (skip_dc) lv[0] = 0;
    for (int i = 0; i < 16; ++i) out_scan[i] = static_cast<int16_t>(lv[kZigzag4x4[i]]);
    if (skip_dc) out_scan[0] = 0;
    for (int r = 0; r < 16; ++r) res[r] = dequant_w(lv[r], qp, r, wl);
    // caller supplies DC (if skip_dc) before inverse
  }

  int avail(int mx, int my) const {
    int av = 0;
    if (mx > 0) av |= AV_LEFT;
    if (my > 0) av |= AV_TOP;
    if (mx > 0 && my > 0) av |= AV_TOPLEFT;
    if (my > 0 && mx < wmb_ - 1) av |= AV_TOPRIGHT;
    return av;
  }

  // ---------------------------------------------------------------- intra 4x4
  int i4_pred_mode(int mx, int my, const uint8_t* cur_modes, int blk) const {
    int bx = kBlkX[blk], by = kBlkY[blk];
    int ma, mb;
    if (bx > 0) ma = cur_modes[kRasterToBlk[(bx - 1) + 4 * by]];
    else if (mx > 0) {
      const MbHeader& a = mbs_[my * wmb_ + mx - 1];
      ma = a.kind == MBK_I4x4 ? a.i4_modes[kRasterToBlk[3 + 4 * by]] : 2;
    } else return 2;
    if (by > 0) mb = cur_modes[kRasterToBlk[bx + 4 * (by - 1)]];
    else if (my > 0) {
      const MbHeader& b = mbs_[(my - 1) * wmb_ + mx];
      mb = b.kind == MBK_I4x4 ? b.i4_modes[kRasterToBlk[bx + 12]] : 2;
    } else return 2;
    return std::min(ma, mb);
  }

  // encode the MB as I4x4 into a scratch recon; returns cost. Writes modes/coefs to hdr/coef, pixels into rec_.
  int encode_i4x4(int mx, int my, int qp, MbHeader& hdr, int16_t* coef) {
    int X0 = mx * 16, Y0 = my * 16, W = rec_.W;
    int mbav = avail(mx, my);
    int total = 0;
    for (int blk = 0; blk < 16; ++blk) {
      int bx = kBlkX[blk], by = kBlkY[blk];
      int x0 = X0 + bx * 4, y0 = Y0 + by * 4;
      int av = 0;
      bool left = bx > 0 || (mbav & AV_LEFT), top = by > 0 || (mbav & AV_TOP);
      if (left) av |= AV_LEFT;
      if (top) av |= AV_TOP;
      if (left && top) av |= AV_TOPLEFT;
      bool tr;
      if (blk == 3 || blk == 7 || blk == 11 || blk == 13 || blk == 15) tr = false;
      else if (blk == 5) tr = (mbav & AV_TOPRIGHT) != 0;
      else if (blk == 0 || blk == 1 || blk == 4) tr = (mbav & AV_TOP) != 0;
      else tr = true;
      if (tr) av |= AV_TOPRIGHT;
      int e[13] = {0};
      if (av & AV_TOPLEFT) e[0] = rec_.y[static_cast<size_t>(y0 - 1) * W + x0 - 1];
      if (top) {
        for (int i = 0; i < 4; ++i) e[1 + i] = rec_.y[static_cast<size_t>(y0 - 1) * W + x0 + i];
        for (int i = 4; i < 8; ++i) e[1 + i] = tr ? rec_.y[static_cast<size_t>(y0 - 1) * W + x0 + i] : e[4];
      }
      if (left)
        for (int i = 0; i < 4; ++i) e[9 + i] = rec_.y[static_cast<size_t>(y0 + i) * W + x0 - 1];
      int pm = i4_pred_mode(mx, my, hdr.i4_modes, blk);
      int best = INT_MAX, best_mode = 2;
      for (int mode = 0; mode < 9; ++mode) {
        if (!i4_mode_ok(mode, av)) continue;
        int r[16];
        for (int y = 0; y < 4; ++y)
          for (int x = 0; x < 4; ++x) r[y * 4 + x] = sy(x0 + x, y0 + y) - i4_pred_sample(mode, av, e, x, y);
        int cost = satd4x4(r) + lambda_ * (mode == pm ? 1 : 4);
        if (cost < best) {
          best = cost;
          best_mode = mode;
        }
      }
      hdr.i4_modes[blk] = static_cast<uint8_t>(best_mode);
      int pred[16], res[16];
      for (int y = 0; y < 4; ++y)
        for (int x = 0; x < 4; ++x) {
          pred[y * 4 + x] = i4_pred_sample(best_mode, av, e, x, y);
          res[y * 4 + x] = sy(x0 + x, y0 + y) - pred[y * 4 + x];
        }
      tq4x4(res, qp, true, coef + COEF_LUMA + blk * 16, false, 0);
      inverse_core4x4(res);
      for (int y = 0; y < 4; ++y)
        for (int x = 0; x < 4; ++x)
          rec_.y[static_cast<size_t>(y0 + y) * W + x0 + x] = static_cast<uint8_t>(clip1(pred[y * 4 + x] + res[y * 4 + x]));
      total += best;
    }
    return total + lambda_ * 8;
  }

  // ---------------------------------------------------------------- intra 16x16
  void gather16(int mx, int my, int* top, int* left, int* tl) const {
    int X0 = mx * 16, Y0 = my * 16, W = rec_.W;
    for (int i = 0; i < 16; ++i) {
      top[i] = my > 0 ? rec_.y[static_cast<size_t>(Y0 - 1) * W + X0 + i] : 0;
      left[i] = mx > 0 ? rec_.y[static_cast<size_t>(Y0 + i) * W + X0 - 1] : 0;
    }
    *tl = (mx > 0 && my > 0) ? rec_.y[static_cast<size_t>(Y0 - 1) * W + X0 - 1] : 0;
  }
  void pred16(int mode, int av, const int* top, const int* left, int tl, int* pred) const {
    int a = 0, b = 0, c = 0, dc = 0;
    if (mode == 3) i16_plane_params(top, left, tl, &a, &b, &c);
    if (mode == 2) dc = i16_dc(top, left, av);
    for (int y = 0; y < 16; ++y)
      for (int x = 0; x < 16; ++x) {
        int v;
        if (mode == 0) v = top[x];
        else if (mode == 1) v = left[y];
        else if (mode == 2) v = dc;
        else v = clip1((a + b * (x - 7) + c * (y - 7) + 16) >> 5);
        pred[y * 16 + x] = v;
      }
  }
  int best_i16(int mx, int my, int* mode_out) const {
    int top[16], left[16], tl;
    gather16(mx, my, top, left, &tl);
    int av = avail(mx, my);
    int best = INT_MAX;
    for (int mode = 0; mode < 4; ++mode) {
      if (!i16_mode_ok(mode, av)) continue;
      int pred[256];
      pred16(mode, av, top, left, tl, pred);
      int cost = 0;
      for (int b = 0; b < 16; ++b) {
        int r[16];
        int bx = (b & 3) * 4, by = (b >> 2) * 4;
        for (int y = 0; y < 4; ++y)
          for (int x = 0; x < 4; ++x)
            r[y * 4 + x] = sy(mx * 16 + bx + x, my * 16 + by + y) - pred[(by + y) * 16 + bx + x];
        cost += satd4x4(r);
      }
      cost += lambda_ * 4;
      if (cost < best) {
        best = cost;
        *mode_out = mode;
      }
    }
    return best;
  }
  void encode_i16(int mx, int my, int mode, int qp, int16_t* coef) {
    int top[16], left[16], tl;
    gather16(mx, my, top, left, &tl);
    int pred[256];
    pred16(mode, avail(mx, my), top, left, tl, pred);
    int X0 = mx * 16, Y0 = my * 16, W = rec_.W;
    int res[16][16];
    int dcs[16];
    for (int blk = 0; blk < 16; ++blk) {
      int bx = kBlkX[blk] * 4, by = kBlkY[blk] * 4;
      for (int y = 0; y < 4; ++y)
        for (int x = 0; x < 4; ++x) res[blk][y * 4 + x] = sy(X0 + bx + x, Y0 + by + y) - pred[(by + y) * 16 + bx + x];
      int w[16];
      for (int i = 0; i < 16; ++i) w[i] = res[blk][i];
      forward_core4x4(w);
      dcs[kBlkX[blk] + 4 * kBlkY[blk]] = w[0];
      tq4x4(res[blk], qp, true, coef + COEF_LUMA + blk * 16, true, 0);
    }
    // DC: Hadamard, /2, quantise with qbits+1
    hadamard4x4(dcs);
    int qbits = 15 + qp / 6;
    int dcl[16];
    for (int r = 0; r < 16; ++r) dcl[r] = quant_coef(dcs[r] >> 1, kQuantMF[qp % 6][0] * 16 / sl4_[0][0], qbits + 1, 21);
    for (int i = 0; i < 16; ++i) coef[COEF_LUMA_DC + i] = static_cast<int16_t>(dcl[kZigzag4x4[i]]);
    // encoder-side reconstruction of the DC path (mirrors 8.5.10)
    int f[16];
    for (int i = 0; i < 16; ++i) f[i] = dcl[i];
    hadamard4x4(f);
    int ls = sl4_[0][0] * kDequantV[qp % 6][0];
    for (int blk = 0; blk < 16; ++blk) {
      int rpos = kBlkX[blk] + 4 * kBlkY[blk];
      int fv = f[rpos];
      int dcv = qp >= 36 ? (fv * ls) << (qp / 6 - 6) : (fv * ls + (1 << (5 - qp / 6))) >> (6 - qp / 6);
      res[blk][0] = dcv;
      inverse_core4x4(res[blk]);
      int bx = kBlkX[blk] * 4, by = kBlkY[blk] * 4;
      for (int y = 0; y < 4; ++y)
        for (int x = 0; x < 4; ++x)
          rec_.y[static_cast<size_t>(Y0 + by + y) * W + X0 + bx + x] =
              static_cast<uint8_t>(clip1(pred[(by + y) * 16 + bx + x] + res[blk][y * 4 + x]));
    }
  }

  // ---------------------------------------------------------------- chroma
  void chroma_pred(int comp, int mx, int my, int mode, int* pred) const {
    const std::vector<uint8_t>& pl = comp == 0 ? rec_.u : rec_.v;
    int cw = rec_.W / 2, X0 = mx * 8, Y0 = my * 8;
    int top[8], left[8], tl = 0;
    for (int i = 0; i < 8; ++i) {
      top[i] = my > 0 ? pl[static_cast<size_t>(Y0 - 1) * cw + X0 + i] : 0;
      left[i] = mx > 0 ? pl[static_cast<size_t>(Y0 + i) * cw + X0 - 1] : 0;
    }
    if (mx > 0 && my > 0) tl = pl[static_cast<size_t>(Y0 - 1) * cw + X0 - 1];
    int av = avail(mx, my);
    int a = 0, b = 0, c = 0;
    if (mode == 3) chroma_plane_params(top, left, tl, &a, &b, &c);
    for (int y = 0; y < 8; ++y)
      for (int x = 0; x < 8; ++x) {
        int v;
        if (mode == 0) v = chroma_dc(top, left, av, x >> 2, y >> 2);
        else if (mode == 1) v = left[y];
        else if (mode == 2) v = top[x];
        else v = clip1((a + b * (x - 3) + c * (y - 3) + 16) >> 5);
        pred[y * 8 + x] = v;
      }
  }
  int choose_chroma_mode(int mx, int my) const {
    int av = avail(mx, my);
    int best = INT_MAX, bm = 0;
    for (int mode = 0; mode < 4; ++mode) {
      if (!chroma_mode_ok(mode, av)) continue;
      int cost = 0;
      for (int comp = 0; comp < 2; ++comp) {
        const std::vector<uint8_t>& sp = comp == 0 ? src_->u : src_->v;
        int pred[64];
        chroma_pred(comp, mx, my, mode, pred);
        for (int b = 0; b < 4; ++b) {
          int r[16];
          int bx = (b & 1) * 4, by = (b >> 1) * 4;
          for (int y = 0; y < 4; ++y)
            for (int x = 0; x < 4; ++x)
              r[y * 4 + x] = sp[static_cast<size_t>(my * 8 + by + y) * (src_->W / 2) + mx * 8 + bx + x] - pred[(by + y) * 8 + bx + x];
          cost += satd4x4(r);
        }
      }
      if (cost < best) {
        best = cost;
        bm = mode;
      }
    }
    return bm;
  }
  // residual + TQ + recon for both chroma planes given predictions
  void encode_chroma(int mx, int my, const int* pred_u, const int* pred_v, int qp, bool intra, int16_t* coef) {
    int qpc = chroma_qp(qp, cfg_.chroma_qp_offset);
    int cw = rec_.W / 2;
    for (int comp = 0; comp < 2; ++comp) {
      const std::vector<uint8_t>& sp = comp == 0 ? src_->u : src_->v;
      std::vector<uint8_t>& rp = comp == 0 ? rec_.u : rec_.v;
      const int* pred = comp == 0 ? pred_u : pred_v;
      int res[4][16], dcs[4];
      for (int b = 0; b < 4; ++b) {
        int bx = (b & 1) * 4, by = (b >> 1) * 4;
        for (int y = 0; y < 4; ++y)
          for (int x = 0; x < 4; ++x)
            res[b][y * 4 + x] = sp[static_cast<size_t>(my * 8 + by + y) * cw + mx * 8 + bx + x] - pred[(by + y) * 8 + bx + x];
        int w[16];
        for (int i = 0; i < 16; ++i) w[i] = res[b][i];
        forward_core4x4(w);
        dcs[b] = w[0];
        tq4x4(res[b], qpc, intra, coef + COEF_CHROMA_AC + (comp * 4 + b) * 16, true, (intra ? 1 : 4) + comp);
      }
      int y0 = dcs[0] + dcs[1] + dcs[2] + dcs[3];
      int y1 = dcs[0] - dcs[1] + dcs[2] - dcs[3];
      int y2 = dcs[0] + dcs[1] - dcs[2] - dcs[3];
      int y3 = dcs[0] - dcs[1] - dcs[2] + dcs[3];
      int yd[4] = {y0, y1, y2, y3};
      int qbits = 15 + qpc / 6;
      int lv[4];
      for (int i = 0; i < 4; ++i) {
        lv[i] = quant_coef(yd[i], kQuantMF[qpc % 6][0] * 16 / sl4_[(intra ? 1 : 4) + comp][0], qbits + 1, intra ? 21 : 11);
        coef[COEF_CHROMA_DC + comp * 4 + i] = static_cast<int16_t>(lv[i]);
      }
      int f[4] = {lv[0] + lv[1] + lv[2] + lv[3], lv[0] - lv[1] + lv[2] - lv[3], lv[0] + lv[1] - lv[2] - lv[3],
                  lv[0] - lv[1] - lv[2] + lv[3]};
      int ls = sl4_[(intra ? 1 : 4) + comp][0] * kDequantV[qpc % 6][0];
      bool any = false;
      for (int i = 0; i < 4; ++i) any |= lv[i] != 0;
      for (int b = 0; b < 4 && !any; ++b)
        for (int i = 1; i < 16; ++i) any |= coef[COEF_CHROMA_AC + (comp * 4 + b) * 16 + i] != 0;
      for (int b = 0; b < 4; ++b) {
        res[b][0] = ((f[b] * ls) << (qpc / 6)) >> 5;
        if (any) inverse_core4x4(res[b]);
        int bx = (b & 1) * 4, by = (b >> 1) * 4;
        for (int y = 0; y < 4; ++y)
          for (int x = 0; x < 4; ++x)
            rp[static_cast<size_t>(my * 8 + by + y) * cw + mx * 8 + bx + x] =
                static_cast<uint8_t>(clip1(pred[(by + y) * 8 + bx + x] + (any ? res[b][y * 4 + x] : 0)));
      }
    }
  }
  // The chroma residual is dropped entirely when the writer will not code it (cbp chroma == 0),
  // which happens exactly when every level is zero -- handled by `any` above.

  // ---------------------------------------------------------------- inter
  int mv_cost(int mvx, int mvy, int px, int py) const { return lambda_ * (se_bits(mvx - px) + se_bits(mvy - py)); }
  int sad16_int(int mx, int my, int dx, int dy) const {
    ClampRef r{ref_->y.data(), ref_->W, ref_->H};
    int s = 0;
    for (int y = 0; y < 16; ++y)
      for (int x = 0; x < 16; ++x) {
        int a = sy(mx * 16 + x, my * 16 + y) - r(mx * 16 + x + dx, my * 16 + y + dy);
        s += a < 0 ? -a : a;
      }
    return s;
  }
  void pred_luma16(int mx, int my, int mvx, int mvy, int* pred) const {
    ClampRef r{ref_->y.data(), ref_->W, ref_->H};
    for (int y = 0; y < 16; ++y)
      for (int x = 0; x < 16; ++x) {
        int px = mx * 16 + x, py = my * 16 + y;
        pred[y * 16 + x] = mc_luma_sample(r, px + (mvx >> 2), py + (mvy >> 2), mvx & 3, mvy & 3);
      }
  }
  int satd16(int mx, int my, const int* pred) const {
    int cost = 0;
    for (int b = 0; b < 16; ++b) {
      int r[16];
      int bx = (b & 3) * 4, by = (b >> 2) * 4;
      for (int y = 0; y < 4; ++y)
        for (int x = 0; x < 4; ++x) r[y * 4 + x] = sy(mx * 16 + bx + x, my * 16 + by + y) - pred[(by + y) * 16 + bx + x];
      cost += satd4x4(r);
    }
    return cost;
  }
  void motion_search(int mx, int my, int* bmx, int* bmy, int* bcost) {
    // predictor: left MB's motion (approximation of the median predictor)
    int px = 0, py = 0;
    if (mx > 0) {
      px = mvs_[2 * (my * wmb_ + mx - 1)];
      py = mvs_[2 * (my * wmb_ + mx - 1) + 1];
    }
    int R = cfg_.me_range;
    int best = INT_MAX, bx = 0, by = 0;
    int cands[3][2] = {{0, 0}, {px >> 2, py >> 2}, {0, 0}};
    if (my > 0) {
      cands[2][0] = mvs_[2 * ((my - 1) * wmb_ + mx)] >> 2;
      cands[2][1] = mvs_[2 * ((my - 1) * wmb_ + mx) + 1] >> 2;
    }
    for (auto& c : cands) {
      int cost = sad16_int(mx, my, c[0], c[1]) + mv_cost(c[0] * 4, c[1] * 4, px, py);
      if (cost < best) {
        best = cost;
        bx = c[0];
        by = c[1];
      }
    }
    // small diamond descent then exhaustive refinement in a +-2 window, bounded by R
    bool improved = true;
    int iters = 0;
    while (improved && iters++ < 2 * R) {
      improved = false;
      static const int d[4][2] = {{1, 0}, {-1, 0}, {0, 1}, {0, -1}};
      for (auto& dd : d) {
        int cx = bx + dd[0], cy = by + dd[1];
        if (std::abs(cx) > R || std::abs(cy) > R) continue;
        int cost = sad16_int(mx, my, cx, cy) + mv_cost(cx * 4, cy * 4, px, py);
        if (cost < best) {
          best = cost;
          bx = cx;
          by = cy;
          improved = true;
        }
      }
    }
    int mvx = bx * 4, mvy = by * 4;
    int pred[256];
    pred_luma16(mx, my, mvx, mvy, pred);
    int bestq = satd16(mx, my, pred) + mv_cost(mvx, mvy, px, py);
    // sub-pel refinement: half then quarter
    for (int step = 2; step >= (cfg_.subpel >= 2 ? 1 : 2) && cfg_.subpel > 0; step >>= 1) {
      int cx0 = mvx, cy0 = mvy;
      for (int dy = -step; dy <= step; dy += step)
        for (int dx = -step; dx <= step; dx += step) {
          if (!dx && !dy) continue;
          int cx = cx0 + dx, cy = cy0 + dy;
          pred_luma16(mx, my, cx, cy, pred);
          int cost = satd16(mx, my, pred) + mv_cost(cx, cy, px, py);
          if (cost < bestq) {
            bestq = cost;
            mvx = cx;
            mvy = cy;
          }
        }
    }
    *bmx = mvx;
    *bmy = mvy;
    *bcost = bestq;
  }

  // ---------------------------------------------------------------- per MB
  void encode_mb(int mx, int my) {
    int addr = my * wmb_ + mx;
    MbHeader& hdr = mbs_[addr];
    int16_t* coef = coef_.data() + static_cast<size_t>(addr) * kCoefPerMb;
    hdr.qp = static_cast<int8_t>(qp_);
    mvs_[2 * addr] = mvs_[2 * addr + 1] = 0;
    int i16_mode = 2;
    int c16 = best_i16(mx, my, &i16_mode);
    if (!islice_) {
      int mvx, mvy, cinter;
      motion_search(mx, my, &mvx, &mvy, &cinter);
      if (cinter <= c16) {
        hdr.kind = MBK_P16x16;
        for (int q = 0; q < 4; ++q) {
          hdr.mv[0][q][0] = static_cast<int16_t>(mvx);
          hdr.mv[0][q][1] = static_cast<int16_t>(mvy);
          hdr.ref[0][q] = 0;
        }
        mvs_[2 * addr] = mvx;
        mvs_[2 * addr + 1] = mvy;
        int pred[256];
        pred_luma16(mx, my, mvx, mvy, pred);
        int X0 = mx * 16, Y0 = my * 16, W = rec_.W;
        for (int blk = 0; blk < 16; ++blk) {
          int bx = kBlkX[blk] * 4, by = kBlkY[blk] * 4;
          int res[16];
          for (int y = 0; y < 4; ++y)
            for (int x = 0; x < 4; ++x) res[y * 4 + x] = sy(X0 + bx + x, Y0 + by + y) - pred[(by + y) * 16 + bx + x];
          tq4x4(res, qp_, false, coef + COEF_LUMA + blk * 16, false, 3);
        }
        // drop 8x8 blocks whose only content is a few +-1 levels (cheap decimation)
        for (int b8 = 0; b8 < 4; ++b8) {
          int score = 0;
          for (int b = 0; b < 4; ++b)
            for (int i = 0; i < 16; ++i) {
              int v = coef[COEF_LUMA + (b8 * 4 + b) * 16 + i];
              score += v == 0 ? 0 : (v == 1 || v == -1 ? 1 : 10);
            }
          if (score < 4)
            for (int b = 0; b < 4; ++b)
              for (int i = 0; i < 16; ++i) coef[COEF_LUMA + (b8 * 4 + b) * 16 + i] = 0;
        }
        for (int blk = 0; blk < 16; ++blk) {
          int bx = kBlkX[blk] * 4, by = kBlkY[blk] * 4;
          int res[16];
          for (int r = 0; r < 16; ++r) res[r] = 0;
          for (int i = 0; i < 16; ++i) {
            int r = kZigzag4x4[i];
            res[r] = dequant_w(coef[COEF_LUMA + blk * 16 + i], qp_, r, sl4_[3]);
          }
          inverse_core4x4(res);
          for (int y = 0; y < 4; ++y)
            for (int x = 0; x < 4; ++x)
              rec_.y[static_cast<size_t>(Y0 + by + y) * W + X0 + bx + x] =
                  static_cast<uint8_t>(clip1(pred[(by + y) * 16 + bx + x] + res[y * 4 + x]));
        }
        // chroma MC
        int pu[64], pv[64];
        ClampRef ru{ref_->u.data(), ref_->W / 2, ref_->H / 2}, rv{ref_->v.data(), ref_->W / 2, ref_->H / 2};
        for (int y = 0; y < 8; ++y)
          for (int x = 0; x < 8; ++x) {
            int px = mx * 8 + x + (mvx >> 3), py = my * 8 + y + (mvy >> 3);
            pu[y * 8 + x] = mc_chroma_sample(ru, px, py, mvx & 7, mvy & 7);
            pv[y * 8 + x] = mc_chroma_sample(rv, px, py, mvx & 7, mvy & 7);
          }
        encode_chroma(mx, my, pu, pv, qp_, false, coef);
        return;
      }
    }
    // intra: compare I16x16 against I4x4 (I4x4 writes rec_ directly; restore if I16 wins)
    if (cfg_.use_i4x4) {
      int X0 = mx * 16, Y0 = my * 16, W = rec_.W;
      uint8_t save[256];
      for (int y = 0; y < 16; ++y) std::memcpy(save + y * 16, &rec_.y[static_cast<size_t>(Y0 + y) * W + X0], 16);
      MbHeader tmp = hdr;
      tmp.kind = MBK_I4x4;
      int16_t c4[kCoefPerMb];
      std::memset(c4, 0, sizeof(c4));
      int c4cost = encode_i4x4(mx, my, qp_, tmp, c4);
      if (c4cost < c16) {
        hdr = tmp;
        std::memcpy(coef, c4, sizeof(c4));
      } else {
        for (int y = 0; y < 16; ++y) std::memcpy(&rec_.y[static_cast<size_t>(Y0 + y) * W + X0], save + y * 16, 16);
        hdr.kind = MBK_I16x16;
        hdr.i16_mode = static_cast<uint8_t>(i16_mode);
        encode_i16(mx, my, i16_mode, qp_, coef);
      }
    } else {
      hdr.kind = MBK_I16x16;
      hdr.i16_mode = static_cast<uint8_t>(i16_mode);
      encode_i16(mx, my, i16_mode, qp_, coef);
    }
    int cm = choose_chroma_mode(mx, my);
    hdr.chroma_mode = static_cast<uint8_t>(cm);
    int pu[64], pv[64];
    chroma_pred(0, mx, my, cm, pu);
    chroma_pred(1, mx, my, cm, pv);
    encode_chroma(mx, my, pu, pv, qp_, true, coef);
  }

  const EncoderConfig& cfg_;
  int wmb_, hmb_;
  const Planes* src_ = nullptr;
  const Planes* ref_ = nullptr;
  bool islice_ = true;
  int qp_ = 26;
  int lambda_ = 4;
  std::vector<int> mvs_;
};

void pad_frame(const uint8_t* f, int w, int h, Planes& out) {
  int W = out.W, H = out.H;
  for (int y = 0; y < H; ++y) {
    const uint8_t* row = f + static_cast<size_t>(std::min(y, h - 1)) * w;
    uint8_t* dst = &out.y[static_cast<size_t>(y) * W];
    std::memcpy(dst, row, w);
    for (int x = w; x < W; ++x) dst[x] = row[w - 1];
  }
  int w2 = w / 2, h2 = h / 2, W2 = W / 2, H2 = H / 2;
  const uint8_t* u = f + static_cast<size_t>(w) * h;
  const uint8_t* v = u + static_cast<size_t>(w2) * h2;
  for (int y = 0; y < H2; ++y) {
    const uint8_t* ru = u + static_cast<size_t>(std::min(y, h2 - 1)) * w2;
    const uint8_t* rv = v + static_cast<size_t>(std::min(y, h2 - 1)) * w2;
    uint8_t* du = &out.u[static_cast<size_t>(y) * W2];
    uint8_t* dv = &out.v[static_cast<size_t>(y) * W2];
    std::memcpy(du, ru, w2);
    std::memcpy(dv, rv, w2);
    for (int x = w2; x < W2; ++x) {
      du[x] = ru[w2 - 1];
      dv[x] = rv[w2 - 1];
    }
  }
}

}  // namespace

CpuEncoder::CpuEncoder(const EncoderConfig& cfg) : cfg_(cfg) {
  if (cfg.width <= 0 || cfg.height <= 0 || (cfg.width & 1) || (cfg.height & 1))
    throw std::runtime_error("width/height must be positive and even");
}

std::vector<uint8_t> CpuEncoder::encode(const uint8_t* frames, int nframes, int idr_pic_id) {
  SPS sps = make_sps(cfg_);
  PPS pps = make_pps(cfg_);
  std::vector<uint8_t> out = write_parameter_sets(sps, pps);
  Decoder dec;
  dec.decode(out.data(), out.size());
  FrameEncoder fe(cfg_, sps.width_mbs, sps.height_mbs);
  // the lists the decoder derives from what was written (fall-back rules included)
  {
    uint8_t sl8[2][64];
    dec.pps_scaling(pps.pps_id, &fe.sl4_[0][0], &sl8[0][0]);
  }
  Planes src, ref;
  src.alloc(sps.width_mbs * 16, sps.height_mbs * 16);
  ref.alloc(src.W, src.H);
  stats_.clear();
  recon_.clear();
  recon_unf_.clear();
  size_t fsize = static_cast<size_t>(cfg_.width) * cfg_.height * 3 / 2;
  int frame_num = 0;
  // keyint <= 0: the first picture is the only IDR (as the GPU encoders' keyint 0)
  const int keyint = cfg_.keyint > 0 ? cfg_.keyint : std::max(1, nframes);
  for (int f = 0; f < nframes; ++f) {
    pad_frame(frames + f * fsize, cfg_.width, cfg_.height, src);
    bool idr = (f % keyint) == 0;
    if (idr) frame_num = 0;
    int qp = std::max(0, std::min(51, cfg_.qp + (idr ? -3 : 0)));
    fe.encode(src, idr ? nullptr : &ref, idr, qp);
    SliceHeader sh;
    sh.nal_unit_type = idr ? NAL_IDR : NAL_SLICE;
    sh.nal_ref_idc = idr ? 3 : 2;
    sh.slice_type = idr ? SLICE_I : SLICE_P;
    sh.frame_num = frame_num;
    sh.idr_pic_id = (idr_pic_id + f / keyint) & 0xFFFF;
    sh.slice_qp_delta = qp - pps.pic_init_qp;
    sh.disable_deblocking_filter_idc = cfg_.deblock ? 0 : 1;
    std::vector<uint8_t> nal =
        pps.entropy_coding_mode
            ? write_slice_nal_cabac(sps, pps, sh, fe.mbs_.data(), fe.coef_.data(), sps.width_mbs * sps.height_mbs)
            : write_slice_nal(sps, pps, sh, fe.mbs_.data(), fe.coef_.data(), sps.width_mbs * sps.height_mbs);
    out.insert(out.end(), nal.begin(), nal.end());
    recon_unf_.insert(recon_unf_.end(), fe.rec_.y.begin(), fe.rec_.y.end());
    recon_unf_.insert(recon_unf_.end(), fe.rec_.u.begin(), fe.rec_.u.end());
    recon_unf_.insert(recon_unf_.end(), fe.rec_.v.begin(), fe.rec_.v.end());
    // decode to obtain the deblocked reference (drift-free by construction)
    dec.decode(nal.data(), nal.size());
    dec.flush();
    DecodedPicture& pic = dec.out().back();
    ref.y = pic.y;
    ref.u = pic.u;
    ref.v = pic.v;
    std::vector<uint8_t> crop = pic.cropped_i420();
    // PSNR-Y against the source
    double se = 0;
    const uint8_t* s = frames + f * fsize;
    for (size_t i = 0; i < static_cast<size_t>(cfg_.width) * cfg_.height; ++i) {
      double d = static_cast<double>(s[i]) - crop[i];
      se += d * d;
    }
    double mse = se / (static_cast<double>(cfg_.width) * cfg_.height);
    FrameStats st;
    st.type = sh.slice_type;
    st.qp = qp;
    st.bytes = static_cast<int>(nal.size());
    st.psnr_y = mse <= 1e-10 ? 100.0 : 10.0 * std::log10(255.0 * 255.0 / mse);
    stats_.push_back(st);
    recon_.insert(recon_.end(), crop.begin(), crop.end());
    dec.out().clear();
    ++frame_num;
  }
  return out;
}

}  // namespace h264
}  // namespace mivc
