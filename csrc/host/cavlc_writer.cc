#include "cavlc_writer.h"

#include <algorithm>
#include <cstdlib>
#include <stdexcept>

namespace mivc {
namespace h264 {

namespace {

inline int coeff_token_table(int nc) {
  if (nc < 2) return 0;
  if (nc < 4) return 1;
  if (nc < 8) return 2;
  return 3;
}

// level_prefix / level_suffix coding for one level (clause 9.2.2.1 inverted)
inline void write_level(BitWriter& bw, int level_code, int suffix_len) {
  int prefix, suffix = 0, suffix_size = 0, base;
  if (suffix_len == 0) {
    if (level_code < 14) {
      bw.put(1, level_code + 1);  // level_code zeros then a one
      return;
    }
    if (level_code < 30) {
      bw.put(1, 15);  // prefix 14
      bw.put(static_cast<uint32_t>(level_code - 14), 4);
      return;
    }
    base = 30;
  } else {
    if (level_code < (15 << suffix_len)) {
      prefix = level_code >> suffix_len;
      bw.put(1, prefix + 1);
      bw.put(static_cast<uint32_t>(level_code & ((1 << suffix_len) - 1)), suffix_len);
      return;
    }
    base = 15 << suffix_len;
  }
  int rem = level_code - base;
  if (rem < 4096) {
    prefix = 15;
    suffix = rem;
  } else {
    prefix = 16;
    while (true) {
      int r = rem - ((1 << (prefix - 3)) - 4096);
      if (r < (1 << (prefix - 3))) {
        suffix = r;
        break;
      }
      ++prefix;
    }
  }
  suffix_size = prefix - 3;
  bw.put(0, prefix);
  bw.put(1, 1);
  bw.put(static_cast<uint32_t>(suffix), suffix_size);
}

}  // namespace

int cavlc_write_block(BitWriter& bw, const int16_t* coef, int start, int end, int max_num_coeff, int nc) {
  int levels[16], runs[16];
  int total = 0, total_zeros = 0;
  // gather non-zero coefficients from the highest frequency down
  int last = -1;
  for (int i = end; i >= start; --i)
    if (coef[i]) {
      last = i;
      break;
    }
  if (last >= 0) {
    int run = 0;
    for (int i = last; i >= start; --i) {
      if (coef[i]) {
        if (total > 0) runs[total - 1] = run;
        levels[total++] = coef[i];
        run = 0;
      } else {
        ++run;
        ++total_zeros;
      }
    }
    runs[total - 1] = run;  // zeros below the lowest coefficient (implicit, = zerosLeft at the end)
  }
  int t1 = 0;
  for (int i = 0; i < total && t1 < 3; ++i) {
    if (levels[i] == 1 || levels[i] == -1) ++t1; else break;
  }
  // coeff_token
  if (nc == -1) {
    bw.put(kChromaDcCoeffTokenBits[total * 4 + t1], kChromaDcCoeffTokenLen[total * 4 + t1]);
  } else {
    int t = coeff_token_table(nc);
    bw.put(kCoeffTokenBits[t][total * 4 + t1], kCoeffTokenLen[t][total * 4 + t1]);
  }
  if (total == 0) return 0;
  for (int i = 0; i < t1; ++i) bw.put_bit(levels[i] < 0);
  int suffix_len = (total > 10 && t1 < 3) ? 1 : 0;
  for (int i = t1; i < total; ++i) {
    int lv = levels[i];
    int level_code = lv > 0 ? 2 * lv - 2 : -2 * lv - 1;
    if (i == t1 && t1 < 3) level_code -= 2;
    write_level(bw, level_code, suffix_len);
    if (suffix_len == 0) suffix_len = 1;
    if (std::abs(lv) > (3 << (suffix_len - 1)) && suffix_len < 6) ++suffix_len;
  }
  int span = end - start + 1;
  if (total < span) {
    if (max_num_coeff == 4) {
      bw.put(kChromaDcTotalZerosBits[total - 1][total_zeros], kChromaDcTotalZerosLen[total - 1][total_zeros]);
    } else {
      bw.put(kTotalZerosBits[total - 1][total_zeros], kTotalZerosLen[total - 1][total_zeros]);
    }
  }
  int zeros_left = total_zeros;
  for (int i = 0; i < total - 1 && zeros_left > 0; ++i) {
    int rb = runs[i];
    int tab = std::min(zeros_left, 7) - 1;
    bw.put(kRunBeforeBits[tab][rb], kRunBeforeLen[tab][rb]);
    zeros_left -= rb;
  }
  return total;
}

int derive_cbp(const MbHeader& mb, const int16_t* coef) {
  if (mb.kind == MBK_IPCM || mb.kind == MBK_PSKIP) {
    if (mb.kind == MBK_IPCM) return 0x2F;
  }
  int luma = 0;
  for (int b8 = 0; b8 < 4; ++b8) {
    bool nz = false;
    for (int b = 0; b < 4 && !nz; ++b) {
      const int16_t* c = coef + COEF_LUMA + (b8 * 4 + b) * 16;
      for (int i = (mb.kind == MBK_I16x16 && !(mb.flags & MBF_T8x8) ? 1 : 0); i < 16; ++i)
        if (c[i]) {
          nz = true;
          break;
        }
    }
    if (nz) luma |= 1 << b8;
  }
  if (mb.kind == MBK_I16x16 && luma) luma = 15;
  int chroma = 0;
  for (int i = 0; i < 2 * 4 * 16; ++i)
    if ((i & 15) && coef[COEF_CHROMA_AC + i]) {
      chroma = 2;
      break;
    }
  if (!chroma)
    for (int i = 0; i < 8; ++i)
      if (coef[COEF_CHROMA_DC + i]) {
        chroma = 1;
        break;
      }
  return luma | (chroma << 4);
}

namespace {

struct MbCtx {
  int kind = -1;      // final coded kind (MBK_PSKIP when skipped); -1 = not available
  uint8_t tc[16 + 8]; // TotalCoeff per luma 4x4 (AC for I16x16), then Cb[4], Cr[4] AC
  int8_t ref[16];     // per 4x4 block, -1 intra
  int16_t mv[16][2];
  uint8_t i4[16];
};

inline int median3(int a, int b, int c) { return std::max(std::min(a, b), std::min(std::max(a, b), c)); }

class SliceWriter {
 public:
  SliceWriter(const SPS& sps, const PPS& pps, const SliceHeader& sh, const MbHeader* mbs, const int16_t* coef,
              int num_mbs)
      : sps_(sps), pps_(pps), sh_(sh), mbs_(mbs), coef_(coef), w_(sps.width_mbs), h_(sps.height_mbs),
        num_(num_mbs), ctx_(static_cast<size_t>(sps.width_mbs) * sps.height_mbs) {}

  void run(BitWriter& bw, SliceStats* st) {
    int qp_prev = pps_.pic_init_qp + sh_.slice_qp_delta;
    int skip_run = 0;
    const bool pslice = sh_.slice_type == SLICE_P;
    for (int addr = sh_.first_mb; addr < sh_.first_mb + num_; ++addr) {
      const MbHeader& mb = mbs_[addr];
      const int16_t* c = coef_ + static_cast<size_t>(addr) * kCoefPerMb;
      MbCtx& m = ctx_[addr];
      int mx = addr % w_, my = addr / w_;
      int cbp = derive_cbp(mb, c);
      if (mb.kind == MBK_PSKIP && (cbp != 0 || !pslice)) throw std::runtime_error("P_Skip hint with residual");
      bool inter = !mbk_is_intra(mb.kind);
      if (inter && !pslice) throw std::runtime_error("inter MB in I slice");
      // ---- skip decision (clause 8.4.1.1)
      if (pslice && inter && cbp == 0 && (mb.kind == MBK_P16x16 || mb.kind == MBK_PSKIP)) {
        int smv[2];
        skip_mv(mx, my, addr, smv);
        if (smv[0] == mb.mv[0][0][0] && smv[1] == mb.mv[0][0][1]) {
          m.kind = MBK_PSKIP;
          std::fill(m.tc, m.tc + 24, 0);
          for (int b = 0; b < 16; ++b) {
            m.ref[b] = 0;
            m.mv[b][0] = smv[0];
            m.mv[b][1] = smv[1];
            m.i4[b] = 2;
          }
          ++skip_run;
          if (st) ++st->skipped;
          continue;
        }
      }
      if (pslice) {
        bw.put_ue(skip_run);
        skip_run = 0;
      }
      write_mb(bw, mb, c, cbp, addr, mx, my, pslice, qp_prev);
      if (st) {
        if (inter) ++st->coded_inter; else ++st->intra;
      }
    }
    if (pslice && skip_run > 0) bw.put_ue(skip_run);
  }

 private:
  bool avail(int mx, int my) const {
    if (mx < 0 || my < 0 || mx >= w_ || my >= h_) return false;
    int a = my * w_ + mx;
    return a >= sh_.first_mb && ctx_[a].kind >= 0;
  }
  const MbCtx* at(int mx, int my) const { return avail(mx, my) ? &ctx_[my * w_ + mx] : nullptr; }

  // neighbour 4x4 block (bx,by may be -1 or 4) relative to the current MB
  // returns the ctx of the MB holding it and the block's raster index; nullptr if unavailable
  const MbCtx* nb_block(int mx, int my, const MbCtx* cur, int bx, int by, int* blk_raster) const {
    int dmx = 0, dmy = 0;
    if (bx < 0) { dmx = -1; bx += 4; }
    if (bx > 3) { dmx = 1; bx -= 4; }
    if (by < 0) { dmy = -1; by += 4; }
    *blk_raster = bx + 4 * by;
    if (dmx == 0 && dmy == 0) return cur;
    return at(mx + dmx, my + dmy);
  }

  // MV predictor for a partition whose top-left 4x4 block is (bx,by) with width bw4 (in 4x4 units)
  void mvp(int mx, int my, const MbCtx* cur, int bx, int by, int bw4, int part_shape, int part_idx, int out[2]) {
    int ra, rb, rc;
    const MbCtx* A = nb_block(mx, my, cur, bx - 1, by, &ra);
    const MbCtx* B = nb_block(mx, my, cur, bx, by - 1, &rb);
    const MbCtx* C = nb_block(mx, my, cur, bx + bw4, by - 1, &rc);
    // C is unavailable when it lies in the current MB but is not yet decoded, or to the right
    if (C == cur && !cur_decoded_[rc]) C = nullptr;
    if (C && C != cur && (bx + bw4 > 3) && by > 0) C = nullptr;  // right MB, not yet decoded
    if (!C) {
      C = nb_block(mx, my, cur, bx - 1, by - 1, &rc);
      if (C == cur && !cur_decoded_[rc]) C = nullptr;
    }
    int refA = -1, refB = -1, refC = -1, mA[2] = {0, 0}, mB[2] = {0, 0}, mC[2] = {0, 0};
    auto load = [&](const MbCtx* N, int r, int& ref, int* m) {
      if (!N) return;
      if (N == cur) {
        ref = cur_ref_[r];
        m[0] = cur_mv_[r][0];
        m[1] = cur_mv_[r][1];
      } else {
        ref = N->ref[r];
        m[0] = N->mv[r][0];
        m[1] = N->mv[r][1];
      }
    };
    load(A, ra, refA, mA);
    load(B, rb, refB, mB);
    load(C, rc, refC, mC);
    if (!B && !C && A) {
      refB = refC = refA;
      mB[0] = mC[0] = mA[0];
      mB[1] = mC[1] = mA[1];
    }
    const int ref = 0;
    if (part_shape == 1) {  // 16x8
      if (part_idx == 0 && refB == ref) { out[0] = mB[0]; out[1] = mB[1]; return; }
      if (part_idx == 1 && refA == ref) { out[0] = mA[0]; out[1] = mA[1]; return; }
    } else if (part_shape == 2) {  // 8x16
      if (part_idx == 0 && refA == ref) { out[0] = mA[0]; out[1] = mA[1]; return; }
      if (part_idx == 1 && refC == ref) { out[0] = mC[0]; out[1] = mC[1]; return; }
    }
    int n = (refA == ref) + (refB == ref) + (refC == ref);
    if (n == 1) {
      const int* m = refA == ref ? mA : (refB == ref ? mB : mC);
      out[0] = m[0];
      out[1] = m[1];
      return;
    }
    out[0] = median3(mA[0], mB[0], mC[0]);
    out[1] = median3(mA[1], mB[1], mC[1]);
  }

  void reset_cur() {
    for (int i = 0; i < 16; ++i) {
      cur_decoded_[i] = false;
      cur_ref_[i] = -1;
      cur_mv_[i][0] = cur_mv_[i][1] = 0;
    }
  }

  void skip_mv(int mx, int my, int addr, int out[2]) {
    (void)addr;
    out[0] = out[1] = 0;
    const MbCtx* A = at(mx - 1, my);
    const MbCtx* B = at(mx, my - 1);
    if (!A || !B) return;
    if (A->ref[3] == 0 && A->mv[3][0] == 0 && A->mv[3][1] == 0) return;   // block (3,0)
    if (B->ref[12] == 0 && B->mv[12][0] == 0 && B->mv[12][1] == 0) return; // block (0,3)
    reset_cur();
    MbCtx dummy;
    mvp(mx, my, &dummy, 0, 0, 4, 0, 0, out);
  }

  int nc_luma(int mx, int my, const MbCtx& cur, int bx, int by) {
    int r;
    const MbCtx* A = nb_block(mx, my, &cur, bx - 1, by, &r);
    int nA = A ? A->tc[kRasterToBlk[r]] : 0;
    int rb;
    const MbCtx* B = nb_block(mx, my, &cur, bx, by - 1, &rb);
    int nB = B ? B->tc[kRasterToBlk[rb]] : 0;
    if (A && B) return (nA + nB + 1) >> 1;
    if (A) return nA;
    if (B) return nB;
    return 0;
  }
  int nc_chroma(int mx, int my, const MbCtx& cur, int comp, int cx, int cy) {
    const MbCtx* A = cx > 0 ? &cur : at(mx - 1, my);
    const MbCtx* B = cy > 0 ? &cur : at(mx, my - 1);
    int ax = cx > 0 ? cx - 1 : 1, by_ = cy > 0 ? cy - 1 : 1;
    int nA = A ? A->tc[16 + comp * 4 + cy * 2 + ax] : 0;
    int nB = B ? B->tc[16 + comp * 4 + by_ * 2 + cx] : 0;
    if (A && B) return (nA + nB + 1) >> 1;
    if (A) return nA;
    if (B) return nB;
    return 0;
  }

  int pred_i4_mode(int mx, int my, const MbCtx& cur, int bx, int by) {
    int ra, rb;
    const MbCtx* A = nb_block(mx, my, &cur, bx - 1, by, &ra);
    const MbCtx* B = nb_block(mx, my, &cur, bx, by - 1, &rb);
    if (!A || !B) return 2;
    // dcPredModePredictedFlag also when a neighbour is inter-coded under constrained intra
    // prediction (8.3.1.1)
    if (pps_.constrained_intra_pred && (!mbk_is_intra(A->kind) || !mbk_is_intra(B->kind))) return 2;
    int ma = (A->kind == MBK_I4x4 || A->kind == MBK_I8x8) ? A->i4[kRasterToBlk[ra]] : 2;
    int mb = (B->kind == MBK_I4x4 || B->kind == MBK_I8x8) ? B->i4[kRasterToBlk[rb]] : 2;
    return std::min(ma, mb);
  }

  void write_mb(BitWriter& bw, const MbHeader& mb, const int16_t* c, int cbp, int addr, int mx, int my,
                bool pslice, int& qp_prev) {
    MbCtx& m = ctx_[addr];
    int kind = mb.kind == MBK_PSKIP ? MBK_P16x16 : mb.kind;
    m.kind = kind;
    std::fill(m.tc, m.tc + 24, 0);
    for (int b = 0; b < 16; ++b) {
      m.ref[b] = -1;
      m.mv[b][0] = m.mv[b][1] = 0;
      m.i4[b] = 2;
    }
    int cbp_luma = cbp & 15, cbp_chroma = cbp >> 4;
    // ---- mb_type
    int intra_offset = pslice ? 5 : 0;
    switch (kind) {
      case MBK_P16x16: bw.put_ue(0); break;
      case MBK_P16x8: bw.put_ue(1); break;
      case MBK_P8x16: bw.put_ue(2); break;
      case MBK_P8x8: bw.put_ue(3); break;
      case MBK_I4x4:
      case MBK_I8x8: bw.put_ue(intra_offset + 0); break;
      case MBK_I16x16:
        bw.put_ue(intra_offset + 1 + mb.i16_mode + 4 * cbp_chroma + (cbp_luma ? 12 : 0));
        break;
      case MBK_IPCM: bw.put_ue(intra_offset + 25); break;
      default: throw std::runtime_error("bad mb kind");
    }
    if (kind == MBK_IPCM) {
      bw.align_zero();
      // pcm_sample_luma / chroma: BitDepthY / BitDepthC bits each (7.3.5)
      for (int i = 0; i < 384; ++i) {
        const int bd = i < 256 ? sps_.bit_depth_luma : sps_.bit_depth_chroma;
        bw.put(static_cast<uint32_t>(c[i]) & ((1u << bd) - 1), bd);
      }
      std::fill(m.tc, m.tc + 24, 16);
      qp_prev = qp_prev;  // QP unchanged (QP'Y of I_PCM for deblocking handled by decoder: qPp = 0)
      return;
    }
    const bool t8 = (kind == MBK_I8x8) || ((mb.flags & MBF_T8x8) && !mbk_is_intra(kind));
    if ((kind == MBK_I4x4 || kind == MBK_I8x8) && pps_.transform_8x8_mode) bw.put_bit(kind == MBK_I8x8);
    if (kind == MBK_I8x8 && !pps_.transform_8x8_mode) throw std::runtime_error("I8x8 without transform_8x8_mode");
    // ---- prediction info
    if (kind == MBK_I8x8) {
      for (int b8 = 0; b8 < 4; ++b8) {
        int bx = (b8 & 1) * 2, by = (b8 >> 1) * 2;
        int pred = pred_i4_mode(mx, my, m, bx, by);
        int mode = mb.i4_modes[b8 * 4];
        if (mode == pred) {
          bw.put_bit(1);
        } else {
          bw.put_bit(0);
          bw.put(mode < pred ? mode : mode - 1, 3);
        }
        for (int k = 0; k < 4; ++k) m.i4[kRasterToBlk[bx + (k & 1) + 4 * (by + (k >> 1))]] = static_cast<uint8_t>(mode);
      }
    }
    if (kind == MBK_I4x4) {
      for (int blk = 0; blk < 16; ++blk) {
        int bx = kBlkX[blk], by = kBlkY[blk];
        int pred = pred_i4_mode(mx, my, m, bx, by);
        int mode = mb.i4_modes[blk];
        if (mode == pred) {
          bw.put_bit(1);
        } else {
          bw.put_bit(0);
          bw.put(mode < pred ? mode : mode - 1, 3);
        }
        m.i4[blk] = static_cast<uint8_t>(mode);
      }
    }
    if (kind == MBK_I4x4 || kind == MBK_I16x16 || kind == MBK_I8x8) bw.put_ue(mb.chroma_mode);
    if (!mbk_is_intra(kind)) {
      reset_cur();
      auto set_part = [&](int bx, int by, int w4, int h4, int mvx, int mvy) {
        for (int y = by; y < by + h4; ++y)
          for (int x = bx; x < bx + w4; ++x) {
            int r = x + 4 * y;
            cur_ref_[r] = 0;
            cur_mv_[r][0] = mvx;
            cur_mv_[r][1] = mvy;
            cur_decoded_[r] = true;
          }
      };
      int p[2];
      if (kind == MBK_P16x16) {
        mvp(mx, my, &m, 0, 0, 4, 0, 0, p);
        bw.put_se(mb.mv[0][0][0] - p[0]);
        bw.put_se(mb.mv[0][0][1] - p[1]);
        set_part(0, 0, 4, 4, mb.mv[0][0][0], mb.mv[0][0][1]);
      } else if (kind == MBK_P16x8) {
        for (int part = 0; part < 2; ++part) {
          const int16_t* v = mb.mv[0][part * 2];
          mvp(mx, my, &m, 0, part * 2, 4, 1, part, p);
          bw.put_se(v[0] - p[0]);
          bw.put_se(v[1] - p[1]);
          set_part(0, part * 2, 4, 2, v[0], v[1]);
        }
      } else if (kind == MBK_P8x16) {
        for (int part = 0; part < 2; ++part) {
          const int16_t* v = mb.mv[0][part];
          mvp(mx, my, &m, part * 2, 0, 2, 2, part, p);
          bw.put_se(v[0] - p[0]);
          bw.put_se(v[1] - p[1]);
          set_part(part * 2, 0, 2, 4, v[0], v[1]);
        }
      } else {  // P_8x8, all sub_mb_type 0 (8x8)
        for (int s = 0; s < 4; ++s) bw.put_ue(0);
        for (int s = 0; s < 4; ++s) {
          int bx = (s & 1) * 2, by = (s >> 1) * 2;
          mvp(mx, my, &m, bx, by, 2, 0, 0, p);
          bw.put_se(mb.mv[0][s][0] - p[0]);
          bw.put_se(mb.mv[0][s][1] - p[1]);
          set_part(bx, by, 2, 2, mb.mv[0][s][0], mb.mv[0][s][1]);
        }
      }
      for (int r = 0; r < 16; ++r) {
        m.ref[r] = cur_ref_[r];
        m.mv[r][0] = cur_mv_[r][0];
        m.mv[r][1] = cur_mv_[r][1];
      }
    }
    // ---- coded_block_pattern
    if (kind != MBK_I16x16) {
      const uint8_t* tab = mbk_is_intra(kind) ? kGolombToIntraCbp : kGolombToInterCbp;
      int code = -1;
      for (int i = 0; i < 48; ++i)
        if (tab[i] == cbp) {
          code = i;
          break;
        }
      bw.put_ue(code);
      if (cbp_luma && pps_.transform_8x8_mode && !mbk_is_intra(kind)) bw.put_bit(t8 ? 1 : 0);
    }
    if (cbp_luma == 0 && cbp_chroma == 0 && kind != MBK_I16x16) return;
    // ---- mb_qp_delta
    // mb_qp_delta in -(26 + QpBdOffsetY / 2) .. 25 + QpBdOffsetY / 2, modulo 52 + QpBdOffsetY (7.4.5)
    const int qpbd = 6 * (sps_.bit_depth_luma - 8);
    int d = mb.qp - qp_prev;
    if (d < -(26 + qpbd / 2)) d += 52 + qpbd;
    if (d > 25 + qpbd / 2) d -= 52 + qpbd;
    bw.put_se(d);
    qp_prev = mb.qp;
    // ---- residual
    if (kind == MBK_I16x16) {
      int nc = nc_luma(mx, my, m, 0, 0);
      cavlc_write_block(bw, c + COEF_LUMA_DC, 0, 15, 16, nc);
    }
    for (int b8 = 0; b8 < 4; ++b8) {
      for (int b4 = 0; b4 < 4; ++b4) {
        int blk = b8 * 4 + b4;
        if (!(cbp_luma & (1 << b8))) continue;
        int nc = nc_luma(mx, my, m, kBlkX[blk], kBlkY[blk]);
        const int16_t* blkc = c + COEF_LUMA + blk * 16;
        int16_t il[16];
        if (t8 && pps_.transform_8x8_mode) {  // 8x8 levels as four interleaved 4x4 blocks (7.3.5.3.2)
          for (int i = 0; i < 16; ++i) il[i] = c[COEF_LUMA + b8 * 64 + 4 * i + b4];
          blkc = il;
        }
        int tc = kind == MBK_I16x16 ? cavlc_write_block(bw, blkc, 1, 15, 15, nc)
                                    : cavlc_write_block(bw, blkc, 0, 15, 16, nc);
        m.tc[blk] = static_cast<uint8_t>(tc);
      }
    }
    if (cbp_chroma) {
      for (int comp = 0; comp < 2; ++comp) cavlc_write_block(bw, c + COEF_CHROMA_DC + comp * 4, 0, 3, 4, -1);
    }
    if (cbp_chroma & 2) {
      for (int comp = 0; comp < 2; ++comp)
        for (int b = 0; b < 4; ++b) {
          int nc = nc_chroma(mx, my, m, comp, b & 1, b >> 1);
          int tc = cavlc_write_block(bw, c + COEF_CHROMA_AC + (comp * 4 + b) * 16, 1, 15, 15, nc);
          m.tc[16 + comp * 4 + b] = static_cast<uint8_t>(tc);
        }
    }
  }

  const SPS& sps_;
  const PPS& pps_;
  const SliceHeader& sh_;
  const MbHeader* mbs_;
  const int16_t* coef_;
  int w_, h_, num_;
  std::vector<MbCtx> ctx_;
  bool cur_decoded_[16];
  int cur_ref_[16];
  int cur_mv_[16][2];
};

}  // namespace

std::vector<uint8_t> write_slice_nal(const SPS& sps, const PPS& pps, const SliceHeader& sh, const MbHeader* mbs,
                                     const int16_t* coef, int num_mbs, SliceStats* stats) {
  if (pps.entropy_coding_mode) throw std::runtime_error("CAVLC writer called with CABAC PPS");
  BitWriter bw;
  write_slice_header(bw, sh, sps, pps);
  SliceWriter w(sps, pps, sh, mbs, coef, num_mbs);
  w.run(bw, stats);
  bw.trailing();
  std::vector<uint8_t> out;
  out.reserve(bw.bytes().size() + bw.bytes().size() / 64 + 16);
  append_nal(out, sh.nal_ref_idc, sh.nal_unit_type, bw.bytes());
  if (stats) stats->bits = static_cast<int>(out.size() * 8);
  return out;
}

std::vector<uint8_t> write_parameter_sets(const SPS& sps, const PPS& pps) {
  std::vector<uint8_t> out;
  BitWriter a;
  write_sps(a, sps);
  append_nal(out, 3, NAL_SPS, a.bytes());
  BitWriter b;
  write_pps(b, pps);
  append_nal(out, 3, NAL_PPS, b.bytes());
  return out;
}

}  // namespace h264
}  // namespace mivc
