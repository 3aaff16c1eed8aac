// gfx950 HEVC decode: sample reconstruction of host-parsed pictures (csrc/host/hevc_dec.cc
// resolves every syntax element, vector, reference and boundary strength; this file does
// the sample work of clauses 8.4 - 8.7) for B independent segments per launch.
//
// Reference parity: the reference worker decodes its piece with `ffmpeg -i` before
// re-encoding (client.go:115); the north star names H.264/HEVC decode as native kernels.
//
// Per picture step (picture t of every slot, DPB slots chosen by the host):
//   hevcd_residual   one wave per coded transform block: scaling (flat or scaling list),
//                    inverse DCT 4..32 / DST 4x4 as two wave-level matrix products, transform
//                    skip, cu_transquant_bypass, PCM samples -> residual planes
//   hevcd_inter      one wave per 8x8 luma block: 8-tap / 4-tap fractional interpolation
//                    from the slot's DPB, uni / bi / explicit weighted prediction + residual
//   hevcd_intra      one workgroup per slot, waves own CTB rows (2-CTB wavefront lag, row
//                    progress in LDS): every intra transform block in decoding order --
//                    reference availability (z-scan / slice / tile / constrained intra),
//                    substitution, [1 2 1] or strong filtering, planar / DC / angular
//   hevcd_deblock    vertical then horizontal edges, one lane per 4-sample edge segment
//                    (luma) and per 2-sample chroma segment
//   hevcd_sao        band / edge offsets per CTB from the deblocked copy
#include "hevc_common.h"
#include "hevc_decode.h"

namespace mivc {
namespace gpu {

namespace {

// 32-point DCT matrix (8.6.4.2) as a compile-time table in constant memory
constexpr int dct_val(int k, int n) {
  if (k == 0) return 64;
  int t = ((2 * n + 1) * k) & 127;
  int sign = 1;
  if (t > 64) t = 128 - t;
  if (t > 32) {
    t = 64 - t;
    sign = -1;
  }
  int mag = 0;
  if (t & 1) {
    const int v[16] = {90, 90, 88, 85, 82, 78, 73, 67, 61, 54, 46, 38, 31, 22, 13, 4};
    mag = v[(t - 1) >> 1];
  } else if (t & 2) {
    const int v[8] = {90, 87, 80, 70, 57, 43, 25, 9};
    mag = v[((t >> 1) - 1) >> 1];
  } else if (t & 4) {
    const int v[4] = {89, 75, 50, 18};
    mag = v[((t >> 2) - 1) >> 1];
  } else if (t & 8) {
    mag = (t >> 3) == 1 ? 83 : 36;
  } else if (t == 16) {
    mag = 64;
  }
  return sign * mag;
}
struct DctTab {
  int8_t m[32][32];
  int8_t dst[4][4];
  constexpr DctTab() : m(), dst() {
    for (int k = 0; k < 32; ++k)
      for (int n = 0; n < 32; ++n) m[k][n] = static_cast<int8_t>(dct_val(k, n));
    const int d[16] = {29, 55, 74, 84, 74, 74, 0, -74, 84, -29, -74, 55, 55, -84, 74, -29};
    for (int i = 0; i < 16; ++i) dst[i >> 2][i & 3] = static_cast<int8_t>(d[i]);
  }
};
__constant__ DctTab kDctTab = DctTab();

__device__ __forceinline__ int clip3d(int lo, int hi, int v) { return v < lo ? lo : (v > hi ? hi : v); }

struct Tu {
  int x, y, log2, cidx, qp, flags;
  uint32_t coef;
};
__device__ __forceinline__ Tu load_tu(const uint8_t* p) {
  const uint32_t w0 = *reinterpret_cast<const uint32_t*>(p);
  const uint32_t w1 = *reinterpret_cast<const uint32_t*>(p + 4);
  Tu t;
  t.x = static_cast<int>(w0 & 0xFFFF);
  t.y = static_cast<int>(w0 >> 16);
  t.log2 = static_cast<int>(w1 & 255);
  t.cidx = static_cast<int>((w1 >> 8) & 255);
  t.qp = static_cast<int>((w1 >> 16) & 255);
  t.flags = static_cast<int>(w1 >> 24);
  t.coef = *reinterpret_cast<const uint32_t*>(p + 8);
  return t;
}

constexpr uint8_t DM_INTRA = 1, DM_NOFILTER = 2, DM_INTER = 4, DM_SPLIT = 8;  // hevc_dec.h DecMv4

struct Mv4 {
  int mv[2][2];
  int ref[2];
  int flags, qp;
};
__device__ __forceinline__ Mv4 load_mv4(const uint8_t* p) {
  const int16_t* m = reinterpret_cast<const int16_t*>(p);
  Mv4 r;
  r.mv[0][0] = m[0];
  r.mv[0][1] = m[1];
  r.mv[1][0] = m[2];
  r.mv[1][1] = m[3];
  r.ref[0] = p[8];
  r.ref[1] = p[9];
  r.flags = p[10];
  r.qp = static_cast<int8_t>(p[11]);
  return r;
}

// motion of the 4x4 luma block at (x, y): the 8x8 record, or for a DM_SPLIT record the
// 4x4 entry its first 4 bytes index in mvf_sub (csrc/host/hevc_dec.h DecPicture::mvf)
__device__ __forceinline__ Mv4 mv_at(const HevcDecParams& a, const uint8_t* mvf8, int x, int y) {
  const uint8_t* p = mvf8 + (static_cast<size_t>(y >> 3) * (a.W >> 3) + (x >> 3)) * 12;
  if (p[10] & DM_SPLIT) {
    const uint32_t idx = *reinterpret_cast<const uint32_t*>(p);
    p = a.mvf_sub + (static_cast<size_t>(idx) * 4 + ((y >> 2) & 1) * 2 + ((x >> 2) & 1)) * 12;
  }
  return load_mv4(p);
}

constexpr uint8_t DT_DST = 1, DT_TSKIP = 2, DT_BYPASS = 4, DT_INTRA = 8, DT_SCALING = 16, DT_PCM = 32;

__device__ __forceinline__ size_t plane_size(const HevcDecParams& a, int c) {
  return c ? static_cast<size_t>(a.W / 2) * (a.H / 2) : static_cast<size_t>(a.W) * a.H;
}
__device__ __forceinline__ uint16_t* dpb_plane(const HevcDecParams& a, int b, int buf, int c) {
  return a.dpb[c] + (static_cast<size_t>(b) * a.D + buf) * plane_size(a, c);
}

}  // namespace

// ------------------------------------------------------------------ residuals (8.6.2 - 8.6.4)
__global__ __launch_bounds__(64) void hevcd_residual(HevcDecParams a) {
  __shared__ int R[32 * 32];
  __shared__ int S[32 * 32];
  const int b = blockIdx.y;
  if (!a.run[b]) return;
  const int i = a.tu_base[b] + static_cast<int>(blockIdx.x);
  if (i >= a.tu_base[b + 1]) return;
  const Tu t = load_tu(a.tus + static_cast<size_t>(i) * 12);
  const int lane = lane_id();
  const int n = 1 << t.log2, nn = n * n;
  const int bdv = t.cidx ? a.bdc : a.bd;
  // sparse levels (hevc_dec.cc push_tu): 64-bit mask of the coded 4x4 groups, then 16
  // levels per coded group
  const int16_t* lp = a.coefs + a.coef_base[b] + t.coef;
  uint64_t cgm = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) cgm |= static_cast<uint64_t>(static_cast<uint16_t>(lp[k])) << (16 * k);
  const int16_t* cgv = lp + 4;
  const int gs = n >> 2;
  auto lv = [&](int k) -> int {  // level at raster position k of the block
    const int y = k >> t.log2, x = k & (n - 1);
    const int cg = (y >> 2) * gs + (x >> 2);
    if (!((cgm >> cg) & 1ull)) return 0;
    const int idx = __popcll(cgm & ((1ull << cg) - 1ull));
    return cgv[idx * 16 + (y & 3) * 4 + (x & 3)];
  };
  const int pw = t.cidx ? a.W / 2 : a.W;
  int16_t* dst = a.res[t.cidx] + static_cast<size_t>(b) * plane_size(a, t.cidx) + static_cast<size_t>(t.y) * pw + t.x;
  if (t.flags & (DT_BYPASS | DT_PCM)) {  // residual = the coded values (PCM: the samples)
    for (int k = lane; k < nn; k += 64) dst[(k >> t.log2) * pw + (k & (n - 1))] = static_cast<int16_t>(lv(k));
    return;
  }
  // scaling (8.6.3): m = 16 (flat) or ScalingFactor; transform-skipped blocks > 4x4 stay flat
  const int qp = t.qp, bdshift = bdv + t.log2 - 5;
  const int ls = hevc::kLevelScale[qp % 6] << (qp / 6);
  const bool tskip = (t.flags & DT_TSKIP) != 0;
  const uint8_t* sl = nullptr;
  if ((t.flags & DT_SCALING) && a.scaling && !(tskip && t.log2 > 2))
    sl = a.scaling + static_cast<size_t>(b) * 8160 + (t.log2 == 2 ? 0 : t.log2 == 3 ? 96 : t.log2 == 4 ? 480 : 2016) +
         (((t.flags & DT_INTRA) ? 0 : 3) + t.cidx) * nn;
  for (int k = lane; k < nn; k += 64) {
    const int m = sl ? sl[k] : 16;
    const long long v = static_cast<long long>(lv(k)) * m * ls + (1ll << (bdshift - 1));
    R[(k >> t.log2) * 32 + (k & (n - 1))] = clip3d(-32768, 32767, static_cast<int>(v >> bdshift));
  }
  wave_sync();
  const int sh2 = 20 - bdv, rnd2 = 1 << (sh2 - 1);
  if (tskip) {
    const int ts = 5 + t.log2;
    for (int k = lane; k < nn; k += 64) {
      const int y = k >> t.log2, x = k & (n - 1);
      dst[y * pw + x] = static_cast<int16_t>(((R[y * 32 + x] << ts) + rnd2) >> sh2);
    }
    return;
  }
  const bool dst4 = (t.flags & DT_DST) != 0;
  const int step = 32 >> t.log2;
  auto C = [&](int k, int m) { return dst4 ? static_cast<int>(kDctTab.dst[k][m]) : static_cast<int>(kDctTab.m[k * step][m]); };
  // columns: S[y][x] = clip16((sum_k C[k][y] * R[k][x] + 64) >> 7)
  hv::wave_matmul(n, [&](int y, int k) { return C(k, y); }, [&](int k, int x) { return R[k * 32 + x]; },
                  [&](int y, int x, int v) { S[y * 32 + x] = clip3d(-32768, 32767, (v + 64) >> 7); });
  wave_sync();
  // rows: r[y][x] = (sum_k S[y][k] * C[k][x] + rnd) >> (20 - bitDepth)
  hv::wave_matmul(n, [&](int y, int k) { return S[y * 32 + k]; }, [&](int k, int x) { return C(k, x); },
                  [&](int y, int x, int v) { dst[y * pw + x] = static_cast<int16_t>((v + rnd2) >> sh2); });
}

// ------------------------------------------------------------------ inter prediction (8.5.3.3)
namespace {
__constant__ int8_t kLumaTap[4][8] = {{0, 0, 0, 64, 0, 0, 0, 0},
                                      {-1, 4, -10, 58, 17, -5, 1, 0},
                                      {-1, 4, -11, 40, 40, -11, 4, -1},
                                      {0, 1, -5, 17, 58, -10, 4, -1}};
__constant__ int8_t kChromaTap[8][4] = {{0, 64, 0, 0},    {-2, 58, 10, -2}, {-4, 54, 16, -2}, {-6, 46, 28, -4},
                                        {-4, 36, 36, -4}, {-4, 28, 46, -6}, {-2, 16, 54, -4}, {-2, 10, 58, -2}};

// one predicted sample at 14-bit intermediate precision (predSamplesLX)
__device__ __forceinline__ int mc_sample(const uint16_t* rp, int pw, int ph, int x, int y, int mvx, int mvy, bool chroma,
                                         int bdv) {
  const int fx = chroma ? (mvx & 7) : (mvx & 3), fy = chroma ? (mvy & 7) : (mvy & 3);
  const int xi = x + (chroma ? (mvx >> 3) : (mvx >> 2)), yi = y + (chroma ? (mvy >> 3) : (mvy >> 2));
  const int sh1 = min(4, bdv - 8), sh3 = 14 - bdv;
  auto R = [&](int xx, int yy) { return static_cast<int>(rp[static_cast<size_t>(clip3d(0, ph - 1, yy)) * pw + clip3d(0, pw - 1, xx)]); };
  const int ntap = chroma ? 4 : 8, half = chroma ? 1 : 3;
  auto tap = [&](int f, int i) { return chroma ? static_cast<int>(kChromaTap[f][i]) : static_cast<int>(kLumaTap[f][i]); };
  if (fx == 0 && fy == 0) return R(xi, yi) << sh3;
  if (fy == 0) {
    int s = 0;
    for (int i = 0; i < ntap; ++i) s += tap(fx, i) * R(xi + i - half, yi);
    return s >> sh1;
  }
  if (fx == 0) {
    int s = 0;
    for (int i = 0; i < ntap; ++i) s += tap(fy, i) * R(xi, yi + i - half);
    return s >> sh1;
  }
  int s = 0;
  for (int j = 0; j < ntap; ++j) {
    int h = 0;
    for (int i = 0; i < ntap; ++i) h += tap(fx, i) * R(xi + i - half, yi + j - half);
    s += tap(fy, j) * (h >> sh1);
  }
  return s >> 6;
}

struct RefE {
  int buf, log2wd_y, log2wd_c, weighted, w[3], o[3];
};
__device__ __forceinline__ RefE load_ref(const HevcDecParams& a, int b, int e) {
  const uint8_t* p = a.refs + static_cast<size_t>(a.ref_base[b] + e) * 16;
  RefE r;
  const int pic = static_cast<int8_t>(p[0]);
  r.buf = (pic >= 0 && pic < 16) ? a.reftab[b * 16 + pic] : -1;
  r.log2wd_y = p[1];
  r.log2wd_c = p[2];
  r.weighted = p[3];
  const int16_t* w = reinterpret_cast<const int16_t*>(p + 4);
  for (int c = 0; c < 3; ++c) {
    r.w[c] = w[c];
    r.o[c] = w[3 + c];
  }
  return r;
}
}  // namespace

__global__ __launch_bounds__(64) void hevcd_inter(HevcDecParams a) {
  const int b = blockIdx.y;
  if (!a.run[b]) return;
  const int w8 = a.W / 8;
  const int bx8 = static_cast<int>(blockIdx.x) % w8, by8 = static_cast<int>(blockIdx.x) / w8;
  const int lane = lane_id();
  const uint8_t* mvf = a.mvf + static_cast<size_t>(b) * (a.H / 8) * (a.W / 8) * 12;
  const int cur = a.cur[b];
  // luma: one sample per lane
  {
    const int x = bx8 * 8 + (lane & 7), y = by8 * 8 + (lane >> 3);
    const Mv4 m = mv_at(a, mvf, x, y);
    if (m.flags & DM_INTER) {
      int p[2] = {0, 0};
      RefE e[2];
      bool use[2] = {false, false};
      for (int l = 0; l < 2; ++l) {
        if (m.ref[l] == 0xFF) continue;
        e[l] = load_ref(a, b, m.ref[l]);
        if (e[l].buf < 0 || e[l].buf >= a.D) {
          atomicOr(a.err, 16);
          return;
        }
        use[l] = true;
        p[l] = mc_sample(dpb_plane(a, b, e[l].buf, 0), a.W, a.H, x, y, m.mv[l][0], m.mv[l][1], false, a.bd);
      }
      const int shift1 = 14 - a.bd, mx = (1 << a.bd) - 1;
      int v;
      const int l0 = use[0] ? 0 : 1;
      if (!e[l0].weighted) {
        if (use[0] && use[1]) {
          const int sh2 = 15 - a.bd;
          v = (p[0] + p[1] + (1 << (sh2 - 1))) >> sh2;
        } else {
          v = (p[l0] + (1 << (shift1 - 1))) >> shift1;
        }
      } else {
        const int log2wd = e[l0].log2wd_y + shift1;
        if (use[0] && use[1]) {
          v = (p[0] * e[0].w[0] + p[1] * e[1].w[0] + ((e[0].o[0] + e[1].o[0] + 1) << log2wd)) >> (log2wd + 1);
        } else {
          v = log2wd >= 1 ? ((p[l0] * e[l0].w[0] + (1 << (log2wd - 1))) >> log2wd) + e[l0].o[0] : p[l0] * e[l0].w[0] + e[l0].o[0];
        }
      }
      const size_t o = static_cast<size_t>(y) * a.W + x;
      v = clip3d(0, mx, clip3d(0, mx, v) + a.res[0][static_cast<size_t>(b) * plane_size(a, 0) + o]);
      dpb_plane(a, b, cur, 0)[o] = static_cast<uint16_t>(v);
    }
  }
  // chroma: lanes 0..15 Cb, 16..31 Cr of the 4x4 chroma block
  if (lane < 32) {
    const int c = 1 + (lane >> 4), i = lane & 15;
    const int cx = bx8 * 4 + (i & 3), cy = by8 * 4 + (i >> 2);
    const int lx = cx * 2, ly = cy * 2;
    const Mv4 m = mv_at(a, mvf, lx, ly);
    if (m.flags & DM_INTER) {
      const int cw = a.W / 2, ch = a.H / 2;
      int p[2] = {0, 0};
      RefE e[2];
      bool use[2] = {false, false};
      for (int l = 0; l < 2; ++l) {
        if (m.ref[l] == 0xFF) continue;
        e[l] = load_ref(a, b, m.ref[l]);
        if (e[l].buf < 0 || e[l].buf >= a.D) {
          atomicOr(a.err, 16);
          return;
        }
        use[l] = true;
        p[l] = mc_sample(dpb_plane(a, b, e[l].buf, c), cw, ch, cx, cy, m.mv[l][0], m.mv[l][1], true, a.bdc);
      }
      const int shift1 = 14 - a.bdc, mx = (1 << a.bdc) - 1;
      int v;
      const int l0 = use[0] ? 0 : 1;
      if (!e[l0].weighted) {
        if (use[0] && use[1]) {
          const int sh2 = 15 - a.bdc;
          v = (p[0] + p[1] + (1 << (sh2 - 1))) >> sh2;
        } else {
          v = (p[l0] + (1 << (shift1 - 1))) >> shift1;
        }
      } else {
        const int log2wd = e[l0].log2wd_c + shift1;
        if (use[0] && use[1]) {
          v = (p[0] * e[0].w[c] + p[1] * e[1].w[c] + ((e[0].o[c] + e[1].o[c] + 1) << log2wd)) >> (log2wd + 1);
        } else {
          v = log2wd >= 1 ? ((p[l0] * e[l0].w[c] + (1 << (log2wd - 1))) >> log2wd) + e[l0].o[c] : p[l0] * e[l0].w[c] + e[l0].o[c];
        }
      }
      const size_t o = static_cast<size_t>(cy) * cw + cx;
      v = clip3d(0, mx, clip3d(0, mx, v) + a.res[c][static_cast<size_t>(b) * plane_size(a, c) + o]);
      dpb_plane(a, b, cur, c)[o] = static_cast<uint16_t>(v);
    }
  }
}

// ------------------------------------------------------------------ intra (8.4.4.2), CTB wavefront
constexpr int kDecIntraWaves = 16;

namespace {
__device__ __forceinline__ uint32_t zorder4d(int bx, int by) {
  uint32_t z = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) z |= (((bx >> i) & 1u) << (2 * i)) | (((by >> i) & 1u) << (2 * i + 1));
  return z;
}
// order global stores of this wave before its later loads (other lanes read them)
__device__ __forceinline__ void wave_sync_global() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
}  // namespace

__global__ __launch_bounds__(64 * kDecIntraWaves) void hevcd_intra(HevcDecParams a) {
  __shared__ int prog[kMaxRows];
  __shared__ int refs_lds[kDecIntraWaves][2][132];
  const int b = blockIdx.x;
  if (!a.run[b]) return;
  const int wave = wave_id(), lane = lane_id();
  for (int r = threadIdx.x; r < a.hctb; r += blockDim.x) prog[r] = 0;
  __syncthreads();
  const int nctb = a.wctb * a.hctb, w8 = a.W / 8;
  const int32_t* meta = a.meta + b * HM_COLS;
  const bool cip = meta[HM_CONSTRAINED_INTRA] != 0, strong = meta[HM_STRONG_INTRA] != 0;
  const uint8_t* ctbs = a.ctbs + static_cast<size_t>(b) * nctb * 8;
  const uint8_t* slices = a.slices + static_cast<size_t>(a.slice_base[b]) * 8;
  const uint8_t* mvf = a.mvf + static_cast<size_t>(b) * (a.H / 8) * w8 * 12;
  const uint32_t* cops = a.ctb_ops + static_cast<size_t>(b) * (nctb + 1);
  const uint8_t* ops = a.ops + static_cast<size_t>(a.op_base[b]) * 12;
  const int cur = a.cur[b];
  const int l4 = a.log2_ctb - 2, zm = (1 << l4) - 1;
  auto ctb_slice_addr = [&](int rs) {
    const int s = *reinterpret_cast<const uint16_t*>(ctbs + rs * 8);
    return *reinterpret_cast<const uint32_t*>(slices + s * 8 + 4);
  };
  auto ctb_tile = [&](int rs) { return static_cast<int>(*reinterpret_cast<const uint16_t*>(ctbs + rs * 8 + 2)); };
  auto ctb_ts = [&](int rs) { return *reinterpret_cast<const uint32_t*>(ctbs + rs * 8 + 4); };
  int* p = refs_lds[wave][0];
  int* q = refs_lds[wave][1];
  for (int ry = wave; ry < a.hctb; ry += kDecIntraWaves) {
    for (int rx = 0; rx < a.wctb; ++rx) {
      if (ry > 0) row_wait(prog, ry - 1, min(rx + 2, a.wctb), a.err);
      const int rs = ry * a.wctb + rx;
      const uint32_t o0 = cops[rs], o1 = cops[rs + 1];
      const uint32_t cur_ts = ctb_ts(rs), cur_slice = ctb_slice_addr(rs);
      const int cur_tile = ctb_tile(rs);
      for (uint32_t oi = o0; oi < o1; ++oi) {
        const uint8_t* op = ops + static_cast<size_t>(oi) * 12;
        const uint32_t w0 = *reinterpret_cast<const uint32_t*>(op);
        const int x0 = static_cast<int>(w0 & 0xFFFF), y0 = static_cast<int>(w0 >> 16);
        const int log2 = op[4], c = op[5], mode = op[6];
        const uint32_t tu = *reinterpret_cast<const uint32_t*>(op + 8);
        const int n = 1 << log2, sc = c ? 1 : 0;
        const int pw = c ? a.W / 2 : a.W, ph = c ? a.H / 2 : a.H;
        const int bdv = c ? a.bdc : a.bd, mx = (1 << bdv) - 1;
        uint16_t* pl = dpb_plane(a, b, cur, c);
        const int16_t* res = a.res[c] + static_cast<size_t>(b) * plane_size(a, c);
        const bool has_res = tu != 0xFFFFFFFFu;
        if (mode == 0xFF) {  // PCM: the residual plane holds the samples
          for (int k = lane; k < n * n; k += 64) {
            const int y = y0 + (k >> log2), x = x0 + (k & (n - 1));
            pl[static_cast<size_t>(y) * pw + x] = static_cast<uint16_t>(clip3d(0, mx, res[static_cast<size_t>(y) * pw + x]));
          }
          wave_sync_global();
          continue;
        }
        // reference samples: index i -> component position (8.4.4.2.1 ordering of hevc_common build_refs)
        const int xl = x0 << sc, yl = y0 << sc;  // luma position of the block
        const uint32_t zc = zorder4d((xl >> 2) & zm, (yl >> 2) & zm);
        auto pos = [&](int i, int* xc, int* yc) {
          if (i < 2 * n) {
            *xc = x0 - 1;
            *yc = y0 + 2 * n - 1 - i;
          } else if (i == 2 * n) {
            *xc = x0 - 1;
            *yc = y0 - 1;
          } else {
            *xc = x0 + (i - 2 * n - 1);
            *yc = y0 - 1;
          }
        };
        auto avail = [&](int i) {
          int xc, yc;
          pos(i, &xc, &yc);
          if (xc < 0 || yc < 0 || xc >= pw || yc >= ph) return false;
          const int xn = xc << sc, yn = yc << sc;
          const int rsn = (yn >> a.log2_ctb) * a.wctb + (xn >> a.log2_ctb);
          if (rsn == rs) {
            if (zorder4d((xn >> 2) & zm, (yn >> 2) & zm) > zc) return false;
          } else {
            if (ctb_ts(rsn) > cur_ts) return false;
            if (ctb_slice_addr(rsn) != cur_slice || ctb_tile(rsn) != cur_tile) return false;
          }
          if (cip && !(mvf[(static_cast<size_t>(yn >> 3) * w8 + (xn >> 3)) * 12 + 10] & DM_INTRA)) return false;
          return true;
        };
        auto fetch = [&](int i) {
          int xc, yc;
          pos(i, &xc, &yc);
          return static_cast<int>(pl[static_cast<size_t>(yc) * pw + xc]);
        };
        hv::build_refs(p, n, bdv, avail, fetch);
        const int* pr = p;
        if (c == 0 && hv::intra_filter_flag(mode, n)) {
          hv::filter_refs(p, q, n, bdv, strong);
          pr = q;
        }
        const int dc = mode == 1 ? hv::intra_dc(pr, n, log2) : 0;
        const bool edge = c == 0 && n < 32;
        for (int k = lane; k < n * n; k += 64) {
          const int yy = k >> log2, xx = k & (n - 1);
          int v = hv::intra_pred_sample(pr, n, log2, mode, xx, yy, dc, edge, mx);
          const size_t o = static_cast<size_t>(y0 + yy) * pw + x0 + xx;
          if (has_res) v = clip3d(0, mx, v + res[o]);
          pl[o] = static_cast<uint16_t>(v);
        }
        wave_sync_global();
      }
      row_publish(prog, ry, rx + 1);
    }
  }
}

// ------------------------------------------------------------------ deblocking (8.7.2)
namespace {
__device__ __forceinline__ void filter_luma_seg(uint16_t* s, int step, int across, int bsv, int qpl, int beta_off,
                                                int tc_off, bool np, bool nq, int bd) {
  const int mx = (1 << bd) - 1;
  const int qb = clip3d(0, 51, qpl + beta_off);
  const int qt = clip3d(0, 53, qpl + 2 * (bsv - 1) + tc_off);
  const int beta = hevc::kBetaTable[qb] * (1 << (bd - 8)), tc = hevc::kTcTable[qt] * (1 << (bd - 8));
  int P[4][4], Q[4][4];
#pragma unroll
  for (int l = 0; l < 4; ++l)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      P[l][i] = s[l * step - (i + 1) * across];
      Q[l][i] = s[l * step + i * across];
    }
  const int dp0 = abs(P[0][2] - 2 * P[0][1] + P[0][0]), dp3 = abs(P[3][2] - 2 * P[3][1] + P[3][0]);
  const int dq0 = abs(Q[0][2] - 2 * Q[0][1] + Q[0][0]), dq3 = abs(Q[3][2] - 2 * Q[3][1] + Q[3][0]);
  const int dpq0 = dp0 + dq0, dpq3 = dp3 + dq3, dpv = dp0 + dp3, dqv = dq0 + dq3;
  if (dpq0 + dpq3 >= beta) return;
  auto dsam = [&](int l, int dpq) {
    return 2 * dpq < (beta >> 2) && abs(P[l][3] - P[l][0]) + abs(Q[l][0] - Q[l][3]) < (beta >> 3) &&
           abs(P[l][0] - Q[l][0]) < ((5 * tc + 1) >> 1);
  };
  const bool strong = dsam(0, dpq0) && dsam(3, dpq3);
  const bool dep = dpv < ((beta + (beta >> 1)) >> 3), deq = dqv < ((beta + (beta >> 1)) >> 3);
#pragma unroll
  for (int l = 0; l < 4; ++l) {
    const int p0 = P[l][0], p1 = P[l][1], p2 = P[l][2], p3 = P[l][3];
    const int q0 = Q[l][0], q1 = Q[l][1], q2 = Q[l][2], q3 = Q[l][3];
    uint16_t* r = s + l * step;
    if (strong) {
      if (!np) {
        r[-across] = static_cast<uint16_t>(clip3d(p0 - 2 * tc, p0 + 2 * tc, (p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3));
        r[-2 * across] = static_cast<uint16_t>(clip3d(p1 - 2 * tc, p1 + 2 * tc, (p2 + p1 + p0 + q0 + 2) >> 2));
        r[-3 * across] = static_cast<uint16_t>(clip3d(p2 - 2 * tc, p2 + 2 * tc, (2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3));
      }
      if (!nq) {
        r[0] = static_cast<uint16_t>(clip3d(q0 - 2 * tc, q0 + 2 * tc, (p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3));
        r[across] = static_cast<uint16_t>(clip3d(q1 - 2 * tc, q1 + 2 * tc, (p0 + q0 + q1 + q2 + 2) >> 2));
        r[2 * across] = static_cast<uint16_t>(clip3d(q2 - 2 * tc, q2 + 2 * tc, (p0 + q0 + q1 + 3 * q2 + 2 * q3 + 4) >> 3));
      }
    } else {
      int delta = (9 * (q0 - p0) - 3 * (q1 - p1) + 8) >> 4;
      if (abs(delta) >= tc * 10) continue;
      delta = clip3d(-tc, tc, delta);
      if (!np) r[-across] = static_cast<uint16_t>(clip3d(0, mx, p0 + delta));
      if (!nq) r[0] = static_cast<uint16_t>(clip3d(0, mx, q0 - delta));
      if (dep && !np)
        r[-2 * across] = static_cast<uint16_t>(clip3d(0, mx, p1 + clip3d(-(tc >> 1), tc >> 1, (((p2 + p0 + 1) >> 1) - p1 + delta) >> 1)));
      if (deq && !nq)
        r[across] = static_cast<uint16_t>(clip3d(0, mx, q1 + clip3d(-(tc >> 1), tc >> 1, (((q2 + q0 + 1) >> 1) - q1 - delta) >> 1)));
    }
  }
}
}  // namespace

__global__ __launch_bounds__(256) void hevcd_deblock(HevcDecParams a, int dir) {
  const int b = blockIdx.y;
  if (!a.run[b]) return;
  const int w4 = a.W / 4, h4 = a.H / 4;
  const int k = static_cast<int>(blockIdx.x) * 256 + static_cast<int>(threadIdx.x);
  if (k >= w4 * h4) return;
  const int bsv = (a.bs[static_cast<size_t>(b) * w4 * h4 + k] >> (2 * dir)) & 3;
  if (!bsv) return;
  const int x = (k % w4) * 4, y = (k / w4) * 4;
  const int xp = dir == 0 ? x - 1 : x, yp = dir == 0 ? y : y - 1;
  const uint8_t* mvf = a.mvf + static_cast<size_t>(b) * (w4 / 2) * (h4 / 2) * 12;
  const uint8_t* mq = mvf + (static_cast<size_t>(y >> 3) * (w4 / 2) + (x >> 3)) * 12;
  const uint8_t* mp = mvf + (static_cast<size_t>(yp >> 3) * (w4 / 2) + (xp >> 3)) * 12;
  const int qpl = (static_cast<int8_t>(mp[11]) + static_cast<int8_t>(mq[11]) + 1) >> 1;
  const bool np = (mp[10] & DM_NOFILTER) != 0, nq = (mq[10] & DM_NOFILTER) != 0;
  const int nctb = a.wctb * a.hctb;
  const int rs = (y >> a.log2_ctb) * a.wctb + (x >> a.log2_ctb);
  const int s = *reinterpret_cast<const uint16_t*>(a.ctbs + (static_cast<size_t>(b) * nctb + rs) * 8);
  const uint8_t* sl = a.slices + static_cast<size_t>(a.slice_base[b] + s) * 8;
  const int beta_off = static_cast<int8_t>(sl[0]), tc_off = static_cast<int8_t>(sl[1]);
  const int cur = a.cur[b];
  uint16_t* py = dpb_plane(a, b, cur, 0) + static_cast<size_t>(y) * a.W + x;
  filter_luma_seg(py, dir == 0 ? a.W : 1, dir == 0 ? 1 : a.W, bsv, qpl, beta_off, tc_off, np, nq, a.bd);
  // chroma: edges on the 8x8 chroma grid (16 luma samples) with bS 2, two chroma rows per segment
  if (bsv == 2 && (dir == 0 ? (x % 16) : (y % 16)) == 0) {
    const int32_t* meta = a.meta + b * HM_COLS;
    const int cw = a.W / 2, mx = (1 << a.bdc) - 1;
    for (int c = 1; c < 3; ++c) {
      const int off = c == 1 ? meta[HM_CB_QP_OFF] : meta[HM_CR_QP_OFF];
      const int qpc = hevc::chroma_qp_map(qpl + off);
      const int qt = clip3d(0, 53, qpc + 2 + tc_off);
      const int tc = hevc::kTcTable[qt] * (1 << (a.bdc - 8));
      uint16_t* sc = dpb_plane(a, b, cur, c) + static_cast<size_t>(y / 2) * cw + x / 2;
      const int step = dir == 0 ? cw : 1, across = dir == 0 ? 1 : cw;
      for (int l = 0; l < 2; ++l) {
        uint16_t* r = sc + l * step;
        const int p0 = r[-across], p1 = r[-2 * across], q0 = r[0], q1 = r[across];
        const int delta = clip3d(-tc, tc, ((((q0 - p0) << 2) + p1 - q1 + 4) >> 3));
        if (!np) r[-across] = static_cast<uint16_t>(clip3d(0, mx, p0 + delta));
        if (!nq) r[0] = static_cast<uint16_t>(clip3d(0, mx, q0 - delta));
      }
    }
  }
}

// ------------------------------------------------------------------ SAO (8.7.3)
__global__ __launch_bounds__(256) void hevcd_sao(HevcDecParams a) {
  const int b = blockIdx.y;
  if (!a.run[b]) return;
  const size_t ny = static_cast<size_t>(a.W) * a.H, nc = ny / 4;
  const size_t k = static_cast<size_t>(blockIdx.x) * 256 + threadIdx.x;
  if (k >= ny + 2 * nc) return;
  const int c = k < ny ? 0 : (k < ny + nc ? 1 : 2);
  const size_t kk = c == 0 ? k : (c == 1 ? k - ny : k - ny - nc);
  const int pw = c ? a.W / 2 : a.W, ph = c ? a.H / 2 : a.H, sc = c ? 1 : 0;
  const int x = static_cast<int>(kk % pw), y = static_cast<int>(kk / pw);
  const int xl = x << sc, yl = y << sc;
  const int nctb = a.wctb * a.hctb;
  const int rs = (yl >> a.log2_ctb) * a.wctb + (xl >> a.log2_ctb);
  const uint8_t* sp = a.sao + (static_cast<size_t>(b) * nctb + rs) * 24;
  const int type = sp[c];
  if (!type) return;
  const int w8 = a.W / 8;
  const uint8_t* mvf = a.mvf + static_cast<size_t>(b) * (a.H / 8) * w8 * 12;
  if (mvf[(static_cast<size_t>(yl >> 3) * w8 + (xl >> 3)) * 12 + 10] & DM_NOFILTER) return;
  const uint16_t* src = a.tmp[c] + static_cast<size_t>(b) * plane_size(a, c);
  const int v = src[static_cast<size_t>(y) * pw + x];
  const int bdv = c ? a.bdc : a.bd, mx = (1 << bdv) - 1;
  const int8_t* off = reinterpret_cast<const int8_t*>(sp + 10 + 4 * c);
  int o = 0;
  if (type == 1) {
    const int band = v >> (bdv - 5), k0 = (band - sp[3 + c]) & 31;
    if (k0 < 4) o = off[k0];
  } else {
    const int cl = sp[6 + c];
    const int hp0 = cl == 1 ? 0 : (cl == 3 ? 1 : -1), vp0 = cl == 0 ? 0 : -1;
    const int xa[2] = {x + hp0, x - hp0}, ya[2] = {y + vp0, y - vp0};
    const uint8_t* ctbs = a.ctbs + static_cast<size_t>(b) * nctb * 8;
    const uint8_t* slices = a.slices + static_cast<size_t>(a.slice_base[b]) * 8;
    const int32_t* meta = a.meta + b * HM_COLS;
    const int s_cur = *reinterpret_cast<const uint16_t*>(ctbs + rs * 8);
    const uint32_t sa_cur = *reinterpret_cast<const uint32_t*>(slices + s_cur * 8 + 4);
    int e = 2;
    for (int j = 0; j < 2; ++j) {
      if (xa[j] < 0 || ya[j] < 0 || xa[j] >= pw || ya[j] >= ph) return;
      const int rn = ((ya[j] << sc) >> a.log2_ctb) * a.wctb + ((xa[j] << sc) >> a.log2_ctb);
      if (rn != rs) {
        const int s_n = *reinterpret_cast<const uint16_t*>(ctbs + rn * 8);
        const uint32_t sa_n = *reinterpret_cast<const uint32_t*>(slices + s_n * 8 + 4);
        if (sa_n != sa_cur) {
          const bool nb_first = *reinterpret_cast<const uint32_t*>(ctbs + rn * 8 + 4) < *reinterpret_cast<const uint32_t*>(ctbs + rs * 8 + 4);
          if (nb_first && !slices[s_cur * 8 + 3]) return;
          if (!nb_first && !slices[s_n * 8 + 3]) return;
        }
        if (!meta[HM_LF_ACROSS_TILES] &&
            *reinterpret_cast<const uint16_t*>(ctbs + rn * 8 + 2) != *reinterpret_cast<const uint16_t*>(ctbs + rs * 8 + 2))
          return;
      }
      const int nv = src[static_cast<size_t>(ya[j]) * pw + xa[j]];
      e += (v > nv) - (v < nv);
    }
    if (e <= 2) e = (e == 2) ? 0 : e + 1;
    if (e) o = off[e - 1];
  }
  if (o) dpb_plane(a, b, a.cur[b], c)[static_cast<size_t>(y) * pw + x] = static_cast<uint16_t>(clip3d(0, mx, v + o));
}

// stage 7: deblocked picture -> tmp (the SAO input), every running slot; 8-byte vectors
// (plane sizes are multiples of 4 samples: W, H multiples of 8)
__global__ __launch_bounds__(256) void hevcd_snapshot(HevcDecParams a) {
  const int b = blockIdx.y;
  if (!a.run[b]) return;
  const size_t ny = static_cast<size_t>(a.W) * a.H / 4, nc = ny / 4;  // in uint64 units
  for (size_t k = static_cast<size_t>(blockIdx.x) * 256 + threadIdx.x; k < ny + 2 * nc; k += static_cast<size_t>(gridDim.x) * 256) {
    const int c = k < ny ? 0 : (k < ny + nc ? 1 : 2);
    const size_t kk = c == 0 ? k : (c == 1 ? k - ny : k - ny - nc);
    const uint64_t* src = reinterpret_cast<const uint64_t*>(dpb_plane(a, b, a.cur[b], c));
    uint64_t* dst = reinterpret_cast<uint64_t*>(a.tmp[c] + static_cast<size_t>(b) * plane_size(a, c));
    dst[kk] = src[kk];
  }
}

// stage 6: the step's pictures (cropped to the conformance window) to their display
// positions of the [B, Fo, h, w] output -- uint8 for 8-bit output, else the int16 samples
__global__ __launch_bounds__(256) void hevcd_emit(HevcDecParams a) {
  const int b = blockIdx.y;
  if (!a.run[b]) return;
  const int d = a.disp[b];
  if (d < 0 || d >= a.Fo) return;
  const int w = a.out_w, h = a.out_h;
  const size_t ny = static_cast<size_t>(w) * h, nc = static_cast<size_t>(w / 2) * (h / 2);
  for (size_t k = static_cast<size_t>(blockIdx.x) * 256 + threadIdx.x; k < ny + 2 * nc; k += static_cast<size_t>(gridDim.x) * 256) {
    const int c = k < ny ? 0 : (k < ny + nc ? 1 : 2);
    const size_t kk = c == 0 ? k : (c == 1 ? k - ny : k - ny - nc);
    const int ow = c ? w / 2 : w;
    const int x = static_cast<int>(kk % ow), y = static_cast<int>(kk / ow);
    const int pw = c ? a.W / 2 : a.W;
    const int sx = x + (c ? a.crop_x / 2 : a.crop_x), sy = y + (c ? a.crop_y / 2 : a.crop_y);
    const uint16_t v = dpb_plane(a, b, a.cur[b], c)[static_cast<size_t>(sy) * pw + sx];
    const size_t o = (static_cast<size_t>(b) * a.Fo + d) * (c ? nc : ny) + kk;
    if (a.out_u8) static_cast<uint8_t*>(a.out[c])[o] = static_cast<uint8_t>(v);
    else static_cast<int16_t*>(a.out[c])[o] = static_cast<int16_t>(v);
  }
}

}  // namespace gpu
}  // namespace mivc

using mivc::gpu::HevcDecParams;

// stage: 0 residual, 1 inter, 2 intra, 3 deblock vertical, 4 deblock horizontal, 5 SAO,
// 6 emit (display-order output), 7 snapshot (deblocked copy for SAO)
extern "C" int mivc_launch_hevc_decode(const HevcDecParams* p, int stage, void* stream) {
  const HevcDecParams& a = *p;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (a.B <= 0 || a.W <= 0 || a.H <= 0 || (a.W & 7) || (a.H & 7) || a.hctb > mivc::gpu::kMaxRows) return -1;
  switch (stage) {
    case 0:
      if (a.max_tus <= 0) return 0;
      hipLaunchKernelGGL(mivc::gpu::hevcd_residual, dim3(a.max_tus, a.B), dim3(64), 0, s, a);
      break;
    case 1:
      hipLaunchKernelGGL(mivc::gpu::hevcd_inter, dim3((a.W / 8) * (a.H / 8), a.B), dim3(64), 0, s, a);
      break;
    case 2:
      hipLaunchKernelGGL(mivc::gpu::hevcd_intra, dim3(a.B), dim3(64 * mivc::gpu::kDecIntraWaves), 0, s, a);
      break;
    case 3:
    case 4: {
      const int n = (a.W / 4) * (a.H / 4);
      hipLaunchKernelGGL(mivc::gpu::hevcd_deblock, dim3((n + 255) / 256, a.B), dim3(256), 0, s, a, stage - 3);
      break;
    }
    case 5: {
      const long long n = static_cast<long long>(a.W) * a.H * 3 / 2;
      hipLaunchKernelGGL(mivc::gpu::hevcd_sao, dim3(static_cast<unsigned>((n + 255) / 256), a.B), dim3(256), 0, s, a);
      break;
    }
    case 6:
      if (!a.disp || !a.out[0] || !a.out[1] || !a.out[2] || a.Fo <= 0 || a.out_w <= 0 || a.out_h <= 0 ||
          a.crop_x + a.out_w > a.W || a.crop_y + a.out_h > a.H || (a.out_w & 1) || (a.out_h & 1))
        return -1;
      hipLaunchKernelGGL(mivc::gpu::hevcd_emit, dim3(1024, a.B), dim3(256), 0, s, a);
      break;
    case 7:
      hipLaunchKernelGGL(mivc::gpu::hevcd_snapshot, dim3(512, a.B), dim3(256), 0, s, a);
      break;
    default:
      return -2;
  }
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
