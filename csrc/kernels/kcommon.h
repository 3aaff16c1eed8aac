// Device-side helpers shared by the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../common/h264_enc_math.h"
#include "../common/h264_mb.h"
#include "../common/h264_pred.h"
#include "../common/h264_tables.h"
#include "route.h"

namespace mivc {
namespace gpu {

// Batched frame geometry: B independent segment slots, coded size W x H (multiple of 16).
struct Geom {
  int B;        // slots in flight
  int wmb, hmb; // macroblocks
  int W, H;     // coded luma size
  __host__ __device__ int cw() const { return W / 2; }
  __host__ __device__ int ch() const { return H / 2; }
  __host__ __device__ int nmb() const { return wmb * hmb; }
  __host__ __device__ size_t ysize() const { return static_cast<size_t>(W) * H; }
  __host__ __device__ size_t csize() const { return static_cast<size_t>(W / 2) * (H / 2); }
};

// Planar YUV 4:2:0 batch: plane p of slot b at base + b * stride
struct FrameBatch {
  uint8_t* y;
  uint8_t* u;
  uint8_t* v;
};

// routed launches (route.h): does `slot` take part -- its picture this step is of `kind`
// (kind < 0: any coded picture)?  Unrouted launches: every slot.
__device__ __forceinline__ bool route_active(const SlotRoute* rt, int slot, int kind) {
  if (!rt) return true;
  const int k = rt[slot].kind;
  return kind < 0 ? k >= 0 : k == kind;
}

// half-sample planes of one picture: [3, H + 8, W + 8] (me_halfpel_planes, margin 4)
__host__ __device__ inline size_t hp_plane_bytes(int W, int H) { return static_cast<size_t>(3) * (W + 8) * (H + 8); }

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// Sum of absolute differences of 4 packed bytes + accumulator (v_sad_u8)
__device__ __forceinline__ uint32_t sad4(uint32_t a, uint32_t b, uint32_t acc) {
  return __builtin_amdgcn_sad_u8(a, b, acc);
}

// 4x4 SATD from 16 residuals in registers (x264 normalisation: sum|H| / 2)
__device__ __forceinline__ int satd16(int* r) {
  return h264::satd4x4(r);
}

// 4x4 SATD of packed 8-bit rows (s: source, p: prediction, 4 samples per dword) on packed
// 16-bit lanes: equal to satd16 of the residual, with about half the VALU work.
//   * bytes 0/2 and 1/3 of each row go to the two 16-bit halves of two registers (v_perm),
//     so one v_pk_sub_i16 forms two residuals and the vertical Hadamard is 16 packed ops;
//   * the horizontal pass needs e = c0 + c1, f = c0 - c1 per half (columns (0, 1) / (2, 3)),
//     and |a + b| + |a - b| = 2 max(|a|, |b|) replaces the last butterfly stage: the SATD
//     (sum / 2) is the sum of max(|e.lo|, |e.hi|) + max(|f.lo|, |f.hi|), formed by one
//     v_perm pairing the halves, a v_pk_max_i16 and a v_dot2 accumulate.
// Ranges: residuals +-255, after the vertical pass +-1020, e / f +-2040: int16 throughout.
typedef short v2i16 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ v2i16 as_v2i16(uint32_t x) { return __builtin_bit_cast(v2i16, x); }
__device__ __forceinline__ uint32_t as_u32(v2i16 x) { return __builtin_bit_cast(uint32_t, x); }
__device__ __forceinline__ int satd4x4_u8(const uint32_t (&s)[4], const uint32_t (&p)[4]) {
  v2i16 lo[4], hi[4];  // row y: (x0, x2) and (x1, x3) residuals
#pragma unroll
  for (int y = 0; y < 4; ++y) {
    // v_perm_b32 selector bytes: 0x0c = zero; byte 0/2 -> halves of lo, 1/3 -> halves of hi
    const uint32_t s02 = __builtin_amdgcn_perm(0u, s[y], 0x0c020c00u), s13 = __builtin_amdgcn_perm(0u, s[y], 0x0c030c01u);
    const uint32_t p02 = __builtin_amdgcn_perm(0u, p[y], 0x0c020c00u), p13 = __builtin_amdgcn_perm(0u, p[y], 0x0c030c01u);
    lo[y] = as_v2i16(s02) - as_v2i16(p02);
    hi[y] = as_v2i16(s13) - as_v2i16(p13);
  }
  // vertical 4-point Hadamard on both register sets
  const v2i16 a0 = lo[0] + lo[1], a1 = lo[0] - lo[1], a2 = lo[2] + lo[3], a3 = lo[2] - lo[3];
  const v2i16 b0 = hi[0] + hi[1], b1 = hi[0] - hi[1], b2 = hi[2] + hi[3], b3 = hi[2] - hi[3];
  const v2i16 vl[4] = {a0 + a2, a0 - a2, a1 + a3, a1 - a3};
  const v2i16 vh[4] = {b0 + b2, b0 - b2, b1 + b3, b1 - b3};
  int acc = 0;
  const v2i16 one = {1, 1};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v2i16 e = vl[k] + vh[k], f = vl[k] - vh[k];  // (c0 + c1, c2 + c3), (c0 - c1, c2 - c3)
    e = __builtin_elementwise_max(e, -e);
    f = __builtin_elementwise_max(f, -f);
    // (|e.lo|, |f.lo|) vs (|e.hi|, |f.hi|)
    const uint32_t ue = as_u32(e), uf = as_u32(f);
    const v2i16 m = __builtin_elementwise_max(as_v2i16(__builtin_amdgcn_perm(uf, ue, 0x05040100u)),
                                              as_v2i16(__builtin_amdgcn_perm(uf, ue, 0x07060302u)));
    acc = __builtin_amdgcn_sdot2(m, one, acc, false);
  }
  return acc;
}

// ---------------------------------------------------------------- in-workgroup wavefront
// The serial stages (intra coding, deblocking) run one workgroup per frame with
// kWaves waves; wave w owns MB rows w, w + kWaves, ...  Row progress lives in LDS
// and is exchanged at workgroup scope: all waves of a workgroup share one CU and
// its vector L1, so release/acquire at workgroup scope is an s_waitcnt, not a
// cache write-back/invalidate (agent-scope fences cost 1.7-7 us per hand-off on
// MI355X, guide §Persistent kernels price list; the first version of these
// kernels spent ~20 us per MB step there).
constexpr int kMaxRows = 272;

// Keep memory freed with hipFreeAsync in the device's default pool (release threshold
// "never"): by default the pool hands it back to the driver at every synchronisation, and
// the next stream-ordered allocation of the same size re-maps it (~100 ms for a GB-sized
// per-batch workspace).  Host-side helper for the launchers.
inline void keep_async_pool() {
  static bool done[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64 || done[dev]) return;
  hipMemPool_t pool;
  if (hipDeviceGetDefaultMemPool(&pool, dev) == hipSuccess) {
    uint64_t thr = ~0ull;
    (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr);
  }
  done[dev] = true;
}  // 8K: 4320 / 16 = 270 MB rows

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }

// order LDS/global accesses between lanes of one wave (no hardware barrier needed)
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// wait until prog[row] >= target (bounded: a bug must not hang the GPU)
__device__ __forceinline__ void row_wait(int* prog, int row, int target, int* err) {
  int spins = 0;
  while (__hip_atomic_load(prog + row, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < target) {
    __builtin_amdgcn_s_sleep(2);
    if (++spins > (1 << 24)) {
      if (lane_id() == 0) atomicOr(err, 1);
      break;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// row_wait whose acquire orders LDS only (the producer hands data over through LDS)
__device__ __forceinline__ void row_wait_lds(int* prog, int row, int target, int* err) {
  int spins = 0;
  while (__hip_atomic_load(prog + row, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < target) {
    __builtin_amdgcn_s_sleep(1);
    if (++spins > (1 << 22)) {
      atomicOr(err, 1);  // any waiting lane (callers wait from divergent lane subsets)
      break;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// four values in [0, 255] -> one little-endian word, via v_perm_b32 only.  (A shift/or
// packing of clip((x + r) >> n) values gets selected to gfx950's v_ashr_pk_u8_i32, whose
// high half the backend wrongly assumes is zero.)
__device__ __forceinline__ uint32_t pack4_u8(const int* v) {
  const uint32_t lo = __builtin_amdgcn_perm(static_cast<uint32_t>(v[1]), static_cast<uint32_t>(v[0]), 0x0c0c0400u);
  const uint32_t hi = __builtin_amdgcn_perm(static_cast<uint32_t>(v[3]), static_cast<uint32_t>(v[2]), 0x0c0c0400u);
  return __builtin_amdgcn_perm(hi, lo, 0x05040100u);
}

// publish prog[row] = value after this wave's LDS stores only (global stores are not
// waited for: the consumer reads nothing this wave stored to global memory)
__device__ __forceinline__ void row_publish_lds(int* prog, int row, int value) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  if (lane_id() == 0) __hip_atomic_store(prog + row, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// device-scope progress counters (several workgroups share one wavefront): the acquire /
// release order the reconstruction's global loads and stores across CUs (and XCDs)
// returns the progress it observed (>= target): the acquire covers everything up to it
__device__ __forceinline__ int row_wait_agent(int* prog, int row, int target, int* err) {
  int spins = 0, v;
  while ((v = __hip_atomic_load(prog + row, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) < target) {
    __builtin_amdgcn_s_sleep(2);
    if (++spins > (1 << 22)) {
      if (lane_id() == 0) atomicOr(err, 1);
      v = target;
      break;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  return v;
}
__device__ __forceinline__ void row_publish_agent(int* prog, int row, int value) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  if (lane_id() == 0) __hip_atomic_store(prog + row, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// publish prog[row] = value after this wave's global stores
__device__ __forceinline__ void row_publish(int* prog, int row, int value) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if (lane_id() == 0) __hip_atomic_store(prog + row, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// ---------------------------------------------------------------- cross-lane primitives
// HIP's __shfl* lower to ds_bpermute_b32, which goes through the LDS crossbar (~50+
// cycles of latency per hop).  The wavefront kernels are chains of small cross-lane
// steps (4x4 transforms, SATD, mode minima), so every hop here is a DPP modifier on a
// VALU op (quad_perm / row mirrors, a few cycles) or a gfx950 v_permlane{16,32}_swap.
constexpr int kDppQuadXor1 = 0xB1;      // quad_perm [1,0,3,2]
constexpr int kDppQuadXor2 = 0x4E;      // quad_perm [2,3,0,1]
constexpr int kDppRowMirror = 0x140;    // lane i <- 15 - i within a row of 16
constexpr int kDppRowHalfMirror = 0x141;// lane i <- 7 - i within each half row

template <int CTRL>
__device__ __forceinline__ int dpp(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
// value of lane (lane & ~3) + K, for every lane of the quad
template <int K>
__device__ __forceinline__ int quad_bcast(int v) {
  return dpp<K * 0x55>(v);
}
// reductions: results are valid on every lane of the reduced group
__device__ __forceinline__ int sum4(int v) {
  v += dpp<kDppQuadXor1>(v);
  return v + dpp<kDppQuadXor2>(v);
}
__device__ __forceinline__ int sum8(int v) {  // within each 8-lane half row
  v = sum4(v);
  return v + dpp<kDppRowHalfMirror>(v);
}
__device__ __forceinline__ int sum16(int v) {
  v = sum4(v);
  v += dpp<kDppRowHalfMirror>(v);
  return v + dpp<kDppRowMirror>(v);
}
__device__ __forceinline__ int sum32(int v) {  // within each half wave
  v = sum16(v);
  auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  return static_cast<int>(p[0]) + static_cast<int>(p[1]);
}
__device__ __forceinline__ int sum64(int v) {
  v = sum32(v);
  auto p = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return static_cast<int>(p[0]) + static_cast<int>(p[1]);
}
// int8 / int32 MFMA operands (v_mfma_i32_16x16x64_i8: A / B 16 bytes per lane, D 4 ints)
typedef int mfma_i32x4 __attribute__((ext_vector_type(4)));
// v(l) + v(l ^ 16) + v(l ^ 32) + v(l ^ 48): a 16x16 MFMA result column summed over its four
// lane groups (rows 4 g .. 4 g + 3 of the tile live in lane group g)
__device__ __forceinline__ int sum_row_groups(int v) {
  auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  v = static_cast<int>(p[0]) + static_cast<int>(p[1]);
  auto q = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return static_cast<int>(q[0]) + static_cast<int>(q[1]);
}
__device__ __forceinline__ int min16(int v) {
  v = min(v, dpp<kDppQuadXor1>(v));
  v = min(v, dpp<kDppQuadXor2>(v));
  v = min(v, dpp<kDppRowHalfMirror>(v));
  return min(v, dpp<kDppRowMirror>(v));
}
__device__ __forceinline__ int min64(int v) {
  v = min16(v);
  auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  v = min(static_cast<int>(p[0]), static_cast<int>(p[1]));
  auto q = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return min(static_cast<int>(q[0]), static_cast<int>(q[1]));
}

// ---------------------------------------------------------------- lane-parallel 4x4 transforms
// A 4x4 block lives in a group of 4 consecutive lanes (base = lane & ~3); lane base+y
// holds row y in v[0..3].  Row passes are in-register, column passes exchange the
// group's rows with DPP quad broadcasts.  Every lane of the wave must execute these
// (uniform control flow) because shuffles read other lanes' registers.
// XCD-aware workgroup order for (x = unit within a slot, y = slot) grids: the hardware
// deals workgroups round-robin over the 8 XCDs, so consecutive units (neighbouring MBs,
// whose reference rows overlap) would land on 8 different L2s and every cache line would
// be fetched 8 times; remap so each XCD walks one contiguous eighth of the grid.
__device__ __forceinline__ void xcd_unit_slot(int& x, int& y) {
  const int gx = static_cast<int>(gridDim.x), total = gx * static_cast<int>(gridDim.y);
  int lin = static_cast<int>(blockIdx.y) * gx + static_cast<int>(blockIdx.x);
  if ((total & 7) == 0) lin = (lin & 7) * (total >> 3) + (lin >> 3);
  y = lin / gx;
  x = lin - y * gx;
}

__device__ __forceinline__ int sel4(int y, int a, int b, int c, int d) { return y == 0 ? a : (y == 1 ? b : (y == 2 ? c : d)); }

// forward integer core transform (encoder side)
__device__ __forceinline__ void grp_fwd4x4(int* v, int base, int y) {
  int s03 = v[0] + v[3], d03 = v[0] - v[3], s12 = v[1] + v[2], d12 = v[1] - v[2];
  int t[4] = {s03 + s12, 2 * d03 + d12, s03 - s12, d03 - 2 * d12};
#pragma unroll
  for (int x = 0; x < 4; ++x) {
    int c0 = quad_bcast<0>(t[x]), c1 = quad_bcast<1>(t[x]);
    int c2 = quad_bcast<2>(t[x]), c3 = quad_bcast<3>(t[x]);
    int a = c0 + c3, b = c0 - c3, c = c1 + c2, d = c1 - c2;
    v[x] = sel4(y, a + c, 2 * b + d, a - c, b - 2 * d);
  }
}

// normative inverse core transform (clause 8.5.12.2: rows, then columns, then (x+32)>>6)
__device__ __forceinline__ void grp_inv4x4(int* v, int base, int y) {
  int e0 = v[0] + v[2], e1 = v[0] - v[2], e2 = (v[1] >> 1) - v[3], e3 = v[1] + (v[3] >> 1);
  int f[4] = {e0 + e3, e1 + e2, e1 - e2, e0 - e3};
#pragma unroll
  for (int x = 0; x < 4; ++x) {
    int c0 = quad_bcast<0>(f[x]), c1 = quad_bcast<1>(f[x]);
    int c2 = quad_bcast<2>(f[x]), c3 = quad_bcast<3>(f[x]);
    int g0 = c0 + c2, g1 = c0 - c2, g2 = (c1 >> 1) - c3, g3 = c1 + (c3 >> 1);
    v[x] = (sel4(y, g0 + g3, g1 + g2, g1 - g2, g0 - g3) + 32) >> 6;
  }
}

// SATD of the group's block (sum |Hadamard| / 2), returned on every lane of the group
__device__ __forceinline__ int grp_satd4x4(const int* v, int y) {
  int a = v[0] + v[1], b = v[2] + v[3], c = v[0] - v[1], d = v[2] - v[3];
  int h[4] = {a + b, a - b, c - d, c + d};
  int s = 0;
#pragma unroll
  for (int x = 0; x < 4; ++x) {
    int p = dpp<kDppQuadXor1>(h[x]);
    int u = (y & 1) ? p - h[x] : h[x] + p;
    int q = dpp<kDppQuadXor2>(u);
    int w = (y & 2) ? q - u : u + q;
    s += w < 0 ? -w : w;
  }
  return sum4(s) >> 1;
}

// inverse 4x4 zigzag (raster (x, y) -> scan index) without a memory table: one packed
// word per column, so a lane-varying y never turns into a vector load from __constant__
__device__ __forceinline__ int zzinv(int x, int y) {
  const uint32_t w = x == 0 ? (0u | 2u << 8 | 3u << 16 | 9u << 24)
                   : x == 1 ? (1u | 4u << 8 | 8u << 16 | 10u << 24)
                   : x == 2 ? (5u | 7u << 8 | 11u << 16 | 14u << 24)
                            : (6u | 12u << 8 | 13u << 16 | 15u << 24);
  return static_cast<int>((w >> (8 * y)) & 255u);
}

__device__ __forceinline__ int pos_class(int x, int y) {
  return ((x | y) & 1) == 0 ? 0 : (((x & y) & 1) ? 1 : 2);
}


// ---------------------------------------------------------------- intra neighbourhood tiles
// Luma tile of the intra kernels (encoder and decoder): row 0 = the row above the MB
// (x = -1 .. 19, top-right included), column 0 = the column to its left.
constexpr int kTileStride = 24;

// Intra4x4 neighbour vector e[13] of block blk (see h264::i4_pred_sample) + availability
// Intra4x4 neighbour vector e[0..12] of block blk (0: top-left, 1-8: above and above-right,
// 9-12: left) from the tile: lane i < 13 returns entry i (the other lanes 0) -- one register
// per lane instead of the 13-entry vector in every lane.  *av_out: availability (uniform).
// luma4x4BlkIdx <-> 4x4 block column / row and raster index, by bit arithmetic (a table lookup
// with a run-time index is a memory load on the dependency chain of every block)
__device__ __forceinline__ int blkidx_x(int b) { return (b & 1) | ((b >> 1) & 2); }
__device__ __forceinline__ int blkidx_y(int b) { return ((b >> 1) & 1) | ((b >> 2) & 2); }
__device__ __forceinline__ int raster_to_blkidx(int r) {
  const int x = r & 3, y = r >> 2;
  return (x & 1) | ((y & 1) << 1) | ((x & 2) << 1) | ((y & 2) << 2);
}

__device__ __forceinline__ int i4_neighbour_lane(const uint8_t* t, int blk, int mbav, int lane, int* av_out) {
  int bx = blkidx_x(blk), by = blkidx_y(blk);
  bool left = bx > 0 || (mbav & h264::AV_LEFT), top = by > 0 || (mbav & h264::AV_TOP);
  int av = 0;
  if (left) av |= h264::AV_LEFT;
  if (top) av |= h264::AV_TOP;
  if (left && top) av |= h264::AV_TOPLEFT;
  bool tr;
  if (blk == 3 || blk == 7 || blk == 11 || blk == 13 || blk == 15) tr = false;
  else if (blk == 5) tr = (mbav & h264::AV_TOPRIGHT) != 0;
  else if (blk == 0 || blk == 1 || blk == 4) tr = (mbav & h264::AV_TOP) != 0;
  else tr = true;
  if (tr) av |= h264::AV_TOPRIGHT;
  *av_out = av;
  const uint8_t* row = t + (by * 4) * kTileStride + bx * 4;  // tile row above the block, col of x = -1
  if (lane >= 13) return 0;
  if (lane < 5) return row[lane];
  if (lane < 9) return tr ? row[lane] : row[4];
  return t[(by * 4 + 1 + lane - 9) * kTileStride + bx * 4];
}

}  // namespace gpu
}  // namespace mivc
