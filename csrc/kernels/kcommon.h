// Device-side helpers shared by the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../common/h264_enc_math.h"
#include "../common/h264_mb.h"
#include "../common/h264_pred.h"
#include "../common/h264_tables.h"

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

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// Sum of absolute differences of 4 packed bytes + accumulator (v_sad_u8)
__device__ __forceinline__ uint32_t sad4(uint32_t a, uint32_t b, uint32_t acc) {
  return __builtin_amdgcn_sad_u8(a, b, acc);
}

// 4x4 SATD from 16 residuals in registers (x264 normalisation: sum|H| / 2)
__device__ __forceinline__ int satd16(int* r) {
  return h264::satd4x4(r);
}

// ---------------------------------------------------------------- in-workgroup wavefront
// The serial stages (intra coding, deblocking) run one workgroup per frame with
// kWaves waves; wave w owns MB rows w, w + kWaves, ...  Row progress lives in LDS
// and is exchanged at workgroup scope: all waves of a workgroup share one CU and
// its vector L1, so release/acquire at workgroup scope is an s_waitcnt, not a
// cache write-back/invalidate (agent-scope fences cost 1.7-7 us per hand-off on
// MI355X, guide §Persistent kernels price list; the first version of these
// kernels spent ~20 us per MB step there).
constexpr int kMaxRows = 272;  // 8K: 4320 / 16 = 270 MB rows

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

// publish prog[row] = value after this wave's global stores
__device__ __forceinline__ void row_publish(int* prog, int row, int value) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if (lane_id() == 0) __hip_atomic_store(prog + row, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

}  // namespace gpu
}  // namespace mivc
