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

// ---------------------------------------------------------------- inter-workgroup hand-off
// Producer (all threads of the workgroup call): publish `value` into *flag after every
// thread's global stores are complete.  Recipe per MI355X guide §6 Guideline 16 R1.
__device__ __forceinline__ void publish_progress(int* flag, int value) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(flag, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Consumer: wait until *flag >= target (bounded spin), then acquire.
// Returns false on timeout (the kernel then sets an error word and bails out).
__device__ __forceinline__ bool wait_progress(int* flag, int target, int* err) {
  __shared__ int ok;
  if (threadIdx.x == 0) {
    long long spins = 0;
    int v = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (v < target) {
      __builtin_amdgcn_s_sleep(1);
      v = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (++spins > (1ll << 26)) break;  // ~seconds: never hang the GPU
      if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
    }
    ok = v >= target;
    if (!ok) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  return ok;
}

// Dynamic row ticket (deadlock-free wavefront order regardless of dispatch order):
// the workgroup that draws ticket t processes row t; row t-1 was drawn earlier by a
// workgroup that is already running.
__device__ __forceinline__ int draw_ticket(int* counter) {
  __shared__ int t;
  if (threadIdx.x == 0) t = atomicAdd(counter, 1);
  __syncthreads();
  return t;
}

}  // namespace gpu
}  // namespace mivc
