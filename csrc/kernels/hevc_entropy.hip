// HEVC CABAC slice data on the GPU: the host writer's coder (csrc/common/hevc_ctu_coder.h)
// run per picture on the device, so the entropy stage no longer binds to the host cores of a
// rank (profiles/r6_hevc_rank_rehearsal.md: 2 cores per rank held config 4 to 731 fps).
//
// One workgroup per picture, one lane per WPP substream (CTU row).  The rows advance as a
// wavefront in lock step: at step t row r codes CTU t - 2r, so CTU (x, r - 1) and (x + 1,
// r - 1), the above and above-right neighbours, were coded at steps <= t - 1, and row r starts
// (step 2r) with the contexts row r - 1 saved after its CTU 1 (step 2r - 1) -- 9.3.2.4.  A
// barrier between steps orders the rows' writes to the picture state (global) and contexts
// (LDS).  Without WPP lane 0 codes the slice alone.  Each lane writes its substream to its own
// bounded region; hevc_entropy_scan / _gather then pack the substreams into pinned host memory
// at 16-byte aligned offsets, so only the coded bytes cross to the host, where
// hevc_assemble_slice (hevc_writer.cc) adds the slice header, entry points and emulation
// prevention.
#include <hip/hip_runtime.h>

#include "../common/hevc_ctu_coder.h"
#include "kcommon.h"

namespace mivc {
namespace gpu {

using hevc::CoderLevels;
using hevc::CoderPic;
using hevc::CoderState;
using hevc::CtxState;
using hevc::CtuCoder;
using hevc::CtuInfo;
using hevc::CuInfo;
using hevc::Motion;

// bounded substream sink: bits MSB first, bytes past `cap` are counted but not written
struct DevSink {
  uint8_t* buf;
  uint32_t cap;
  uint32_t n;
  uint64_t acc;
  int nacc;
  __device__ void byte(uint32_t b) {
    if (n < cap) buf[n] = static_cast<uint8_t>(b);
    ++n;
  }
  __device__ void put(uint32_t v, int nbits) {
    if (nbits <= 0) return;
    if (nbits < 32) v &= (1u << nbits) - 1u;
    acc = (acc << nbits) | v;
    nacc += nbits;
    while (nacc >= 8) {
      nacc -= 8;
      byte(static_cast<uint32_t>(acc >> nacc) & 0xFFu);
    }
  }
  __device__ void align_zero() {
    if (nacc) put(0, 8 - nacc);
  }
};

struct HevcEntropyArgs {
  CoderPic pic;                // per-step picture parameters (qp per picture from `qp`)
  const int* qp;               // [B] SliceQpY
  const CtuInfo* ctu;          // [B][nctb]
  const CuInfo* cu;            // [B][nctb * 16]
  const CuInfo* col;           // [B][nctb * 16] collocated records, or null
  const unsigned long long* nzmap;  // [B][nctb][2]
  const int16_t* coef[3];      // level planes [B][H][W], [B][H / 2][W / 2]
  uint8_t* state;              // [B][state_bytes] picture state (hevc_entropy_state_bytes)
  long long state_bytes;
  uint8_t* out;                // [B][nsub][cap] substreams
  unsigned cap;
  unsigned* sizes;             // [B][nsub] bytes written (may exceed cap: overflow)
  int* errs;                   // [B][nsub] CoderError
  int nsub;
};

__host__ __device__ inline long long entropy_state_bytes(int W, int H) {
  const long long n = static_cast<long long>(W / 8) * (H / 8);
  return ((9 * n + 15) / 16) * 16 + 12 * n;  // depth, skip, pred, coded, qpy (n each), mode4 (4n); motion
}

__device__ inline CoderState entropy_state(uint8_t* base, int W, int H) {
  const long long n = static_cast<long long>(W / 8) * (H / 8);
  CoderState s;
  s.depth = reinterpret_cast<int8_t*>(base);
  s.skip = s.depth + n;
  s.pred = s.skip + n;
  s.coded = reinterpret_cast<uint8_t*>(s.pred + n);
  s.qpy = reinterpret_cast<int8_t*>(s.coded + n);
  s.mode4 = s.qpy + n;
  s.mot = reinterpret_cast<Motion*>(base + ((9 * n + 15) / 16) * 16);
  return s;
}

__global__ __launch_bounds__(256) void hevc_entropy(HevcEntropyArgs a) {
  extern __shared__ CtxState s_ctx[];  // [2][nsub][kNumCtx]: working contexts, saved after CTU 1
  __shared__ CoderPic sP;
  const int b = blockIdx.x, r = threadIdx.x, nl = blockDim.x;
  const int W = a.pic.W, H = a.pic.H, nctb = a.pic.wctb * a.pic.hctb;
  if (r == 0) {
    sP = a.pic;
    sP.qp = a.qp[b];
  }
  uint8_t* st = a.state + static_cast<size_t>(b) * a.state_bytes;
  const CoderState cs = entropy_state(st, W, H);
  const long long n8 = static_cast<long long>(W / 8) * (H / 8);
  for (long long i = r; i < n8; i += nl) cs.coded[i] = 0;
  __syncthreads();
  CoderLevels lv;
  lv.nzmap = reinterpret_cast<const uint64_t*>(a.nzmap) + static_cast<size_t>(b) * nctb * 2;
  lv.plane[0] = a.coef[0] + static_cast<size_t>(b) * W * H;
  lv.plane[1] = a.coef[1] + static_cast<size_t>(b) * (W / 2) * (H / 2);
  lv.plane[2] = a.coef[2] + static_cast<size_t>(b) * (W / 2) * (H / 2);
  const CtuInfo* ctu = a.ctu + static_cast<size_t>(b) * nctb;
  const CuInfo* cu = a.cu + static_cast<size_t>(b) * nctb * hevc::kCusPerCtb;
  const CuInfo* col = (a.col && sP.col_set && sP.tmvp && sP.slice_type != 2)
                          ? a.col + static_cast<size_t>(b) * nctb * hevc::kCusPerCtb
                          : nullptr;
  const bool active = r < a.nsub;
  DevSink sink{a.out + (static_cast<size_t>(b) * a.nsub + (active ? r : 0)) * a.cap, a.cap, 0, 0, 0};
  CtxState* ctx = s_ctx + static_cast<size_t>(r) * hevc::kNumCtx;  // valid for active lanes
  CtxState* saved = s_ctx + static_cast<size_t>(a.nsub + r) * hevc::kNumCtx;
  CtuCoder<DevSink> w;
  if (active) w.begin(&sP, ctu, cu, col, lv, cs, ctx, &sink);
  const int wctu = sP.wctu, hctu = sP.hctu;
  if (!sP.wpp) {
    if (r == 0)
      for (int i = 0; i < wctu * hctu; ++i) w.code_ctu(i % wctu, i / wctu);
  } else {
    const int steps = wctu + 2 * (hctu - 1);
    for (int t = 0; t < steps; ++t) {
      const int rx = t - 2 * r;
      if (active && rx >= 0 && rx < wctu) {
        if (rx == 0 && r > 0 && wctu >= 2) {  // 9.3.2.4 sync from CTU (1, r - 1)
          const CtxState* src = s_ctx + static_cast<size_t>(a.nsub + r - 1) * hevc::kNumCtx;
          for (int i = 0; i < hevc::kNumCtx; ++i) ctx[i] = src[i];
        }
        w.code_ctu(rx, r);
        if (rx == 1)
          for (int i = 0; i < hevc::kNumCtx; ++i) saved[i] = ctx[i];
      }
      __syncthreads();
    }
  }
  if (active) {
    const size_t o = static_cast<size_t>(b) * a.nsub + r;
    a.sizes[o] = sink.n;
    a.errs[o] = w.err ? w.err : (sink.n > a.cap ? static_cast<int>(hevc::CE_OVERFLOW) : 0);
  }
}

// exclusive scan of the substream sizes rounded up to 16 bytes (all pictures of the step):
// offs[i] (device and host copies), offs[n] = total; total > dst_cap flags *overflow
__global__ __launch_bounds__(1024) void hevc_entropy_scan(int n, const unsigned* __restrict__ sizes, unsigned cap,
                                                          unsigned long long* __restrict__ offs,
                                                          unsigned long long* __restrict__ offs_host,
                                                          unsigned long long dst_cap, int* __restrict__ overflow) {
  __shared__ unsigned long long s_sum[1024];
  const int per = (n + blockDim.x - 1) / blockDim.x;
  const int i0 = threadIdx.x * per, i1 = min(n, i0 + per);
  auto padded = [cap](unsigned v) { return static_cast<unsigned long long>((min(v, cap) + 15u) & ~15u); };
  unsigned long long sum = 0;
  for (int i = i0; i < i1; ++i) sum += padded(sizes[i]);
  s_sum[threadIdx.x] = sum;
  __syncthreads();
  for (int d = 1; d < blockDim.x; d <<= 1) {
    const unsigned long long v = threadIdx.x >= d ? s_sum[threadIdx.x - d] : 0;
    __syncthreads();
    s_sum[threadIdx.x] += v;
    __syncthreads();
  }
  unsigned long long run = threadIdx.x > 0 ? s_sum[threadIdx.x - 1] : 0;
  for (int i = i0; i < i1; ++i) {
    offs[i] = run;
    offs_host[i] = run;
    run += padded(sizes[i]);
  }
  if (threadIdx.x == blockDim.x - 1) {
    offs[n] = s_sum[threadIdx.x];
    offs_host[n] = s_sum[threadIdx.x];
    *overflow = s_sum[threadIdx.x] > dst_cap ? 1 : 0;
  }
}

// substream i -> dst + offs[i] in 16-byte stores (dst: pinned host memory)
__global__ __launch_bounds__(256) void hevc_entropy_gather(const uint8_t* __restrict__ src, unsigned cap,
                                                           const unsigned* __restrict__ sizes,
                                                           const unsigned long long* __restrict__ offs, int n,
                                                           uint8_t* __restrict__ dst, const int* __restrict__ overflow) {
  const int i = blockIdx.x;
  if (i >= n || *overflow) return;
  const unsigned len = (min(sizes[i], cap) + 15u) & ~15u;
  const uint4* s = reinterpret_cast<const uint4*>(src + static_cast<size_t>(i) * cap);
  uint4* d = reinterpret_cast<uint4*>(dst + offs[i]);
  for (unsigned k = threadIdx.x; k < len / 16; k += blockDim.x) d[k] = s[k];
}

}  // namespace gpu
}  // namespace mivc

using namespace mivc::gpu;

extern "C" long long mivc_hevc_entropy_state_bytes(int W, int H) { return entropy_state_bytes(W, H); }

// B pictures of one coding step.  pic: the step's CoderPic (hevc_coder_pic); sizes / errs:
// [B, nsub]; offs: [B * nsub + 1] device, offs_host the same in pinned host memory; dst:
// pinned host memory of dst_cap bytes.  Returns -1 on bad geometry.
extern "C" int mivc_launch_hevc_entropy(const void* pic, int B, const int* qp, const void* ctu, const void* cu,
                                        const void* col, const unsigned long long* nzmap, const int16_t* cy,
                                        const int16_t* cb, const int16_t* cr, uint8_t* state, long long state_bytes,
                                        uint8_t* out, unsigned cap, unsigned* sizes, int* errs,
                                        unsigned long long* offs, unsigned long long* offs_host, uint8_t* dst,
                                        unsigned long long dst_cap, int* overflow, void* stream) {
  HevcEntropyArgs a{};
  a.pic = *static_cast<const CoderPic*>(pic);
  const int nsub = a.pic.wpp ? a.pic.hctu : 1;
  if (nsub < 1 || nsub > 100 || (cap & 15) || a.pic.W % 32 || a.pic.H % 32 ||
      state_bytes < entropy_state_bytes(a.pic.W, a.pic.H))
    return -1;
  a.qp = qp;
  a.ctu = static_cast<const CtuInfo*>(ctu);
  a.cu = static_cast<const CuInfo*>(cu);
  a.col = static_cast<const CuInfo*>(col);
  a.nzmap = nzmap;
  a.coef[0] = cy;
  a.coef[1] = cb;
  a.coef[2] = cr;
  a.state = state;
  a.state_bytes = state_bytes;
  a.out = out;
  a.cap = cap;
  a.sizes = sizes;
  a.errs = errs;
  a.nsub = nsub;
  const int lanes = ((nsub + 63) / 64) * 64;
  const size_t lds = static_cast<size_t>(2) * nsub * mivc::hevc::kNumCtx * sizeof(CtxState);  // <= 60 KB
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(hevc_entropy, dim3(B), dim3(lanes), lds, s, a);
  const int n = B * nsub;
  hipLaunchKernelGGL(hevc_entropy_scan, dim3(1), dim3(1024), 0, s, n, sizes, cap, offs, offs_host, dst_cap, overflow);
  hipLaunchKernelGGL(hevc_entropy_gather, dim3(n), dim3(256), 0, s, out, cap, sizes, offs, n, dst, overflow);
  return 0;
}
