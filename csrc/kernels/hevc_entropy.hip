// HEVC CABAC slice data on the GPU: the host writer's coder (csrc/common/hevc_ctu_coder.h)
// run per picture on the device, so the entropy stage no longer binds to the host cores of a
// rank (profiles/r6_hevc_rank_rehearsal.md: 2 cores per rank held config 4 to 731 fps).
//
// One workgroup per picture; lane 0 of each of its (up to 16) waves codes WPP substreams (CTU
// rows wave, wave + 16, ...): one active lane per wave, because the rows' code paths differ and
// lanes of one wavefront would serialise them.  The rows advance as a wavefront: in each round
// a row codes its next CTU x when the row above has coded CTU x + 1 (the above-right
// neighbour), and row r starts with the contexts row r - 1 saved after its CTU 1 (9.3.2.4).
// Barriers between the rounds order the rows' writes to the picture state (global) and the
// contexts / progress (LDS).  Without WPP lane 0 of wave 0 codes the slice alone.  Each lane writes its substream to its own
// bounded region; hevc_entropy_scan / _gather then pack the substreams into pinned host memory
// at 16-byte aligned offsets, so only the coded bytes cross to the host, where
// hevc_assemble_slice (hevc_writer.cc) adds the slice header, entry points and emulation
// prevention.
#include <hip/hip_runtime.h>

#include <cstdlib>

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
  unsigned long long* prof;    // diagnostics: [B][16 waves][CP_N + 2] cycle counters, or null
  // workgroups per picture: 1 = the rows advance in barrier-separated rounds inside one
  // workgroup; K > 1 (narrow batches: few pictures, many CTU rows) = the picture's rows are
  // dealt to K x waves waves, which hand progress and row contexts over through device memory
  int K;
  int* gprog;                  // [B][nsub] CTUs coded per row (K > 1; zeroed by the launcher)
  CtxState* gctx;              // [B][nsub][kNumCtx] contexts after each row's CTU 1 (K > 1)
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

constexpr int kStageBlocks = 128;  // 4x4 level blocks staged per CTU and wave (4 KiB)

// kMW: the most waves a launch uses (8 or 16); it sizes the per-wave LDS, so the default
// 8-wave launch leaves more of a CU's LDS to the concurrent compute stream's kernels.
// __launch_bounds__(1024) either way: the 128-VGPR budget measured best
template <bool kMulti, int kMW>
__global__ __launch_bounds__(1024) void hevc_entropy(HevcEntropyArgs a) {
  // working contexts per wave [nwave][kNumCtx], then (one workgroup per picture) the contexts
  // of each row after its CTU 1 [nsub][kNumCtx]
  extern __shared__ CtxState s_ctx[];
  __shared__ CoderPic sP;
  __shared__ int s_prog[128];          // CTUs coded per row
  // the coder's constant tables in LDS (read once or more per bin / coefficient)
  __shared__ uint32_t s_step[256];
  __shared__ uint8_t s_scans[sizeof(hevc::kScans.t)];
  __shared__ uint8_t s_sig[sizeof(hevc::kSig.t)];
  // workgroup kk of picture b is blockIdx kk * B + b: with B a multiple of 8 a picture's
  // workgroups share an XCD (blockIdx mod 8)
  const int B = gridDim.x / a.K;
  const int kk = blockIdx.x / B, b = blockIdx.x - kk * B, tid = threadIdx.x, nt = blockDim.x;
  const int wave = tid >> 6, nwave = nt >> 6;
  const bool lead = (tid & 63) == 0;
  const int W = a.pic.W, H = a.pic.H, nctb = a.pic.wctb * a.pic.hctb;
  if (tid == 0) {
    sP = a.pic;
    sP.qp = a.qp[b];
  }
  for (int i = tid; i < a.nsub; i += nt) s_prog[i] = 0;
  for (int i = tid; i < 256; i += nt) s_step[i] = hevc::kCabacStep.t[i];
  for (int i = tid; i < static_cast<int>(sizeof(s_scans)); i += nt) s_scans[i] = (&hevc::kScans.t[0][0][0])[i];
  for (int i = tid; i < static_cast<int>(sizeof(s_sig)); i += nt) s_sig[i] = (&hevc::kSig.t[0][0][0][0][0][0])[i];
  uint8_t* st = a.state + static_cast<size_t>(b) * a.state_bytes;
  const CoderState cs = entropy_state(st, W, H);
  const long long n8 = static_cast<long long>(W / 8) * (H / 8);
  if (!kMulti)  // K > 1: the launcher zeroed the state (every workgroup of the picture reads it)
    for (long long i = tid; i < n8; i += nt) cs.coded[i] = 0;
  __syncthreads();
  CoderLevels lv;
  lv.nzmap = reinterpret_cast<const uint64_t*>(a.nzmap) + static_cast<size_t>(b) * nctb * 2;
  lv.plane[0] = a.coef[0] + static_cast<size_t>(b) * W * H;
  lv.plane[1] = a.coef[1] + static_cast<size_t>(b) * (W / 2) * (H / 2);
  lv.plane[2] = a.coef[2] + static_cast<size_t>(b) * (W / 2) * (H / 2);
  lv.stage_ctu = 1;  // with WPP (below) levels come from the per-CTU staging area first
  const CtuInfo* ctu = a.ctu + static_cast<size_t>(b) * nctb;
  const CuInfo* cu = a.cu + static_cast<size_t>(b) * nctb * hevc::kCusPerCtb;
  const CuInfo* col = (a.col && sP.col_set && sP.tmvp && sP.slice_type != 2)
                          ? a.col + static_cast<size_t>(b) * nctb * hevc::kCusPerCtb
                          : nullptr;
  const int wctu = sP.wctu, hctu = sP.hctu;
  // lane 0 of each wave codes rows wave, wave + nwave, ...: one active lane per wave, so the
  // rows' different code paths never share (serialise within) a wavefront
  int row = wave;
  // each wave's coder and sink in LDS: their fields are read and written around every bin, and
  // the out-of-line calls would otherwise keep them in scratch memory
  __shared__ __attribute__((aligned(16))) unsigned char s_coder[kMW][sizeof(CtuCoder<DevSink>)];
  __shared__ DevSink s_sink[kMW];
  __shared__ __attribute__((aligned(16))) int16_t s_lv[kMW][kStageBlocks * 16];
  __shared__ CuInfo s_cu[kMW][4 * hevc::kCusPerCtb];
  CtuCoder<DevSink>& w = *reinterpret_cast<CtuCoder<DevSink>*>(s_coder[wave]);
  DevSink& sink = s_sink[wave];
  auto start_row = [&](int r) {
    sink = DevSink{a.out + (static_cast<size_t>(b) * a.nsub + r) * a.cap, a.cap, 0, 0, 0};
    w.begin(&sP, ctu, cu, col, lv, cs, s_ctx + static_cast<size_t>(wave) * hevc::kNumCtx, &sink, s_step, s_scans, s_sig);
  };
  auto end_row = [&](int r) {
    const size_t o = static_cast<size_t>(b) * a.nsub + r;
    a.sizes[o] = sink.n;
    a.errs[o] = w.err ? w.err : (sink.n > a.cap ? static_cast<int>(hevc::CE_OVERFLOW) : 0);
  };
  if (!sP.wpp) {  // one substream: lane 0 of wave 0 codes the slice
    sink = DevSink{nullptr, a.cap, 0, 0, 0};
    if (tid == 0) {
      start_row(0);
      for (int i = 0; i < wctu * hctu; ++i) w.code_ctu(i % wctu, i / wctu);
      end_row(0);
    }
    return;
  }
  // this wave's staging area: the current CTU's records and its first kStageBlocks non-zero
  // 4x4 level blocks, copied by all 64 lanes at once (one memory latency instead of one per
  // access of the serial coder)
  const int lane = tid & 63;
  auto stage = [&](int cx, int cy) {
    const int per = sP.ctu64 ? 2 : 1;
    int base = 0;
    for (int q = 0; q < per * per; ++q) {
      const int bx = cx * per + (q & 1), by = cy * per + (q >> 1);
      if (bx >= sP.wctb || by >= sP.hctb) continue;
      const size_t ci = static_cast<size_t>(by) * sP.wctb + bx;
      if (lane < hevc::kCusPerCtb) s_cu[wave][q * hevc::kCusPerCtb + lane] = cu[ci * hevc::kCusPerCtb + lane];
      const unsigned long long lm = lv.nzmap[2 * ci], cm = lv.nzmap[2 * ci + 1] & 0xFFFFFFFFull;
      if ((lm >> lane) & 1ull) {
        const int rank = base + __popcll(lm & ((1ull << lane) - 1ull));
        if (rank < kStageBlocks) {
          const int16_t* src = lv.plane[0] + static_cast<size_t>(by * 32 + (lane >> 3) * 4) * W + bx * 32 + (lane & 7) * 4;
          uint64_t* d = reinterpret_cast<uint64_t*>(&s_lv[wave][rank * 16]);
#pragma unroll
          for (int r = 0; r < 4; ++r) d[r] = *reinterpret_cast<const uint64_t*>(src + static_cast<size_t>(r) * W);
        }
      }
      if (lane < 32 && ((cm >> lane) & 1ull)) {
        const int rank = base + __popcll(lm) + __popcll(cm & ((1ull << lane) - 1ull));
        if (rank < kStageBlocks) {
          const int k = lane & 15, cw = W / 2;
          const int16_t* src = lv.plane[lane < 16 ? 1 : 2] + static_cast<size_t>(by * 16 + (k >> 2) * 4) * cw + bx * 16 + (k & 3) * 4;
          uint64_t* d = reinterpret_cast<uint64_t*>(&s_lv[wave][rank * 16]);
#pragma unroll
          for (int r = 0; r < 4; ++r) d[r] = *reinterpret_cast<const uint64_t*>(src + static_cast<size_t>(r) * cw);
        }
      }
      base += __popcll(lm) + __popcll(cm);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  if constexpr (kMulti) {
    // each wave on its own: wait (device scope) until the row above has coded the above-right
    // CTU, code, publish; row contexts after CTU 1 go through device memory
    // workgroup kk codes the contiguous rows [kk R, (kk + 1) R), its waves round-robin: every
    // row waits only on rows of its own workgroup or of workgroup kk - 1 (a lower blockIdx,
    // dispatched first), so progress never depends on a workgroup that is not yet resident
    const int R = (a.nsub + a.K - 1) / a.K;
    const int r_end = min(a.nsub, (kk + 1) * R);
    int* prog = a.gprog + static_cast<size_t>(b) * a.nsub;
    CtxState* gctx = a.gctx + static_cast<size_t>(b) * a.nsub * hevc::kNumCtx;
    CtxState* ctx = s_ctx + static_cast<size_t>(wave) * hevc::kNumCtx;
    for (int r = kk * R + wave; r < r_end; r += nwave) {
      if (lead) {
        sink = DevSink{a.out + (static_cast<size_t>(b) * a.nsub + r) * a.cap, a.cap, 0, 0, 0};
        w.begin(&sP, ctu, cu, col, lv, cs, ctx, &sink, s_step, s_scans, s_sig);
      }
      bool timeout = false;
      for (int x = 0; x < wctu && !timeout; ++x) {
        if (r > 0) {
          const int target = min(x + 2, wctu);
          int spins = 0;
          while (__hip_atomic_load(prog + r - 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            __builtin_amdgcn_s_sleep(2);
            if (++spins > (1 << 24)) {
              timeout = true;
              break;
            }
          }
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          if (timeout) break;
        }
        stage(x, r);
        if (lead) {
          if (x == 0 && r > 0 && wctu >= 2)  // sync from CTU (1, r - 1)
            for (int i = 0; i < hevc::kNumCtx; ++i) ctx[i] = gctx[static_cast<size_t>(r - 1) * hevc::kNumCtx + i];
          w.lv.levels = &s_lv[wave][0];
          w.lv.nblocks = kStageBlocks;
          w.cu_stage = &s_cu[wave][0];
          w.stage_cx = x;
          w.stage_cy = r;
          w.prof = nullptr;
          w.code_ctu(x, r);
          if (x == 1)
            for (int i = 0; i < hevc::kNumCtx; ++i) gctx[static_cast<size_t>(r) * hevc::kNumCtx + i] = ctx[i];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        if (lead) __hip_atomic_store(prog + r, x + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_wave_barrier();  // lane 0 is done with the staging area
      }
      if (lead) {
        const size_t o = static_cast<size_t>(b) * a.nsub + r;
        a.sizes[o] = sink.n;
        a.errs[o] = timeout ? static_cast<int>(hevc::CE_TIMEOUT)
                            : (w.err ? w.err : (sink.n > a.cap ? static_cast<int>(hevc::CE_OVERFLOW) : 0));
        if (timeout)  // let the rows below finish (their bytes are discarded with this error)
          __hip_atomic_store(prog + r, wctu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    return;
  }
  __shared__ uint64_t s_prof[kMW][hevc::CP_N + 2];  // + cycles waiting at barriers, + CTUs coded
  if (a.prof && lead) {
    for (int k = 0; k < hevc::CP_N + 2; ++k) s_prof[wave][k] = 0;
  }
  uint64_t t_wait = 0;
  if (lead && row < a.nsub) start_row(row);
  for (;;) {
    const uint64_t tw = a.prof ? __builtin_readcyclecounter() : 0;
    // barrier: the previous iteration's CTUs (picture state, contexts, progress) are visible.
    // Every lane of a wave follows its row (wave-uniform control), lane 0 codes.
    if (!__syncthreads_or(lead && row < a.nsub)) break;
    int x = 0;
    bool ready = false;
    if (row < a.nsub) {
      x = s_prog[row];
      ready = row == 0 || s_prog[row - 1] >= min(x + 2, wctu);  // above-right CTU coded (9.3.2.4: CTU 1)
    }
    __syncthreads();  // every wave has read the progress before any wave advances it
    if (a.prof) t_wait += __builtin_readcyclecounter() - tw;
    if (ready) {
      stage(x, row);
      if (lead) {
        CtxState* ctx = s_ctx + static_cast<size_t>(wave) * hevc::kNumCtx;
        if (x == 0 && row > 0 && wctu >= 2) {  // sync from CTU (1, row - 1)
          const CtxState* src = s_ctx + static_cast<size_t>(nwave + row - 1) * hevc::kNumCtx;
          for (int i = 0; i < hevc::kNumCtx; ++i) ctx[i] = src[i];
        }
        w.lv.levels = &s_lv[wave][0];
        w.lv.nblocks = kStageBlocks;
        w.cu_stage = &s_cu[wave][0];
        w.stage_cx = x;
        w.stage_cy = row;
        w.prof = a.prof ? &s_prof[wave][0] : nullptr;
        w.code_ctu(x, row);
        if (a.prof) s_prof[wave][hevc::CP_N + 1] += 1;
        if (x == 1) {
          CtxState* sv = s_ctx + static_cast<size_t>(nwave + row) * hevc::kNumCtx;
          for (int i = 0; i < hevc::kNumCtx; ++i) sv[i] = ctx[i];
        }
        s_prog[row] = x + 1;
        if (x + 1 == wctu) end_row(row);
      }
      if (x + 1 == wctu) {
        row += nwave;
        if (lead && row < a.nsub) start_row(row);
      }
      __builtin_amdgcn_wave_barrier();  // lane 0 is done with the staging area
    }
  }
  if (a.prof && lead) {
    s_prof[wave][hevc::CP_N] = t_wait;
    unsigned long long* o = a.prof + (static_cast<size_t>(b) * 16 + wave) * (hevc::CP_N + 2);
    for (int k = 0; k < hevc::CP_N + 2; ++k) o[k] = s_prof[wave][k];
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
                                        unsigned long long dst_cap, int* overflow, void* stream,
                                        unsigned long long* prof, int* gprog, void* gctx) {
  HevcEntropyArgs a{};
  a.prof = prof;
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
  // a wave per row up to MIVC_HEVC_ENTROPY_WAVES (default 8: config 4 2052 fps vs 1953 at 16
  // and 1986 at 4, profiles/r6_hevc_gpu_entropy.md) per picture, further rows
  // round-robin: fewer waves leave more of each CU's registers to the compute stream's
  // kernels running concurrently, at a longer critical path per picture
  static const int max_waves = [] {
    const char* e = std::getenv("MIVC_HEVC_ENTROPY_WAVES");
    const int v = e ? std::atoi(e) : 8;
    return v < 1 ? 1 : (v > 16 ? 16 : v);
  }();
  const int nw = nsub < max_waves ? nsub : max_waves;
  const int lanes = 64 * nw;
  // narrow batches (fewer than 512 substream waves, e.g. 10 x 8K) spread each picture's rows
  // over ceil(rows / waves) workgroups (contiguous row blocks); MIVC_HEVC_ENTROPY_WG forces K
  static const int wg_env = [] {
    const char* e = std::getenv("MIVC_HEVC_ENTROPY_WG");
    return e ? std::atoi(e) : 0;
  }();
  int K = 1;
  if (a.pic.wpp && gprog && gctx) {
    // K workgroups per picture while the launch stays at most 1024 waves (a quarter of the
    // device's resident waves at this kernel's registers: room for the concurrent compute)
    // and at most nw rows per workgroup (a wave per row: a second row of a wave would wait for
    // its first to finish and delay every row below it)
    const int need = (nsub + nw - 1) / nw;
    K = wg_env > 0 ? wg_env : (B * nw < 512 && B * need * nw <= 1024 ? need : 1);
    K = K < 1 ? 1 : (K > 16 ? 16 : (K > need ? need : K));
  }
  a.K = K;
  a.gprog = gprog;
  a.gctx = static_cast<CtxState*>(gctx);
  // working contexts per wave, plus (K == 1) each row's contexts after CTU 1: <= 35 KB
  const size_t lds = static_cast<size_t>(K > 1 ? nw : nw + nsub) * mivc::hevc::kNumCtx * sizeof(CtxState);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (K > 1) {
    (void)hipMemsetAsync(gprog, 0, static_cast<size_t>(B) * nsub * sizeof(int), s);
    (void)hipMemsetAsync(state, 0, static_cast<size_t>(B) * state_bytes, s);
  }
  if (K > 1) {
    if (nw <= 8) hipLaunchKernelGGL((hevc_entropy<true, 8>), dim3(B * K), dim3(lanes), lds, s, a);
    else hipLaunchKernelGGL((hevc_entropy<true, 16>), dim3(B * K), dim3(lanes), lds, s, a);
  } else {
    if (nw <= 8) hipLaunchKernelGGL((hevc_entropy<false, 8>), dim3(B), dim3(lanes), lds, s, a);
    else hipLaunchKernelGGL((hevc_entropy<false, 16>), dim3(B), dim3(lanes), lds, s, a);
  }
  const int n = B * nsub;
  hipLaunchKernelGGL(hevc_entropy_scan, dim3(1), dim3(1024), 0, s, n, sizes, cap, offs, offs_host, dst_cap, overflow);
  hipLaunchKernelGGL(hevc_entropy_gather, dim3(n), dim3(256), 0, s, out, cap, sizes, offs, n, dst, overflow);
  return 0;
}
