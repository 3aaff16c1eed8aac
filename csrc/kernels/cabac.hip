// CABAC slice coding on the GPU (x264's default entropy coder behind
// the reference's `-vcodec libx264`, server.go:69-70 / client.go:115).
//
// CABAC is serial only in its arithmetic coder: every context index is a function of
// the decision records (csrc/common/h264_cabac.h: cabac_prepare_mb + cabac_qp_chain), so
// the binarisation of every macroblock of every slot runs in parallel and records
// 16-bit symbols; the serial stage is a tight arithmetic-coding loop over them.  The
// binariser and the symbol coder are the shared host/device code, so the bytes equal the
// host writer's (tests/test_cabac.py pins the decomposition on the CPU).
//
// Two launches:
//   mivc_launch_cabac_bin   one frame step (B slots, S slices each), into a symbol pool
//     cabac_mask    (nmb/2 x B, wave64)    non-zero mask of every 4x4 / DC block
//     cabac_prep    (nmb/64 x B, 64)       lane per MB: coding state (skip, cbp, mvd, cbf ...)
//     cabac_chain   (B, 64)                mb_qp_delta chain (QP_pred scan) per slot
//     cabac_count   (nmb/64 x B, 64)       lane per MB: symbol count
//     cabac_offsets (B, 64)                per-slot exclusive scan of the counts
//     cabac_alloc   (1, 64)                slot regions in the pool (scan over slots)
//     cabac_bins    (nmb/64 x B, 64)       lane per MB: symbols, staged to 16-byte stores
//   mivc_launch_cabac_code  G frame steps at once (G * B slices: one lane each)
//     cabac_arith   (G*B/lpw, 64)          context states in LDS (one column per lane),
//                                          header bytes + arithmetic coding, output written
//                                          in place over the slice's consumed symbols
//     cabac_compact (G*B, 256)             slice outputs packed (16-byte aligned starts),
//                                          straight into pinned host memory when they fit
// The serial stage is latency-bound (a chain of dependent LDS reads per bin), so its
// throughput scales with the number of independent slices in flight: grouping G frame
// steps multiplies the waves the chip runs at once by G.
#include "kcommon.h"
// after kcommon.h: the shared headers' MIVC_HD needs the HIP runtime declarations
#include "../common/h264_cabac.h"

namespace mivc {
namespace gpu {

using h264::CabacNb;
using h264::CabacSliceInfo;
using h264::MbHeader;

// symbols reserved in front of every slice's symbols: the slice header bytes are written
// there, so the in-place output (<= header + 10 bits per symbol) never overtakes the reads
constexpr int kCabacGap = 64;
// symbols past a slice's end the arithmetic coder may load (its next-block prefetch)
constexpr int kArithReadAhead = 160;

struct CabacBinArgs {
  Geom g;
  const MbHeader* hdr;    // [B, nmb]
  const int16_t* coef;    // [B, nmb, 408]
  uint32_t* mask;         // [B, nmb]
  CabacNb* nb;            // [B, nmb]
  int* cnt;               // [B, nmb] symbols per MB
  long long* off;         // [B, nmb] symbol offset of the MB inside its slice
  int* tot;               // [B] symbols per slice (scratch)
  uint16_t* pool;         // symbol pool of the group
  long long pool_cap;     // symbols
  long long* pool_used;   // [1] running allocation of the group
  long long* base;        // [B] out: slice region start (symbols, a multiple of 8)
  int* total;             // [B] out: symbols of the slice (-1: pool exhausted)
  const int* slot_qp;     // [B] slice QP
  int slice_type;
  int num_ref_l0, num_ref_l1;
  int t8x8_mode;
  int* err;
  // routed (route.h): every slot's own slice type (its picture kind) and active list-0 size
  const SlotRoute* rt;
  // slices (H264Params.slices): every picture is `per_slot` slices of `slice_mbs` MBs (whole
  // MB rows; the last one may be shorter).  Slice index ls = slot * per_slot + mb / slice_mbs
  // addresses tot / base / total; symbol offsets are relative to the slice.
  int slice_mbs, per_slot;
};

__device__ __forceinline__ int slice_first(const CabacBinArgs& a, int mb) { return (mb / a.slice_mbs) * a.slice_mbs; }
__device__ __forceinline__ int slice_end(const CabacBinArgs& a, int mb) {
  return min(slice_first(a, mb) + a.slice_mbs, a.g.nmb());
}
__device__ __forceinline__ int slice_index(const CabacBinArgs& a, int slot, int mb) {
  return slot * a.per_slot + mb / a.slice_mbs;
}

__device__ __forceinline__ CabacSliceInfo slice_info(const CabacBinArgs& a, int slot, int mb) {
  CabacSliceInfo si{};
  si.slice_type = a.rt ? a.rt[slot].kind : a.slice_type;
  si.wmb = a.g.wmb;
  si.hmb = a.g.hmb;
  si.first_mb = slice_first(a, mb);
  si.num_ref[0] = a.rt ? (a.rt[slot].kind == SK_I ? 1 : a.rt[slot].n0) : a.num_ref_l0;
  si.num_ref[1] = a.num_ref_l1;
  si.t8x8_mode = a.t8x8_mode;
  si.slice_qp = a.slot_qp[slot];
  return si;
}

// one wave = two MBs per step, kMaskSpan steps per workgroup (a workgroup per MB pair made
// the launch dispatch-bound: a million one-wave workgroups per 1080p frame step)
constexpr int kMaskSpan = 16;

__global__ __launch_bounds__(64) void cabac_mask(CabacBinArgs a) {
  const Geom& g = a.g;
  const int lane = threadIdx.x, sub = lane & 31;
  const int slot = blockIdx.y;
  for (int it = 0; it < kMaskSpan; ++it) {
  const int mb = (blockIdx.x * kMaskSpan + it) * 2 + (lane >> 5);
  if ((blockIdx.x * kMaskSpan + it) * 2 >= g.nmb()) break;  // (uniform)
  const bool live = mb < g.nmb();
  const size_t o = static_cast<size_t>(slot) * g.nmb() + (live ? mb : 0);
  const int16_t* c = a.coef + o * h264::kCoefPerMb;
  const bool i16 = a.hdr[o].kind == h264::MBK_I16x16;
  bool nz = false;
  if (sub < 16 || (sub >= 19 && sub < 27)) {
    const int16_t* p = sub < 16 ? c + h264::COEF_LUMA + sub * 16 : c + h264::COEF_CHROMA_AC + (sub - 19) * 16;
    const uint4 q0 = reinterpret_cast<const uint4*>(p)[0];
    const uint4 q1 = reinterpret_cast<const uint4*>(p)[1];
    const bool skip_dc = sub >= 19 || i16;  // AC-only blocks: level 0 is not coded
    nz = ((skip_dc ? (q0.x & 0xFFFF0000u) : q0.x) | q0.y | q0.z | q0.w | q1.x | q1.y | q1.z | q1.w) != 0;
  } else if (sub == 16) {
    const uint4 q0 = reinterpret_cast<const uint4*>(c + h264::COEF_LUMA_DC)[0];
    const uint4 q1 = reinterpret_cast<const uint4*>(c + h264::COEF_LUMA_DC)[1];
    nz = i16 && (q0.x | q0.y | q0.z | q0.w | q1.x | q1.y | q1.z | q1.w) != 0;
  } else if (sub == 17 || sub == 18) {
    const uint2 q = reinterpret_cast<const uint2*>(c + h264::COEF_CHROMA_DC)[sub - 17];
    nz = (q.x | q.y) != 0;
  }
  const unsigned long long bal = __ballot(nz);
  const uint32_t m = static_cast<uint32_t>((bal >> (lane & 32)) & 0x7FFFFFFull);
  if (live && sub == 0) a.mask[o] = m;
  }
}

// The 64 records of a wave are built in LDS and leave as one contiguous run of 16-byte stores:
// cabac_prepare_mb's field-by-field byte stores straight to global memory (64 lanes at a
// 112-byte stride) made this launch fetch 4.2 GB per 1080p x 256 step for 0.23 GB of records
// (round-4 PMC), and it runs beside the encode kernels.
static_assert(sizeof(CabacNb) % 16 == 0, "CabacNb rows leave as 16-byte chunks");
__global__ __launch_bounds__(64) void cabac_prep(CabacBinArgs a) {
  __shared__ __attribute__((aligned(16))) CabacNb s_nb[64];
  const int mb0 = blockIdx.x * 64, mb = mb0 + threadIdx.x, slot = blockIdx.y, nmb = a.g.nmb();
  const size_t base = static_cast<size_t>(slot) * nmb;
  if (mb < nmb) {
    const CabacSliceInfo si = slice_info(a, slot, mb);
    h264::cabac_prepare_mb(si, a.hdr + base, mb, a.mask[base + mb], s_nb[threadIdx.x]);
  }
  __syncthreads();
  const int n16 = min(64, nmb - mb0) * static_cast<int>(sizeof(CabacNb) / 16);
  const uint4* src = reinterpret_cast<const uint4*>(s_nb);
  uint4* dst = reinterpret_cast<uint4*>(a.nb + base + mb0);
  for (int i = threadIdx.x; i < n16; i += 64) dst[i] = src[i];
}

// Wave-wide inclusive scans (one-wave workgroups: the per-slot scans below run beside the
// encode kernels on the copy stream, and a 1024-thread workgroup waited for a whole CU's
// worth of free wave slots -- 4-8 ms per launch instead of tens of microseconds).
__device__ __forceinline__ long long wave_scan_add(long long v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const long long y = __shfl_up(v, o, 64);
    if (lane >= o) v += y;
  }
  return v;
}
__device__ __forceinline__ int wave_scan_max(int v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(v, o, 64);
    if (lane >= o) v = max(v, y);
  }
  return v;
}

// mb_qp_delta chain (cabac_qp_chain as a scan): MB i codes a delta iff it is not skipped
// and (cbp != 0 or I16x16); its delta is QP_i - QP of the last earlier delta MB (or the
// slice QP); its first-bin context is "MB i-1 coded a non-zero delta".  One wave per slice.
__global__ __launch_bounds__(64) void cabac_chain(CabacBinArgs a) {
  const int slot = blockIdx.x / a.per_slot, first = (blockIdx.x - slot * a.per_slot) * a.slice_mbs;
  const int n = min(a.g.nmb() - first, a.slice_mbs), lane = threadIdx.x;
  CabacNb* nb = a.nb + static_cast<size_t>(slot) * a.g.nmb() + first;
  const int per = (n + 63) / 64;
  const int i0 = lane * per, i1 = min(n, i0 + per);
  auto has = [&](int i) { return !nb[i].skip && (nb[i].cbp != 0 || nb[i].kind == h264::MBK_I16x16); };
  int ld = -1;
  for (int i = i0; i < i1; ++i)
    if (has(i)) ld = i;
  const int incl = wave_scan_max(ld);
  ld = __shfl_up(incl, 1, 64);
  if (lane == 0) ld = -1;
  int last_qp = ld >= 0 ? nb[ld].qp : a.slot_qp[slot];
  for (int i = i0; i < i1; ++i) {
    if (has(i)) {
      int d = nb[i].qp - last_qp;
      if (d < -26) d += 52;
      if (d > 25) d -= 52;
      nb[i].dqp = static_cast<int8_t>(d);
      last_qp = nb[i].qp;
    } else {
      nb[i].dqp = 0;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  for (int i = lane; i < n; i += 64)
    nb[i].prev_dqp_nz = static_cast<uint8_t>(i > 0 && has(i - 1) && nb[i - 1].dqp != 0);
}

__global__ __launch_bounds__(64) void cabac_count(CabacBinArgs a) {
  const int mb = blockIdx.x * 64 + threadIdx.x, slot = blockIdx.y, n = a.g.nmb();
  if (mb >= n) return;
  const CabacSliceInfo si = slice_info(a, slot, mb);
  const size_t base = static_cast<size_t>(slot) * n;
  h264::CabacSymbolPacker<h264::CabacCountEmit> s;
  h264::CabacMbCoder<h264::CabacSymbolPacker<h264::CabacCountEmit>> coder(s, si, a.nb + base);
  coder.code_mb(mb, a.hdr[base + mb], a.coef + (base + mb) * h264::kCoefPerMb, mb == slice_end(a, mb) - 1);
  s.flush_bypass();
  a.cnt[base + mb] = s.out.n;
}

// Symbol offsets of every MB inside its slice: one wave per slice.
__global__ __launch_bounds__(64) void cabac_offsets(CabacBinArgs a) {
  const int slot = blockIdx.x / a.per_slot, first = (blockIdx.x - slot * a.per_slot) * a.slice_mbs;
  const int n = min(a.g.nmb() - first, a.slice_mbs), lane = threadIdx.x;
  const size_t base = static_cast<size_t>(slot) * a.g.nmb() + first;
  const int per = (n + 63) / 64;
  const int i0 = lane * per, i1 = min(n, i0 + per);
  long long loc = 0;
  for (int i = i0; i < i1; ++i) loc += a.cnt[base + i];
  const long long incl = wave_scan_add(loc);
  long long p = incl - loc;
  for (int i = i0; i < i1; ++i) {
    a.off[base + i] = p;
    p += a.cnt[base + i];
  }
  if (lane == 63) a.tot[blockIdx.x] = static_cast<int>(incl);
}

// Slice regions of this frame step in the group's pool: kCabacGap + symbols, rounded to
// 8 symbols (16-byte aligned), allocated back to back after the group's earlier steps.
// One wave.
__global__ __launch_bounds__(64) void cabac_alloc(CabacBinArgs a) {
  const int B = a.g.B * a.per_slot, lane = threadIdx.x;  // slices of the step
  const int per = (B + 63) / 64;
  const int i0 = lane * per, i1 = min(B, i0 + per);
  auto region = [&](int s) { return (static_cast<long long>(a.tot[s]) + kCabacGap + 7) & ~7ll; };
  long long loc = 0;
  for (int i = i0; i < i1; ++i) loc += region(i);
  const long long incl = wave_scan_add(loc);
  const long long sum = __shfl(incl, 63, 64);
  long long p = incl - loc;
  const long long start = *a.pool_used;
  const bool fits = start + sum + kArithReadAhead <= a.pool_cap;  // the coder's read-ahead
  for (int i = i0; i < i1; ++i) {
    a.base[i] = start + p;
    a.total[i] = fits ? a.tot[i] : -1;
    p += region(i);
  }
  if (lane == 0) {
    if (fits) *a.pool_used = start + sum;
    else atomicOr(a.err, 4);
  }
}

// Symbol sink of cabac_bins: symbols go through an 8-entry LDS stage per lane and leave
// as 16-byte stores (an MB's first and last partial chunks element by element, since the
// neighbouring MBs' lanes own the rest of those chunks).
struct StagedEmit {
  uint16_t* g;     // slice symbols (16-byte aligned)
  uint16_t* lds;   // this lane's stage
  long long start; // first symbol index of this MB
  long long pos;   // next symbol index
  int n;
  __device__ __forceinline__ void emit(uint16_t s) {
    lds[pos & 7] = s;
    ++pos;
    ++n;
    if ((pos & 7) == 0) {
      const long long c0 = pos - 8;
      if (c0 >= start) {
        const uint32_t* w = reinterpret_cast<const uint32_t*>(lds);
        *reinterpret_cast<uint4*>(g + c0) = make_uint4(w[0], w[1], w[2], w[3]);
      } else {
        for (long long i = start; i < pos; ++i) g[i] = lds[i & 7];
      }
    }
  }
  __device__ __forceinline__ void finish() {
    const long long c0 = pos & ~7ll;
    for (long long i = c0 > start ? c0 : start; i < pos; ++i) g[i] = lds[i & 7];
  }
};

// 6 waves per SIMD: 80 VGPRs instead of 94, no extra spill (it runs beside the encode kernels)
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(6, 8))) void cabac_bins(CabacBinArgs a) {
  __shared__ __attribute__((aligned(16))) uint16_t stage[64 * 8];
  const int mb = blockIdx.x * 64 + threadIdx.x, slot = blockIdx.y, n = a.g.nmb();
  if (mb >= n) return;
  const int ls = slice_index(a, slot, mb);
  if (a.total[ls] < 0) return;
  const CabacSliceInfo si = slice_info(a, slot, mb);
  const size_t base = static_cast<size_t>(slot) * n;
  h264::CabacSymbolPacker<StagedEmit> s;
  s.out.g = a.pool + a.base[ls] + kCabacGap;
  s.out.lds = stage + threadIdx.x * 8;
  s.out.start = s.out.pos = a.off[base + mb];
  s.out.n = 0;
  h264::CabacMbCoder<h264::CabacSymbolPacker<StagedEmit>> coder(s, si, a.nb + base);
  coder.code_mb(mb, a.hdr[base + mb], a.coef + (base + mb) * h264::kCoefPerMb, mb == slice_end(a, mb) - 1);
  s.flush_bypass();
  s.out.finish();
}

// ---------------------------------------------------------------- serial arithmetic coding
struct CabacCodeArgs {
  int L;                     // slices: G frame steps x B slots (lane l = step * B + slot)
  int B;
  int lpw;                   // live lanes per wave (the coder is latency-bound: spreading few
                             // slices over more waves / SIMDs buys throughput)
  uint16_t* pool;
  const long long* base;     // [L]
  const int* total;          // [L]
  const uint32_t* hdr_bits;  // [L, 16] slice header incl. cabac_alignment_one_bits, big-endian words
  const int* hdr_nbits;      // [L] (a multiple of 8)
  const int* slot_qp;        // [L] slice QP
  unsigned long long itypes; // bit g: frame step g is an I slice (else P)
  int* bytes;                // [L] out: slice RBSP bytes (-1: error)
  uint8_t* out;              // compacted slices (device; used when they exceed host_cap)
  long long* out_off;        // [L]
  int* err;
  uint8_t* host_out;         // pinned host buffer, device-visible (nullable)
  long long host_cap;
};

// Output of one lane's slice: bytes collect in a 256-byte LDS ring and leave as aligned
// dword stores at block ends, so no global store sits between a symbol block's load and
// its use (stores count in vmcnt on CDNA: a store inside the coding loop made every
// prefetch wait drain to vmcnt(0)).  Carries are resolved in the ring: `hold` is the last
// byte that can still take one (the last non-0xFF arithmetic byte; the 0xFF bytes after it
// become 0x00), and only bytes before it are flushed.
struct RingOut {
  uint8_t* p;          // global slice output (in place over the consumed symbols; 16-byte aligned)
  uint8_t* ring;       // this lane's LDS ring
  long long n, flushed, cap;
  long long arith0;    // first arithmetic byte (after the slice header)
  long long hold;      // -1 until the first non-0xFF arithmetic byte
  int ovf;
  __device__ void start(long long header_bytes) {
    arith0 = header_bytes;
    hold = -1;
  }
  __device__ void flush_words() {
    const long long e = (hold >= 0 ? hold : arith0) & ~3ll;
    for (; flushed < e; flushed += 4) {
      const uint32_t w = *reinterpret_cast<const uint32_t*>(ring + (flushed & 255));
      if (flushed + 4 <= cap) *reinterpret_cast<uint32_t*>(p + flushed) = w;
    }
  }
  __device__ void put(int b) {  // slice header bytes
    ring[n & 255] = static_cast<uint8_t>(b);
    ++n;
  }
  __device__ bool byte9(uint32_t v) {
    if (v >> 8) {
      if (hold < 0) return false;
      ring[hold & 255] += 1;
      for (long long i = hold + 1; i < n; ++i) ring[i & 255] = 0;
    }
    if (n - flushed >= 240) flush_words();
    if (n - flushed >= 256) {  // a 0xFF run longer than the ring: never seen in practice
      ovf = 1;
      return false;
    }
    const uint32_t b = v & 0xFFu;
    ring[n & 255] = static_cast<uint8_t>(b);
    if (b != 0xFFu) hold = n;
    ++n;
    return true;
  }
  __device__ __forceinline__ void finish() {
    hold = n;  // every byte is final
    flush_words();
    for (; flushed < n; ++flushed)
      if (flushed < cap) p[flushed] = ring[flushed & 255];
  }
};

// Branch-free symbol step of the GPU coder (the bytes equal CabacSymbolCoder::step_nodrain,
// which the host tests pin): every symbol reads and writes a context state -- bypass and
// terminate symbols use a dummy context row -- and one 8-byte table entry per state holds
// the four rLPS values and both transitions, so a symbol costs two dependent LDS reads and
// no exec-mask branches (the generic step branched around its LDS accesses).
constexpr int kDummyCtx = h264::kCabacContexts;  // extra LDS row absorbing non-decision symbols

template <class C>
__device__ __forceinline__ void fast_step(C& c, uint32_t sym, uint8_t* st_lane, const uint2* tab) {
  const bool dec = !(sym & 0x8000u);
  const bool byp = (sym & 0xC000u) == 0x8000u;
  uint8_t* sp = st_lane + (dec ? (sym & 0x1FFu) : static_cast<uint32_t>(kDummyCtx)) * 64u;
  const uint32_t sv = *sp;
  const uint32_t pst = sv >> 1, mps = sv & 1u;
  const uint2 t = tab[pst];
  const uint32_t rl = (t.x >> ((c.range >> 3) & 24u)) & 0xFFu;
  const uint32_t rlps = dec ? rl : 2u;
  const uint32_t r1 = c.range - rlps;
  const bool lpsb = dec && ((sym >> 9) & 1u) != mps;
  const uint32_t nr = lpsb ? rlps : r1;
  const uint32_t add = lpsb ? r1 : 0u;
  const uint32_t npst = lpsb ? (t.y & 0xFFu) : ((t.y >> 8) & 0xFFu);
  const uint32_t nmps = mps ^ ((lpsb && pst == 0) ? 1u : 0u);
  *sp = static_cast<uint8_t>((npst << 1) | nmps);
  const int shd = h264::cabac_clz32(nr) - 23;
  const int n = byp ? static_cast<int>((sym >> 10) & 15u) : (shd > 0 ? shd : 0);
  const uint32_t bterm = c.range * (byp ? (sym & 0x3FFu) : 0u);  // < 2^19
  const uint32_t nrs = nr << n;
  c.low = ((c.low + add) << n) + bterm;
  c.range = byp ? c.range : nrs;
  c.nbits += n;
}

constexpr int kArithBlock = 64;         // symbols per lane per block (8 x 16-byte loads)
constexpr int kArithInStride = 9;       // uint4 per lane in LDS (8 + 1 pad: conflict-free b128 reads)
constexpr int kArithRingStride = 260;   // bytes per lane ring (256 + 4 pad)

// One lane per slice (a.lpw live lanes per wave).  Per block of 64 symbols: the next block's 8 loads are issued first,
// the current block is coded from LDS (context states, symbols and output ring are all
// LDS, so the loop waits only on lgkmcnt), then the next block lands in LDS and the ring's
// complete dwords are stored.  The only vmcnt wait per block covers loads and stores issued
// a whole block earlier.
__global__ __launch_bounds__(64) void cabac_arith(CabacCodeArgs a) {
  __shared__ uint8_t st[(h264::kCabacContexts + 1) * 64];
  __shared__ uint2 tab[64];
  __shared__ uint4 sin[64 * kArithInStride];
  __shared__ __attribute__((aligned(16))) uint8_t ring[64 * kArithRingStride];
  const int lane = threadIdx.x;
  const int l = blockIdx.x * a.lpw + lane;
  const bool live = lane < a.lpw && l < a.L;
  tab[lane] = make_uint2(static_cast<uint32_t>(h264::kCabacRangeLPS[lane][0]) |
                            (static_cast<uint32_t>(h264::kCabacRangeLPS[lane][1]) << 8) |
                            (static_cast<uint32_t>(h264::kCabacRangeLPS[lane][2]) << 16) |
                            (static_cast<uint32_t>(h264::kCabacRangeLPS[lane][3]) << 24),
                        static_cast<uint32_t>(h264::kCabacTransLPS[lane]) |
                            (static_cast<uint32_t>(lane < 62 ? lane + 1 : 62) << 8));
  st[kDummyCtx * 64 + lane] = 0;
  // context states of this lane's slice (its slice type and QP; cabac_init_idc 0)
  const int qp = live ? h264::clip3(0, 51, a.slot_qp[l]) : 26;
  const int table = live && ((a.itypes >> (l / a.B)) & 1ull) ? 0 : 1;
  for (int i = 0; i < h264::kCabacContexts; ++i) {
    const int r = i < 276 ? i : (i >= 399 && i <= 435 ? i - 399 + 276 : -1);
    uint8_t v = 0;
    if (r >= 0) {
      const h264::CabacInitMN mn = h264::kCabacInit[table][r];
      const int pre = h264::clip3(1, 126, ((mn.m * qp) >> 4) + mn.n);
      v = pre <= 63 ? static_cast<uint8_t>((63 - pre) << 1) : static_cast<uint8_t>(((pre - 64) << 1) | 1);
    }
    st[i * 64 + lane] = v;
  }
  __syncthreads();
  if (!live) return;
  const int total = a.total[l];
  const uint16_t* sy = a.pool + a.base[l] + kCabacGap;
  if (total < 0) {  // pool exhausted (reported by cabac_alloc)
    a.bytes[l] = -1;
    return;
  }
  if (total == 0 || sy[total - 1] != 0xC001u) {
    a.bytes[l] = -1;
    atomicOr(a.err, 8);
    return;
  }
  h264::CabacSymbolCoder<RingOut> c;
  c.out.p = reinterpret_cast<uint8_t*>(a.pool + a.base[l]);
  c.out.ring = ring + lane * kArithRingStride;
  c.out.cap = 2ll * (((static_cast<long long>(total) + kCabacGap + 7) & ~7ll));
  c.out.n = c.out.flushed = 0;
  c.out.ovf = 0;
  const uint4* q = reinterpret_cast<const uint4*>(sy);
  uint4* my = sin + lane * kArithInStride;
  {
    uint4 t[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) t[k] = q[k];
#pragma unroll
    for (int k = 0; k < 8; ++k) my[k] = t[k];
  }
  const int hbytes = a.hdr_nbits[l] >> 3;
  for (int i = 0; i < hbytes; ++i) c.out.put(static_cast<uint8_t>(a.hdr_bits[l * 16 + (i >> 2)] >> (24 - 8 * (i & 3))));
  c.out.start(hbytes);
  c.init();
  const int n = total - 1;  // the last symbol is end_of_slice_flag = 1: finish()
  for (int b0 = 0; b0 < n; b0 += kArithBlock) {
    // read-ahead (the pool keeps slack past every slice): plain registers, not an array,
    // so nothing is staged through scratch
    const uint4* nq = q + (b0 >> 3) + 8;
    const uint4 n0 = nq[0], n1 = nq[1], n2 = nq[2], n3 = nq[3], n4 = nq[4], n5 = nq[5], n6 = nq[6], n7 = nq[7];
    const int m = min(kArithBlock, n - b0);
    for (int ch = 0; ch * 8 < m; ++ch) {
      const uint4 cw = my[ch];
      const int mm = min(8, m - ch * 8);
      // lazy draining: at most 4 symbols (<= 40 bits) between drains (see CabacSymbolCoder).
      // Symbols past the slice's end become 0x8000 (a bypass batch of no bins: a no-op),
      // so every lane runs the same straight-line code.
      auto sym = [&](uint32_t w, int k) { return k < mm ? w : 0x8000u; };
      fast_step(c, sym(cw.x & 0xFFFFu, 0), st + lane, tab);
      fast_step(c, sym(cw.x >> 16, 1), st + lane, tab);
      fast_step(c, sym(cw.y & 0xFFFFu, 2), st + lane, tab);
      fast_step(c, sym(cw.y >> 16, 3), st + lane, tab);
      c.drain();
      fast_step(c, sym(cw.z & 0xFFFFu, 4), st + lane, tab);
      fast_step(c, sym(cw.z >> 16, 5), st + lane, tab);
      fast_step(c, sym(cw.w & 0xFFFFu, 6), st + lane, tab);
      fast_step(c, sym(cw.w >> 16, 7), st + lane, tab);
      c.drain();
    }
    my[0] = n0;
    my[1] = n1;
    my[2] = n2;
    my[3] = n3;
    my[4] = n4;
    my[5] = n5;
    my[6] = n6;
    my[7] = n7;
    c.out.flush_words();
  }
  c.finish();
  const bool bad = c.bad || c.out.n > c.out.cap;
  a.bytes[l] = bad ? -1 : static_cast<int>(c.out.n);
  if (bad) atomicOr(a.err, 8);
}

// Slice outputs packed in l order, each starting on a 16-byte boundary, with 16-byte
// stores (the region bases in the pool are 16-byte aligned).  Into pinned host memory when
// the whole group fits host_cap (zero-copy: the bytes cross PCIe inside this kernel, in
// stream order after the coder, so no D2H copy has to be ordered against the next group),
// else into the device buffer.
__global__ __launch_bounds__(256) void cabac_compact(CabacCodeArgs a) {
  const int l = blockIdx.x;
  __shared__ unsigned long long s_off, s_tot;
  if (threadIdx.x == 0) s_off = s_tot = 0;
  __syncthreads();
  unsigned long long part = 0, tot = 0;
  for (int s = threadIdx.x; s < a.L; s += blockDim.x) {
    const unsigned long long r16 = a.bytes[s] > 0 ? ((static_cast<unsigned long long>(a.bytes[s]) + 15ull) & ~15ull) : 0ull;
    tot += r16;
    if (s < l) part += r16;
  }
  atomicAdd(&s_off, part);
  atomicAdd(&s_tot, tot);
  __syncthreads();
  const long long off = static_cast<long long>(s_off);
  const bool host = a.host_out && static_cast<long long>(s_tot) <= a.host_cap;
  if (threadIdx.x == 0) a.out_off[l] = off;
  const int nbytes = a.bytes[l];
  if (nbytes <= 0) return;
  const uint4* src = reinterpret_cast<const uint4*>(a.pool + a.base[l]);
  uint4* dst = reinterpret_cast<uint4*>((host ? a.host_out : a.out) + off);
  for (int i = threadIdx.x; i < (nbytes + 15) / 16; i += blockDim.x) dst[i] = src[i];
}

}  // namespace gpu
}  // namespace mivc

using namespace mivc::gpu;

extern "C" size_t mivc_cabac_nb_bytes() { return sizeof(CabacNb); }
extern "C" int mivc_cabac_gap() { return kCabacGap; }
extern "C" int mivc_cabac_read_ahead() { return kArithReadAhead; }

// One frame step's slices -> symbols in the group pool (pool_used advances; base/total
// describe each slice's region).  Scratch: mask, nb, cnt, off [B, nmb], tot [B].
extern "C" void mivc_launch_cabac_bin(int B, int wmb, int hmb, const void* hdr, const int16_t* coef, uint32_t* mask,
                                      void* nb, int* cnt, long long* off, int* tot, uint16_t* pool,
                                      long long pool_cap, long long* pool_used, long long* base, int* total,
                                      const int* slot_qp, int slice_type, int num_ref_l0, int num_ref_l1,
                                      int t8x8_mode, int* err, void* stream, const void* route, int slice_rows) {
  CabacBinArgs a;
  const int rows = (slice_rows > 0 && slice_rows < hmb) ? slice_rows : hmb;
  a.slice_mbs = rows * wmb;
  a.per_slot = (hmb + rows - 1) / rows;
  a.rt = static_cast<const SlotRoute*>(route);
  a.g = Geom{B, wmb, hmb, wmb * 16, hmb * 16};
  a.hdr = static_cast<const MbHeader*>(hdr);
  a.coef = coef;
  a.mask = mask;
  a.nb = static_cast<CabacNb*>(nb);
  a.cnt = cnt;
  a.off = off;
  a.tot = tot;
  a.pool = pool;
  a.pool_cap = pool_cap;
  a.pool_used = pool_used;
  a.base = base;
  a.total = total;
  a.slot_qp = slot_qp;
  a.slice_type = slice_type;
  a.num_ref_l0 = num_ref_l0;
  a.num_ref_l1 = num_ref_l1;
  a.t8x8_mode = t8x8_mode;
  a.err = err;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int nmb = wmb * hmb;
  const dim3 mbgrid((nmb + 63) / 64, B);
  hipLaunchKernelGGL(cabac_mask, dim3((nmb + 2 * kMaskSpan - 1) / (2 * kMaskSpan), B), dim3(64), 0, s, a);
  hipLaunchKernelGGL(cabac_prep, mbgrid, dim3(64), 0, s, a);
  hipLaunchKernelGGL(cabac_chain, dim3(B * a.per_slot), dim3(64), 0, s, a);
  hipLaunchKernelGGL(cabac_count, mbgrid, dim3(64), 0, s, a);
  hipLaunchKernelGGL(cabac_offsets, dim3(B * a.per_slot), dim3(64), 0, s, a);
  hipLaunchKernelGGL(cabac_alloc, dim3(1), dim3(64), 0, s, a);
  hipLaunchKernelGGL(cabac_bins, mbgrid, dim3(64), 0, s, a);
}

// L = G * B slices (frame step g of the group, slot b at l = g * B + b) -> slice RBSPs
// (header + CABAC data + stop bit), compacted in l order into `out`.
extern "C" void mivc_launch_cabac_code(int L, int B, uint16_t* pool, const long long* base, const int* total,
                                       const uint32_t* hdr_bits, const int* hdr_nbits, const int* slot_qp,
                                       unsigned long long itypes, int* bytes, uint8_t* out, long long* out_off,
                                       int* err, uint8_t* host_out, long long host_cap, void* stream) {
  CabacCodeArgs a;
  a.L = L;
  a.B = B;
  a.pool = pool;
  a.base = base;
  a.total = total;
  a.hdr_bits = hdr_bits;
  a.hdr_nbits = hdr_nbits;
  a.slot_qp = slot_qp;
  a.itypes = itypes;
  a.bytes = bytes;
  a.out = out;
  a.out_off = out_off;
  a.err = err;
  a.host_out = nullptr;
  a.host_cap = 0;
  if (host_out) {
    void* dp = nullptr;
    if (hipHostGetDevicePointer(&dp, host_out, 0) == hipSuccess && dp) {
      a.host_out = static_cast<uint8_t*>(dp);
      a.host_cap = host_cap;
    }
  }
  hipStream_t s = static_cast<hipStream_t>(stream);
  // full waves: spreading the slices over more, partly empty waves was measured slower
  // (the coder's issue cycles come out of the concurrently running encode kernels)
  a.lpw = 64;
  hipLaunchKernelGGL(cabac_arith, dim3((L + 63) / 64), dim3(64), 0, s, a);
  hipLaunchKernelGGL(cabac_compact, dim3(L), dim3(256), 0, s, a);
}
