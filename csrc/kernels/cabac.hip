// CABAC slice coding on the GPU (x264's default entropy coder behind
// the reference's `-vcodec libx264`, server.go:69-70 / client.go:115).
//
// CABAC is serial only in its arithmetic coder: every context index is a function of
// the decision records (csrc/common/h264_cabac.h: cabac_prepare_mb + cabac_qp_chain), so
// the binarisation of every macroblock of every slot runs in parallel and records
// 16-bit symbols; the serial stage is a tight arithmetic-coding loop over them.  The
// binariser is the shared host/device code, so the bytes equal the host writer's (CPU
// test oracle; tests/test_cabac.py pins the symbol decomposition on the CPU).
//
// Kernels (batched over B slots; each (slot, frame) picture is one slice):
//   cabac_mask    (nmb/2 x B, wave64)    non-zero mask of every 4x4 / DC block of every MB
//   cabac_prep    (nmb/64 x B, 64)       lane per MB: coding state (skip, cbp, mvd, cbf ...)
//   cabac_chain   (B, 1024)              mb_qp_delta chain (QP_pred scan) per slot
//   cabac_count   (nmb/64 x B, 64)       lane per MB: symbol count
//   cabac_offsets (B, 1024)              exclusive scan of the counts, capacity check
//   cabac_bins    (nmb/64 x B, 64)       lane per MB: symbols
//   cabac_arith   (B/64, 64)             lane per slot: context states (LDS, one column per
//                                         lane), slice header bytes, arithmetic coding
//   cabac_compact (B, 256)               slot outputs packed back to back
#include "kcommon.h"
// after kcommon.h: the shared headers' MIVC_HD needs the HIP runtime declarations
#include "../common/h264_cabac.h"

namespace mivc {
namespace gpu {

using h264::CabacNb;
using h264::CabacSliceInfo;
using h264::MbHeader;

struct CabacArgs {
  Geom g;
  const MbHeader* hdr;       // [B, nmb]
  const int16_t* coef;       // [B, nmb, 408]
  uint32_t* mask;            // [B, nmb]
  CabacNb* nb;               // [B, nmb]
  int* cnt;                  // [B, nmb] symbols per MB
  long long* off;            // [B, nmb] symbol offset per MB
  int* total;                // [B] symbols per slot
  uint16_t* syms;            // [B, cap_syms]
  long long cap_syms;
  uint8_t* slot_out;         // [B, cap] per-slot slice RBSP (header + data)
  long long cap;
  int* slot_bytes;           // [B] (-1: overflow)
  const uint32_t* hdr_bits;  // [B, 16] slice header incl. cabac_alignment_one_bits, big-endian words
  const int* hdr_nbits;      // [B] (a multiple of 8)
  const int* slot_qp;        // [B] slice QP
  int slice_type;
  int num_ref_l0, num_ref_l1;
  int t8x8_mode;
  uint8_t* out;              // compacted
  long long* out_off;        // [B]
  int* err;
};

__device__ __forceinline__ CabacSliceInfo slice_info(const CabacArgs& a, int slot) {
  CabacSliceInfo si{};
  si.slice_type = a.slice_type;
  si.wmb = a.g.wmb;
  si.hmb = a.g.hmb;
  si.first_mb = 0;
  si.num_ref[0] = a.num_ref_l0;
  si.num_ref[1] = a.num_ref_l1;
  si.t8x8_mode = a.t8x8_mode;
  si.slice_qp = a.slot_qp[slot];
  return si;
}

__global__ __launch_bounds__(64) void cabac_mask(CabacArgs a) {
  const Geom& g = a.g;
  const int lane = threadIdx.x, sub = lane & 31;
  const int mb = blockIdx.x * 2 + (lane >> 5), slot = blockIdx.y;
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

__global__ __launch_bounds__(64) void cabac_prep(CabacArgs a) {
  const int mb = blockIdx.x * 64 + threadIdx.x, slot = blockIdx.y;
  if (mb >= a.g.nmb()) return;
  const CabacSliceInfo si = slice_info(a, slot);
  const size_t base = static_cast<size_t>(slot) * a.g.nmb();
  h264::cabac_prepare_mb(si, a.hdr + base, mb, a.mask[base + mb], a.nb[base + mb]);
}

// mb_qp_delta chain (cabac_qp_chain as a scan): MB i codes a delta iff it is not skipped
// and (cbp != 0 or I16x16); its delta is QP_i - QP of the last earlier delta MB (or the
// slice QP); its first-bin context is "MB i-1 coded a non-zero delta".
__global__ __launch_bounds__(1024) void cabac_chain(CabacArgs a) {
  const int slot = blockIdx.x, n = a.g.nmb();
  CabacNb* nb = a.nb + static_cast<size_t>(slot) * n;
  __shared__ int s_last[1024];
  const int per = (n + blockDim.x - 1) / blockDim.x;
  const int i0 = threadIdx.x * per, i1 = min(n, i0 + per);
  auto has = [&](int i) { return !nb[i].skip && (nb[i].cbp != 0 || nb[i].kind == h264::MBK_I16x16); };
  int ld = -1;
  for (int i = i0; i < i1; ++i)
    if (has(i)) ld = i;
  s_last[threadIdx.x] = ld;
  __syncthreads();
  for (int o = 1; o < blockDim.x; o <<= 1) {
    const int v = threadIdx.x >= o ? s_last[threadIdx.x - o] : -1;
    __syncthreads();
    s_last[threadIdx.x] = max(s_last[threadIdx.x], v);
    __syncthreads();
  }
  ld = threadIdx.x > 0 ? s_last[threadIdx.x - 1] : -1;
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
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x)
    nb[i].prev_dqp_nz = static_cast<uint8_t>(i > 0 && has(i - 1) && nb[i - 1].dqp != 0);
}

__global__ __launch_bounds__(64) void cabac_count(CabacArgs a) {
  const int mb = blockIdx.x * 64 + threadIdx.x, slot = blockIdx.y, n = a.g.nmb();
  if (mb >= n) return;
  const CabacSliceInfo si = slice_info(a, slot);
  const size_t base = static_cast<size_t>(slot) * n;
  h264::CabacSymbolPacker<h264::CabacCountEmit> s;
  h264::CabacMbCoder<h264::CabacSymbolPacker<h264::CabacCountEmit>> coder(s, si, a.nb + base);
  coder.code_mb(mb, a.hdr[base + mb], a.coef + (base + mb) * h264::kCoefPerMb, mb == n - 1);
  s.flush_bypass();
  a.cnt[base + mb] = s.out.n;
}

__global__ __launch_bounds__(1024) void cabac_offsets(CabacArgs a) {
  const int slot = blockIdx.x, n = a.g.nmb();
  const size_t base = static_cast<size_t>(slot) * n;
  __shared__ long long s_sum[1024];
  const int per = (n + blockDim.x - 1) / blockDim.x;
  const int i0 = threadIdx.x * per, i1 = min(n, i0 + per);
  long long loc = 0;
  for (int i = i0; i < i1; ++i) loc += a.cnt[base + i];
  s_sum[threadIdx.x] = loc;
  __syncthreads();
  for (int o = 1; o < blockDim.x; o <<= 1) {
    const long long v = threadIdx.x >= o ? s_sum[threadIdx.x - o] : 0;
    __syncthreads();
    s_sum[threadIdx.x] += v;
    __syncthreads();
  }
  long long p = threadIdx.x > 0 ? s_sum[threadIdx.x - 1] : 0;
  for (int i = i0; i < i1; ++i) {
    a.off[base + i] = p;
    p += a.cnt[base + i];
  }
  if (threadIdx.x == blockDim.x - 1) {
    const long long tot = s_sum[blockDim.x - 1];
    const bool fits = tot <= a.cap_syms;
    a.total[slot] = fits ? static_cast<int>(tot) : -1;
    if (!fits) atomicOr(a.err, 2);
  }
}

__global__ __launch_bounds__(64) void cabac_bins(CabacArgs a) {
  const int mb = blockIdx.x * 64 + threadIdx.x, slot = blockIdx.y, n = a.g.nmb();
  if (mb >= n || a.total[slot] < 0) return;
  const CabacSliceInfo si = slice_info(a, slot);
  const size_t base = static_cast<size_t>(slot) * n;
  h264::CabacSymbolPacker<h264::CabacStoreEmit> s;
  s.out.p = a.syms + static_cast<size_t>(slot) * a.cap_syms + a.off[base + mb];
  h264::CabacMbCoder<h264::CabacSymbolPacker<h264::CabacStoreEmit>> coder(s, si, a.nb + base);
  coder.code_mb(mb, a.hdr[base + mb], a.coef + (base + mb) * h264::kCoefPerMb, mb == n - 1);
  s.flush_bypass();
}

// ---------------------------------------------------------------- serial arithmetic coding
// One lane per slot (64 slots per wave).  The context states of lane l live in LDS column
// l (st[ctx * 64 + l]: lanes reading the same context hit distinct bytes), the LPS tables
// in LDS; coder registers stay in VGPRs.  Byte-oriented coder of h264::CabacEncoder.
struct ArithState {
  uint32_t low, range;
  int nbits, pend, nff, bad;
  uint8_t* o;
  long long n, cap;
};

__device__ __forceinline__ void ar_out(ArithState& s, int b) {
  if (s.n < s.cap) s.o[s.n] = static_cast<uint8_t>(b);
  ++s.n;
}
__device__ __forceinline__ void ar_put_byte(ArithState& s, uint32_t v) {
  const int b = static_cast<int>(v & 0xFFu);
  if (v >> 8) {
    if (s.pend < 0) s.bad = 1;
    if (s.nff > 0) {
      ar_out(s, s.pend + 1);
      for (int k = 0; k < s.nff - 1; ++k) ar_out(s, 0);
      s.pend = 0;
      s.nff = 0;
    } else {
      s.pend += 1;
    }
  }
  if (b == 0xFF) {
    ++s.nff;
  } else {
    if (s.pend >= 0) {
      ar_out(s, s.pend);
      for (int k = 0; k < s.nff; ++k) ar_out(s, 0xFF);
    }
    s.pend = b;
    s.nff = 0;
  }
}
__device__ __forceinline__ void ar_drain(ArithState& s) {
  while (s.nbits >= 8) {
    const int sh = s.nbits + 2;
    const uint32_t v = s.low >> sh;
    s.low &= (1u << sh) - 1u;
    s.nbits -= 8;
    ar_put_byte(s, v);
  }
}

__global__ __launch_bounds__(64) void cabac_arith(CabacArgs a) {
  __shared__ uint8_t st[h264::kCabacContexts * 64];
  __shared__ uint8_t lps[64 * 4];
  __shared__ uint8_t trans[64];
  const int lane = threadIdx.x;
  const int slot = blockIdx.x * 64 + lane;
  const bool live = slot < a.g.B;
  for (int i = lane; i < 256; i += 64) lps[i] = h264::kCabacRangeLPS[i >> 2][i & 3];
  trans[lane] = h264::kCabacTransLPS[lane];
  // context states of every lane's slice (its own slice QP)
  const int qp = live ? h264::clip3(0, 51, a.slot_qp[slot]) : 26;
  const int table = a.slice_type == h264::SLICE_I ? 0 : 1;  // cabac_init_idc 0
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
  const int total = a.total[slot];
  if (total < 0) {
    a.slot_bytes[slot] = -1;
    return;
  }
  ArithState s;
  s.o = a.slot_out + static_cast<size_t>(slot) * a.cap;
  s.cap = a.cap;
  const int hbytes = a.hdr_nbits[slot] >> 3;
  for (int i = 0; i < hbytes; ++i) s.o[i] = static_cast<uint8_t>(a.hdr_bits[slot * 16 + (i >> 2)] >> (24 - 8 * (i & 3)));
  s.n = hbytes;
  s.low = 0;
  s.range = 510;
  s.nbits = -1;
  s.pend = -1;
  s.nff = 0;
  s.bad = 0;
  const uint16_t* sy = a.syms + static_cast<size_t>(slot) * a.cap_syms;
  uint4 buf = make_uint4(0, 0, 0, 0);
  for (int i = 0; i < total; ++i) {
    if ((i & 7) == 0) buf = *reinterpret_cast<const uint4*>(sy + i);  // 8 symbols (cap is a multiple of 8)
    const uint32_t w = (i & 4) ? ((i & 2) ? buf.w : buf.z) : ((i & 2) ? buf.y : buf.x);
    const uint32_t sym = (i & 1) ? (w >> 16) : (w & 0xFFFFu);
    if (!(sym & 0x8000u)) {
      // EncodeDecision
      const int ctx = sym & 0x1FF, bin = (sym >> 9) & 1;
      uint8_t* sp = &st[ctx * 64 + lane];
      const int sv = *sp;
      int pst = sv >> 1, mps = sv & 1;
      const uint32_t rlps = lps[pst * 4 + ((s.range >> 6) & 3)];
      s.range -= rlps;
      if (bin != mps) {
        s.low += s.range;
        s.range = rlps;
        mps ^= pst == 0;
        pst = trans[pst];
      } else {
        pst = min(pst + 1, 62);
      }
      *sp = static_cast<uint8_t>((pst << 1) | mps);
      if (s.range < 256) {
        const int sh = __clz(static_cast<int>(s.range)) - 23;
        s.range <<= sh;
        s.low <<= sh;
        s.nbits += sh;
      }
    } else if (!(sym & 0x4000u)) {
      // n bypass bins at once
      const int nb = (sym >> 10) & 15;
      s.low = (s.low << nb) + s.range * (sym & 0x3FFu);
      s.nbits += nb;
    } else {
      // EncodeTerminate (+ EncodeFlush and the stop bit on the last MB)
      s.range -= 2;
      if (!(sym & 1)) {
        if (s.range < 256) {
          s.range <<= 1;
          s.low <<= 1;
          s.nbits += 1;
        }
      } else {
        s.low += s.range;
        s.range = 2;
        s.low <<= 7;
        s.nbits += 7;
        ar_drain(s);
        s.low |= 0x80u;
        s.low <<= 3;
        s.nbits += 3;
        ar_drain(s);
        if (s.nbits > 0) {
          s.low <<= 8 - s.nbits;
          s.nbits = 8;
          ar_drain(s);
        }
        if (s.pend >= 0) ar_out(s, s.pend);
        for (int k = 0; k < s.nff; ++k) ar_out(s, 0xFF);
        s.pend = -1;
        s.nff = 0;
      }
    }
    if (s.nbits >= 8) ar_drain(s);
  }
  const bool bad = s.bad || s.n > s.cap;
  a.slot_bytes[slot] = bad ? -1 : static_cast<int>(s.n);
  if (bad) atomicOr(a.err, 2);
}

__global__ __launch_bounds__(256) void cabac_compact(CabacArgs a) {
  const int slot = blockIdx.x;
  long long off = 0;
  for (int s = 0; s < slot; ++s) off += a.slot_bytes[s] > 0 ? a.slot_bytes[s] : 0;
  if (threadIdx.x == 0) a.out_off[slot] = off;
  const int nbytes = a.slot_bytes[slot];
  if (nbytes <= 0) return;
  const uint8_t* src = a.slot_out + static_cast<size_t>(slot) * a.cap;
  uint8_t* dst = a.out + off;
  for (int i = threadIdx.x; i < nbytes; i += blockDim.x) dst[i] = src[i];
}

}  // namespace gpu
}  // namespace mivc

using namespace mivc::gpu;

extern "C" size_t mivc_cabac_nb_bytes() { return sizeof(CabacNb); }

// Scratch (all device memory, caller-owned): mask [B, nmb] u32, nb [B, nmb] CabacNb,
// cnt [B, nmb] i32, off [B, nmb] i64, total [B] i32, syms [B, cap_syms] u16 (cap_syms a
// multiple of 8), slot_out [B, cap] u8.  hdr_bits / hdr_nbits: slice header incl. the
// cabac_alignment_one_bits (byte-aligned).  Results: out (compacted), slot_bytes,
// out_off; err |= 2 on overflow.
extern "C" void mivc_launch_cabac(int B, int wmb, int hmb, const void* hdr, const int16_t* coef, uint32_t* mask,
                                  void* nb, int* cnt, long long* off, int* total, uint16_t* syms, long long cap_syms,
                                  uint8_t* slot_out, long long cap, int* slot_bytes, const uint32_t* hdr_bits,
                                  const int* hdr_nbits, const int* slot_qp, int slice_type, int num_ref_l0,
                                  int num_ref_l1, int t8x8_mode, uint8_t* out, long long* out_off, int* err,
                                  void* stream) {
  CabacArgs a;
  a.g = Geom{B, wmb, hmb, wmb * 16, hmb * 16};
  a.hdr = static_cast<const MbHeader*>(hdr);
  a.coef = coef;
  a.mask = mask;
  a.nb = static_cast<CabacNb*>(nb);
  a.cnt = cnt;
  a.off = off;
  a.total = total;
  a.syms = syms;
  a.cap_syms = cap_syms;
  a.slot_out = slot_out;
  a.cap = cap;
  a.slot_bytes = slot_bytes;
  a.hdr_bits = hdr_bits;
  a.hdr_nbits = hdr_nbits;
  a.slot_qp = slot_qp;
  a.slice_type = slice_type;
  a.num_ref_l0 = num_ref_l0;
  a.num_ref_l1 = num_ref_l1;
  a.t8x8_mode = t8x8_mode;
  a.out = out;
  a.out_off = out_off;
  a.err = err;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int nmb = wmb * hmb;
  const dim3 mbgrid((nmb + 63) / 64, B);
  hipLaunchKernelGGL(cabac_mask, dim3((nmb + 1) / 2, B), dim3(64), 0, s, a);
  hipLaunchKernelGGL(cabac_prep, mbgrid, dim3(64), 0, s, a);
  hipLaunchKernelGGL(cabac_chain, dim3(B), dim3(1024), 0, s, a);
  hipLaunchKernelGGL(cabac_count, mbgrid, dim3(64), 0, s, a);
  hipLaunchKernelGGL(cabac_offsets, dim3(B), dim3(1024), 0, s, a);
  hipLaunchKernelGGL(cabac_bins, mbgrid, dim3(64), 0, s, a);
  hipLaunchKernelGGL(cabac_arith, dim3((B + 63) / 64), dim3(64), 0, s, a);
  hipLaunchKernelGGL(cabac_compact, dim3(B), dim3(256), 0, s, a);
}
