// CABAC slice coding on the GPU (x264's default entropy coder behind
// the reference's `-vcodec libx264`, server.go:69-70 / client.go:115).
//
// CABAC is serial inside a slice, but every (slot, frame) picture of the batched encoder
// is its own slice, so B slices are coded at once: one workgroup per slot.  The
// macroblock-layer coder is the shared host/device implementation in
// csrc/common/h264_cabac.h, so the bytes are identical to the host writer's (the CPU test
// oracle) by construction.
//
// Kernels (batched over B slots):
//   cabac_mask    (nmb/2 x B, wave64)   non-zero mask of every 4x4 / DC block of every MB
//                                        (fully parallel; the serial coder then never loads
//                                        an all-zero block)
//   cabac_slices  (B, 64)               lanes initialise the 460 context states and the
//                                        neighbour row in LDS in parallel, copy the slice
//                                        header bytes; lane 0 then codes the slice data
//   cabac_compact (B, 256)              slot outputs packed back to back
#include "kcommon.h"
// after kcommon.h: the shared headers' MIVC_HD needs the HIP runtime declarations
#include "../common/h264_cabac.h"

namespace mivc {
namespace gpu {

using h264::CabacBuf;
using h264::CabacMbWriter;
using h264::CabacNb;
using h264::CabacSliceInfo;
using h264::MbHeader;

constexpr int kCabacMaxCols = 512;  // 8192 luma samples wide

struct CabacArgs {
  Geom g;
  const MbHeader* hdr;       // [B, nmb]
  const int16_t* coef;       // [B, nmb, 408]
  uint32_t* mask;            // [B, nmb]
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

__global__ __launch_bounds__(64) void cabac_slices(CabacArgs a) {
  __shared__ uint8_t st[h264::kCabacContexts];
  __shared__ CabacNb row[kCabacMaxCols];
  const Geom& g = a.g;
  const int slot = blockIdx.x, lane = threadIdx.x;
  const int qp = a.slot_qp[slot];
  const int table = a.slice_type == h264::SLICE_I ? 0 : 1;  // cabac_init_idc 0
  // ---- parallel prologue: context states, neighbour row, slice header bytes
  for (int i = lane; i < h264::kCabacContexts; i += 64) {
    const int r = i < 276 ? i : (i >= 399 && i <= 435 ? i - 399 + 276 : -1);
    uint8_t v = 0;
    if (r >= 0) {
      const h264::CabacInitMN mn = h264::kCabacInit[table][r];
      const int pre = h264::clip3(1, 126, ((mn.m * h264::clip3(0, 51, qp)) >> 4) + mn.n);
      v = pre <= 63 ? static_cast<uint8_t>((63 - pre) << 1) : static_cast<uint8_t>(((pre - 64) << 1) | 1);
    }
    st[i] = v;
  }
  for (int i = lane; i < g.wmb; i += 64) row[i].avail = 0;
  uint8_t* out = a.slot_out + static_cast<size_t>(slot) * a.cap;
  const int hbytes = a.hdr_nbits[slot] >> 3;
  for (int i = lane; i < hbytes; i += 64)
    out[i] = static_cast<uint8_t>(a.hdr_bits[slot * 16 + (i >> 2)] >> (24 - 8 * (i & 3)));
  __syncthreads();
  if (lane != 0) return;
  // ---- serial slice data
  CabacSliceInfo si{};
  si.slice_type = a.slice_type;
  si.wmb = g.wmb;
  si.hmb = g.hmb;
  si.first_mb = 0;
  si.num_ref[0] = a.num_ref_l0;
  si.num_ref[1] = a.num_ref_l1;
  si.t8x8_mode = a.t8x8_mode;
  si.slice_qp = qp;
  CabacBuf buf{out, static_cast<size_t>(a.cap), static_cast<size_t>(hbytes), 0};
  CabacMbWriter w;
  const size_t base = static_cast<size_t>(slot) * g.nmb();
  h264::cabac_write_slice_data(w, si, row, st, &buf, a.hdr + base, a.coef + base * h264::kCoefPerMb, g.nmb(), nullptr,
                               nullptr, a.mask + base, true, true);
  const bool bad = buf.overflow || w.e.bad;
  a.slot_bytes[slot] = bad ? -1 : static_cast<int>(buf.n);
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

// hdr_bits / hdr_nbits: slice header incl. the cabac_alignment_one_bits (byte-aligned);
// slot_out: [B, cap] scratch; out: compacted result; slot_bytes / out_off: per slot.
extern "C" void mivc_launch_cabac(int B, int wmb, int hmb, const void* hdr, const int16_t* coef, uint32_t* mask,
                                  uint8_t* slot_out, long long cap, int* slot_bytes, const uint32_t* hdr_bits,
                                  const int* hdr_nbits, const int* slot_qp, int slice_type, int num_ref_l0,
                                  int num_ref_l1, int t8x8_mode, uint8_t* out, long long* out_off, int* err,
                                  void* stream) {
  if (wmb > kCabacMaxCols) return;
  CabacArgs a;
  a.g = Geom{B, wmb, hmb, wmb * 16, hmb * 16};
  a.hdr = static_cast<const MbHeader*>(hdr);
  a.coef = coef;
  a.mask = mask;
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
  hipLaunchKernelGGL(cabac_mask, dim3((nmb + 1) / 2, B), dim3(64), 0, s, a);
  hipLaunchKernelGGL(cabac_slices, dim3(B), dim3(64), 0, s, a);
  hipLaunchKernelGGL(cabac_compact, dim3(B), dim3(256), 0, s, a);
}
