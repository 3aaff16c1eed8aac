// Per-slot picture routing of the batched H.264 encoder (models/h264_gpu.py, models/gop.py).
//
// Every slot of a batch follows its own GOP plan (x264 --b-adapt places B pictures per
// segment, --b-pyramid keeps some of them as references), so at one coding step slot 3 may
// code a P picture predicting from its buffer 2 while slot 4 codes a reference B picture
// between its buffers 0 and 1.  Reconstructions, half-sample planes and decision records of
// the reference pictures live in per-slot pools ([B, NB, plane], slot-major like the
// decoder's DPB); one SlotRoute per slot and step says which pool buffer plays which role.
// Kernels take a `const SlotRoute* rt` (the step's [B] row) plus the pool size NB: with
// rt == nullptr they behave as before (uniform batch, plane pointers as passed), so the HEVC
// encoder and the tools keep calling them unrouted.
//
// Plain C++ (shared by the .hip kernels and the pybind11 shim); the layout is mirrored by
// ROUTE_DTYPE in models/h264_gpu.py.
#pragma once
#include <cstdint>

namespace mivc {
namespace gpu {

enum SlotKind : int8_t { SK_IDLE = -1, SK_P = 0, SK_B = 1, SK_I = 2 };  // = the SliceType codes

enum SlotFlags : uint8_t {
  SF_REF = 1,      // a reference picture: its half-sample planes and records are kept
  SF_DEBLOCK = 2,  // run the in-loop filter on its reconstruction
};

// roles of a routed plane pointer: RefPicList0[0..3], RefPicList1[0], the picture being coded
enum RouteRole : int { RO_L0 = 0, RO_L1 = 4, RO_CUR = 5 };

struct SlotRoute {  // 32 bytes
  int8_t kind;      // SlotKind
  int8_t cur;       // pool buffer of the picture being coded
  int8_t n0;        // active RefPicList0 entries (P / B), 1..4
  int8_t l1;        // pool buffer of RefPicList1[0] (B)
  int8_t l0[4];     // pool buffers of RefPicList0[0..3]
  int16_t w1[4];    // B: implicit bi-prediction weight of list 1 per refIdxL0 (8.4.2.3.1; 32 = average)
  int16_t dsf[4];   // B: temporal-direct DistScaleFactor per refIdxL0 (8.4.1.2.3)
  int8_t dcopy[4];  // B: td == 0 (direct vectors copied, not scaled)
  uint8_t flags;    // SlotFlags
  int8_t col_l1;    // B: 1 = RefPicList1[0] is a B picture (its records carry list-1 motion)
  int16_t disp;     // display index of the picture (MB-tree offsets), -1 = none
};
static_assert(sizeof(SlotRoute) == 32, "SlotRoute layout is mirrored in Python");

// the pool index (slot-major [B, nbuf]) of a role's buffer; without routing, the slot itself
#if defined(__HIPCC__)
__host__ __device__
#endif
inline size_t route_index(const SlotRoute* rt, int nbuf, int slot, int role) {
  if (!rt) return static_cast<size_t>(slot);
  const SlotRoute& r = rt[slot];
  const int b = role == RO_CUR ? r.cur : (role == RO_L1 ? r.l1 : r.l0[role & 3]);
  return static_cast<size_t>(slot) * nbuf + (b < 0 ? 0 : b);
}

}  // namespace gpu
}  // namespace mivc
