// Synthetic raw-YUV source generator (BASELINE.json: "on synthetic raw-YUV
// input") -- writes frames straight into HBM so no PCIe/disk feed sits in the
// encode loop.
//
// Content model (deterministic in (seed, slot, frame)): a panning value-noise
// texture with sub-pixel global motion, three moving textured objects (local
// motion with occlusion), a slow luminance ramp, and +-2 LSB temporal sensor
// noise -- chosen to exercise motion estimation, intra prediction and residual
// coding the way camera content does.
//
// Content classes (SynthGeom::kind; the RD suite, tools/content_rd.py, measures encoder
// defaults on all of them, not on the headline content alone):
//   0 default   pan of up to +-3 / +-1.5 px per frame, objects at +-5 / +-3, a drifting sine
//   1 pan-fast  pan of 16..32 px per frame (sports, fast camera moves)
//   2 static    static background (no pan, no drifting pattern), small slow movers
//   3 fade      the default content faded to near black and back (48-frame period)
//   4 zoom      a steady zoom-in (1 % per frame) about the picture centre
//   5 cuts      a scene cut every 30 frames (new background region, inverted luma, objects moved)
//   6 noise     the default content with +-12 LSB sensor noise
//
// Cost structure: the 3-octave value noise is evaluated ONCE per slot into a
// periodic canvas (its lattice wraps at the canvas size), and the three object
// textures once into per-slot tiles; a frame is then a bilinear sample of the
// canvas at the frame's fractional pan offset (uniform weights), the object tiles
// at integer positions, one sine per pixel and one hash per 4 pixels (see the
// frame kernels below for the launch shape).
#include <algorithm>

#include "kcommon.h"

namespace mivc {
namespace gpu {

__device__ __forceinline__ uint32_t hash3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t h = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u) * 0x85EBCA77u ^ (c + 0x165667B1u) * 0xC2B2AE3Du;
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  h *= 0x297A2D39u;
  h ^= h >> 15;
  return h;
}

// smooth value noise in [0,1) on a lattice of `cell` pixels, periodic with (px, py) lattice cells
__device__ float value_noise_p(int x, int y, int cell, int px, int py, uint32_t seed) {
  const int xi = x / cell, yi = y / cell;
  float tx = static_cast<float>(x - xi * cell) / cell, ty = static_cast<float>(y - yi * cell) / cell;
  tx = tx * tx * (3.f - 2.f * tx);
  ty = ty * ty * (3.f - 2.f * ty);
  auto L = [&](int a, int b) {
    a = a % px;
    b = b % py;
    return (hash3(static_cast<uint32_t>(a), static_cast<uint32_t>(b), seed) >> 8) * (1.0f / 16777216.0f);
  };
  float v00 = L(xi, yi), v10 = L(xi + 1, yi), v01 = L(xi, yi + 1), v11 = L(xi + 1, yi + 1);
  return (v00 * (1 - tx) + v10 * tx) * (1 - ty) + (v01 * (1 - tx) + v11 * tx) * ty;
}

struct SynthGeom {
  int width, height;    // display size (even)
  int cw, ch;           // luma canvas (periodic), multiples of 192
  int ow[3], oh[3];     // object tile sizes
  int frames, slots, frame0;
  uint32_t seed;
  int slot0;            // global index of slot 0 (content depends on seed and slot0 + slot only)
  int kind;             // content class (see the file comment)
};

enum SynthKind : int { SK_DEFAULT = 0, SK_PAN_FAST, SK_STATIC, SK_FADE, SK_ZOOM, SK_CUTS, SK_NOISE, SK_NKINDS };

// the luma pan offset (pixels) of slot seed ss at frame f
__device__ __forceinline__ void pan_at(const SynthGeom& g, uint32_t ss, int f, float* px, float* py) {
  const float h1 = (hash3(ss, 1, 0) & 255) / 255.f, h2 = (hash3(ss, 2, 0) & 255) / 255.f;
  float vx = (h1 - 0.5f) * 6.f, vy = (h2 - 0.5f) * 3.f;
  if (g.kind == SK_PAN_FAST) {
    vx = (h1 < 0.5f ? -1.f : 1.f) * (16.f + 32.f * fabsf(h1 - 0.5f));
    vy = (h2 - 0.5f) * 8.f;
  } else if (g.kind == SK_STATIC || g.kind == SK_ZOOM) {
    vx = vy = 0.f;
  }
  float ox = 0.f, oy = 0.f;
  if (g.kind == SK_CUTS) {  // every 30 frames: a jump to another region of the canvas
    const uint32_t hs = hash3(ss, 77, static_cast<uint32_t>(f / 30));
    ox = static_cast<float>(hs % 997u);
    oy = static_cast<float>((hs >> 12) % 613u);
  }
  *px = vx * f + ox;
  *py = vy * f + oy;
}

// luma gain of the fade class at frame f (1 elsewhere)
__device__ __forceinline__ float fade_gain(const SynthGeom& g, int f) {
  if (g.kind != SK_FADE) return 1.f;
  return 0.15f + 0.85f * (0.5f + 0.5f * __cosf(6.2831853f * f / 48.f));
}

__device__ __forceinline__ uint32_t slot_seed(const SynthGeom& g, int slot) {
  return g.seed * 7919u + static_cast<uint32_t>(g.slot0 + slot) * 104729u;
}

// ---- once per slot: background canvas (luma + 2 chroma) and object tiles
__global__ void synth_canvas(SynthGeom g, uint8_t* cy, uint8_t* cu, uint8_t* cv) {
  const int x4 = (blockIdx.x * blockDim.x + threadIdx.x) * 4, y = blockIdx.y, slot = blockIdx.z;
  const uint32_t ss = slot_seed(g, slot);
  if (x4 < g.cw) {
    uint32_t w = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int x = x4 + k;
      float t = 0.55f * value_noise_p(x, y, 48, g.cw / 48, g.ch / 48, ss) +
                0.30f * value_noise_p(x, y, 12, g.cw / 12, g.ch / 12, ss + 1) +
                0.15f * value_noise_p(x, y, 4, g.cw / 4, g.ch / 4, ss + 2);
      w |= static_cast<uint32_t>(40.f + 170.f * t + 0.5f) << (8 * k);
    }
    *reinterpret_cast<uint32_t*>(cy + (static_cast<size_t>(slot) * g.ch + y) * g.cw + x4) = w;
  }
  const int ccw = g.cw / 2, cch = g.ch / 2;
  if (x4 < ccw && y < cch) {
    uint32_t wu = 0, wv = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int x = x4 + k;
      float a = 128.f + 40.f * (value_noise_p(x, y, 32, ccw / 32, cch / 32, ss + 5) - 0.5f);
      float b = 128.f + 40.f * (value_noise_p(x, y, 48, ccw / 48, cch / 48, ss + 6) - 0.5f);
      wu |= static_cast<uint32_t>(a + 0.5f) << (8 * k);
      wv |= static_cast<uint32_t>(b + 0.5f) << (8 * k);
    }
    const size_t off = (static_cast<size_t>(slot) * cch + y) * ccw + x4;
    *reinterpret_cast<uint32_t*>(cu + off) = wu;
    *reinterpret_cast<uint32_t*>(cv + off) = wv;
  }
}

__global__ void synth_objects(SynthGeom g, uint8_t* tiles, size_t tile_stride) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  const int o = blockIdx.z % 3, slot = blockIdx.z / 3;
  if (x >= g.ow[o] || y >= g.oh[o]) return;
  const uint32_t os = hash3(slot_seed(g, slot), 10 + o, 0);
  const int cell = 6 + 4 * o;
  // object-local texture (non-periodic: large period)
  float t = value_noise_p(x + 1000 * o, y, cell, 1 << 20, 1 << 20, os);
  uint8_t* tile = tiles + (static_cast<size_t>(slot) * 3 + o) * tile_stride;
  tile[static_cast<size_t>(y) * g.ow[o] + x] = static_cast<uint8_t>(60.f + 150.f * t + 0.5f);
}

// object o of a slot at frame f: integer top-left (px, py) in display coordinates (wrapping)
__device__ __forceinline__ void object_pos(const SynthGeom& g, int slot, int o, int f, int w, int h, int ow, int oh,
                                           float vscale, int* px, int* py) {
  const uint32_t os = hash3(slot_seed(g, slot), 10 + o, 0);
  float cx = (os & 1023) / 1023.f * w, cy = ((os >> 10) & 1023) / 1023.f * h;
  float ovx = (((os >> 20) & 63) / 63.f - 0.5f) * 10.f * vscale, ovy = (((os >> 26) & 63) / 63.f - 0.5f) * 6.f * vscale;
  int x = static_cast<int>(floorf(cx + ovx * f)) - ow / 2, y = static_cast<int>(floorf(cy + ovy * f)) - oh / 2;
  x %= w;
  y %= h;
  *px = x < 0 ? x + w : x;
  *py = y < 0 ? y + h : y;
}

struct FrameArgs {
  SynthGeom g;
  const uint8_t *cy, *cu, *cv, *tiles;
  size_t tile_stride;
  void *y, *u, *v;  // [slots*frames, h, w] display-size frames (uint8, or uint16 at BD 10)
};

// 16 output samples of a run: one 16-byte store at 8 bits, two at 10 bits (uint16 samples)
template <int BD>
__device__ __forceinline__ void store_run(void* base, size_t idx, const int (&v)[16], int valid) {
  if constexpr (BD == 8) {
    uint8_t* dst = static_cast<uint8_t*>(base) + idx;
    uint32_t o[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      int p4[4] = {v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
      o[q] = pack4_u8(p4);
    }
    if (valid >= 16 && (reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
      *reinterpret_cast<uint4*>(dst) = make_uint4(o[0], o[1], o[2], o[3]);
    } else {
      for (int k = 0; k < 16 && k < valid; ++k) dst[k] = static_cast<uint8_t>(v[k]);
    }
  } else {
    uint16_t* dst = static_cast<uint16_t*>(base) + idx;
    uint32_t o[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = static_cast<uint32_t>(v[2 * q]) | (static_cast<uint32_t>(v[2 * q + 1]) << 16);
    if (valid >= 16 && (reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
      reinterpret_cast<uint4*>(dst)[0] = make_uint4(o[0], o[1], o[2], o[3]);
      reinterpret_cast<uint4*>(dst)[1] = make_uint4(o[4], o[5], o[6], o[7]);
    } else {
      for (int k = 0; k < 16 && k < valid; ++k) dst[k] = static_cast<uint16_t>(v[k]);
    }
  }
}

// A frame step is B*F frames of W x H: the per-row launch of the first version issued
// ~50M 256-thread workgroups per 1080p batch and was bound by workgroup dispatch
// (131 ms for 15360 frames, ~250 GB/s).  Here a fixed grid strides over 16-pixel
// runs: one unit = 16 consecutive pixels of one row, one 16-byte store; the canvas
// bytes of a run come from 5 aligned dword loads + v_alignbyte, and one hash feeds the
// sensor noise of 4 pixels.
__device__ __forceinline__ int noise5(uint32_t h, int k) { return static_cast<int>(((h >> (8 * k)) & 255u) % 5u) - 2; }
// the same +-2 (8-bit) LSB noise amplitude at 10 bits: +-8 in 10-bit steps
__device__ __forceinline__ int noise17(uint32_t h, int k) { return static_cast<int>(((h >> (8 * k)) & 255u) % 17u) - 8; }

struct FrameConst {
  int slot, f;
  uint32_t ss;
  int obx[3], oby[3];
};

__device__ __forceinline__ FrameConst frame_const(const SynthGeom& g, int fz) {
  FrameConst c;
  c.slot = fz / g.frames;
  c.f = fz % g.frames + g.frame0;
  c.ss = slot_seed(g, c.slot);
  // static: small slow movers; cuts: the objects jump at every cut
  const float vs = g.kind == SK_STATIC ? 0.4f : 1.f;
  const int fo = g.kind == SK_CUTS ? c.f + 1000 * (c.f / 30) : c.f;
#pragma unroll
  for (int o = 0; o < 3; ++o) object_pos(g, c.slot, o, fo, g.width, g.height, g.ow[o], g.oh[o], vs, &c.obx[o], &c.oby[o]);
  return c;
}

// Per-frame constants are computed once per workgroup (grid = (run blocks, frames)), the
// objects are tested once per 16-pixel run (per-pixel tests only where a run meets one),
// and the per-pixel sine comes from one sin/cos pair per run by angle addition.
struct FrameShared {
  FrameConst fc;
  int ix, iy;
  float w00, w10, w01, w11;
};

// sin(a + d * k), cos(d * k) for k = 0..15 by angle addition from one sin/cos pair
template <int N>
__device__ __forceinline__ void sin_run(float a, float d, float (&out)[N]) {
  const float s0 = __sinf(a), c0 = __cosf(a);
#pragma unroll
  for (int k = 0; k < N; ++k) out[k] = s0 * cosf(d * k) + c0 * sinf(d * k);  // constants after unrolling
}

// does the run [x16, x16 + 16) of row y meet object o (wrapping display coordinates)?
__device__ __forceinline__ bool run_meets(int x16, int y, int obx, int oby, int ow, int oh, int w, int h) {
  int ly = y - oby;
  ly = ly < 0 ? ly + h : ly;
  if (ly >= oh) return false;
  int lx = x16 - obx;
  lx = lx < 0 ? lx + w : lx;
  return lx < ow || lx + 16 > w;
}

// BD 10: the same content computed at 10-bit precision (canvas interpolation, ramp and
// noise keep their fractional bits; texture tiles scale by 4), not 8-bit samples << 2.
template <int BD>
__global__ __launch_bounds__(256) void synth_frame_luma(FrameArgs a) {
  constexpr float S = BD == 8 ? 1.f : 4.f;
  constexpr int kMax = (1 << BD) - 1;
  const SynthGeom& g = a.g;
  const int runs = (g.width + 15) >> 4;
  const int nfr = g.slots * g.frames;
  __shared__ FrameShared F;
  for (int fz = blockIdx.y; fz < nfr; fz += gridDim.y) {
    __syncthreads();
    if (threadIdx.x == 0) {
      F.fc = frame_const(g, fz);
      // per-slot global motion (pan), sub-pixel
      float fx, fy;
      pan_at(g, F.fc.ss, F.fc.f, &fx, &fy);
      const float ixf = floorf(fx), iyf = floorf(fy);
      const float tx = fx - ixf, ty = fy - iyf;
      F.ix = static_cast<int>(ixf);
      F.iy = static_cast<int>(iyf);
      F.w00 = (1.f - tx) * (1.f - ty);
      F.w10 = tx * (1.f - ty);
      F.w01 = (1.f - tx) * ty;
      F.w11 = tx * ty;
    }
    __syncthreads();
    const FrameConst& fc = F.fc;
    for (int item = blockIdx.x * blockDim.x + threadIdx.x; item < g.height * runs; item += gridDim.x * blockDim.x) {
    const int y = item / runs, x16 = (item - y * runs) * 16;
    int cy0 = (y + F.iy) % g.ch;
    cy0 = cy0 < 0 ? cy0 + g.ch : cy0;
    const int cy1 = cy0 + 1 == g.ch ? 0 : cy0 + 1;
    const uint8_t* r0 = a.cy + (static_cast<size_t>(fc.slot) * g.ch + cy0) * g.cw;
    const uint8_t* r1 = a.cy + (static_cast<size_t>(fc.slot) * g.ch + cy1) * g.cw;
    int cx0 = (x16 + F.ix) % g.cw;
    cx0 = cx0 < 0 ? cx0 + g.cw : cx0;
    uint32_t u0w[5], u1w[5];
    if (cx0 + 17 <= g.cw) {  // the run's 17 canvas bytes are contiguous (cw is a multiple of 4)
      const int ca = cx0 & ~3, sh = cx0 & 3;
      uint32_t w0[6], w1[6];
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        const int o = min(ca + 4 * k, g.cw - 4);
        w0[k] = *reinterpret_cast<const uint32_t*>(r0 + o);
        w1[k] = *reinterpret_cast<const uint32_t*>(r1 + o);
      }
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        u0w[k] = __builtin_amdgcn_alignbyte(w0[k + 1], w0[k], sh);
        u1w[k] = __builtin_amdgcn_alignbyte(w1[k + 1], w1[k], sh);
      }
    } else {
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        uint32_t v0 = 0, v1 = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          int cx = cx0 + 4 * k + b;
          cx = cx >= g.cw ? cx - g.cw : cx;
          v0 |= static_cast<uint32_t>(r0[cx]) << (8 * b);
          v1 |= static_cast<uint32_t>(r1[cx]) << (8 * b);
        }
        u0w[k] = v0;
        u1w[k] = v1;
      }
    }
    auto t0 = [&](int k) { return static_cast<float>((u0w[k >> 2] >> (8 * (k & 3))) & 255u); };
    auto t1 = [&](int k) { return static_cast<float>((u1w[k >> 2] >> (8 * (k & 3))) & 255u); };
    float sn[16];
    sin_run(0.01f * (x16 + y) + (g.kind == SK_STATIC ? 0.f : 0.03f * fc.f), 0.01f, sn);
    float bg[16];
    if (g.kind == SK_ZOOM) {
      // per-pixel bilinear sample of the canvas at the zoomed position (1 % per frame)
      const float inv = 1.f / (1.f + 0.01f * fc.f), cxm = 0.5f * g.width, cym = 0.5f * g.height;
      const float sy = (y - cym) * inv + cym;
      const int iy = static_cast<int>(floorf(sy));
      const float ty = sy - iy;
      int ry0 = iy % g.ch;
      ry0 = ry0 < 0 ? ry0 + g.ch : ry0;
      const int ry1 = ry0 + 1 == g.ch ? 0 : ry0 + 1;
      const uint8_t* q0 = a.cy + (static_cast<size_t>(fc.slot) * g.ch + ry0) * g.cw;
      const uint8_t* q1 = a.cy + (static_cast<size_t>(fc.slot) * g.ch + ry1) * g.cw;
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const float sx = (x16 + k - cxm) * inv + cxm;
        const int ix = static_cast<int>(floorf(sx));
        const float tx = sx - ix;
        int c0 = ix % g.cw;
        c0 = c0 < 0 ? c0 + g.cw : c0;
        const int c1 = c0 + 1 == g.cw ? 0 : c0 + 1;
        bg[k] = (q0[c0] * (1.f - tx) + q0[c1] * tx) * (1.f - ty) + (q1[c0] * (1.f - tx) + q1[c1] * tx) * ty;
      }
    } else {
#pragma unroll
      for (int k = 0; k < 16; ++k) bg[k] = t0(k) * F.w00 + t0(k + 1) * F.w10 + t1(k) * F.w01 + t1(k + 1) * F.w11;
    }
    int lum[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) lum[k] = static_cast<int>(S * (bg[k] + 20.f * sn[k]) + 0.5f);
#pragma unroll
    for (int o = 0; o < 3; ++o) {
      if (run_meets(x16, y, fc.obx[o], fc.oby[o], g.ow[o], g.oh[o], g.width, g.height)) {
        int ly = y - fc.oby[o];
        ly = ly < 0 ? ly + g.height : ly;
        const uint8_t* trow = a.tiles + (static_cast<size_t>(fc.slot) * 3 + o) * a.tile_stride + static_cast<size_t>(ly) * g.ow[o];
        for (int k = 0; k < 16; ++k) {
          int lx = x16 + k - fc.obx[o];
          lx = lx < 0 ? lx + g.width : lx;  // wrap-around
          if (lx < g.ow[o]) lum[k] = static_cast<int>(trow[lx]) * static_cast<int>(S);
        }
      }
    }
    if (g.kind == SK_FADE || g.kind == SK_CUTS) {
      const float gain = fade_gain(g, fc.f);
      const bool inv = g.kind == SK_CUTS && ((fc.f / 30) & 1);
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        int v = static_cast<int>(16.f * S + (lum[k] - 16.f * S) * gain + 0.5f);
        lum[k] = inv ? kMax - v : v;
      }
    }
    const int namp = g.kind == SK_NOISE ? 12 : 2;  // +-LSB at 8 bits
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t h = hash3(static_cast<uint32_t>(x16 + 4 * q), static_cast<uint32_t>(y), fc.ss ^ (fc.f * 2654435761u));
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int nz = namp == 2 ? (BD == 8 ? noise5(h, b) : noise17(h, b))
                                 : (static_cast<int>(((h >> (8 * b)) & 255u) % (2u * namp + 1u)) - namp) * (BD == 8 ? 1 : 4);
        lum[4 * q + b] = clampi(lum[4 * q + b] + nz, 0, kMax);
      }
    }
    store_run<BD>(a.y, (static_cast<size_t>(fz) * g.height + y) * g.width + x16, lum, g.width - x16);
    }
  }
}

template <int BD>
__global__ __launch_bounds__(256) void synth_frame_chroma(FrameArgs a) {
  constexpr int S = BD == 8 ? 1 : 4;
  constexpr int kMax = (1 << BD) - 1;
  const SynthGeom& g = a.g;
  const int w2 = g.width / 2, h2 = g.height / 2, ccw = g.cw / 2, cch = g.ch / 2;
  const int runs = (w2 + 15) >> 4;
  const int nfr = g.slots * g.frames;
  __shared__ FrameShared F;
  for (int fz = blockIdx.y; fz < nfr; fz += gridDim.y) {
    __syncthreads();
    if (threadIdx.x == 0) {
      F.fc = frame_const(g, fz);
      float fx, fy;
      pan_at(g, F.fc.ss, F.fc.f, &fx, &fy);  // chroma moves at half the luma pan
      F.ix = static_cast<int>(floorf(0.5f * fx));
      F.iy = static_cast<int>(floorf(0.5f * fy));
#pragma unroll
      for (int o = 0; o < 3; ++o) {
        F.fc.obx[o] >>= 1;
        F.fc.oby[o] >>= 1;
      }
    }
    __syncthreads();
    const FrameConst& fc = F.fc;
    for (int item = blockIdx.x * blockDim.x + threadIdx.x; item < h2 * runs; item += gridDim.x * blockDim.x) {
    const int y = item / runs, x16 = (item - y * runs) * 16;
    int cyy = (y + F.iy) % cch;
    cyy = cyy < 0 ? cyy + cch : cyy;
    const size_t rowo = (static_cast<size_t>(fc.slot) * cch + cyy) * ccw;
    int cx0 = (x16 + F.ix) % ccw;
    cx0 = cx0 < 0 ? cx0 + ccw : cx0;
    uint32_t uw[4], vw[4];
    if (cx0 + 20 <= ccw) {  // contiguous: 5 aligned words + alignbyte
      const int ca = cx0 & ~3, sh = cx0 & 3;
      uint32_t a0[5], b0[5];
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        a0[k] = *reinterpret_cast<const uint32_t*>(a.cu + rowo + ca + 4 * k);
        b0[k] = *reinterpret_cast<const uint32_t*>(a.cv + rowo + ca + 4 * k);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        uw[k] = __builtin_amdgcn_alignbyte(a0[k + 1], a0[k], sh);
        vw[k] = __builtin_amdgcn_alignbyte(b0[k + 1], b0[k], sh);
      }
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        uint32_t p = 0, q = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          int cx = cx0 + 4 * k + b;
          cx = cx >= ccw ? cx - ccw : cx;
          p |= static_cast<uint32_t>(a.cu[rowo + cx]) << (8 * b);
          q |= static_cast<uint32_t>(a.cv[rowo + cx]) << (8 * b);
        }
        uw[k] = p;
        vw[k] = q;
      }
    }
    float sn[16];
    sin_run(0.02f * x16, 0.02f, sn);
    const int cv_row = static_cast<int>(10.f * S * __cosf(0.02f * y));
    int cu[16], cv[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      cu[k] = static_cast<int>((uw[k >> 2] >> (8 * (k & 3))) & 255u) * S + static_cast<int>(10.f * S * sn[k]);
      cv[k] = static_cast<int>((vw[k >> 2] >> (8 * (k & 3))) & 255u) * S + cv_row;
    }
#pragma unroll
    for (int o = 0; o < 3; ++o) {
      if (run_meets(x16, y, fc.obx[o], fc.oby[o], g.ow[o] / 2, g.oh[o] / 2, w2, h2)) {
        for (int k = 0; k < 16; ++k) {
          int lx = x16 + k - fc.obx[o];
          lx = lx < 0 ? lx + w2 : lx;
          if (lx < g.ow[o] / 2) {
            cu[k] = (90 + 50 * o) * S;
            cv[k] = (170 - 40 * o) * S;
          }
        }
      }
    }
    if (g.kind == SK_FADE || g.kind == SK_CUTS) {
      const float gain = fade_gain(g, fc.f);
      const bool swap = g.kind == SK_CUTS && ((fc.f / 30) & 1);
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int a0 = static_cast<int>(128.f * S + (cu[k] - 128.f * S) * gain + 0.5f);
        const int b0 = static_cast<int>(128.f * S + (cv[k] - 128.f * S) * gain + 0.5f);
        cu[k] = swap ? b0 : a0;
        cv[k] = swap ? a0 : b0;
      }
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      cu[k] = clampi(cu[k], 0, kMax);
      cv[k] = clampi(cv[k], 0, kMax);
    }
    const size_t idx = (static_cast<size_t>(fz) * h2 + y) * w2 + x16;
    store_run<BD>(a.u, idx, cu, w2 - x16);
    store_run<BD>(a.v, idx, cv, w2 - x16);
    }
  }
}

}  // namespace gpu
}  // namespace mivc

using namespace mivc::gpu;

// bit_depth 8: uint8 planes; 10: uint16 planes holding 10-bit samples
extern "C" void mivc_launch_synth(void* y, void* u, void* v, int width, int height, int slots, int frames, int frame0,
                                  uint32_t seed, int bit_depth, int slot0, void* stream, int kind) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  SynthGeom g{};
  g.kind = kind;
  g.width = width;
  g.height = height;
  g.cw = (width + 191) / 192 * 192 + 192;
  g.ch = (height + 191) / 192 * 192 + 192;
  size_t tile_stride = 0;
  for (int o = 0; o < 3; ++o) {
    g.ow[o] = (static_cast<int>(width * (0.08f + 0.05f * o)) * 2 + 1) & ~1;
    g.oh[o] = (static_cast<int>(height * (0.10f + 0.06f * o)) * 2 + 1) & ~1;
    tile_stride = std::max(tile_stride, static_cast<size_t>(g.ow[o]) * g.oh[o]);
  }
  tile_stride = (tile_stride + 255) & ~static_cast<size_t>(255);
  g.frames = frames;
  g.slots = slots;
  g.frame0 = frame0;
  g.seed = seed;
  g.slot0 = slot0;
  const size_t ysz = static_cast<size_t>(g.cw) * g.ch, csz = ysz / 4;
  const size_t bytes = slots * (ysz + 2 * csz + 3 * tile_stride);
  uint8_t* ws = nullptr;
  keep_async_pool();
  if (hipMallocAsync(reinterpret_cast<void**>(&ws), bytes, s) != hipSuccess) return;
  uint8_t* cy = ws;
  uint8_t* cu = cy + slots * ysz;
  uint8_t* cv = cu + slots * csz;
  uint8_t* tiles = cv + slots * csz;
  hipLaunchKernelGGL(synth_canvas, dim3((g.cw / 4 + 255) / 256, g.ch, slots), dim3(256), 0, s, g, cy, cu, cv);
  int omw = std::max(g.ow[0], std::max(g.ow[1], g.ow[2])), omh = std::max(g.oh[0], std::max(g.oh[1], g.oh[2]));
  hipLaunchKernelGGL(synth_objects, dim3((omw + 255) / 256, omh, slots * 3), dim3(256), 0, s, g, tiles, tile_stride);
  FrameArgs fa{g, cy, cu, cv, tiles, tile_stride, y, u, v};
  // grid: (16-pixel-run blocks of one frame, frames); frames beyond 65535 stride
  const long long fr = static_cast<long long>(slots) * frames;
  const unsigned gy = static_cast<unsigned>(fr < 65535 ? fr : 65535);
  const int lruns = height * ((width + 15) / 16), cruns = (height / 2) * ((width / 2 + 15) / 16);
  // 8 runs per thread: per-frame setup and workgroup dispatch amortised over 2048 runs
  if (bit_depth == 10) {
    hipLaunchKernelGGL(synth_frame_luma<10>, dim3((lruns + 2047) / 2048, gy), dim3(256), 0, s, fa);
    hipLaunchKernelGGL(synth_frame_chroma<10>, dim3((cruns + 2047) / 2048, gy), dim3(256), 0, s, fa);
  } else {
    hipLaunchKernelGGL(synth_frame_luma<8>, dim3((lruns + 2047) / 2048, gy), dim3(256), 0, s, fa);
    hipLaunchKernelGGL(synth_frame_chroma<8>, dim3((cruns + 2047) / 2048, gy), dim3(256), 0, s, fa);
  }
  hipFreeAsync(ws, s);
}
