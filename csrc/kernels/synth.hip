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
};

__device__ __forceinline__ uint32_t slot_seed(const SynthGeom& g, int slot) {
  return g.seed * 7919u + static_cast<uint32_t>(slot) * 104729u;
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
  uint8_t *y, *u, *v;  // [slots*frames, h, w] display-size frames
};

// A frame step is B*F frames of W x H: the per-row launch of the first version issued
// ~50M 256-thread workgroups per 1080p batch and was bound by workgroup dispatch
// (131 ms for 15360 frames, ~250 GB/s).  Here a fixed grid strides over 16-pixel
// runs: one unit = 16 consecutive pixels of one row, one 16-byte store; the canvas
// bytes of a run come from 5 aligned dword loads + v_alignbyte, and one hash feeds the
// sensor noise of 4 pixels.
__device__ __forceinline__ int noise5(uint32_t h, int k) { return static_cast<int>(((h >> (8 * k)) & 255u) % 5u) - 2; }

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
#pragma unroll
  for (int o = 0; o < 3; ++o) object_pos(g, c.slot, o, c.f, g.width, g.height, g.ow[o], g.oh[o], 1.f, &c.obx[o], &c.oby[o]);
  return c;
}

__global__ __launch_bounds__(256) void synth_frame_luma(FrameArgs a) {
  const SynthGeom& g = a.g;
  const int runs = (g.width + 15) >> 4;
  const long long total = static_cast<long long>(g.slots) * g.frames * g.height * runs;
  for (long long i = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += static_cast<long long>(gridDim.x) * blockDim.x) {
    const int fz = static_cast<int>(i / (static_cast<long long>(g.height) * runs));
    const int rem = static_cast<int>(i - static_cast<long long>(fz) * g.height * runs);
    const int y = rem / runs, x16 = (rem - y * runs) * 16;
    const FrameConst fc = frame_const(g, fz);
    // per-slot global motion (pan) in pixels/frame, sub-pixel
    const float vx = ((hash3(fc.ss, 1, 0) & 255) / 255.f - 0.5f) * 6.f;
    const float vy = ((hash3(fc.ss, 2, 0) & 255) / 255.f - 0.5f) * 3.f;
    const float fx = vx * fc.f, fy = vy * fc.f;
    const float ixf = floorf(fx), iyf = floorf(fy);
    const float tx = fx - ixf, ty = fy - iyf;
    int cy0 = (y + static_cast<int>(iyf)) % g.ch;
    cy0 = cy0 < 0 ? cy0 + g.ch : cy0;
    const int cy1 = cy0 + 1 == g.ch ? 0 : cy0 + 1;
    const uint8_t* r0 = a.cy + (static_cast<size_t>(fc.slot) * g.ch + cy0) * g.cw;
    const uint8_t* r1 = a.cy + (static_cast<size_t>(fc.slot) * g.ch + cy1) * g.cw;
    int cx0 = (x16 + static_cast<int>(ixf)) % g.cw;
    cx0 = cx0 < 0 ? cx0 + g.cw : cx0;
    uint8_t t0[20], t1[20];
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
        const uint32_t u0 = __builtin_amdgcn_alignbyte(w0[k + 1], w0[k], sh);
        const uint32_t u1 = __builtin_amdgcn_alignbyte(w1[k + 1], w1[k], sh);
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          t0[4 * k + b] = static_cast<uint8_t>(u0 >> (8 * b));
          t1[4 * k + b] = static_cast<uint8_t>(u1 >> (8 * b));
        }
      }
    } else {
#pragma unroll
      for (int k = 0; k < 17; ++k) {
        const int cx = cx0 + k >= g.cw ? cx0 + k - g.cw : cx0 + k;
        t0[k] = r0[cx];
        t1[k] = r1[cx];
      }
    }
    const float w00 = (1.f - tx) * (1.f - ty), w10 = tx * (1.f - ty), w01 = (1.f - tx) * ty, w11 = tx * ty;
    uint32_t h4[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      h4[q] = hash3(static_cast<uint32_t>(x16 + 4 * q), static_cast<uint32_t>(y), fc.ss ^ (fc.f * 2654435761u));
    uint32_t out[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint32_t w = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int k = 4 * q + b, x = x16 + k;
        float lum = t0[k] * w00 + t0[k + 1] * w10 + t1[k] * w01 + t1[k + 1] * w11 +
                    20.f * __sinf(0.01f * (x + y) + 0.03f * fc.f);
#pragma unroll
        for (int o = 0; o < 3; ++o) {
          int lx = x - fc.obx[o], ly = y - fc.oby[o];
          lx = lx < 0 ? lx + g.width : lx;  // wrap-around
          ly = ly < 0 ? ly + g.height : ly;
          if (lx < g.ow[o] && ly < g.oh[o])
            lum = a.tiles[(static_cast<size_t>(fc.slot) * 3 + o) * a.tile_stride + static_cast<size_t>(ly) * g.ow[o] + lx];
        }
        int v = static_cast<int>(lum + 0.5f) + noise5(h4[q], b);
        v = v < 0 ? 0 : (v > 255 ? 255 : v);
        w |= static_cast<uint32_t>(v) << (8 * b);
      }
      out[q] = w;
    }
    uint8_t* dst = a.y + (static_cast<size_t>(fz) * g.height + y) * g.width + x16;
    if (x16 + 16 <= g.width && (reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
      *reinterpret_cast<uint4*>(dst) = make_uint4(out[0], out[1], out[2], out[3]);
    } else {
      for (int k = 0; k < 16 && x16 + k < g.width; ++k) dst[k] = static_cast<uint8_t>(out[k >> 2] >> (8 * (k & 3)));
    }
  }
}

__global__ __launch_bounds__(256) void synth_frame_chroma(FrameArgs a) {
  const SynthGeom& g = a.g;
  const int w2 = g.width / 2, h2 = g.height / 2, ccw = g.cw / 2, cch = g.ch / 2;
  const int runs = (w2 + 15) >> 4;
  const long long total = static_cast<long long>(g.slots) * g.frames * h2 * runs;
  for (long long i = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += static_cast<long long>(gridDim.x) * blockDim.x) {
    const int fz = static_cast<int>(i / (static_cast<long long>(h2) * runs));
    const int rem = static_cast<int>(i - static_cast<long long>(fz) * h2 * runs);
    const int y = rem / runs, x16 = (rem - y * runs) * 16;
    FrameConst fc = frame_const(g, fz);
    const float vx = ((hash3(fc.ss, 1, 0) & 255) / 255.f - 0.5f) * 3.f;
    const float vy = ((hash3(fc.ss, 2, 0) & 255) / 255.f - 0.5f) * 1.5f;
    const int ix = static_cast<int>(floorf(vx * fc.f)), iy = static_cast<int>(floorf(vy * fc.f));
    int cyy = (y + iy) % cch;
    cyy = cyy < 0 ? cyy + cch : cyy;
    const size_t rowo = (static_cast<size_t>(fc.slot) * cch + cyy) * ccw;
#pragma unroll
    for (int o = 0; o < 3; ++o) {
      fc.obx[o] >>= 1;
      fc.oby[o] >>= 1;
    }
    const float cv_row = 10.f * __cosf(0.02f * y);
    uint32_t ou[4], ov[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint32_t wu = 0, wv = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int x = x16 + 4 * q + b;
        int cxx = (x + ix) % ccw;
        cxx = cxx < 0 ? cxx + ccw : cxx;
        int cu = a.cu[rowo + cxx] + static_cast<int>(10.f * __sinf(0.02f * x));
        int cv = a.cv[rowo + cxx] + static_cast<int>(cv_row);
#pragma unroll
        for (int o = 0; o < 3; ++o) {
          int lx = x - fc.obx[o], ly = y - fc.oby[o];
          lx = lx < 0 ? lx + w2 : lx;
          ly = ly < 0 ? ly + h2 : ly;
          if (lx < g.ow[o] / 2 && ly < g.oh[o] / 2) {
            cu = 90 + 50 * o;
            cv = 170 - 40 * o;
          }
        }
        wu |= static_cast<uint32_t>(clampi(cu, 0, 255)) << (8 * b);
        wv |= static_cast<uint32_t>(clampi(cv, 0, 255)) << (8 * b);
      }
      ou[q] = wu;
      ov[q] = wv;
    }
    const size_t idx = (static_cast<size_t>(fz) * h2 + y) * w2 + x16;
    if (x16 + 16 <= w2 && ((reinterpret_cast<uintptr_t>(a.u + idx) | reinterpret_cast<uintptr_t>(a.v + idx)) & 15) == 0) {
      *reinterpret_cast<uint4*>(a.u + idx) = make_uint4(ou[0], ou[1], ou[2], ou[3]);
      *reinterpret_cast<uint4*>(a.v + idx) = make_uint4(ov[0], ov[1], ov[2], ov[3]);
    } else {
      for (int k = 0; k < 16 && x16 + k < w2; ++k) {
        a.u[idx + k] = static_cast<uint8_t>(ou[k >> 2] >> (8 * (k & 3)));
        a.v[idx + k] = static_cast<uint8_t>(ov[k >> 2] >> (8 * (k & 3)));
      }
    }
  }
}

}  // namespace gpu
}  // namespace mivc

using namespace mivc::gpu;

extern "C" void mivc_launch_synth(uint8_t* y, uint8_t* u, uint8_t* v, int width, int height, int slots, int frames,
                                  int frame0, uint32_t seed, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  SynthGeom g{};
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
  const size_t ysz = static_cast<size_t>(g.cw) * g.ch, csz = ysz / 4;
  const size_t bytes = slots * (ysz + 2 * csz + 3 * tile_stride);
  uint8_t* ws = nullptr;
  if (hipMallocAsync(reinterpret_cast<void**>(&ws), bytes, s) != hipSuccess) return;
  uint8_t* cy = ws;
  uint8_t* cu = cy + slots * ysz;
  uint8_t* cv = cu + slots * csz;
  uint8_t* tiles = cv + slots * csz;
  hipLaunchKernelGGL(synth_canvas, dim3((g.cw / 4 + 255) / 256, g.ch, slots), dim3(256), 0, s, g, cy, cu, cv);
  int omw = std::max(g.ow[0], std::max(g.ow[1], g.ow[2])), omh = std::max(g.oh[0], std::max(g.oh[1], g.oh[2]));
  hipLaunchKernelGGL(synth_objects, dim3((omw + 255) / 256, omh, slots * 3), dim3(256), 0, s, g, tiles, tile_stride);
  FrameArgs fa{g, cy, cu, cv, tiles, tile_stride, y, u, v};
  // grid-stride over 16-pixel runs: 32 workgroups per CU (256 CUs) at most
  auto grid = [](long long units) {
    const long long g = (units + 255) / 256;
    return dim3(static_cast<unsigned>(g < 8192 ? (g > 0 ? g : 1) : 8192));
  };
  const long long fr = static_cast<long long>(slots) * frames;
  hipLaunchKernelGGL(synth_frame_luma, grid(fr * height * ((width + 15) / 16)), dim3(256), 0, s, fa);
  hipLaunchKernelGGL(synth_frame_chroma, grid(fr * (height / 2) * ((width / 2 + 15) / 16)), dim3(256), 0, s, fa);
  hipFreeAsync(ws, s);
}
