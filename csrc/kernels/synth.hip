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
// at integer positions, one sine and one hash per pixel.  Four pixels per thread,
// one dword store each.
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

__global__ void synth_frame_luma(FrameArgs a) {
  const SynthGeom& g = a.g;
  const int x4 = (blockIdx.x * blockDim.x + threadIdx.x) * 4, y = blockIdx.y, fz = blockIdx.z;
  if (x4 >= g.width) return;
  const int slot = fz / g.frames, f = fz % g.frames + g.frame0;
  const uint32_t ss = slot_seed(g, slot);
  // per-slot global motion (pan) in pixels/frame, sub-pixel
  const float vx = ((hash3(ss, 1, 0) & 255) / 255.f - 0.5f) * 6.f;
  const float vy = ((hash3(ss, 2, 0) & 255) / 255.f - 0.5f) * 3.f;
  const float fx = vx * f, fy = vy * f;
  const float ix = floorf(fx), iy = floorf(fy);
  const float tx = fx - ix, ty = fy - iy;
  int cy0 = (y + static_cast<int>(iy)) % g.ch;
  cy0 = cy0 < 0 ? cy0 + g.ch : cy0;
  const int cy1 = cy0 + 1 == g.ch ? 0 : cy0 + 1;
  const uint8_t* r0 = a.cy + (static_cast<size_t>(slot) * g.ch + cy0) * g.cw;
  const uint8_t* r1 = a.cy + (static_cast<size_t>(slot) * g.ch + cy1) * g.cw;
  int obx[3], oby[3];
#pragma unroll
  for (int o = 0; o < 3; ++o) object_pos(g, slot, o, f, g.width, g.height, g.ow[o], g.oh[o], 1.f, &obx[o], &oby[o]);
  uint32_t w = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int x = x4 + k;
    int cx0 = (x + static_cast<int>(ix)) % g.cw;
    cx0 = cx0 < 0 ? cx0 + g.cw : cx0;
    const int cx1 = cx0 + 1 == g.cw ? 0 : cx0 + 1;
    float top = r0[cx0] * (1.f - tx) + r0[cx1] * tx, bot = r1[cx0] * (1.f - tx) + r1[cx1] * tx;
    float lum = top * (1.f - ty) + bot * ty + 20.f * __sinf(0.01f * (x + y) + 0.03f * f);
#pragma unroll
    for (int o = 0; o < 3; ++o) {
      int lx = x - obx[o], ly = y - oby[o];
      lx = lx < 0 ? lx + g.width : lx;  // wrap-around
      ly = ly < 0 ? ly + g.height : ly;
      if (lx < g.ow[o] && ly < g.oh[o])
        lum = a.tiles[(static_cast<size_t>(slot) * 3 + o) * a.tile_stride + static_cast<size_t>(ly) * g.ow[o] + lx];
    }
    const int n = static_cast<int>(hash3(static_cast<uint32_t>(x), static_cast<uint32_t>(y), ss ^ (f * 2654435761u)) % 5u) - 2;
    int v = static_cast<int>(lum + 0.5f) + n;
    v = v < 0 ? 0 : (v > 255 ? 255 : v);
    w |= static_cast<uint32_t>(v) << (8 * k);
  }
  uint8_t* dst = a.y + (static_cast<size_t>(fz) * g.height + y) * g.width + x4;
  if (x4 + 4 <= g.width && (reinterpret_cast<uintptr_t>(dst) & 3) == 0) {
    *reinterpret_cast<uint32_t*>(dst) = w;
  } else {
    for (int k = 0; k < 4 && x4 + k < g.width; ++k) dst[k] = static_cast<uint8_t>(w >> (8 * k));
  }
}

__global__ void synth_frame_chroma(FrameArgs a) {
  const SynthGeom& g = a.g;
  const int w2 = g.width / 2, h2 = g.height / 2, ccw = g.cw / 2, cch = g.ch / 2;
  const int x4 = (blockIdx.x * blockDim.x + threadIdx.x) * 4, y = blockIdx.y, fz = blockIdx.z;
  if (x4 >= w2) return;
  const int slot = fz / g.frames, f = fz % g.frames + g.frame0;
  const uint32_t ss = slot_seed(g, slot);
  const float vx = ((hash3(ss, 1, 0) & 255) / 255.f - 0.5f) * 3.f;
  const float vy = ((hash3(ss, 2, 0) & 255) / 255.f - 0.5f) * 1.5f;
  const int ix = static_cast<int>(floorf(vx * f)), iy = static_cast<int>(floorf(vy * f));
  int cyy = (y + iy) % cch;
  cyy = cyy < 0 ? cyy + cch : cyy;
  const size_t rowo = (static_cast<size_t>(slot) * cch + cyy) * ccw;
  int obx[3], oby[3];
#pragma unroll
  for (int o = 0; o < 3; ++o) {
    object_pos(g, slot, o, f, g.width, g.height, g.ow[o], g.oh[o], 1.f, &obx[o], &oby[o]);
    obx[o] >>= 1;
    oby[o] >>= 1;
  }
  uint32_t wu = 0, wv = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int x = x4 + k;
    int cxx = (x + ix) % ccw;
    cxx = cxx < 0 ? cxx + ccw : cxx;
    int cu = a.cu[rowo + cxx] + static_cast<int>(10.f * __sinf(0.02f * x));
    int cv = a.cv[rowo + cxx] + static_cast<int>(10.f * __cosf(0.02f * y));
#pragma unroll
    for (int o = 0; o < 3; ++o) {
      int lx = x - obx[o], ly = y - oby[o];
      lx = lx < 0 ? lx + w2 : lx;
      ly = ly < 0 ? ly + h2 : ly;
      if (lx < g.ow[o] / 2 && ly < g.oh[o] / 2) {
        cu = 90 + 50 * o;
        cv = 170 - 40 * o;
      }
    }
    wu |= static_cast<uint32_t>(clampi(cu, 0, 255)) << (8 * k);
    wv |= static_cast<uint32_t>(clampi(cv, 0, 255)) << (8 * k);
  }
  const size_t idx = (static_cast<size_t>(fz) * h2 + y) * w2 + x4;
  if (x4 + 4 <= w2 && ((reinterpret_cast<uintptr_t>(a.u + idx) | reinterpret_cast<uintptr_t>(a.v + idx)) & 3) == 0) {
    *reinterpret_cast<uint32_t*>(a.u + idx) = wu;
    *reinterpret_cast<uint32_t*>(a.v + idx) = wv;
  } else {
    for (int k = 0; k < 4 && x4 + k < w2; ++k) {
      a.u[idx + k] = static_cast<uint8_t>(wu >> (8 * k));
      a.v[idx + k] = static_cast<uint8_t>(wv >> (8 * k));
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
  hipLaunchKernelGGL(synth_frame_luma, dim3((width / 4 + 255) / 256 + 1, height, slots * frames), dim3(256), 0, s, fa);
  hipLaunchKernelGGL(synth_frame_chroma, dim3((width / 8 + 255) / 256 + 1, height / 2, slots * frames), dim3(256), 0, s,
                     fa);
  hipFreeAsync(ws, s);
}
