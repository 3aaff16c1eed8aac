// Synthetic raw-YUV source generator (BASELINE.json: "on synthetic raw-YUV
// input") -- writes frames straight into HBM so no PCIe/disk feed sits in the
// encode loop.
//
// Content model (deterministic in (seed, slot, frame)): a panning value-noise
// texture (global motion), three moving textured objects (local motion with
// occlusion), a slow luminance ramp, and +-2 LSB temporal sensor noise.  It is
// chosen to exercise motion estimation, intra prediction and residual coding the
// way camera content does; random-noise-only frames would make every encoder
// look identical (incompressible).
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

// smooth value noise in [0,1) on a lattice of `cell` pixels
__device__ float value_noise(float x, float y, float cell, uint32_t seed) {
  float fx = x / cell, fy = y / cell;
  float ix = floorf(fx), iy = floorf(fy);
  float tx = fx - ix, ty = fy - iy;
  tx = tx * tx * (3.f - 2.f * tx);
  ty = ty * ty * (3.f - 2.f * ty);
  int xi = static_cast<int>(ix), yi = static_cast<int>(iy);
  auto L = [&](int a, int b) { return (hash3(static_cast<uint32_t>(a), static_cast<uint32_t>(b), seed) >> 8) * (1.0f / 16777216.0f); };
  float v00 = L(xi, yi), v10 = L(xi + 1, yi), v01 = L(xi, yi + 1), v11 = L(xi + 1, yi + 1);
  return (v00 * (1 - tx) + v10 * tx) * (1 - ty) + (v01 * (1 - tx) + v11 * tx) * ty;
}

struct SynthArgs {
  uint8_t* y;   // [B*F, H, W] display-size frames (tightly packed I420 planes, see below)
  uint8_t* u;
  uint8_t* v;
  int width, height;  // display size (even)
  int frames;         // frames per slot
  int slots;
  int frame0;         // index of the first frame (temporal position) for this batch
  uint32_t seed;
};

__global__ void synth_luma(SynthArgs a) {
  int x = blockIdx.x * blockDim.x + threadIdx.x;
  int y = blockIdx.y;
  int fz = blockIdx.z;  // slot * frames + f
  if (x >= a.width) return;
  int slot = fz / a.frames, f = fz % a.frames + a.frame0;
  uint32_t sseed = a.seed * 7919u + static_cast<uint32_t>(slot) * 104729u;
  // per-slot global motion (pan) in pixels/frame
  float vx = ((hash3(sseed, 1, 0) & 255) / 255.f - 0.5f) * 6.f;
  float vy = ((hash3(sseed, 2, 0) & 255) / 255.f - 0.5f) * 3.f;
  float bx = x + vx * f, by = y + vy * f;
  float t = 0.55f * value_noise(bx, by, 48.f, sseed) + 0.30f * value_noise(bx, by, 12.f, sseed + 1) +
            0.15f * value_noise(bx, by, 4.f, sseed + 2);
  float lum = 40.f + 170.f * t + 20.f * __sinf(0.01f * (x + y) + 0.03f * f);
  // three moving objects with their own texture and motion
  for (int o = 0; o < 3; ++o) {
    uint32_t os = hash3(sseed, 10 + o, 0);
    float cx = (os & 1023) / 1023.f * a.width, cy = ((os >> 10) & 1023) / 1023.f * a.height;
    float ovx = (((os >> 20) & 63) / 63.f - 0.5f) * 10.f, ovy = (((os >> 26) & 63) / 63.f - 0.5f) * 6.f;
    float px = cx + ovx * f, py = cy + ovy * f;
    // wrap around the frame
    px = px - floorf(px / a.width) * a.width;
    py = py - floorf(py / a.height) * a.height;
    float rw = a.width * (0.08f + 0.05f * o), rh = a.height * (0.10f + 0.06f * o);
    float dx = fabsf(x - px), dy = fabsf(y - py);
    if (dx < rw && dy < rh) {
      float ox = x - px, oy = y - py;
      lum = 60.f + 150.f * value_noise(ox + 1000.f * o, oy, 6.f + 4.f * o, os);
    }
  }
  // temporal sensor noise (+-2)
  int n = static_cast<int>(hash3(static_cast<uint32_t>(x), static_cast<uint32_t>(y), sseed ^ (f * 2654435761u)) % 5u) - 2;
  int v = static_cast<int>(lum + 0.5f) + n;
  v = v < 0 ? 0 : (v > 255 ? 255 : v);
  a.y[(static_cast<size_t>(fz) * a.height + y) * a.width + x] = static_cast<uint8_t>(v);
}

__global__ void synth_chroma(SynthArgs a) {
  int x = blockIdx.x * blockDim.x + threadIdx.x;
  int y = blockIdx.y;
  int fz = blockIdx.z;
  int w2 = a.width / 2, h2 = a.height / 2;
  if (x >= w2) return;
  int slot = fz / a.frames, f = fz % a.frames + a.frame0;
  uint32_t sseed = a.seed * 7919u + static_cast<uint32_t>(slot) * 104729u;
  float vx = ((hash3(sseed, 1, 0) & 255) / 255.f - 0.5f) * 3.f;
  float vy = ((hash3(sseed, 2, 0) & 255) / 255.f - 0.5f) * 1.5f;
  float bx = x + vx * f, by = y + vy * f;
  float cu = 128.f + 40.f * (value_noise(bx, by, 40.f, sseed + 5) - 0.5f) + 10.f * __sinf(0.02f * x);
  float cv = 128.f + 40.f * (value_noise(bx, by, 56.f, sseed + 6) - 0.5f) + 10.f * __cosf(0.02f * y);
  for (int o = 0; o < 3; ++o) {
    uint32_t os = hash3(sseed, 10 + o, 0);
    float cx = (os & 1023) / 1023.f * w2, cy = ((os >> 10) & 1023) / 1023.f * h2;
    float ovx = (((os >> 20) & 63) / 63.f - 0.5f) * 5.f, ovy = (((os >> 26) & 63) / 63.f - 0.5f) * 3.f;
    float px = cx + ovx * f, py = cy + ovy * f;
    px = px - floorf(px / w2) * w2;
    py = py - floorf(py / h2) * h2;
    float rw = w2 * (0.08f + 0.05f * o), rh = h2 * (0.10f + 0.06f * o);
    if (fabsf(x - px) < rw && fabsf(y - py) < rh) {
      cu = 90.f + 50.f * o;
      cv = 170.f - 40.f * o;
    }
  }
  size_t idx = (static_cast<size_t>(fz) * h2 + y) * w2 + x;
  a.u[idx] = static_cast<uint8_t>(cu < 0 ? 0 : (cu > 255 ? 255 : cu));
  a.v[idx] = static_cast<uint8_t>(cv < 0 ? 0 : (cv > 255 ? 255 : cv));
}

}  // namespace gpu
}  // namespace mivc

using namespace mivc::gpu;

extern "C" void mivc_launch_synth(uint8_t* y, uint8_t* u, uint8_t* v, int width, int height, int slots, int frames,
                                  int frame0, uint32_t seed, void* stream) {
  SynthArgs a{y, u, v, width, height, frames, slots, frame0, seed};
  hipStream_t s = static_cast<hipStream_t>(stream);
  dim3 gl((width + 255) / 256, height, slots * frames);
  hipLaunchKernelGGL(synth_luma, gl, dim3(256), 0, s, a);
  dim3 gc((width / 2 + 255) / 256, height / 2, slots * frames);
  hipLaunchKernelGGL(synth_chroma, gc, dim3(256), 0, s, a);
}
