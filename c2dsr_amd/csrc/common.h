// Shared device helpers for the C2DSR gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#define C2_API extern "C" __attribute__((visibility("default")))

#define C2_CHECK_LAUNCH()                         \
  do {                                            \
    hipError_t e__ = hipGetLastError();           \
    if (e__ != hipSuccess) return (int)e__;       \
  } while (0)

namespace c2 {

constexpr int WAVE = 64;

// Counter-based dropout hash (restated in oracle/c2dsr_oracle.py:keep_mask).
// keep(idx) = lowbias32(lowbias32(lo(idx) ^ k0) ^ hi(idx) ^ k1) >= thr,
// thr = floor(p * 2^32).  Stateless, so fwd and bwd regenerate the same mask.
__device__ __forceinline__ uint32_t lowbias32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x7feb352dU;
  h ^= h >> 15;
  h *= 0x846ca68bU;
  h ^= h >> 16;
  return h;
}

struct Drop {
  uint32_t k0, k1, thr;
  float scale;  // 1/(1-p); thr == 0 means "no dropout"
  __device__ __forceinline__ bool active() const { return thr != 0; }
  __device__ __forceinline__ float mul(uint64_t idx) const {
    if (thr == 0) return 1.0f;
    uint32_t h = lowbias32((uint32_t)idx ^ k0);
    h = lowbias32(h ^ (uint32_t)(idx >> 32) ^ k1);
    return h >= thr ? scale : 0.0f;
  }
};

inline Drop make_drop(uint32_t k0, uint32_t k1, float p) {
  Drop d;
  d.k0 = k0;
  d.k1 = k1;
  if (p <= 0.0f) {
    d.thr = 0;
    d.scale = 1.0f;
  } else {
    double t = (double)p * 4294967296.0;
    d.thr = t >= 4294967295.0 ? 0xffffffffu : (uint32_t)t;
    if (d.thr == 0) d.thr = 1;  // p so small it rounds to 0: still "active" but keeps ~all
    d.scale = (float)(1.0 / (1.0 - (double)p));
  }
  return d;
}

__device__ __forceinline__ float4 f4(float a) { return make_float4(a, a, a, a); }
__device__ __forceinline__ float4 operator+(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
__device__ __forceinline__ float4 operator*(float4 a, float4 b) { return make_float4(a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w); }
__device__ __forceinline__ float4 operator*(float s, float4 a) { return make_float4(s * a.x, s * a.y, s * a.z, s * a.w); }
__device__ __forceinline__ float4 fma4(float s, float4 a, float4 c) {
  return make_float4(fmaf(s, a.x, c.x), fmaf(s, a.y, c.y), fmaf(s, a.z, c.z), fmaf(s, a.w, c.w));
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
// reduce within aligned groups of G lanes (G power of two <= 64)
template <int G>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

inline int ceil_div(long a, long b) { return (int)((a + b - 1) / b); }

}  // namespace c2
