// Shared device helpers for the C2DSR gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#include "c2dsr.h"  // the C ABI: every C2_API definition is checked against its declaration

#define C2_API extern "C" __attribute__((visibility("default")))

#define C2_CHECK_LAUNCH()                         \
  do {                                            \
    hipError_t e__ = hipGetLastError();           \
    if (e__ != hipSuccess) return (int)e__;       \
  } while (0)

namespace c2 {

constexpr int WAVE = 64;

// Counter-based dropout hash (restated in oracle/c2dsr_oracle.py:keep_mask).  One 32-bit hash per PAIR of
// elements, a 16-bit half for each:
//   h(q)     = lowbias32(lowbias32(lo(q) ^ k0) ^ hi(q) ^ k1),   q = idx >> 1
//   keep(idx) = ((h(q) >> (16 · (idx & 1))) & 0xffff) >= thr,   thr = floor(p · 2^16)
// (p resolved to 2^-16; torch's own Bernoulli draws are float-resolution too).  Stateless, so fwd and bwd
// regenerate the same mask; a float4 of consecutive elements costs two hashes (mul4).
__device__ __forceinline__ uint32_t lowbias32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x7feb352dU;
  h ^= h >> 15;
  h *= 0x846ca68bU;
  h ^= h >> 16;
  return h;
}

__device__ __forceinline__ uint32_t pair_hash(uint64_t q, uint32_t k0, uint32_t k1) {
  const uint32_t h = lowbias32((uint32_t)q ^ k0);
  return lowbias32(h ^ (uint32_t)(q >> 32) ^ k1);
}

struct Drop {
  uint32_t k0, k1, thr;  // thr: 16-bit threshold (1..65535) or 0 = "no dropout"
  float scale;           // 1/(1-p)
  __device__ __forceinline__ bool active() const { return thr != 0; }
  __device__ __forceinline__ float mul(uint64_t idx) const {
    if (thr == 0) return 1.0f;
    const uint32_t h = pair_hash(idx >> 1, k0, k1);
    return ((h >> (16 * (uint32_t)(idx & 1))) & 0xffffu) >= thr ? scale : 0.0f;
  }
  // the multipliers of elements idx .. idx+3 (idx a multiple of 2): two hashes
  __device__ __forceinline__ float4 mul4(uint64_t idx) const {
    if (thr == 0) return make_float4(1.f, 1.f, 1.f, 1.f);
    const uint32_t h0 = pair_hash(idx >> 1, k0, k1), h1 = pair_hash((idx >> 1) + 1, k0, k1);
    return make_float4((h0 & 0xffffu) >= thr ? scale : 0.f, (h0 >> 16) >= thr ? scale : 0.f,
                       (h1 & 0xffffu) >= thr ? scale : 0.f, (h1 >> 16) >= thr ? scale : 0.f);
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
    double t = (double)p * 65536.0;
    d.thr = t >= 65535.0 ? 0xffffu : (uint32_t)t;
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

// 4 consecutive elements of an embedding-table row stored as fp32 (float4 access) or bf16 (8-byte access,
// RNE on store): the C5 roofline run keeps its [N, d] tables in bf16; arithmetic is fp32
typedef __bf16 tbf16;
typedef tbf16 tbf16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ld4(const float* p) { return *(const float4*)p; }
__device__ __forceinline__ float4 ld4(const tbf16* p) {
  const tbf16x4 v = *(const tbf16x4*)p;
  return make_float4((float)v[0], (float)v[1], (float)v[2], (float)v[3]);
}
__device__ __forceinline__ void st4(float* p, float4 v) { *(float4*)p = v; }
__device__ __forceinline__ void st4(tbf16* p, float4 v) {
  tbf16x4 r;
  r[0] = (tbf16)v.x; r[1] = (tbf16)v.y; r[2] = (tbf16)v.z; r[3] = (tbf16)v.w;
  *(tbf16x4*)p = r;
}

// A lane's slice of a table row per step, as fp32 arithmetic: 16 bytes = VW elements (4 fp32 or 8 bf16) → VW/4
// float4 (a 32-byte bf16 slice — two rows per wave — measured 20 % slower in the C5 SpMM)
template <typename T>
constexpr int VW = 16 / (int)sizeof(T);
template <typename T>
struct RowV {
  float4 v[VW<T> / 4];
};
__device__ __forceinline__ RowV<float> ldv(const float* p) { return RowV<float>{{*(const float4*)p}}; }
__device__ __forceinline__ RowV<tbf16> ldv(const tbf16* p) {
  typedef tbf16 tbf16x8 __attribute__((ext_vector_type(8)));
  const tbf16x8 x = *(const tbf16x8*)p;
  return RowV<tbf16>{{make_float4((float)x[0], (float)x[1], (float)x[2], (float)x[3]),
                      make_float4((float)x[4], (float)x[5], (float)x[6], (float)x[7])}};
}
__device__ __forceinline__ void stv(float* p, const RowV<float>& r) { *(float4*)p = r.v[0]; }
__device__ __forceinline__ void stv(tbf16* p, const RowV<tbf16>& r) {
  typedef tbf16 tbf16x8 __attribute__((ext_vector_type(8)));
  tbf16x8 x;
  x[0] = (tbf16)r.v[0].x; x[1] = (tbf16)r.v[0].y; x[2] = (tbf16)r.v[0].z; x[3] = (tbf16)r.v[0].w;
  x[4] = (tbf16)r.v[1].x; x[5] = (tbf16)r.v[1].y; x[6] = (tbf16)r.v[1].z; x[7] = (tbf16)r.v[1].w;
  *(tbf16x8*)p = x;
}

// non-temporal forms (streamed rows touched once per launch: they should not evict re-read rows from L2 / MALL)
typedef float nt_f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ RowV<float> ldv_nt(const float* p) {
  const nt_f32x4 v = __builtin_nontemporal_load((const nt_f32x4*)p);
  return RowV<float>{{make_float4(v[0], v[1], v[2], v[3])}};
}
__device__ __forceinline__ RowV<tbf16> ldv_nt(const tbf16* p) {
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  typedef tbf16 tbf16x8 __attribute__((ext_vector_type(8)));
  const tbf16x8 x = __builtin_bit_cast(tbf16x8, __builtin_nontemporal_load((const s16x8*)p));
  return RowV<tbf16>{{make_float4((float)x[0], (float)x[1], (float)x[2], (float)x[3]),
                      make_float4((float)x[4], (float)x[5], (float)x[6], (float)x[7])}};
}
__device__ __forceinline__ void stv_nt(float* p, const RowV<float>& r) {
  const nt_f32x4 v = {r.v[0].x, r.v[0].y, r.v[0].z, r.v[0].w};
  __builtin_nontemporal_store(v, (nt_f32x4*)p);
}
__device__ __forceinline__ void stv_nt(tbf16* p, const RowV<tbf16>& r) {
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  typedef tbf16 tbf16x8 __attribute__((ext_vector_type(8)));
  tbf16x8 x;
  x[0] = (tbf16)r.v[0].x; x[1] = (tbf16)r.v[0].y; x[2] = (tbf16)r.v[0].z; x[3] = (tbf16)r.v[0].w;
  x[4] = (tbf16)r.v[1].x; x[5] = (tbf16)r.v[1].y; x[6] = (tbf16)r.v[1].z; x[7] = (tbf16)r.v[1].w;
  __builtin_nontemporal_store(__builtin_bit_cast(s16x8, x), (s16x8*)p);
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
