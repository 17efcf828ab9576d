// K1: item-graph propagation (GCN) — CSR SpMM with fused dropout and fused mean.
//
// Replaces models/encoders.py:42-48 (F.dropout + torch.spmm + stack/mean) as called
// by models/C2DSR.py:59-62, and its autograd backward.
//
//   P[i]  = Σ_e val[e] * (Min ⊙ X)[col[e]]          (mask on the gathered row:  forward)
//   P[i]  = Mout_i ⊙ Σ_e val[e] * X[col[e]]          (mask on the output row:    backward, CSR of Aᵀ)
//   Y[i]  = alpha * P[i] + (beta + (i != pad_row ? delta : 0)) * Z[i] + gamma * Y[i]
//   Y2[i] = P[i]   (optional: the next GCN layer's input)
//
// Load balance: item popularity is Zipf-like, so a few rows hold a large share of
// the edges.  The host splits every row into pieces of at most SPLIT edges (a
// static "work" list built once per graph, c2dsr_amd/graph.py); a piece of an
// unsplit row runs the full epilogue, pieces of split rows write raw partial sums
// to a scratch slab that a second pass adds up in piece order (deterministic).
// One work item per group of LPR lanes, float4 per lane (d <= 4*LPR per pass).
#include "common.h"

namespace {

struct Epi {
  float alpha;
  const float* Z;
  float beta, delta;
  int pad_row;
  float gamma;
  float* Y;
  float* Y2;
  c2::Drop drop;
};

template <bool MASK_OUT>
__device__ __forceinline__ void epilogue(float4 acc, long row, int c, int d, const Epi& ep) {
  if (MASK_OUT && ep.drop.active()) {
    const uint64_t b = (uint64_t)row * d + c;
    acc = acc * ep.drop.mul4(b);
  }
  if (ep.Y2) *(float4*)(ep.Y2 + row * d + c) = acc;
  float4 y = ep.alpha * acc;
  if (ep.Z) {
    const float zc = ep.beta + (row != ep.pad_row ? ep.delta : 0.f);
    y = c2::fma4(zc, *(const float4*)(ep.Z + row * d + c), y);
  }
  if (ep.gamma != 0.f) y = c2::fma4(ep.gamma, *(const float4*)(ep.Y + row * d + c), y);
  *(float4*)(ep.Y + row * d + c) = y;
}

// work[w] = {row, e_begin, e_end, slot}; slot < 0: whole row (epilogue), else partial slab index.
template <int LPR, bool MASK_OUT>
__global__ __launch_bounds__(256) void spmm_kernel(const int4* __restrict__ work, int n_work,
                                                   const int* __restrict__ col, const float* __restrict__ val, int d,
                                                   const float* __restrict__ X, Epi ep, float* __restrict__ part) {
  constexpr int GROUPS = 256 / LPR;
  const int g = threadIdx.x / LPR;
  const int lane = threadIdx.x % LPR;
  const long w = (long)blockIdx.x * GROUPS + g;
  if (w >= n_work) return;
  const int4 wk = work[w];
  const long row = wk.x;
  const int e0 = wk.y, e1 = wk.z, slot = wk.w;
  const c2::Drop& drop = ep.drop;
  for (int c = lane * 4; c < d; c += LPR * 4) {
    float4 acc = c2::f4(0.f);
    int e = e0;
    for (; e + 3 < e1; e += 4) {
      const int j0 = col[e], j1 = col[e + 1], j2 = col[e + 2], j3 = col[e + 3];
      const float v0 = val[e], v1 = val[e + 1], v2 = val[e + 2], v3 = val[e + 3];
      float4 x0 = *(const float4*)(X + (long)j0 * d + c);
      float4 x1 = *(const float4*)(X + (long)j1 * d + c);
      float4 x2 = *(const float4*)(X + (long)j2 * d + c);
      float4 x3 = *(const float4*)(X + (long)j3 * d + c);
      if (!MASK_OUT && drop.active()) {
        const uint64_t b0 = (uint64_t)j0 * d + c, b1 = (uint64_t)j1 * d + c;
        const uint64_t b2 = (uint64_t)j2 * d + c, b3 = (uint64_t)j3 * d + c;
        x0 = x0 * drop.mul4(b0);
        x1 = x1 * drop.mul4(b1);
        x2 = x2 * drop.mul4(b2);
        x3 = x3 * drop.mul4(b3);
      }
      acc = c2::fma4(v0, x0, acc);
      acc = c2::fma4(v1, x1, acc);
      acc = c2::fma4(v2, x2, acc);
      acc = c2::fma4(v3, x3, acc);
    }
    for (; e < e1; ++e) {
      const int j = col[e];
      float4 x = *(const float4*)(X + (long)j * d + c);
      if (!MASK_OUT && drop.active()) {
        const uint64_t b = (uint64_t)j * d + c;
        x = x * drop.mul4(b);
      }
      acc = c2::fma4(val[e], x, acc);
    }
    if (slot >= 0)
      *(float4*)(part + (long)slot * d + c) = acc;
    else
      epilogue<MASK_OUT>(acc, row, c, d, ep);
  }
}

#ifndef COMBINE_U
#define COMBINE_U 16
#endif

// split[s] = {row, slot_begin, slot_end}: sum the row's pieces in order, then the epilogue.
template <int LPR, bool MASK_OUT>
__global__ __launch_bounds__(256) void combine_kernel(const int4* __restrict__ split, int n_split, int d, Epi ep,
                                                      const float* __restrict__ part) {
  constexpr int GROUPS = 256 / LPR;
  const int g = threadIdx.x / LPR;
  const int lane = threadIdx.x % LPR;
  const long s = (long)blockIdx.x * GROUPS + g;
  if (s >= n_split) return;
  const int4 sp = split[s];
  for (int c = lane * 4; c < d; c += LPR * 4) {
    float4 acc = c2::f4(0.f);
    int k = sp.y;
    // A hub row's combine is a latency chain (up to ~200 pieces at bench sizes): COMBINE_U pieces' loads in
    // flight per round trip, then eight, added in piece order either way.
    for (; k + COMBINE_U <= sp.z; k += COMBINE_U) {
      float4 v[COMBINE_U];
#pragma unroll
      for (int u = 0; u < COMBINE_U; ++u) v[u] = *(const float4*)(part + (long)(k + u) * d + c);
#pragma unroll
      for (int u = 0; u < COMBINE_U; ++u) acc = acc + v[u];
    }
    for (; k + 8 <= sp.z; k += 8) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = *(const float4*)(part + (long)(k + u) * d + c);
#pragma unroll
      for (int u = 0; u < 8; ++u) acc = acc + v[u];
    }
    for (; k < sp.z; ++k) acc = acc + *(const float4*)(part + (long)k * d + c);
    epilogue<MASK_OUT>(acc, sp.x, c, d, ep);
  }
}

int lpr_for(int d) { return d / 4 >= 64 ? 64 : (d / 4 >= 32 ? 32 : (d / 4 >= 16 ? 16 : (d / 4 >= 8 ? 8 : 4))); }

template <bool MASK_OUT>
int launch(const int4* work, int n_work, const int4* split, int n_split, const int* col, const float* val, int d,
           const float* X, const Epi& ep, float* part, hipStream_t s) {
  const int lpr = lpr_for(d);
  const int groups = 256 / lpr;
#define C2_SPMM(L)                                                                                              \
  spmm_kernel<L, MASK_OUT><<<c2::ceil_div(n_work, groups), 256, 0, s>>>(work, n_work, col, val, d, X, ep, part); \
  if (n_split > 0) combine_kernel<L, MASK_OUT><<<c2::ceil_div(n_split, groups), 256, 0, s>>>(split, n_split, d, ep, part);
  switch (lpr) {
    case 64: C2_SPMM(64) break;
    case 32: C2_SPMM(32) break;
    case 16: C2_SPMM(16) break;
    case 8: C2_SPMM(8) break;
    default: C2_SPMM(4) break;
  }
#undef C2_SPMM
  C2_CHECK_LAUNCH();
  return 0;
}

}  // namespace

C2_API int c2dsr_gcn_spmm(const int* work, int n_work, const int* split, int n_split, float* part, const int* col,
                          const float* val, int d, const float* X, uint32_t k0, uint32_t k1, float p,
                          int mask_on_output, float alpha, const float* Z, float beta, float delta, int pad_row,
                          float gamma, float* Y, float* Y2, void* stream) {
  if (d % 4) return (int)hipErrorInvalidValue;
  if (n_work == 0) return 0;
  Epi ep{alpha, Z, beta, delta, pad_row, gamma, Y, Y2, c2::make_drop(k0, k1, p)};
  hipStream_t s = (hipStream_t)stream;
  if (mask_on_output)
    return launch<true>((const int4*)work, n_work, (const int4*)split, n_split, col, val, d, X, ep, part, s);
  return launch<false>((const int4*)work, n_work, (const int4*)split, n_split, col, val, d, X, ep, part, s);
}
