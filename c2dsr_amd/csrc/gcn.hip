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
// One work item per group of LPR lanes, 4 elements per lane (d <= 4*LPR per pass).  Tables (X, Z, Y, Y2) are
// fp32, or bf16 for the C5 roofline run (c2dsr_gcn_spmm_b16: SURVEY.md §8(d); fp32 arithmetic, RNE stores).
#include "common.h"

#include <type_traits>

// GCN_NT 1: the epilogue's row streams (Z, the accumulated Y, the Y / Y2 stores) bypass the caches' normal
// retention, leaving L2 / MALL to the gathered rows X[col] (Zipf-popular rows are re-read)
#ifndef GCN_NT
#define GCN_NT 1
#endif

// edges' rows in flight per lane group in the whole-batch loop: 4 for fp32 rows, 2 for bf16 rows (C5 bf16 tables
// 4934 → 5387 GB/s; MB fp32 at 2: fwd 99.6 → 104.0 µs, bwd 60.7 → 71.3 µs; 8: slower for both)
#ifndef GCN_UE
#define GCN_UE 4
#endif
#ifndef GCN_UE_B16
#define GCN_UE_B16 2
#endif

namespace {

template <typename T>
__device__ __forceinline__ c2::RowV<T> ld_stream(const T* p) {
  if constexpr (GCN_NT) return c2::ldv_nt(p);
  else return c2::ldv(p);
}
template <typename T>
__device__ __forceinline__ void st_stream(T* p, const c2::RowV<T>& r) {
  if constexpr (GCN_NT) c2::stv_nt(p, r);
  else c2::stv(p, r);
}

template <typename T>
struct Epi {
  float alpha;
  const T* Z;
  float beta, delta;
  int pad_row;
  float gamma;
  T* Y;
  T* Y2;
  c2::Drop drop;
};

template <bool MASK_OUT, typename T>
__device__ __forceinline__ void epilogue(c2::RowV<T> acc, long row, int c, int d, const Epi<T>& ep) {
  constexpr int NH = c2::VW<T> / 4;
  if (MASK_OUT && ep.drop.active()) {
#pragma unroll
    for (int h = 0; h < NH; ++h) acc.v[h] = acc.v[h] * ep.drop.mul4((uint64_t)row * d + c + 4 * h);
  }
  if (ep.Y2) st_stream(ep.Y2 + row * d + c, acc);
  c2::RowV<T> y;
#pragma unroll
  for (int h = 0; h < NH; ++h) y.v[h] = ep.alpha * acc.v[h];
  if (ep.Z) {
    const float zc = ep.beta + (row != ep.pad_row ? ep.delta : 0.f);
    const c2::RowV<T> z = ld_stream(ep.Z + row * d + c);
#pragma unroll
    for (int h = 0; h < NH; ++h) y.v[h] = c2::fma4(zc, z.v[h], y.v[h]);
  }
  if (ep.gamma != 0.f) {
    const c2::RowV<T> o = ld_stream(ep.Y + row * d + c);
#pragma unroll
    for (int h = 0; h < NH; ++h) y.v[h] = c2::fma4(ep.gamma, o.v[h], y.v[h]);
  }
  st_stream(ep.Y + row * d + c, y);
}

// work[w] = {row, e_begin, e_end, slot}; slot < 0: whole row (epilogue), else partial slab index.
// A lane handles 16 bytes of a table row per step (4 fp32 or 8 bf16 elements).
template <int LPR, bool MASK_OUT, typename T>
__global__ __launch_bounds__(256) void spmm_kernel(const int4* __restrict__ work, int n_work,
                                                   const int* __restrict__ col, const float* __restrict__ val, int d,
                                                   const T* __restrict__ X, Epi<T> ep, float* __restrict__ part) {
  constexpr int GROUPS = 256 / LPR;
  constexpr int V = c2::VW<T>, NH = V / 4;
  const int g = threadIdx.x / LPR;
  const int lane = threadIdx.x % LPR;
  const long w = (long)blockIdx.x * GROUPS + g;
  if (w >= n_work) return;
  const int4 wk = work[w];
  const long row = wk.x;
  const int e0 = wk.y, e1 = wk.z, slot = wk.w;
  const c2::Drop& drop = ep.drop;
  for (int c = lane * V; c < d; c += LPR * V) {
    c2::RowV<T> acc;
#pragma unroll
    for (int h = 0; h < NH; ++h) acc.v[h] = c2::f4(0.f);
    int e = e0;
    // UE rows in flight per lane group (most rows of a Zipf item graph have one or two edges: deeper batches only
    // push edges into the one-at-a-time tail)
    constexpr int UE = sizeof(T) == 2 ? GCN_UE_B16 : GCN_UE;
    for (; e + UE - 1 < e1; e += UE) {
      int j[UE];
      float vv[UE];
#pragma unroll
      for (int u = 0; u < UE; ++u) {
        j[u] = col[e + u];
        vv[u] = val[e + u];
      }
      c2::RowV<T> x[UE];
#pragma unroll
      for (int u = 0; u < UE; ++u) x[u] = c2::ldv(X + (long)j[u] * d + c);
      if (!MASK_OUT && drop.active()) {
#pragma unroll
        for (int u = 0; u < UE; ++u)
#pragma unroll
          for (int h = 0; h < NH; ++h) x[u].v[h] = x[u].v[h] * drop.mul4((uint64_t)j[u] * d + c + 4 * h);
      }
#pragma unroll
      for (int h = 0; h < NH; ++h)
#pragma unroll
        for (int u = 0; u < UE; ++u) acc.v[h] = c2::fma4(vv[u], x[u].v[h], acc.v[h]);
    }
    for (; e < e1; ++e) {
      const int j = col[e];
      c2::RowV<T> x = c2::ldv(X + (long)j * d + c);
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        if (!MASK_OUT && drop.active()) x.v[h] = x.v[h] * drop.mul4((uint64_t)j * d + c + 4 * h);
        acc.v[h] = c2::fma4(val[e], x.v[h], acc.v[h]);
      }
    }
    if (slot >= 0) {
#pragma unroll
      for (int h = 0; h < NH; ++h) *(float4*)(part + (long)slot * d + c + 4 * h) = acc.v[h];
    } else {
      epilogue<MASK_OUT>(acc, row, c, d, ep);
    }
  }
}

// The same with NC 16-byte slices of the row per lane, loaded together (d == LPR·VW·NC): every edge's whole row
// is in flight at once instead of one slice per pass over the edges — and with LPR = 32 two work items share a
// wave.  Same accumulation order per element as spmm_kernel (edges in order).
template <int LPR, int NC, bool MASK_OUT, typename T>
__global__ __launch_bounds__(256) void spmm_nc_kernel(const int4* __restrict__ work, int n_work,
                                                      const int* __restrict__ col, const float* __restrict__ val,
                                                      int d, const T* __restrict__ X, Epi<T> ep,
                                                      float* __restrict__ part) {
  constexpr int GROUPS = 256 / LPR;
  constexpr int V = c2::VW<T>, NH = V / 4;
  constexpr int UE = NC >= 2 ? 2 : 4;  // row slices in flight per lane: UE·NC
  const int g = threadIdx.x / LPR;
  const int lane = threadIdx.x % LPR;
  const long w = (long)blockIdx.x * GROUPS + g;
  if (w >= n_work) return;
  const int4 wk = work[w];
  const long row = wk.x;
  const int e0 = wk.y, e1 = wk.z, slot = wk.w;
  const c2::Drop& drop = ep.drop;
  c2::RowV<T> acc[NC];
#pragma unroll
  for (int k = 0; k < NC; ++k)
#pragma unroll
    for (int h = 0; h < NH; ++h) acc[k].v[h] = c2::f4(0.f);
  auto cof = [&](int k) { return lane * V + k * LPR * V; };
  int e = e0;
  for (; e + UE - 1 < e1; e += UE) {
    int j[UE];
    float vv[UE];
#pragma unroll
    for (int u = 0; u < UE; ++u) {
      j[u] = col[e + u];
      vv[u] = val[e + u];
    }
    c2::RowV<T> x[UE][NC];
#pragma unroll
    for (int u = 0; u < UE; ++u)
#pragma unroll
      for (int k = 0; k < NC; ++k) x[u][k] = c2::ldv(X + (long)j[u] * d + cof(k));
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      if (!MASK_OUT && drop.active()) {
#pragma unroll
        for (int u = 0; u < UE; ++u)
#pragma unroll
          for (int h = 0; h < NH; ++h) x[u][k].v[h] = x[u][k].v[h] * drop.mul4((uint64_t)j[u] * d + cof(k) + 4 * h);
      }
#pragma unroll
      for (int h = 0; h < NH; ++h)
#pragma unroll
        for (int u = 0; u < UE; ++u) acc[k].v[h] = c2::fma4(vv[u], x[u][k].v[h], acc[k].v[h]);
    }
  }
  for (; e < e1; ++e) {
    const int j = col[e];
    const float v = val[e];
    c2::RowV<T> x[NC];
#pragma unroll
    for (int k = 0; k < NC; ++k) x[k] = c2::ldv(X + (long)j * d + cof(k));
#pragma unroll
    for (int k = 0; k < NC; ++k)
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        if (!MASK_OUT && drop.active()) x[k].v[h] = x[k].v[h] * drop.mul4((uint64_t)j * d + cof(k) + 4 * h);
        acc[k].v[h] = c2::fma4(v, x[k].v[h], acc[k].v[h]);
      }
  }
#pragma unroll
  for (int k = 0; k < NC; ++k) {
    if (slot >= 0) {
#pragma unroll
      for (int h = 0; h < NH; ++h) *(float4*)(part + (long)slot * d + cof(k) + 4 * h) = acc[k].v[h];
    } else {
      epilogue<MASK_OUT>(acc[k], row, cof(k), d, ep);
    }
  }
}

// One-pass rows (d == LPR·VW: the C5 bf16 width) with ITEMS consecutive work items per lane group: every item's
// header and its first two edges' (col, val) are loaded up front, so per item only the row gathers and the epilogue
// streams remain on the dependent-latency chain (work → col → X in spmm_kernel).  Same per-element accumulation
// order (edges in order, one fma each), so bit-identical to spmm_kernel.
template <int LPR, int ITEMS, bool MASK_OUT, typename T>
__global__ __launch_bounds__(256) void spmm_pf_kernel(const int4* __restrict__ work, int n_work,
                                                      const int* __restrict__ col, const float* __restrict__ val,
                                                      int d, const T* __restrict__ X, Epi<T> ep,
                                                      float* __restrict__ part) {
  constexpr int GROUPS = 256 / LPR;
  constexpr int V = c2::VW<T>, NH = V / 4;
  const int g = threadIdx.x / LPR;
  const int c = (threadIdx.x % LPR) * V;
  const long w0 = ((long)blockIdx.x * GROUPS + g) * ITEMS;
  if (w0 >= n_work) return;
  const c2::Drop& drop = ep.drop;
  int4 wk[ITEMS];
#pragma unroll
  for (int i = 0; i < ITEMS; ++i) wk[i] = w0 + i < n_work ? work[w0 + i] : make_int4(0, 0, 0, -2);
  int j0[ITEMS], j1[ITEMS];
  float v0[ITEMS], v1[ITEMS];
#pragma unroll
  for (int i = 0; i < ITEMS; ++i) {
    const int e0 = wk[i].y, e1 = wk[i].z;
    j0[i] = e0 < e1 ? col[e0] : 0;
    v0[i] = e0 < e1 ? val[e0] : 0.f;
    j1[i] = e0 + 1 < e1 ? col[e0 + 1] : 0;
    v1[i] = e0 + 1 < e1 ? val[e0 + 1] : 0.f;
  }
  auto mask = [&](c2::RowV<T>& x, int j) {
    if (!MASK_OUT && drop.active()) {
#pragma unroll
      for (int h = 0; h < NH; ++h) x.v[h] = x.v[h] * drop.mul4((uint64_t)j * d + c + 4 * h);
    }
  };
#pragma unroll
  for (int i = 0; i < ITEMS; ++i) {
    const int e0 = wk[i].y, e1 = wk[i].z, slot = wk[i].w;
    if (slot == -2) break;
    c2::RowV<T> acc;
#pragma unroll
    for (int h = 0; h < NH; ++h) acc.v[h] = c2::f4(0.f);
    if (e0 + 1 < e1) {
      c2::RowV<T> x0 = c2::ldv(X + (long)j0[i] * d + c), x1 = c2::ldv(X + (long)j1[i] * d + c);
      mask(x0, j0[i]);
      mask(x1, j1[i]);
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        acc.v[h] = c2::fma4(v0[i], x0.v[h], acc.v[h]);
        acc.v[h] = c2::fma4(v1[i], x1.v[h], acc.v[h]);
      }
    } else if (e0 < e1) {
      c2::RowV<T> x0 = c2::ldv(X + (long)j0[i] * d + c);
      mask(x0, j0[i]);
#pragma unroll
      for (int h = 0; h < NH; ++h) acc.v[h] = c2::fma4(v0[i], x0.v[h], acc.v[h]);
    }
    int e = e0 + 2;
    for (; e + 1 < e1; e += 2) {
      const int ja = col[e], jb = col[e + 1];
      const float va = val[e], vb = val[e + 1];
      c2::RowV<T> xa = c2::ldv(X + (long)ja * d + c), xb = c2::ldv(X + (long)jb * d + c);
      mask(xa, ja);
      mask(xb, jb);
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        acc.v[h] = c2::fma4(va, xa.v[h], acc.v[h]);
        acc.v[h] = c2::fma4(vb, xb.v[h], acc.v[h]);
      }
    }
    for (; e < e1; ++e) {
      const int j = col[e];
      c2::RowV<T> x = c2::ldv(X + (long)j * d + c);
      mask(x, j);
#pragma unroll
      for (int h = 0; h < NH; ++h) acc.v[h] = c2::fma4(val[e], x.v[h], acc.v[h]);
    }
    if (slot >= 0) {
#pragma unroll
      for (int h = 0; h < NH; ++h) *(float4*)(part + (long)slot * d + c + 4 * h) = acc.v[h];
    } else {
      epilogue<MASK_OUT>(acc, wk[i].x, c, d, ep);
    }
  }
}

#ifndef COMBINE_U
#define COMBINE_U 16
#endif
#ifndef COMBINE_HI
#define COMBINE_HI 1
#endif

// split[s] = {row, slot_begin, slot_end}: sum the row's pieces in order, then the epilogue.
template <int LPR, bool MASK_OUT, typename T>
__global__ __launch_bounds__(256) void combine_kernel(const int4* __restrict__ split, int n_split, int d, Epi<T> ep,
                                                      const float* __restrict__ part) {
  constexpr int GROUPS = 256 / LPR;
  constexpr int V = c2::VW<T>, NH = V / 4;
  const int g = threadIdx.x / LPR;
  const int lane = threadIdx.x % LPR;
  const long s = (long)blockIdx.x * GROUPS + g;
  if (s >= n_split) return;
  const int4 sp = split[s];
  for (int c0 = lane * V; c0 < d; c0 += LPR * V) {
    c2::RowV<T> res;
#if COMBINE_HI
    // all NH float4 slices of the lane's piece rows in flight together (bf16 rows: 2 per piece), each slice still
    // summed in piece order (bit-identical; C5 bf16-table line 5708 → 5807 GB/s, COMBINE_U 32: 5524;
    // profiles/r04_exp30_combine.txt)
#pragma unroll
    for (int h = 0; h < NH; ++h) res.v[h] = c2::f4(0.f);
    int k = sp.y;
    for (; k + COMBINE_U <= sp.z; k += COMBINE_U) {
      float4 v[COMBINE_U][NH];
#pragma unroll
      for (int u = 0; u < COMBINE_U; ++u)
#pragma unroll
        for (int h = 0; h < NH; ++h) v[u][h] = *(const float4*)(part + (long)(k + u) * d + c0 + 4 * h);
#pragma unroll
      for (int u = 0; u < COMBINE_U; ++u)
#pragma unroll
        for (int h = 0; h < NH; ++h) res.v[h] = res.v[h] + v[u][h];
    }
    for (; k + 8 <= sp.z; k += 8) {
      float4 v[8][NH];
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int h = 0; h < NH; ++h) v[u][h] = *(const float4*)(part + (long)(k + u) * d + c0 + 4 * h);
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int h = 0; h < NH; ++h) res.v[h] = res.v[h] + v[u][h];
    }
    for (; k < sp.z; ++k)
#pragma unroll
      for (int h = 0; h < NH; ++h) res.v[h] = res.v[h] + *(const float4*)(part + (long)k * d + c0 + 4 * h);
#else
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      const int c = c0 + 4 * h;
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
      res.v[h] = acc;
    }
#endif
    epilogue<MASK_OUT>(res, sp.x, c0, d, ep);
  }
}

int lpr_for(int d) { return d / 4 >= 64 ? 64 : (d / 4 >= 32 ? 32 : (d / 4 >= 16 ? 16 : (d / 4 >= 8 ? 8 : 4))); }

template <bool MASK_OUT, typename T>
int launch(const int4* work, int n_work, const int4* split, int n_split, const int* col, const float* val, int d,
           const T* X, const Epi<T>& ep, float* part, hipStream_t s) {
  const int lpr = lpr_for(d * 4 / c2::VW<T>);  // lanes per row: VW elements each
  const int groups = 256 / lpr;
#ifndef SPMM_NC
#define SPMM_NC 1
#endif
  // fp32 rows of d = 512: both 16-byte slices of a lane loaded per edge in one pass over the edges (C5 fp32 tables
  // 6838 → 6894 GB/s).  bf16 rows stay one slice per lane, one work item per wave: two work items per wave (32
  // lanes × 2 slices) measured 15.6 → 16.4 ms per launch at C5
  if (SPMM_NC && d == 512 && std::is_same_v<T, float>) {
    constexpr int L = 64;
    spmm_nc_kernel<L, 2, MASK_OUT, T><<<c2::ceil_div(n_work, 256 / L), 256, 0, s>>>(work, n_work, col, val, d, X, ep,
                                                                                  part);
    if (n_split > 0)
      combine_kernel<L, MASK_OUT, T><<<c2::ceil_div(n_split, 256 / L), 256, 0, s>>>(split, n_split, d, ep, part);
    C2_CHECK_LAUNCH();
    return 0;
  }
#ifndef GCN_PF_B16
#define GCN_PF_B16 2
#endif
  // bf16 rows of d = 512 (C5): GCN_PF_B16 work items per wave with their headers and first edges loaded up front
  // (C5 bf16-table line 5350 → 5652 GB/s at 2, 5071 at 4; outputs bit-identical: profiles/r04_exp28_gcn_pf.txt)
  if constexpr (GCN_PF_B16 > 1 && std::is_same_v<T, c2::tbf16>) {
    if (d == 64 * c2::VW<T>) {
      spmm_pf_kernel<64, GCN_PF_B16, MASK_OUT, T><<<c2::ceil_div(n_work, 4 * GCN_PF_B16), 256, 0, s>>>(
          work, n_work, col, val, d, X, ep, part);
      if (n_split > 0)
        combine_kernel<64, MASK_OUT, T><<<c2::ceil_div(n_split, 4), 256, 0, s>>>(split, n_split, d, ep, part);
      C2_CHECK_LAUNCH();
      return 0;
    }
  }
#ifndef GCN_PF_F32
#define GCN_PF_F32 1
#endif
  // the same for fp32 rows of d = 256 (the bench's Movie-Book width): measured and not kept — MB fwd 100.7 → 117.0 µs
  // at 2, 152 µs at 4; bwd 61.8 → 79.6 / 108 µs (profiles/r04_exp29_gcn_pf_f32.txt)
  if constexpr (GCN_PF_F32 > 1 && std::is_same_v<T, float>) {
    if (d == 64 * c2::VW<T>) {
      spmm_pf_kernel<64, GCN_PF_F32, MASK_OUT, T><<<c2::ceil_div(n_work, 4 * GCN_PF_F32), 256, 0, s>>>(
          work, n_work, col, val, d, X, ep, part);
      if (n_split > 0)
        combine_kernel<64, MASK_OUT, T><<<c2::ceil_div(n_split, 4), 256, 0, s>>>(split, n_split, d, ep, part);
      C2_CHECK_LAUNCH();
      return 0;
    }
  }
#define C2_SPMM(L)                                                                                       \
  spmm_kernel<L, MASK_OUT, T><<<c2::ceil_div(n_work, groups), 256, 0, s>>>(work, n_work, col, val, d, X, ep, part); \
  if (n_split > 0) combine_kernel<L, MASK_OUT, T><<<c2::ceil_div(n_split, groups), 256, 0, s>>>(split, n_split, d, ep, part);
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

template <typename T>
int gcn_spmm(const int* work, int n_work, const int* split, int n_split, float* part, const int* col, const float* val,
             int d, const T* X, uint32_t k0, uint32_t k1, float p, int mask_on_output, float alpha, const T* Z,
             float beta, float delta, int pad_row, float gamma, T* Y, T* Y2, void* stream) {
  if (d % c2::VW<T>) return (int)hipErrorInvalidValue;
  if (n_work == 0) return 0;
  Epi<T> ep{alpha, Z, beta, delta, pad_row, gamma, Y, Y2, c2::make_drop(k0, k1, p)};
  hipStream_t s = (hipStream_t)stream;
  if (mask_on_output)
    return launch<true>((const int4*)work, n_work, (const int4*)split, n_split, col, val, d, X, ep, part, s);
  return launch<false>((const int4*)work, n_work, (const int4*)split, n_split, col, val, d, X, ep, part, s);
}

C2_API int c2dsr_gcn_spmm(const int* work, int n_work, const int* split, int n_split, float* part, const int* col,
                          const float* val, int d, const float* X, uint32_t k0, uint32_t k1, float p,
                          int mask_on_output, float alpha, const float* Z, float beta, float delta, int pad_row,
                          float gamma, float* Y, float* Y2, void* stream) {
  return gcn_spmm<float>(work, n_work, split, n_split, part, col, val, d, X, k0, k1, p, mask_on_output, alpha, Z, beta,
                         delta, pad_row, gamma, Y, Y2, stream);
}

// the same on bf16 tables X, Z, Y, Y2 (fp32 arithmetic and partial slab, RNE stores): the C5 roofline run
C2_API int c2dsr_gcn_spmm_b16(const int* work, int n_work, const int* split, int n_split, float* part, const int* col,
                              const float* val, int d, const void* X, uint32_t k0, uint32_t k1, float p,
                              int mask_on_output, float alpha, const void* Z, float beta, float delta, int pad_row,
                              float gamma, void* Y, void* Y2, void* stream) {
  return gcn_spmm<c2::tbf16>(work, n_work, split, n_split, part, col, val, d, (const c2::tbf16*)X, k0, k1, p,
                             mask_on_output, alpha, (const c2::tbf16*)Z, beta, delta, pad_row, gamma, (c2::tbf16*)Y,
                             (c2::tbf16*)Y2, stream);
}
