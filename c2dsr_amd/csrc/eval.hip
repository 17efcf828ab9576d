// Evaluation path: batched candidate scoring + ranking and the
// HR/MRR/NDCG@{5,20} sums, on the device.
//
// Replaces trainer.py:162-181 (Trainer.evaluate_batch: a per-row Python loop that runs
// the full classifier GEMV, indexes 1 + n_neg scores and syncs the host per row) and
// utils/metrics.py:4-19 (cal_metrics).  Per row only the 1 + n_neg candidate rows of the
// classifier weight are read (coalesced 16-B lane loads, G lanes per candidate), never
// the full n_dom × d matrix.
#include "common.h"

namespace {

// One workgroup per evaluation row i:
//   dom  = xory[i] == 0 ? a : b                          (trainer.py:169,176)
//   q    = h_share[i, L-1] + h_dom[i, idx_last_dom[i]]   (trainer.py:167,171,178)
//   s(j) = q · W_dom[j] + b_dom[j]                       (classifier_{a,b}, nn.Linear)
//   rank = 1 + #{k : s(neg[i,k]) > s(gt[i])}             (trainer.py:173,180; ties not counted)
// Every candidate is scored by the same lane mapping and reduction tree, so an item that
// appears as both target and negative gets bit-identical scores (as in the reference's
// single GEMV).  Negative indices wrap as torch indexing does (hx[i, -1] is position L-1,
// scores[-k] is item n_dom-k); indices outside [-L,L) / [-n_dom,n_dom) give rank = -1 (the
// host raises IndexError, as the reference would).
template <int G, bool VEC>
__global__ __launch_bounds__(256) void eval_rank_kernel(
    const float* __restrict__ hs, const float* __restrict__ ha, const float* __restrict__ hb, int L, int d,
    const int64_t* __restrict__ il_a, const int64_t* __restrict__ il_b, const int64_t* __restrict__ xory,
    const int64_t* __restrict__ gt, const int64_t* __restrict__ neg, int n_neg, const float* __restrict__ Wa,
    const float* __restrict__ ba, int n_a, const float* __restrict__ Wb, const float* __restrict__ bb, int n_b,
    int* __restrict__ rank) {
  extern __shared__ float lds[];
  float* q = lds;            // [d]
  float* score = lds + d;    // [1 + n_neg]
  __shared__ int bad;
  __shared__ int cnt[4];
  const int i = blockIdx.x;
  const int tid = threadIdx.x;
  const bool da = xory[i] == 0;
  int64_t il = da ? il_a[i] : il_b[i];
  if (il < 0) il += L;
  const float* hdom = da ? ha : hb;
  const float* W = da ? Wa : Wb;
  const float* bias = da ? ba : bb;
  const int n_dom = da ? n_a : n_b;
  if (tid == 0) bad = (il < 0 || il >= L) ? 1 : 0;
  if (tid < 4) cnt[tid] = 0;
  __syncthreads();
  if (bad) {
    if (tid == 0) rank[i] = -1;
    return;
  }
  const float* hl = hs + ((long)i * L + (L - 1)) * d;
  const float* hd = hdom + ((long)i * L + il) * d;
  for (int c = tid; c < d; c += 256) q[c] = hl[c] + hd[c];
  __syncthreads();

  const int n_cand = n_neg + 1;
  const int lig = tid & (G - 1);
  const int grp = tid / G;
  constexpr int NG = 256 / G;
  for (int j = grp; j < n_cand; j += NG) {
    int64_t item = j == 0 ? gt[i] : neg[(long)i * n_neg + (j - 1)];
    if (item < 0) item += n_dom;
    float acc = 0.f;
    if (item >= 0 && item < n_dom) {
      const float* w = W + item * (long)d;
      if constexpr (VEC) {
        for (int c = lig * 4; c < d; c += G * 4) {
          const float4 wv = *(const float4*)(w + c);
          const float4 qv = *(const float4*)(q + c);
          acc = fmaf(qv.x, wv.x, acc);
          acc = fmaf(qv.y, wv.y, acc);
          acc = fmaf(qv.z, wv.z, acc);
          acc = fmaf(qv.w, wv.w, acc);
        }
      } else {
        for (int c = lig; c < d; c += G) acc = fmaf(q[c], w[c], acc);
      }
      acc = c2::group_sum<G>(acc);
      if (lig == 0) score[j] = acc + bias[item];
    } else if (lig == 0) {
      bad = 1;
    }
  }
  __syncthreads();
  if (bad) {
    if (tid == 0) rank[i] = -1;
    return;
  }
  const float sg = score[0];
  int c = 0;
  for (int k = 1 + tid; k < n_cand; k += 256) c += score[k] > sg ? 1 : 0;
  // wave reduction, then the 4 wave counts in fixed order
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((tid & 63) == 0) cnt[tid >> 6] = c;
  __syncthreads();
  if (tid == 0) rank[i] = 1 + cnt[0] + cnt[1] + cnt[2] + cnt[3];
}

// sums[0..6] += (hr5, hr20, mrr5, mrr20, ndcg5, ndcg20, count) over rows with xory == dom
// (utils/metrics.py:4-19; fp64 like the reference's Python floats).  One workgroup, fixed
// reduction order (deterministic); bad ranks (<= 0) are counted in sums[7].
__global__ __launch_bounds__(256) void rank_metrics_kernel(const int* __restrict__ rank,
                                                           const int64_t* __restrict__ xory, int B, int dom,
                                                           double* __restrict__ sums) {
  __shared__ double red[8][256];
  const int tid = threadIdx.x;
  double v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = tid; i < B; i += 256) {
    const bool mine = dom == 0 ? xory[i] == 0 : xory[i] != 0;
    if (!mine) continue;
    const int r = rank[i];
    if (r <= 0) {
      v[7] += 1.0;
      continue;
    }
    v[6] += 1.0;
    if (r <= 20) {
      const double inv = 1.0 / (double)r;
      const double dg = 1.0 / log2((double)r + 1.0);
      v[1] += 1.0;
      v[3] += inv;
      v[5] += dg;
      if (r <= 5) {
        v[0] += 1.0;
        v[2] += inv;
        v[4] += dg;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) red[k][tid] = v[k];
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (tid < s) {
#pragma unroll
      for (int k = 0; k < 8; ++k) red[k][tid] += red[k][tid + s];
    }
    __syncthreads();
  }
  if (tid < 8) sums[tid] += red[tid][0];
}

template <int G, bool VEC>
int launch_rank(int B, size_t lds, hipStream_t s, const float* hs, const float* ha, const float* hb, int L, int d,
                const int64_t* il_a, const int64_t* il_b, const int64_t* xory, const int64_t* gt, const int64_t* neg,
                int n_neg, const float* Wa, const float* ba, int n_a, const float* Wb, const float* bb, int n_b,
                int* rank) {
  eval_rank_kernel<G, VEC><<<B, 256, lds, s>>>(hs, ha, hb, L, d, il_a, il_b, xory, gt, neg, n_neg, Wa, ba, n_a, Wb,
                                               bb, n_b, rank);
  C2_CHECK_LAUNCH();
  return 0;
}

}  // namespace

C2_API int c2dsr_eval_rank(const float* h_share, const float* h_a, const float* h_b, int B, int L, int d,
                           const int64_t* idx_last_a, const int64_t* idx_last_b, const int64_t* xory,
                           const int64_t* gt, const int64_t* neg, int n_neg, const float* Wa, const float* ba, int n_a,
                           const float* Wb, const float* bb, int n_b, int* rank, void* stream) {
  if (B < 0 || L <= 0 || d <= 0 || n_neg < 0 || n_a <= 0 || n_b <= 0) return (int)hipErrorInvalidValue;
  if (B == 0) return 0;
  const size_t lds = sizeof(float) * ((size_t)d + (size_t)n_neg + 1);
  if (lds > 60 * 1024) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  const bool vec = (d % 4) == 0 && ((uintptr_t)Wa % 16) == 0 && ((uintptr_t)Wb % 16) == 0;
  int lanes = vec ? d / 4 : d;
  int G = 1;
  while (G < lanes && G < 64) G <<= 1;
#define C2_EVAL_CASE(g)                                                                                          \
  case g:                                                                                                        \
    return vec ? launch_rank<g, true>(B, lds, s, h_share, h_a, h_b, L, d, idx_last_a, idx_last_b, xory, gt, neg, \
                                      n_neg, Wa, ba, n_a, Wb, bb, n_b, rank)                                     \
               : launch_rank<g, false>(B, lds, s, h_share, h_a, h_b, L, d, idx_last_a, idx_last_b, xory, gt,    \
                                       neg, n_neg, Wa, ba, n_a, Wb, bb, n_b, rank);
  switch (G) {
    C2_EVAL_CASE(1)
    C2_EVAL_CASE(2)
    C2_EVAL_CASE(4)
    C2_EVAL_CASE(8)
    C2_EVAL_CASE(16)
    C2_EVAL_CASE(32)
    C2_EVAL_CASE(64)
  }
#undef C2_EVAL_CASE
  return (int)hipErrorInvalidValue;
}

C2_API int c2dsr_rank_metrics(const int* rank, const int64_t* xory, int B, int dom, double* sums, void* stream) {
  if (B < 0 || (dom != 0 && dom != 1)) return (int)hipErrorInvalidValue;
  if (B == 0) return 0;
  rank_metrics_kernel<<<1, 256, 0, (hipStream_t)stream>>>(rank, xory, B, dom, sums);
  C2_CHECK_LAUNCH();
  return 0;
}
