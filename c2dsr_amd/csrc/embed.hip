// K2: embedding fuse — gather (H[seq] + E[seq]) * sqrt(d) + P[pos], dropout — and its
// deterministic scatter-add backward.
//
// Replaces models/C2DSR.py:65-71,81-82 (F.embedding + nn.Embedding + in-place *=)
// and models/encoders.py:30-31 (pos_emb += , dropout).  The backward replaces
// embedding_dense_backward: instead of float atomics it radix-sorts the row ids
// (stable LSD, 8-bit digits) and sums each item's rows in position order, so the
// result is bitwise reproducible; runs that span several chunks are combined by
// a second pass in chunk order.
#include "common.h"

#include <algorithm>
#include <vector>

namespace {

// ------------------------------------------------------------------ forward gather
// Index range checks of the lookups (F.embedding / nn.Embedding raise IndexError for an index outside [0, N),
// models/C2DSR.py:65-67,81, encoders.py:30): a bad item index sets IDX_ERR_ITEM, a bad position IDX_ERR_POS in the
// caller's error word (host reads it at its next sync and raises), and the row read is row 0 instead — no load
// ever leaves the tables.
__device__ __forceinline__ long checked_index(int64_t v, int n, int bit, int* err) {
  if (v >= 0 && v < n) return (long)v;
  if (err) atomicOr(err, bit);
  return 0;
}

template <int LPR, bool GATHER, typename T = float>
__global__ __launch_bounds__(256) void embed_fwd_kernel(const int64_t* __restrict__ seq, const int64_t* __restrict__ pos,
                                                        int n_rows, int d, const T* __restrict__ H,
                                                        const T* __restrict__ E, const float* __restrict__ Xin,
                                                        const float* __restrict__ P, float scale, c2::Drop drop,
                                                        int64_t idx_base, float* __restrict__ X, int n_items,
                                                        int n_pos, int* __restrict__ err) {
  constexpr int GROUPS = 256 / LPR;
  const int g = threadIdx.x / LPR;
  const int lane = threadIdx.x % LPR;
  const long r = (long)blockIdx.x * GROUPS + g;
  if (r >= n_rows) return;
  const bool flag = lane == 0;
  const long p = checked_index(pos[r], n_pos, C2DSR_IDX_ERR_POS, flag ? err : nullptr);
  long s = 0;
  if (GATHER) s = checked_index(seq[r], n_items, C2DSR_IDX_ERR_ITEM, flag ? err : nullptr);
  for (int c = lane * 4; c < d; c += LPR * 4) {
    float4 a;
    if (GATHER) {
      const float4 h = c2::ld4(H + s * d + c);
      const float4 e = c2::ld4(E + s * d + c);
      a = scale * (h + e);
    } else {
      a = *(const float4*)(Xin + r * d + c);
    }
    float4 x = a + *(const float4*)(P + p * d + c);
    if (drop.active()) {
      const uint64_t b = (uint64_t)(idx_base + r) * d + c;
      x = x * drop.mul4(b);
    }
    *(float4*)(X + r * d + c) = x;
  }
}

// the same, computing only chosen rows: output row k is input row qi[k] (k < nq) or ki[k - nq] (the row-subset
// encoder layer's query rows and key rows, written side by side: the [B·L, d] embedding is never stored)
template <int LPR>
__global__ __launch_bounds__(256) void embed_fwd_rows_kernel(const int64_t* __restrict__ seq,
                                                             const int64_t* __restrict__ pos, int n_rows, int d,
                                                             const float* __restrict__ H, const float* __restrict__ E,
                                                             const float* __restrict__ P, float scale, c2::Drop drop,
                                                             int64_t idx_base, const int* __restrict__ qi, int nq,
                                                             const int* __restrict__ ki, int nk,
                                                             float* __restrict__ X, int n_items, int n_pos,
                                                             int* __restrict__ err) {
  constexpr int GROUPS = 256 / LPR;
  const int g = threadIdx.x / LPR;
  const int lane = threadIdx.x % LPR;
  const long k = (long)blockIdx.x * GROUPS + g;
  if (k >= nq + nk) return;
  const long r = min(max(k < nq ? qi[k] : ki[k - nq], 0), n_rows - 1);
  int* const e = lane == 0 ? err : nullptr;
  const long p = checked_index(pos[r], n_pos, C2DSR_IDX_ERR_POS, e);
  const long s = checked_index(seq[r], n_items, C2DSR_IDX_ERR_ITEM, e);
  for (int c = lane * 4; c < d; c += LPR * 4) {
    // (the statements of embed_fwd_kernel's gather path: the same rounding)
    const float4 h = c2::ld4(H + s * d + c);
    const float4 e = c2::ld4(E + s * d + c);
    const float4 a = scale * (h + e);
    float4 x = a + *(const float4*)(P + p * d + c);
    if (drop.active()) {
      const uint64_t b = (uint64_t)(idx_base + r) * d + c;
      x = x * drop.mul4(b);
    }
    *(float4*)(X + k * d + c) = x;
  }
}

// ------------------------------------------------------------------ radix sort (stable LSD)
constexpr int RS_THREADS = 256;
constexpr int RS_ROUNDS = 8;
constexpr int RS_TILE = RS_THREADS * RS_ROUNDS;

// ------------------------------------------------------------------ index plans, several per launch
// A training step builds eight plans (the item and position indices of its five lookups, positions shared); one
// launch per pass covers all of them (jobs): the blocks of job j are [beg[j], beg[j+1]) of the launch, and a block
// reads its job's fields through pj() (a select chain over the launch's job table: uniform, no indexed kernel-argument
// access).  Per plan: keys prepared, one LSD pass per 8-bit digit (histogram + scatter), then the split list (count +
// emit) — 1 + 2·passes + 2 launches for any number of plans instead of that many per plan.
constexpr int PJ_MAX = 12;
struct PlanJobs {
  int nj, shift;               // jobs in this launch; the radix passes' digit shift
  int beg[PJ_MAX + 1];         // first block of each job
  int n[PJ_MAX], aux[PJ_MAX];  // entries; n_keys (prep) / radix blocks of the job (hist, scatter)
  const int64_t* idx[PJ_MAX];
  uint32_t *ki[PJ_MAX], *vi[PJ_MAX], *ko[PJ_MAX], *vo[PJ_MAX];  // prep: ki / vi; passes: in → out; plans: ki = sorted keys
  uint32_t* hist[PJ_MAX];      // passes: digit histograms [256][radix blocks]; plans: per-block counts
  int4* splits[PJ_MAX];
  int* suboff[PJ_MAX];
  int2* subs[PJ_MAX];
  int* counts[PJ_MAX];
  int* scnt[PJ_MAX];           // plans: pass B's per-split arrival counters (zeroed here)
};
template <typename T>
__device__ __forceinline__ T pj(const T (&a)[PJ_MAX], int j) {
  T r = a[0];
#pragma unroll
  for (int k = 1; k < PJ_MAX; ++k) r = j == k ? a[k] : r;
  return r;
}
// this block's job and its block index / block count within the job
__device__ __forceinline__ int pj_job(const PlanJobs& P, int& lb, int& nb) {
  int j = 0, b0 = P.beg[0], b1 = P.beg[1];  // (beg[k] = the launch's block total for k >= nj)
#pragma unroll
  for (int k = 1; k < PJ_MAX; ++k)
    if (k < P.nj && (int)blockIdx.x >= P.beg[k]) {
      j = k;
      b0 = P.beg[k];
      b1 = P.beg[k + 1];
    }
  lb = (int)blockIdx.x - b0;
  nb = b1 - b0;
  return j;
}

// an index outside [0, n_keys) becomes the key n_keys (sorted after every valid key; the segment sums never follow
// a key >= n_out) and sets `bit` in the caller's error word: a bad index never reaches a gradient read-modify-write
__global__ __launch_bounds__(256) void prep_keys_kernel(PlanJobs P, int bit, int* __restrict__ err) {
  int lb, nb;
  const int j = pj_job(P, lb, nb);
  const int n = pj(P.n, j), n_keys = pj(P.aux, j);
  const int i = lb * 256 + threadIdx.x;
  if (i < n) {
    const int64_t v = pj(P.idx, j)[i];
    const bool ok = v >= 0 && v < n_keys;
    if (!ok && err) atomicOr(err, bit);
    pj(P.ki, j)[i] = ok ? (uint32_t)v : (uint32_t)n_keys;
    pj(P.vi, j)[i] = (uint32_t)i;
  }
}

__global__ __launch_bounds__(RS_THREADS) void rs_hist_kernel(PlanJobs P) {
  __shared__ uint32_t h[256];
  int lb, nb;
  const int j = pj_job(P, lb, nb);
  const uint32_t* __restrict__ keys = pj(P.ki, j);
  const int n = pj(P.n, j), shift = P.shift;
  h[threadIdx.x] = 0;
  // every round's key loaded up front (one memory round trip per block instead of one per round)
  uint32_t k[RS_ROUNDS];
  const int base = lb * RS_TILE;
#pragma unroll
  for (int r = 0; r < RS_ROUNDS; ++r) {
    const int i = base + r * RS_THREADS + threadIdx.x;
    k[r] = i < n ? keys[i] : 0u;
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < RS_ROUNDS; ++r) {
    const int i = base + r * RS_THREADS + threadIdx.x;
    if (i < n) atomicAdd(&h[(k[r] >> shift) & 255u], 1u);
  }
  __syncthreads();
  pj(P.hist, j)[threadIdx.x * nb + lb] = h[threadIdx.x];
}

__global__ __launch_bounds__(RS_THREADS) void rs_scatter_kernel(PlanJobs P) {
  __shared__ uint32_t wcnt[4][256];
  __shared__ uint32_t woff[4][256];
  __shared__ uint32_t run[256];
  __shared__ uint32_t gbase[256];
  int lb, nblocks;
  const int j = pj_job(P, lb, nblocks);
  const uint32_t* __restrict__ kin = pj(P.ki, j);
  const uint32_t* __restrict__ vin = pj(P.vi, j);
  uint32_t* __restrict__ kout = pj(P.ko, j);
  uint32_t* __restrict__ vout = pj(P.vo, j);
  const uint32_t* __restrict__ offs = pj(P.hist, j);  // digit histograms [256][nblocks]
  const int n = pj(P.n, j), shift = P.shift;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  const int base = lb * RS_TILE;
  // every round's key and row loaded up front: their latency overlaps the offset computation below instead of
  // opening each of the RS_ROUNDS rounds
  uint32_t kr[RS_ROUNDS], vr[RS_ROUNDS];
#pragma unroll
  for (int r = 0; r < RS_ROUNDS; ++r) {
    const int i = base + r * RS_THREADS + t;
    kr[r] = i < n ? kin[i] : 0u;
    vr[r] = i < n ? vin[i] : 0u;
  }
  for (int q = 0; q < 4; ++q) wcnt[q][t] = 0;
  run[t] = 0;
  {
    // this block's first destination of digit t = (entries of smaller digits) + (digit-t entries of earlier
    // blocks): read off the digit histograms of all blocks here instead of a separate single-workgroup scan
    const uint32_t* ht = offs + (long)t * nblocks;
    uint32_t pre = 0, tot = 0;
#pragma unroll 8
    for (int b = 0; b < nblocks; ++b) {
      const uint32_t c = ht[b];
      pre += b < lb ? c : 0u;
      tot += c;
    }
    // exclusive scan of tot over the 256 digits (four waves: in-wave shuffles, then the wave totals)
    uint32_t inc = tot;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u = __shfl_up(inc, o, 64);
      if (lane >= o) inc += u;
    }
    if (lane == 63) woff[0][w] = inc;
    __syncthreads();
    uint32_t base = 0;
    for (int k = 0; k < w; ++k) base += woff[0][k];
    gbase[t] = base + inc - tot + pre;
  }
  __syncthreads();
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
#pragma unroll
  for (int r = 0; r < RS_ROUNDS; ++r) {
    const int i = base + r * RS_THREADS + t;
    const bool act = i < n;
    const uint32_t key = kr[r], val = vr[r];
    const uint32_t dg = act ? (key >> shift) & 255u : 0u;
    uint64_t peers = __ballot(act);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      uint64_t bal = __ballot((dg >> b) & 1u);
      peers &= ((dg >> b) & 1u) ? bal : ~bal;
    }
    const uint32_t rank = (uint32_t)__popcll(peers & lt);
    if (act && rank == 0) wcnt[w][dg] = (uint32_t)__popcll(peers);
    __syncthreads();
    {
      uint32_t b = run[t];
      for (int q = 0; q < 4; ++q) {
        woff[q][t] = b;
        b += wcnt[q][t];
        wcnt[q][t] = 0;
      }
      run[t] = b;
    }
    __syncthreads();
    if (act) {
      const uint32_t dst = gbase[dg] + woff[w][dg] + rank;
      kout[dst] = key;
      vout[dst] = val;
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------ sort plan → split lists
// The sorted entries are cut into chunks of SEG_CH; one lane group walks one chunk (pass A).  A
// run wholly inside a chunk goes to out[key] (+=); a run cut by a chunk edge leaves its pieces in
// the chunks' head/tail slots.  A "split" is a run that continues past the end of its first
// chunk: out[key] += tail[c] + head[c+1] + ... + head[last], summed in chunk order (pass B).  The
// split list depends on the indices only, so it is part of the plan (off the critical path).
// Chunk length (tools/embed_micro.py, MB embedding backward, items + positions in one launch): 16 entries with 2
// rows in flight (SEG_U below) 54.0 µs against 61.7 at 32 / 4 — twice the waves, each half as long; 8 → 64.3,
// 64 → 70.2 (the split passes grow below 16).
#ifndef SEG_CH_CFG
#define SEG_CH_CFG 16
#endif
constexpr int SEG_CH = SEG_CH_CFG;
constexpr int PL_T = 256;         // plan kernels: threads per block
constexpr int PL_E = 4;           // entries per thread
constexpr int PL_B = PL_T * PL_E;  // entries per block
constexpr int SUBP = 128;          // pieces per level-1 block of a split (pass B)

__device__ __forceinline__ bool split_start(const uint32_t* K, int n, int i) {
  if (!(i == 0 || K[i] != K[i - 1])) return false;
  const int ce = (i / SEG_CH + 1) * SEG_CH;
  return ce < n && K[ce] == K[i];
}

// chunks spanned by the run that starts at entry i (keys are sorted: binary search for its end)
__device__ __forceinline__ int split_span(const uint32_t* K, int n, int i) {
  const uint32_t key = K[i];
  int lo = i, hi = n;  // first entry with a larger key
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (K[mid] <= key) lo = mid + 1; else hi = mid;
  }
  return (lo - 1) / SEG_CH - i / SEG_CH + 1;
}

__device__ __forceinline__ uint32_t n_subs(int span) { return (uint32_t)((span + SUBP - 1) / SUBP); }

// per block: the splits starting among its PL_B entries and their SUBP-piece sub-ranges → cnt[b], cnt[nb + b]
__global__ __launch_bounds__(PL_T) void plan_count_kernel(PlanJobs P) {
  __shared__ uint32_t red[2][PL_T / 64];
  int lb, nb;
  const int j = pj_job(P, lb, nb);
  const uint32_t* __restrict__ K = pj(P.ki, j);
  const int n = pj(P.n, j);
  uint32_t q = 0, u = 0;
  for (int e = 0; e < PL_E; ++e) {
    const int i = lb * PL_B + e * PL_T + threadIdx.x;
    if (i < n && split_start(K, n, i)) {
      ++q;
      u += n_subs(split_span(K, n, i));
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    q += __shfl_xor(q, o, 64);
    u += __shfl_xor(u, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = q;
    red[1][threadIdx.x >> 6] = u;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0, v = 0;
    for (int w = 0; w < PL_T / 64; ++w) {
      t += red[0][w];
      v += red[1][w];
    }
    uint32_t* cnt = pj(P.hist, j);
    cnt[lb] = t;
    cnt[nb + lb] = v;
  }
}

// exclusive block-wide prefix of one u32 per thread (PL_T threads)
__device__ __forceinline__ uint32_t block_prefix(uint32_t v, uint32_t* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t inc = v;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t u = __shfl_up(inc, o, 64);
    if (lane >= o) inc += u;
  }
  if (lane == 63) red[w] = inc;
  __syncthreads();
  uint32_t base = 0;
  for (int k = 0; k < w; ++k) base += red[k];
  __syncthreads();
  return base + inc - v;
}

// writes splits[s] = {key, first chunk, chunks spanned, 0} in entry order, and — the work a single-workgroup
// launch (plan_subs) did after it until round 6 — every split's SUBP-piece sub-ranges: suboff[s] = its first sub,
// subs[suboff[s] + y] = (s, y·SUBP), suboff[splits] = counts[2] = the sub total; counts[1] = the split total, and the
// plan's error word (counts[3]) starts at 0.  A block's first output slots are the sums of the earlier blocks'
// counts (plan_count_kernel), read here (≤ a few hundred u32 from L2) instead of a separate scan launch.
__global__ __launch_bounds__(PL_T) void plan_emit_kernel(PlanJobs P) {
  __shared__ uint32_t red[2][PL_T / 64];
  int lb, nb;
  const int j = pj_job(P, lb, nb);
  const uint32_t* __restrict__ K = pj(P.ki, j);
  const uint32_t* __restrict__ cnt = pj(P.hist, j);
  int4* __restrict__ splits = pj(P.splits, j);
  int* __restrict__ suboff = pj(P.suboff, j);
  int2* __restrict__ subs = pj(P.subs, j);
  int* __restrict__ scnt = pj(P.scnt, j);
  const int n = pj(P.n, j);
  uint32_t bs = 0, bu = 0;
  for (int b = threadIdx.x; b < lb; b += PL_T) {
    bs += cnt[b];
    bu += cnt[nb + b];
  }
  for (int o = 32; o > 0; o >>= 1) {
    bs += __shfl_xor(bs, o, 64);
    bu += __shfl_xor(bu, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = bs;
    red[1][threadIdx.x >> 6] = bu;
  }
  __syncthreads();
  uint32_t base_s = 0, base_u = 0;
  for (int k = 0; k < PL_T / 64; ++k) {
    base_s += red[0][k];
    base_u += red[1][k];
  }
  __syncthreads();
  // thread t owns entries [i0, i0 + PL_E): contiguous, so the order is kept
  const int i0 = lb * PL_B + threadIdx.x * PL_E;
  uint32_t fs = 0, nu = 0;
  int span[PL_E];
  for (int e = 0; e < PL_E; ++e) {
    const int i = i0 + e;
    span[e] = 0;
    if (i < n && split_start(K, n, i)) {
      fs |= 1u << e;
      span[e] = split_span(K, n, i);
      nu += n_subs(span[e]);
    }
  }
  uint32_t os = base_s + block_prefix(__popc(fs), red[0]);
  uint32_t ou = base_u + block_prefix(nu, red[1]);
  for (int e = 0; e < PL_E; ++e) {
    if (fs >> e & 1) {
      const int i = i0 + e;
      splits[os] = make_int4((int)K[i], i / SEG_CH, span[e], 0);
      suboff[os] = (int)ou;
      scnt[os] = 0;
      const uint32_t k = n_subs(span[e]);
      for (uint32_t y = 0; y < k; ++y) subs[ou + y] = make_int2((int)os, (int)(y * SUBP));
      ++os;
      ou += k;
    }
  }
  if (lb == nb - 1 && threadIdx.x == PL_T - 1) {  // owns the last entries: os / ou are the totals
    suboff[os] = (int)ou;
    int* counts = pj(P.counts, j);
    counts[1] = (int)os;
    counts[2] = (int)ou;
    counts[3] = 0;
  }
}

// ------------------------------------------------------------------ segment sums
// rows in flight per lane group: 2 with 16-entry chunks (tools/embed_micro.py, items + positions: CH 32 / U 4 61.7 µs,
// CH 16 / U 4 61.1, CH 16 / U 2 54.0–54.9, CH 16 / U 1 54.0, CH 8 / U 2 64.4; round 2 at CH 32: U 8 → 87 µs,
// U 16 → 133); SEG_PIPE 1 = the next batch's rows loaded under this batch's read-modify-writes (no better at 4)
#ifndef SEG_U_CFG
#define SEG_U_CFG 2
#endif
constexpr int SEG_U = SEG_U_CFG;  // rows in flight per lane group
#ifndef SEG_PIPE
#define SEG_PIPE 0
#endif
#ifndef SEG_PREF
#define SEG_PREF 0
#endif
#ifndef SEG_MERGE  // pass B's level 2 by each split's last-arriving level-1 block (no second launch)
#define SEG_MERGE 1
#endif

struct RowSrc {
  const float* gX;
  int d;
  c2::Drop drop;
  int64_t idx_base;
  float scale;
  const float* rs;  // optional per-row multiplier
  // optional: row r is the sum of two compact sources, gX[map1[r]] + gX2[map2[r]] (entries < 0: absent) —
  // the row-subset attention layer's input gradient (query rows + key rows, ops.RowsQKVAttnFn)
  const int *map1, *map2;
  const float* gX2;
  // a, b: map1[r], map2[r] when the maps are set (the caller stages them), else unused
  __device__ __forceinline__ float4 load(uint32_t r, int c, int a = -1, int b = -1) const {
    if (!gX) return make_float4(c == 0 ? (rs ? scale * rs[r] : scale) : 0.f, 0.f, 0.f, 0.f);  // the row (1, 0, …)
    float4 v;
    if (map1) {
      v = a >= 0 ? *(const float4*)(gX + (long)a * d + c) : c2::f4(0.f);
      if (b >= 0) v = v + *(const float4*)(gX2 + (long)b * d + c);
    } else {
      v = *(const float4*)(gX + (long)r * d + c);
    }
    if (drop.active()) {
      const uint64_t b = (uint64_t)(idx_base + r) * d + c;
      v = v * drop.mul4(b);
    }
    return (rs ? scale * rs[r] : scale) * v;
  }
};

// One segment-sum job: out[key] += Σ src rows of every run of a plan.  Several jobs over plans
// of the same row width share one launch of each pass (the embedding backward's item and
// position sums).
struct SegJob {
  const uint32_t *K, *V;       // plan: sorted keys, their rows
  const int4* splits;          // plan: runs that cross a chunk end
  const int2* subs;            // plan: (split, first piece) of every SUBP-piece sub-range
  const int* suboff;           // plan: first sub of every split
  const int* counts;           // plan: [pieces, splits, subs]
  int* scnt;                   // plan: per-split arrival counters of pass B (zero between uses)
  int* err;                    // plan: error word (debug)
  int n, n_out, skip_key, nblocks;
  RowSrc src;
  float *out, *ph, *pt, *slot2;
  c2::tbf16* out16;  // non-null: the output table is bf16 (then out is null; the C5 roofline run)
};

// pass A: one lane group per chunk of SEG_CH sorted entries.  The block stages its keys and row
// ids in LDS (one coalesced load; no dependent index loads in the walk).  Rows are loaded
// SEG_U at a time and summed in entry order; a run that closes inside the chunk leaves its sum in
// the slot of its last row, and the read-modify-writes of out[] for all runs closing in the batch
// are issued together (all loads, then all stores), so short runs do not serialise.  The chunk's
// first run goes to its head slot when it continues the previous chunk, the last run to the tail
// slot when it continues into the next (pass B adds those up).  Keys outside [0, n_out) are never
// followed (err is set; checked by the host in debug runs).
// ROLE only names the instantiation (0: embedding backward, 1: classifier one-hot dW) so PMC passes can tell the
// two callers' launches apart (tools/pmc_traffic.py); the code is the same
template <int LPR, int ROLE = 0>
__global__ __launch_bounds__(256) void seg_chunk_kernel(SegJob j0, SegJob j1) {
  constexpr int GROUPS = 256 / LPR;
  constexpr int ENT = GROUPS * SEG_CH;
  __shared__ uint32_t sk[ENT + 2];  // sk[e + 1] = K[b0 + e]; sk[0], sk[ENT + 1]: the neighbours
  __shared__ uint32_t sv[ENT];
  constexpr bool CANMAP = LPR >= 16;  // two-source rows only at d >= 64 (c2dsr_embed_bwd_planned_rows checks)
  __shared__ int sm[2][CANMAP ? ENT : 1];  // two-source rows: map1 / map2 of each staged row (RowSrc::map1)
  const bool second = (int)blockIdx.x >= j0.nblocks;
  const SegJob& J = second ? j1 : j0;
  const int blk = second ? (int)blockIdx.x - j0.nblocks : (int)blockIdx.x;
  const int n = J.n;
  const long b0 = (long)blk * ENT;
  for (int e = threadIdx.x; e < ENT + 2; e += 256) {
    const long gi = b0 - 1 + e;
    sk[e] = (gi >= 0 && gi < n) ? J.K[gi] : 0xffffffffu;
  }
  const bool mapped = CANMAP && J.src.map1 != nullptr;
  for (int e = threadIdx.x; e < ENT; e += 256) {
    const long gi = b0 + e;
    const uint32_t rv = gi < n ? min(J.V[gi], (uint32_t)(n - 1)) : 0u;
    sv[e] = rv;
    if (mapped) {
      sm[0][e] = J.src.map1[rv];
      sm[1][e] = J.src.map2[rv];
    }
  }
  __syncthreads();
  const int g = threadIdx.x / LPR;
  const int lane = threadIdx.x % LPR;
  const long chunk = (long)blk * GROUPS + g;
  const long start = chunk * SEG_CH;
  if (start >= n) return;
  const int cnt = (int)min((long)SEG_CH, n - start);
  const int o = g * SEG_CH;
  const bool cont_head = start > 0 && sk[o] == sk[o + 1];
  const bool cont_tail = start + cnt < n && sk[o + cnt + 1] == sk[o + cnt];
  const RowSrc& src = J.src;
  const int d = src.d;
  for (int c = lane * 4; c < d; c += LPR * 4) {
    float4 acc = c2::f4(0.f);
    bool first = true;  // the next run to close is the chunk's first
    auto load = [&](float4 (&x)[SEG_U], int h0) {
#pragma unroll
      for (int u = 0; u < SEG_U; ++u) {
        const int e = o + h0 + u;
        x[u] = h0 + u < cnt ? (mapped ? src.load(sv[e], c, sm[0][e], sm[1][e]) : src.load(sv[e], c)) : c2::f4(0.f);
      }
    };
    auto process = [&](float4 (&x)[SEG_U], int h0) {
      int kind[SEG_U];  // 0: nothing closes at u, 1: out[key] +=, 2: head slot, 3: tail slot, 4: bad key
#pragma unroll
      for (int u = 0; u < SEG_U; ++u) {
        const int q = h0 + u;
        kind[u] = 0;
        if (q < cnt) {
          acc = acc + x[u];
          if (q == cnt - 1 || sk[o + q + 2] != sk[o + q + 1]) {
            const uint32_t key = sk[o + q + 1];
            if (first && cont_head)
              kind[u] = 2;
            else if (q == cnt - 1 && cont_tail)
              kind[u] = 3;
            else if (key >= (uint32_t)J.n_out)
              kind[u] = 4;
            else if ((int)key != J.skip_key)
              kind[u] = 1;
            x[u] = acc;  // the run's sum, in the slot of its last row
            acc = c2::f4(0.f);
            first = false;
          }
        }
      }
      float4 prev[SEG_U];
#pragma unroll
      for (int u = 0; u < SEG_U; ++u) {
        const long off = (long)sk[o + h0 + u + 1] * d + c;
        prev[u] = kind[u] != 1 ? c2::f4(0.f) : (J.out16 ? c2::ld4(J.out16 + off) : *(const float4*)(J.out + off));
      }
#pragma unroll
      for (int u = 0; u < SEG_U; ++u) {
        if (kind[u] == 1) {
          const long off = (long)sk[o + h0 + u + 1] * d + c;
          if (J.out16)
            c2::st4(J.out16 + off, prev[u] + x[u]);
          else
            *(float4*)(J.out + off) = prev[u] + x[u];
        }
        else if (kind[u] == 2)
          *(float4*)(J.ph + chunk * d + c) = x[u];
        else if (kind[u] == 3)
          *(float4*)(J.pt + chunk * d + c) = x[u];
        else if (kind[u] == 4 && lane == 0)
          atomicOr(J.err, 2);
      }
    };
#if SEG_PREF
    // the out rows a batch read-modify-writes are known from the staged keys alone (each key's row is written by
    // exactly one run close in the launch: a run cut by a chunk edge goes to the head / tail slots instead), so
    // they are loaded together with the batch's gradient rows: one memory round trip per batch, not two
    for (int h0 = 0; h0 < cnt; h0 += SEG_U) {
      int kind[SEG_U];  // as in process(): 0 nothing closes / 1 out[key] += / 2 head / 3 tail / 4 bad key
      bool closes[SEG_U];
#pragma unroll
      for (int u = 0; u < SEG_U; ++u) {
        const int q = h0 + u;
        kind[u] = 0;
        closes[u] = q < cnt && (q == cnt - 1 || sk[o + q + 2] != sk[o + q + 1]);
        if (closes[u]) {
          const uint32_t key = sk[o + q + 1];
          if (first && cont_head)
            kind[u] = 2;
          else if (q == cnt - 1 && cont_tail)
            kind[u] = 3;
          else if (key >= (uint32_t)J.n_out)
            kind[u] = 4;
          else if ((int)key != J.skip_key)
            kind[u] = 1;
          first = false;
        }
      }
      float4 x[SEG_U], prev[SEG_U];
      load(x, h0);
#pragma unroll
      for (int u = 0; u < SEG_U; ++u) {
        const long off = (long)sk[o + h0 + u + 1] * d + c;
        prev[u] = kind[u] != 1 ? c2::f4(0.f) : (J.out16 ? c2::ld4(J.out16 + off) : *(const float4*)(J.out + off));
      }
#pragma unroll
      for (int u = 0; u < SEG_U; ++u) {
        if (h0 + u < cnt) {
          acc = acc + x[u];
          if (closes[u]) {
            x[u] = acc;
            acc = c2::f4(0.f);
          }
        }
      }
#pragma unroll
      for (int u = 0; u < SEG_U; ++u) {
        if (kind[u] == 1) {
          const long off = (long)sk[o + h0 + u + 1] * d + c;
          if (J.out16)
            c2::st4(J.out16 + off, prev[u] + x[u]);
          else
            *(float4*)(J.out + off) = prev[u] + x[u];
        } else if (kind[u] == 2)
          *(float4*)(J.ph + chunk * d + c) = x[u];
        else if (kind[u] == 3)
          *(float4*)(J.pt + chunk * d + c) = x[u];
        else if (kind[u] == 4 && lane == 0)
          atomicOr(J.err, 2);
      }
    }
    (void)process;
#elif SEG_PIPE
    // the next batch's rows are in flight while this batch's runs are read-modify-written (rows and out
    // are different buffers; a run that closes in a batch never reappears in a later one)
    float4 xa[SEG_U], xb[SEG_U];
    load(xa, 0);
    for (int h0 = 0; h0 < cnt; h0 += 2 * SEG_U) {
      if (h0 + SEG_U < cnt) load(xb, h0 + SEG_U);
      process(xa, h0);
      if (h0 + SEG_U >= cnt) break;
      if (h0 + 2 * SEG_U < cnt) load(xa, h0 + 2 * SEG_U);
      process(xb, h0 + SEG_U);
    }
#else
    for (int h0 = 0; h0 < cnt; h0 += SEG_U) {
      float4 x[SEG_U];
      load(x, h0);
      process(x, h0);
    }
#endif
  }
}

// the job of a pass-B block (blockIdx.y), field by field (uniform selects; no struct copy)
struct SplitView {
  const int4* splits;
  const int2* subs;
  const int* suboff;
  const int* counts;
  int* scnt;
  int* err;
  int n, n_out, skip_key, d;
  float* out;
  const float *ph, *pt;
  float* slot2;
  c2::tbf16* out16;
  __device__ __forceinline__ SplitView(const SegJob& j0, const SegJob& j1, bool y)
      : splits(y ? j1.splits : j0.splits), subs(y ? j1.subs : j0.subs), suboff(y ? j1.suboff : j0.suboff),
        counts(y ? j1.counts : j0.counts), scnt(y ? j1.scnt : j0.scnt), err(y ? j1.err : j0.err), n(y ? j1.n : j0.n),
        n_out(y ? j1.n_out : j0.n_out), skip_key(y ? j1.skip_key : j0.skip_key), d(y ? j1.src.d : j0.src.d),
        out(y ? j1.out : j0.out), ph(y ? j1.ph : j0.ph), pt(y ? j1.pt : j0.pt), slot2(y ? j1.slot2 : j0.slot2),
        out16(y ? j1.out16 : j0.out16) {}
  __device__ __forceinline__ int nchunks() const { return (n + SEG_CH - 1) / SEG_CH; }
  __device__ __forceinline__ int max_sub() const { return nchunks() + 2 + n / (SEG_CH * SUBP); }
};

// pass B, level 1: one block per sub-range of SUBP pieces of a split (grid-stride over the plan's
// sub list, blockIdx.y = job): the pieces (tail of the split's first chunk, heads of the following
// ones) are dealt round-robin to the block's lane groups (eight loads in flight each), the group
// sums added in group order → slot2[sub].  Level 2 (SEG_MERGE, since round 6: in the same launch, by the
// block that finishes the split's last sub-range; else seg_split2_kernel): the split's level-1 sums in sub order
// onto out[key].  Fixed orders → deterministic; a padding run of thousands of pieces is spread over many blocks.
template <int LPR, int ROLE = 0>
__global__ __launch_bounds__(1024) void seg_split1_kernel(SegJob j0, SegJob j1) {
  constexpr int GROUPS = 1024 / LPR;
  extern __shared__ __attribute__((aligned(16))) float red[];  // [GROUPS][d]
  __shared__ int s_last;  // (SEG_MERGE) this block finished the last sub-range of its split
  const SplitView J(j0, j1, blockIdx.y != 0);
  const int g = threadIdx.x / LPR;
  const int lane = threadIdx.x % LPR;
  const int d = J.d, nchunks = J.nchunks();
  const int nsub = J.counts[2], nsplit = J.counts[1];
  if (nsub < 0 || nsub > J.max_sub() || nsplit < 0 || nsplit > nchunks) {
    if (threadIdx.x == 0) atomicOr(J.err, 4);
    return;
  }
  for (int j = blockIdx.x; j < nsub; j += gridDim.x) {
    const int2 sb = J.subs[j];  // (split, first piece of this sub-range)
    const int si = min(max(sb.x, 0), max(nsplit - 1, 0));
    const int4 sp = J.splits[si];
    const int chunk = sp.y, np = sp.z;
    const int q_lo = sb.y, q_hi = min(np, sb.y + SUBP);
    if (sb.x != si || chunk < 0 || np < 2 || chunk + np > nchunks || q_lo < 0 || q_lo >= q_hi) {  // uniform
      if (threadIdx.x == 0) atomicOr(J.err, 8);
      continue;
    }
    const float* tail0 = J.pt + (long)chunk * d;
    const float* head0 = J.ph + (long)chunk * d;
    for (int c = lane * 4; c < d; c += LPR * 4) {
      float4 a[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) a[u] = c2::f4(0.f);
      int q = q_lo + g;
      for (; q + 7 * GROUPS < q_hi; q += 8 * GROUPS) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int qq = q + u * GROUPS;
          a[u] = a[u] + *(const float4*)((qq == 0 ? tail0 : head0 + (long)qq * d) + c);
        }
      }
      for (; q < q_hi; q += GROUPS) a[0] = a[0] + *(const float4*)((q == 0 ? tail0 : head0 + (long)q * d) + c);
      *(float4*)(red + g * d + c) = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
    }
    __syncthreads();
    // level 2 in the same launch (SEG_MERGE): out[key] += the split's level-1 sums in sub order — the order
    // seg_split2_kernel used, so the same bits.  A split of ONE sub-range (all but the hottest keys) is finished here
    // from the sum just computed; a longer one by its LAST sub-range to finish, through the guide's counter hand-off
    // (MI355X_MICROARCH.md §Workgroup dispatch…, cdna_hip_programming.md §6 G16): every wave drains its slot2 stores,
    // barrier, lane 0 releases at agent scope (then waits itself: the fence's own wait can be dropped) and takes a
    // ticket from the plan's per-split counter; the last one acquires at agent scope before the barrier that lets its
    // waves read the other sub-ranges' sums, and puts the counter back to 0 for the plan's next use.
    const int key = sp.x, b0 = J.suboff[si], b1 = J.suboff[si + 1];
    const bool bad2 = key < 0 || key >= J.n_out || b0 < 0 || b1 <= b0 || b1 > nsub;
    const bool direct = SEG_MERGE && b1 - b0 == 1;
    for (int c = threadIdx.x * 4; c < d; c += 1024 * 4) {
      float4 t = *(const float4*)(red + c);
      for (int q = 1; q < GROUPS; ++q) t = t + *(const float4*)(red + q * d + c);
      if (!direct) {
        *(float4*)(J.slot2 + (long)j * d + c) = t;
      } else if (!bad2 && key != J.skip_key) {
        const long o = (long)key * d;
        const float4 u = J.out16 ? c2::ld4(J.out16 + o + c) : *(const float4*)(J.out + o + c);
        if (J.out16)
          c2::st4(J.out16 + o + c, u + t);
        else
          *(float4*)(J.out + o + c) = u + t;
      }
    }
    if (direct && bad2 && threadIdx.x == 0) atomicOr(J.err, 8);
#if SEG_MERGE
    if (!direct) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const bool last = !bad2 && __hip_atomic_fetch_add(J.scnt + si, 1, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT) == b1 - b0 - 1;
        if (last) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        if (bad2) atomicOr(J.err, 8);
        s_last = last;
      }
      __syncthreads();
      if (s_last) {
        if (key != J.skip_key) {
          const long o = (long)key * d;
          for (int c = threadIdx.x * 4; c < d; c += 1024 * 4) {
            float4 t = J.out16 ? c2::ld4(J.out16 + o + c) : *(const float4*)(J.out + o + c);
            for (int k = b0; k < b1; ++k) t = t + *(const float4*)(J.slot2 + (long)k * d + c);
            if (J.out16)
              c2::st4(J.out16 + o + c, t);
            else
              *(float4*)(J.out + o + c) = t;
          }
        }
        if (threadIdx.x == 0) J.scnt[si] = 0;
      }
    }
#endif
    __syncthreads();
  }
}

template <int LPR, int ROLE = 0>
__global__ __launch_bounds__(256) void seg_split2_kernel(SegJob j0, SegJob j1) {
  constexpr int GROUPS = 256 / LPR;
  const SplitView J(j0, j1, blockIdx.y != 0);
  const int lane = threadIdx.x % LPR;
  const int d = J.d, nchunks = J.nchunks();
  const int nsplit = J.counts[1], nsub = J.counts[2];
  if (nsplit < 0 || nsplit > nchunks || nsub < 0 || nsub > J.max_sub()) {
    if (threadIdx.x == 0) atomicOr(J.err, 4);
    return;
  }
  for (int j = blockIdx.x * GROUPS + threadIdx.x / LPR; j < nsplit; j += gridDim.x * GROUPS) {
    const int key = J.splits[j].x;
    const int b0 = J.suboff[j], b1 = J.suboff[j + 1];
    if (key < 0 || key >= J.n_out || b0 < 0 || b1 <= b0 || b1 > nsub) {
      if (lane == 0) atomicOr(J.err, 8);
      continue;
    }
    if (key == J.skip_key) continue;
    const long o = (long)key * d;
    for (int c = lane * 4; c < d; c += LPR * 4) {
      float4 t = J.out16 ? c2::ld4(J.out16 + o + c) : *(const float4*)(J.out + o + c);
      for (int k = b0; k < b1; ++k) t = t + *(const float4*)(J.slot2 + (long)k * d + c);
      if (J.out16)
        c2::st4(J.out16 + o + c, t);
      else
        *(float4*)(J.out + o + c) = t;
    }
  }
}

__global__ void drop_scale_kernel(const float* __restrict__ gX, long n4, int d, c2::Drop drop, int64_t idx_base,
                                  float* __restrict__ out) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  float4 v = ((const float4*)gX)[i];
  if (drop.active()) {
    const uint64_t b = (uint64_t)idx_base * d + (uint64_t)i * 4;
    v = v * drop.mul4(b);
  }
  ((float4*)out)[i] = v;
}

// out[c] += T[c][0] for c < n  (T [n][4], the d = 4 segment sums of the (w_r, 0, 0, 0) rows)
__global__ void col0_add_kernel(const float* __restrict__ T, int n, float* __restrict__ out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < n) out[c] += T[4 * (long)c];
}

// err |= bit if any idx[r·ld + ld - cols + c] (r < rows, c < cols) lies outside [0, hi)
__global__ __launch_bounds__(256) void index_check_kernel(const int64_t* __restrict__ idx, long rows, int ld, int cols,
                                                          int64_t hi, int bit, int* __restrict__ err) {
  const long n = rows * cols;
  bool bad = false;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long r = i / cols;
    const int64_t v = idx[r * ld + (ld - cols) + (i - r * cols)];
    bad |= v < 0 || v >= hi;
  }
  if (__ballot(bad) && (threadIdx.x & 63) == 0) atomicOr(err, bit);
}

int lpr_for(int d) { return d / 4 >= 64 ? 64 : (d / 4 >= 32 ? 32 : (d / 4 >= 16 ? 16 : (d / 4 >= 8 ? 8 : 4))); }

size_t align256(size_t b) { return (b + 255) & ~size_t(255); }

// A plan: keys[n] (sorted ids) | rows[n] | splits[n/SEG_CH+1] int4 | counts[4] = (-, splits, subs,
// error word) | suboff[n/SEG_CH+2] | subs[max_subs] int2 | scratch (second
// LSD buffers, digit histograms, plan block counts).
struct Plan {
  uint32_t *k0, *v0;
  int4* splits;
  int* counts;
  int* suboff;
  int2* subs;
  uint32_t *k1, *v1, *hist, *bcnt;
  int* scnt;
  int nblocks;
};

// sub-ranges of SUBP pieces over all splits: at most one per split plus one per SUBP chunks
int max_subs(int n) { return n / SEG_CH + 2 + n / (SEG_CH * SUBP) + 1; }

size_t plan_layout(int n, Plan* p, char* base) {
  const int nblocks = c2::ceil_div(n, RS_TILE);
  const int pb = c2::ceil_div(n, PL_B);
  size_t off = 0;
  auto take = [&](size_t bytes) {
    size_t o = off;
    off += align256(bytes);
    return base ? base + o : nullptr;
  };
  char* k0 = take((size_t)n * 4);
  char* v0 = take((size_t)n * 4);
  char* sp = take((size_t)(n / SEG_CH + 1) * 16);
  char* ct = take(16);
  char* so = take((size_t)(n / SEG_CH + 2) * 4);
  char* sb = take((size_t)max_subs(n) * 8);
  char* k1 = take((size_t)n * 4);
  char* v1 = take((size_t)n * 4);
  char* hist = take((size_t)256 * nblocks * 4);
  char* bc = take((size_t)pb * 8);  // per plan block: split count, sub count
  char* sc = take((size_t)(n / SEG_CH + 1) * 4);  // per split: pass B arrivals (plan_emit zeroes them)
  if (p)
    *p = Plan{(uint32_t*)k0, (uint32_t*)v0, (int4*)sp, (int*)ct, (int*)so, (int2*)sb,
              (uint32_t*)k1, (uint32_t*)v1, (uint32_t*)hist, (uint32_t*)bc, (int*)sc, nblocks};
  return off;
}

Plan plan_view(const void* base, int n) {
  Plan p;
  plan_layout(n, &p, (char*)base);
  return p;
}

// head/tail partial slots of the segment sums, then the error word
size_t seg_slot_bytes(int n, int d) { return align256((size_t)c2::ceil_div(n, SEG_CH) * d * 4); }
size_t seg_slot2_bytes(int n, int d) { return align256((size_t)max_subs(n) * d * 4); }
size_t seg_ws_bytes(int n, int d) { return 2 * seg_slot_bytes(n, d) + seg_slot2_bytes(n, d); }

// sort idx[0..n) (values < n_keys) → k0/v0 sorted (key, original row), stable; then the work lists.  Several
// plans at once: one launch per pass over all of them (PlanJobs; groups of PJ_MAX).
struct PlanSpec {
  const int64_t* idx;
  int n, n_keys;
  Plan w;
};

void build_plan_group(const PlanSpec* js, int m, hipStream_t s, int* err) {
  uint32_t *ki[PJ_MAX], *vi[PJ_MAX], *ko[PJ_MAX], *vo[PJ_MAX];
  int passes[PJ_MAX], max_passes = 0;
  PlanJobs P{};
  int b = 0;
  for (int k = 0; k < m; ++k) {
    const Plan& w = js[k].w;
    int bits = 1;
    while ((1l << bits) < (long)js[k].n_keys + 1) ++bits;  // keys 0 .. n_keys (n_keys: an out-of-range index)
    passes[k] = (bits + 7) / 8;
    max_passes = std::max(max_passes, passes[k]);
    // the passes alternate between the two buffer pairs: start in the pair the last pass does not write
    const bool odd = passes[k] & 1;
    ki[k] = odd ? w.k1 : w.k0, vi[k] = odd ? w.v1 : w.v0, ko[k] = odd ? w.k0 : w.k1, vo[k] = odd ? w.v0 : w.v1;
    P.beg[k] = b;
    P.n[k] = js[k].n;
    P.aux[k] = js[k].n_keys;
    P.idx[k] = js[k].idx;
    P.ki[k] = ki[k];
    P.vi[k] = vi[k];
    b += c2::ceil_div(js[k].n, 256);
  }
  P.nj = m;
  for (int k = m; k <= PJ_MAX; ++k) P.beg[k] = b;
  prep_keys_kernel<<<b, 256, 0, s>>>(P, C2DSR_IDX_ERR_PLAN, err);
  for (int p = 0; p < max_passes; ++p) {
    PlanJobs Q{};
    Q.shift = 8 * p;
    int q = 0;
    b = 0;
    for (int k = 0; k < m; ++k) {
      if (passes[k] <= p) continue;
      Q.beg[q] = b;
      Q.n[q] = js[k].n;
      Q.aux[q] = js[k].w.nblocks;
      Q.ki[q] = ki[k], Q.vi[q] = vi[k], Q.ko[q] = ko[k], Q.vo[q] = vo[k];
      Q.hist[q] = js[k].w.hist;
      b += js[k].w.nblocks;
      std::swap(ki[k], ko[k]);
      std::swap(vi[k], vo[k]);
      ++q;
    }
    Q.nj = q;
    for (int k = q; k <= PJ_MAX; ++k) Q.beg[k] = b;
    rs_hist_kernel<<<b, RS_THREADS, 0, s>>>(Q);
    rs_scatter_kernel<<<b, RS_THREADS, 0, s>>>(Q);
  }
  PlanJobs C{};
  b = 0;
  for (int k = 0; k < m; ++k) {
    const Plan& w = js[k].w;
    C.beg[k] = b;
    C.n[k] = js[k].n;
    C.ki[k] = w.k0;  // (the start pair makes the last pass land in k0 / v0)
    C.hist[k] = w.bcnt;
    C.splits[k] = w.splits;
    C.suboff[k] = w.suboff;
    C.subs[k] = w.subs;
    C.counts[k] = w.counts;
    C.scnt[k] = w.scnt;
    b += c2::ceil_div(js[k].n, PL_B);
  }
  C.nj = m;
  for (int k = m; k <= PJ_MAX; ++k) C.beg[k] = b;
  plan_count_kernel<<<b, PL_T, 0, s>>>(C);
  plan_emit_kernel<<<b, PL_T, 0, s>>>(C);
}

int build_plans(const PlanSpec* js, int count, hipStream_t s, int* err) {
  PlanSpec g[PJ_MAX];
  int m = 0;
  for (int k = 0; k < count; ++k) {
    if (js[k].n == 0) continue;  // nothing to sort (no launch reads such a plan)
    g[m++] = js[k];
    if (m == PJ_MAX) {
      build_plan_group(g, m, s, err);
      m = 0;
    }
  }
  if (m) build_plan_group(g, m, s, err);
  C2_CHECK_LAUNCH();
  return 0;
}

int build_plan(const int64_t* idx, int n, int n_keys, const Plan& w, hipStream_t s, int* err = nullptr) {
  const PlanSpec j{idx, n, n_keys, w};
  return build_plans(&j, 1, s, err);
}

int g_ncu = 0;
int num_cus() {
  if (!g_ncu) {
    int dev = 0, v = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev);
    g_ncu = v > 0 ? v : 256;
  }
  return g_ncu;
}

template <int LPR, int ROLE>
void seg_launch(SegJob j0, SegJob j1, int njobs, hipStream_t s) {
  constexpr int GROUPS = 256 / LPR;
  j0.nblocks = c2::ceil_div(c2::ceil_div(j0.n, SEG_CH), GROUPS);  // one lane group per chunk
  j1.nblocks = njobs > 1 ? c2::ceil_div(c2::ceil_div(j1.n, SEG_CH), GROUPS) : 0;
  seg_chunk_kernel<LPR, ROLE><<<j0.nblocks + j1.nblocks, 256, 0, s>>>(j0, j1);
  const int nmax = std::max(j0.n, njobs > 1 ? j1.n : 0);
  if (nmax > SEG_CH) {
    dim3 g1(std::max(1, std::min(max_subs(nmax), 2 * num_cus())), njobs);
    seg_split1_kernel<LPR, ROLE><<<g1, 1024, (size_t)(1024 / LPR) * j0.src.d * 4, s>>>(j0, j1);
    if (!SEG_MERGE) {
      dim3 g2(std::max(1, std::min(c2::ceil_div(c2::ceil_div(nmax, SEG_CH), GROUPS), 2 * num_cus())), njobs);
      seg_split2_kernel<LPR, ROLE><<<g2, 256, 0, s>>>(j0, j1);
    }
  }
}

// out[key] += Σ src rows of each run of the plan (keys < n_out); partial slots from ws
SegJob seg_job(const Plan& p, int n, int n_out, const RowSrc& src, float* out, char* ws, int skip_key) {
  SegJob j;
  j.K = p.k0;
  j.V = p.v0;
  j.splits = p.splits;
  j.subs = p.subs;
  j.suboff = p.suboff;
  j.counts = p.counts;
  j.scnt = p.scnt;
  j.err = p.counts + 3;
  j.n = n;
  j.n_out = n_out;
  j.skip_key = skip_key;
  j.nblocks = 0;
  j.src = src;
  j.out = out;
  j.out16 = nullptr;
  j.ph = (float*)ws;
  j.pt = (float*)(ws + seg_slot_bytes(n, src.d));
  j.slot2 = (float*)(ws + 2 * seg_slot_bytes(n, src.d));
  return j;
}

// one or two jobs of the same row width in one launch per pass
template <int ROLE = 0>
void seg_dispatch(const SegJob& j0, const SegJob* j1, hipStream_t s) {
  const SegJob& b = j1 ? *j1 : j0;
  const int nj = j1 ? 2 : 1;
  switch (lpr_for(j0.src.d)) {
    case 64: seg_launch<64, ROLE>(j0, b, nj, s); break;
    case 32: seg_launch<32, ROLE>(j0, b, nj, s); break;
    case 16: seg_launch<16, ROLE>(j0, b, nj, s); break;
    case 8: seg_launch<8, ROLE>(j0, b, nj, s); break;
    default: seg_launch<4, ROLE>(j0, b, nj, s); break;
  }
}

}  // namespace

C2_API int c2dsr_embed_fwd(const int64_t* seq, const int64_t* pos, int n_rows, int d, const float* H, const float* E,
                           const float* Xin, const float* P, float scale, uint32_t k0, uint32_t k1, float p,
                           int64_t idx_base, float* X, int n_items, int n_pos, int* err, void* stream) {
  if (d % 4 || n_rows <= 0) return n_rows == 0 ? 0 : (int)hipErrorInvalidValue;
  if (n_pos <= 0 || (!Xin && n_items <= 0)) return (int)hipErrorInvalidValue;
  c2::Drop dr = c2::make_drop(k0, k1, p);
  hipStream_t s = (hipStream_t)stream;
  const int lpr = lpr_for(d);
  dim3 grid(c2::ceil_div(n_rows, 256 / lpr));
  const bool gather = Xin == nullptr;
#define C2_EMB(L)                                                                                                  \
  if (gather)                                                                                                      \
    embed_fwd_kernel<L, true><<<grid, 256, 0, s>>>(seq, pos, n_rows, d, H, E, Xin, P, scale, dr, idx_base, X,      \
                                                   n_items, n_pos, err);                                           \
  else                                                                                                             \
    embed_fwd_kernel<L, false><<<grid, 256, 0, s>>>(seq, pos, n_rows, d, H, E, Xin, P, scale, dr, idx_base, X,     \
                                                    n_items, n_pos, err);
  switch (lpr) {
    case 64: C2_EMB(64) break;
    case 32: C2_EMB(32) break;
    case 16: C2_EMB(16) break;
    case 8: C2_EMB(8) break;
    default: C2_EMB(4) break;
  }
#undef C2_EMB
  C2_CHECK_LAUNCH();
  return 0;
}

C2_API int c2dsr_embed_fwd_rows(const int64_t* seq, const int64_t* pos, int n_rows, int d, const float* H,
                                const float* E, const float* P, float scale, uint32_t k0, uint32_t k1, float p,
                                int64_t idx_base, const int* q_idx, int nq, const int* k_idx, int nk, float* X,
                                int n_items, int n_pos, int* err, void* stream) {
  if (d % 4 || nq < 0 || nk < 0 || !H || !E || !P || n_items <= 0 || n_pos <= 0) return (int)hipErrorInvalidValue;
  if (nq + nk == 0 || n_rows <= 0) return 0;
  c2::Drop dr = c2::make_drop(k0, k1, p);
  hipStream_t s = (hipStream_t)stream;
  const int lpr = lpr_for(d);
  dim3 grid(c2::ceil_div(nq + nk, 256 / lpr));
#define C2_EMB(L)                                                                                                    \
  embed_fwd_rows_kernel<L><<<grid, 256, 0, s>>>(seq, pos, n_rows, d, H, E, P, scale, dr, idx_base, q_idx, nq, k_idx, \
                                                nk, X, n_items, n_pos, err);
  switch (lpr) {
    case 64: C2_EMB(64) break;
    case 32: C2_EMB(32) break;
    case 16: C2_EMB(16) break;
    case 8: C2_EMB(8) break;
    default: C2_EMB(4) break;
  }
#undef C2_EMB
  C2_CHECK_LAUNCH();
  return 0;
}

C2_API int c2dsr_index_check(const int64_t* idx, long rows, int ld, int cols, int64_t hi, int bit, int* err,
                             void* stream) {
  if (rows < 0 || ld <= 0 || cols < 0 || cols > ld || !err) return (int)hipErrorInvalidValue;
  const long n = rows * cols;
  if (n == 0) return 0;
  const int blocks = (int)std::min<long>(c2::ceil_div(n, 256), 1024);
  index_check_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(idx, rows, ld, cols, hi, bit, err);
  C2_CHECK_LAUNCH();
  return 0;
}

C2_API size_t c2dsr_index_plan_bytes(int n) { return plan_layout(n, nullptr, nullptr); }

// Sort plan of an index array: plan = [keys u32 n | rows u32 n | scratch], keys ascending and
// rows ascending within equal keys (stable LSD radix sort).  Depends on the indices only, so
// the host builds it as soon as a batch's index tensors exist (on a side stream, under the
// forward pass) and the backward's segment sums consume it.
C2_API int c2dsr_index_plan(const int64_t* idx, int n, int n_keys, void* plan, size_t plan_bytes, int* err,
                            void* stream) {
  if (n < 0 || n_keys <= 0 || n_keys >= 0x7fffffff) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  Plan p;
  if (plan_bytes < plan_layout(n, &p, (char*)plan)) return (int)hipErrorInvalidValue;
  return build_plan(idx, n, n_keys, p, (hipStream_t)stream, err);
}

// c2dsr_index_plan over several index tensors, one launch per pass for all of them: desc = HOST array of count
// records of five int64 (idx, n, n_keys, plan, plan_bytes)
C2_API int c2dsr_index_plans(const int64_t* desc, int count, int* err, void* stream) {
  if (count < 0 || (count && !desc)) return (int)hipErrorInvalidValue;
  std::vector<PlanSpec> js;
  js.reserve(count);
  for (int k = 0; k < count; ++k) {
    const int64_t* r = desc + 5 * k;
    const int64_t n = r[1], n_keys = r[2];
    if (n < 0 || n > 0x7fffffff || n_keys <= 0 || n_keys >= 0x7fffffff || (n && (!r[0] || !r[3])))
      return (int)hipErrorInvalidValue;
    PlanSpec j{(const int64_t*)(uintptr_t)r[0], (int)n, (int)n_keys, Plan{}};
    const size_t need = plan_layout((int)n, &j.w, (char*)(uintptr_t)r[3]);
    if (n && (r[4] < 0 || (size_t)r[4] < need)) return (int)hipErrorInvalidValue;  // (an empty job writes nothing)
    js.push_back(j);
  }
  return build_plans(js.data(), count, (hipStream_t)stream, err);
}

// two segment-sum jobs (items, positions) run side by side: two slot regions
C2_API size_t c2dsr_embed_bwd_planned_workspace(int n_rows, int d) { return 2 * seg_ws_bytes(n_rows, d); }

// offset of a plan's device error word (nonzero once a segment sum met an inconsistent plan)
C2_API size_t c2dsr_plan_err_offset(int n) {
  Plan p;
  char* const base = reinterpret_cast<char*>(uintptr_t{4096});  // any non-null base: offsets only
  plan_layout(n, &p, base);
  return (size_t)(reinterpret_cast<char*>(p.counts + 3) - base);
}

// gX: grad w.r.t. the dropout output X [n_rows, d]; seq_plan / pos_plan from c2dsr_index_plan.
//   G[seq[r]]  += scale * drop(gX[r])            (G dense [n_items, d]; skipped if G null)
//   gP[pos[r]] += drop(gX[r])                     (gP dense [n_pos, d]; skipped if null)
//   gXin[r]     = drop(gX[r])                     (optional, for the non-gather mode)
// The item and position sums share one launch of each pass.
static int embed_bwd_planned_impl(const void* seq_plan, const void* pos_plan, int n_rows, int d, const float* gX,
                                  const int* map1, const float* gX2, const int* map2, uint32_t k0, uint32_t k1,
                                  float p, int64_t idx_base, float scale, float* G, int n_items, float* gP, int n_pos,
                                  float* gXin, void* workspace, size_t ws_bytes, void* stream,
                                  c2::tbf16* G16 = nullptr) {
  if (d % 4) return (int)hipErrorInvalidValue;
  if (n_rows == 0) return 0;
  if (ws_bytes < c2dsr_embed_bwd_planned_workspace(n_rows, d) || ((G || G16) && !seq_plan) || (gP && !pos_plan))
    return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  c2::Drop dr = c2::make_drop(k0, k1, p);
  char* ws = (char*)workspace;
  SegJob jobs[2];
  int nj = 0;
  if (G || G16) {
    jobs[nj] = seg_job(plan_view(seq_plan, n_rows), n_rows, n_items,
                       RowSrc{gX, d, dr, idx_base, scale, nullptr, map1, map2, gX2}, G, ws, -1);
    jobs[nj++].out16 = G16;
  }
  if (gP)
    jobs[nj++] = seg_job(plan_view(pos_plan, n_rows), n_rows, n_pos,
                         RowSrc{gX, d, dr, idx_base, 1.0f, nullptr, map1, map2, gX2}, gP,
                         ws + seg_ws_bytes(n_rows, d), -1);
  if (nj) seg_dispatch(jobs[0], nj > 1 ? &jobs[1] : nullptr, s);
  if (gXin) {
    long n4 = (long)n_rows * d / 4;
    drop_scale_kernel<<<c2::ceil_div(n4, 256), 256, 0, s>>>(gX, n4, d, dr, idx_base, gXin);
  }
  C2_CHECK_LAUNCH();
  return 0;
}

C2_API int c2dsr_embed_bwd_planned(const void* seq_plan, const void* pos_plan, int n_rows, int d, const float* gX,
                                   uint32_t k0, uint32_t k1, float p, int64_t idx_base, float scale, float* G,
                                   int n_items, float* gP, int n_pos, float* gXin, void* workspace, size_t ws_bytes,
                                   void* stream) {
  return embed_bwd_planned_impl(seq_plan, pos_plan, n_rows, d, gX, nullptr, nullptr, nullptr, k0, k1, p, idx_base,
                                scale, G, n_items, gP, n_pos, gXin, workspace, ws_bytes, stream);
}

// bf16 item tables (the C5 roofline run): the gather reads bf16 H / E rows, the item segment
// sums read-modify-write a bf16 G (fp32 sums, RNE store); P, X, gX, gP stay fp32
C2_API int c2dsr_embed_fwd_b16(const int64_t* seq, const int64_t* pos, int n_rows, int d, const void* H, const void* E,
                               const float* P, float scale, uint32_t k0, uint32_t k1, float p, int64_t idx_base,
                               float* X, int n_items, int n_pos, int* err, void* stream) {
  if (d % 4 || n_rows <= 0 || !H || !E) return n_rows == 0 ? 0 : (int)hipErrorInvalidValue;
  if (n_items <= 0 || n_pos <= 0) return (int)hipErrorInvalidValue;
  c2::Drop dr = c2::make_drop(k0, k1, p);
  hipStream_t s = (hipStream_t)stream;
  const int lpr = lpr_for(d);
  dim3 grid(c2::ceil_div(n_rows, 256 / lpr));
  const c2::tbf16 *Hb = (const c2::tbf16*)H, *Eb = (const c2::tbf16*)E;
#define C2_EMB(L) \
  embed_fwd_kernel<L, true, c2::tbf16><<<grid, 256, 0, s>>>(seq, pos, n_rows, d, Hb, Eb, nullptr, P, scale, dr, idx_base, X, \
                                                            n_items, n_pos, err);
  switch (lpr) {
    case 64: C2_EMB(64) break;
    case 32: C2_EMB(32) break;
    case 16: C2_EMB(16) break;
    case 8: C2_EMB(8) break;
    default: C2_EMB(4) break;
  }
#undef C2_EMB
  C2_CHECK_LAUNCH();
  return 0;
}
C2_API int c2dsr_embed_bwd_planned_b16(const void* seq_plan, const void* pos_plan, int n_rows, int d, const float* gX,
                                       uint32_t k0, uint32_t k1, float p, int64_t idx_base, float scale, void* G,
                                       int n_items, float* gP, int n_pos, void* workspace, size_t ws_bytes,
                                       void* stream) {
  if (!G) return (int)hipErrorInvalidValue;
  return embed_bwd_planned_impl(seq_plan, pos_plan, n_rows, d, gX, nullptr, nullptr, nullptr, k0, k1, p, idx_base,
                                scale, nullptr, n_items, gP, n_pos, nullptr, workspace, ws_bytes, stream,
                                (c2::tbf16*)G);
}

// the same with gX given as two compact row sources: row r = (inv_a[r] >= 0 ? gXa[inv_a[r]] : 0)
// + (inv_b[r] >= 0 ? gXb[inv_b[r]] : 0)
C2_API int c2dsr_embed_bwd_planned_rows(const void* seq_plan, const void* pos_plan, int n_rows, int d,
                                        const float* gXa, const int* inv_a, const float* gXb, const int* inv_b,
                                        uint32_t k0, uint32_t k1, float p, int64_t idx_base, float scale, float* G,
                                        int n_items, float* gP, int n_pos, void* workspace, size_t ws_bytes,
                                        void* stream) {
  if (!gXa || !inv_a || !gXb || !inv_b || d < 64) return (int)hipErrorInvalidValue;
  return embed_bwd_planned_impl(seq_plan, pos_plan, n_rows, d, gXa, inv_a, gXb, inv_b, k0, k1, p, idx_base, scale,
                                G, n_items, gP, n_pos, nullptr, workspace, ws_bytes, stream);
}

C2_API size_t c2dsr_embed_bwd_workspace(int n_rows, int d) {
  return 2 * align256(plan_layout(n_rows, nullptr, nullptr)) + c2dsr_embed_bwd_planned_workspace(n_rows, d);
}

// unplanned form: both plans built inside, then the planned backward
C2_API int c2dsr_embed_bwd(const int64_t* seq, const int64_t* pos, int n_rows, int d, const float* gX, uint32_t k0,
                           uint32_t k1, float p, int64_t idx_base, float scale, float* G, int n_items, float* gP,
                           int n_pos, float* gXin, void* workspace, size_t ws_bytes, void* stream) {
  if (d % 4) return (int)hipErrorInvalidValue;
  if (n_rows == 0) return 0;
  if (ws_bytes < c2dsr_embed_bwd_workspace(n_rows, d)) return (int)hipErrorInvalidValue;
  const size_t pb = align256(plan_layout(n_rows, nullptr, nullptr));
  char* sp = (char*)workspace;
  char* pp = sp + pb;
  char* seg = pp + pb;
  int e;
  if (G && (e = c2dsr_index_plan(seq, n_rows, n_items, sp, pb, nullptr, stream))) return e;
  if (gP && (e = c2dsr_index_plan(pos, n_rows, n_pos, pp, pb, nullptr, stream))) return e;
  return c2dsr_embed_bwd_planned(G ? sp : nullptr, gP ? pp : nullptr, n_rows, d, gX, k0, k1, p, idx_base, scale, G,
                                 n_items, gP, n_pos, gXin, seg, c2dsr_embed_bwd_planned_workspace(n_rows, d), stream);
}

C2_API size_t c2dsr_ce_onehot_planned_workspace(int M, int n, int D) {
  return seg_ws_bytes(M, D) + align256((size_t)n * 16);
}

// The one-hot part of the classifier-head gradient (trainer.py:131-154 via F.cross_entropy):
//   gW[t_r] -= rw_r·H[r],  gb[t_r] -= rw_r   for rows with 0 <= t_r < n (t_r = n is ignore_index)
// over the target plan (c2dsr_index_plan of tgt with n_keys = n + 1): each target's run is reduced
// in row order (deterministic); the bias part runs the same segment reduction over the rows
// (rw_r, 0, 0, 0).
C2_API int c2dsr_ce_onehot_dw_planned(const void* plan, int M, int n, const float* H, int D, const float* rw,
                                      float* gW, float* gb, void* workspace, size_t ws_bytes, void* stream) {
  if (D % 4) return (int)hipErrorInvalidValue;
  if (M == 0) return 0;
  if (ws_bytes < c2dsr_ce_onehot_planned_workspace(M, n, D)) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  char* seg = (char*)workspace;
  const Plan p = plan_view(plan, M);
  const c2::Drop nodrop = c2::make_drop(0, 0, 0.f);
  if (gW) {
    const SegJob j = seg_job(p, M, n + 1, RowSrc{H, D, nodrop, 0, -1.f, rw}, gW, seg, n);
    seg_dispatch<1>(j, nullptr, s);
  }
  if (gb) {
    float* T = (float*)(seg + seg_ws_bytes(M, D));
    (void)hipMemsetAsync(T, 0, (size_t)n * 16, s);
    const SegJob j = seg_job(p, M, n + 1, RowSrc{nullptr, 4, nodrop, 0, -1.f, rw}, T, seg, n);
    seg_dispatch<1>(j, nullptr, s);
    col0_add_kernel<<<c2::ceil_div(n, 256), 256, 0, s>>>(T, n, gb);
  }
  C2_CHECK_LAUNCH();
  return 0;
}

C2_API size_t c2dsr_ce_onehot_workspace(int M, int n, int D) {
  return align256(plan_layout(M, nullptr, nullptr)) + c2dsr_ce_onehot_planned_workspace(M, n, D);
}

// unplanned form: sorts the targets inside
C2_API int c2dsr_ce_onehot_dw(const int64_t* tgt, int M, int n, const float* H, int D, const float* rw, float* gW,
                              float* gb, void* workspace, size_t ws_bytes, void* stream) {
  if (D % 4) return (int)hipErrorInvalidValue;
  if (M == 0) return 0;
  if (ws_bytes < c2dsr_ce_onehot_workspace(M, n, D)) return (int)hipErrorInvalidValue;
  char* plan = (char*)workspace;
  const size_t pb = align256(plan_layout(M, nullptr, nullptr));
  int e = c2dsr_index_plan(tgt, M, n + 1, plan, pb, nullptr, stream);
  if (e) return e;
  return c2dsr_ce_onehot_dw_planned(plan, M, n, H, D, rw, gW, gb, plan + pb, ws_bytes - pb, stream);
}
