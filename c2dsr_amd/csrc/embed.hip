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

namespace {

// ------------------------------------------------------------------ forward gather
template <int LPR, bool GATHER>
__global__ __launch_bounds__(256) void embed_fwd_kernel(const int64_t* __restrict__ seq, const int64_t* __restrict__ pos,
                                                        int n_rows, int d, const float* __restrict__ H,
                                                        const float* __restrict__ E, const float* __restrict__ Xin,
                                                        const float* __restrict__ P, float scale, c2::Drop drop,
                                                        int64_t idx_base, float* __restrict__ X) {
  constexpr int GROUPS = 256 / LPR;
  const int g = threadIdx.x / LPR;
  const int lane = threadIdx.x % LPR;
  const long r = (long)blockIdx.x * GROUPS + g;
  if (r >= n_rows) return;
  const long p = pos[r];
  long s = 0;
  if (GATHER) s = seq[r];
  for (int c = lane * 4; c < d; c += LPR * 4) {
    float4 a;
    if (GATHER) {
      const float4 h = *(const float4*)(H + s * d + c);
      const float4 e = *(const float4*)(E + s * d + c);
      a = scale * (h + e);
    } else {
      a = *(const float4*)(Xin + r * d + c);
    }
    float4 x = a + *(const float4*)(P + p * d + c);
    if (drop.active()) {
      const uint64_t b = (uint64_t)(idx_base + r) * d + c;
      x = x * make_float4(drop.mul(b), drop.mul(b + 1), drop.mul(b + 2), drop.mul(b + 3));
    }
    *(float4*)(X + r * d + c) = x;
  }
}

// ------------------------------------------------------------------ radix sort (stable LSD)
constexpr int RS_THREADS = 256;
constexpr int RS_ROUNDS = 8;
constexpr int RS_TILE = RS_THREADS * RS_ROUNDS;

__global__ void prep_keys_kernel(const int64_t* __restrict__ idx, int n, uint32_t* __restrict__ keys,
                                 uint32_t* __restrict__ vals) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    keys[i] = (uint32_t)idx[i];
    vals[i] = (uint32_t)i;
  }
}

__global__ __launch_bounds__(RS_THREADS) void rs_hist_kernel(const uint32_t* __restrict__ keys, int n, int shift,
                                                            int nblocks, uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[256];
  h[threadIdx.x] = 0;
  __syncthreads();
  const int base = blockIdx.x * RS_TILE;
  for (int r = 0; r < RS_ROUNDS; ++r) {
    int i = base + r * RS_THREADS + threadIdx.x;
    if (i < n) atomicAdd(&h[(keys[i] >> shift) & 255u], 1u);
  }
  __syncthreads();
  hist[threadIdx.x * nblocks + blockIdx.x] = h[threadIdx.x];
}

// exclusive scan of m counters, single workgroup of 1024 threads
__global__ __launch_bounds__(1024) void rs_scan_kernel(uint32_t* __restrict__ hist, int m) {
  __shared__ uint32_t part[1024];
  const int t = threadIdx.x;
  const int per = (m + 1023) / 1024;
  const int lo = min(m, t * per), hi = min(m, lo + per);
  uint32_t s = 0;
  for (int i = lo; i < hi; ++i) s += hist[i];
  part[t] = s;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    uint32_t v = t >= o ? part[t - o] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint32_t run = part[t] - s;
  for (int i = lo; i < hi; ++i) {
    uint32_t c = hist[i];
    hist[i] = run;
    run += c;
  }
}

__global__ __launch_bounds__(RS_THREADS) void rs_scatter_kernel(const uint32_t* __restrict__ kin,
                                                               const uint32_t* __restrict__ vin, int n, int shift,
                                                               int nblocks, const uint32_t* __restrict__ offs,
                                                               uint32_t* __restrict__ kout,
                                                               uint32_t* __restrict__ vout) {
  __shared__ uint32_t wcnt[4][256];
  __shared__ uint32_t woff[4][256];
  __shared__ uint32_t run[256];
  __shared__ uint32_t gbase[256];
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  for (int q = 0; q < 4; ++q) wcnt[q][t] = 0;
  run[t] = 0;
  gbase[t] = offs[t * nblocks + blockIdx.x];
  __syncthreads();
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const int base = blockIdx.x * RS_TILE;
  for (int r = 0; r < RS_ROUNDS; ++r) {
    const int i = base + r * RS_THREADS + t;
    const bool act = i < n;
    uint32_t key = 0, val = 0, dg = 0;
    if (act) {
      key = kin[i];
      val = vin[i];
      dg = (key >> shift) & 255u;
    }
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

// ------------------------------------------------------------------ segment reduce
constexpr int SEG_CH = 32;

struct RowSrc {
  const float* gX;
  int d;
  c2::Drop drop;
  int64_t idx_base;
  float scale;
  const float* rs;  // optional per-row multiplier
  __device__ __forceinline__ float4 load(uint32_t r, int c) const {
    if (!gX) return make_float4(c == 0 ? (rs ? scale * rs[r] : scale) : 0.f, 0.f, 0.f, 0.f);  // the row (1, 0, …)
    float4 v = *(const float4*)(gX + (long)r * d + c);
    if (drop.active()) {
      const uint64_t b = (uint64_t)(idx_base + r) * d + c;
      v = v * make_float4(drop.mul(b), drop.mul(b + 1), drop.mul(b + 2), drop.mul(b + 3));
    }
    return (rs ? scale * rs[r] : scale) * v;
  }
};

// pass A: every chunk of SEG_CH sorted entries sums its runs; whole runs go straight to
// out[key] (+=), runs cut by a chunk edge go to head/tail partial slots.  The block stages
// its keys and row ids in LDS first (no dependent global loads in the run walk); each
// lane group streams its chunk's rows four at a time.
template <int LPR>
__global__ __launch_bounds__(256) void seg_reduce_a(const uint32_t* __restrict__ K, const uint32_t* __restrict__ V,
                                                    int n, RowSrc src, float* __restrict__ out,
                                                    float* __restrict__ part_head, float* __restrict__ part_tail,
                                                    int skip_key) {
  constexpr int GROUPS = 256 / LPR;
  constexpr int ENT = GROUPS * SEG_CH;
  __shared__ uint32_t sk[ENT + 2];  // sk[e + 1] = K[b0 + e]; sk[0], sk[ENT + 1]: the neighbours
  __shared__ uint32_t sv[ENT];
  const long b0 = (long)blockIdx.x * ENT;
  for (int e = threadIdx.x; e < ENT + 2; e += 256) {
    const long gi = b0 - 1 + e;
    sk[e] = (gi >= 0 && gi < n) ? K[gi] : 0xffffffffu;
  }
  for (int e = threadIdx.x; e < ENT; e += 256) {
    const long gi = b0 + e;
    sv[e] = gi < n ? V[gi] : 0u;
  }
  __syncthreads();
  const int g = threadIdx.x / LPR;
  const int lane = threadIdx.x % LPR;
  const long chunk = (long)blockIdx.x * GROUPS + g;
  const long start = chunk * SEG_CH;
  if (start >= n) return;
  const int cnt = (int)min((long)SEG_CH, n - start);
  const int o = g * SEG_CH;
  const bool cont_head = start > 0 && sk[o] == sk[o + 1];
  const bool cont_tail = start + cnt < n && sk[o + cnt + 1] == sk[o + cnt];
  const int d = src.d;
  for (int c = lane * 4; c < d; c += LPR * 4) {
    float4 acc = c2::f4(0.f);
    int rs = 0;  // first entry of the current run
    auto flush = [&](int q) {
      const uint32_t key = sk[o + q + 1];
      const bool head = rs == 0 && cont_head;
      const bool tail = q == cnt - 1 && cont_tail;
      if (head) {
        *(float4*)(part_head + chunk * d + c) = acc;
      } else if (tail) {
        *(float4*)(part_tail + chunk * d + c) = acc;
      } else if ((int)key != skip_key) {
        float4* dst = (float4*)(out + (long)key * d + c);
        *dst = *dst + acc;
      }
      acc = c2::f4(0.f);
      rs = q + 1;
    };
    for (int q0 = 0; q0 < cnt; q0 += 4) {
      float4 x[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) x[u] = q0 + u < cnt ? src.load(sv[o + q0 + u], c) : c2::f4(0.f);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int q = q0 + u;
        if (q < cnt) {
          acc = acc + x[u];
          if (q == cnt - 1 || sk[o + q + 2] != sk[o + q + 1]) flush(q);
        }
      }
    }
  }
}

// pass B: runs that start in chunk c and continue: out[key] += tail[c] + head[c+1] + ... .
// One block per chunk; the run's partials are dealt round-robin to the block's lane
// groups and the group sums are added in group order (fixed order → deterministic).
template <int LPR>
__global__ __launch_bounds__(1024) void seg_reduce_b(const uint32_t* __restrict__ K, int n, int d,
                                                     float* __restrict__ out, const float* __restrict__ part_head,
                                                     const float* __restrict__ part_tail, int skip_key) {
  constexpr int GROUPS = 1024 / LPR;
  __shared__ int s_np;
  extern __shared__ __attribute__((aligned(16))) float red[];  // [GROUPS][d]
  const int g = threadIdx.x / LPR;
  const int lane = threadIdx.x % LPR;
  const long chunk = blockIdx.x;
  const long start = chunk * SEG_CH;
  const long end = min((long)n, start + SEG_CH);
  const uint32_t key = K[end - 1];
  const bool continues = end < n && K[end] == key;
  const bool whole_cont = K[start] == key && start > 0 && K[start - 1] == key;
  if (!continues || whole_cont || (int)key == skip_key) return;  // uniform over the block
  // last chunk k >= chunk+1 the run reaches: the first k whose end does not continue it.
  // Searched 1024 chunks at a time by the whole block (a hub / padding run spans hundreds).
  if (threadIdx.x == 0) s_np = 0x7fffffff;
  __syncthreads();
  const long nchunks = (n + SEG_CH - 1) / SEG_CH;
  for (long base = chunk + 1; base < nchunks; base += 1024) {
    const long k = base + threadIdx.x;
    if (k < nchunks) {
      const long ek = min((long)n, (k + 1) * SEG_CH);
      if (!(ek < n && K[ek] == key)) atomicMin(&s_np, (int)(k - chunk + 1));  // tail of c + heads of c+1..k
    }
    __syncthreads();
    if (s_np != 0x7fffffff) break;
    __syncthreads();
  }
  const int np = s_np;
  for (int c = lane * 4; c < d; c += LPR * 4) {
    float4 a0 = c2::f4(0.f), a1 = c2::f4(0.f);
    int q = g;
    for (; q + GROUPS < np; q += 2 * GROUPS) {
      const float* s0 = q == 0 ? part_tail + chunk * d : part_head + (chunk + q) * d;
      a0 = a0 + *(const float4*)(s0 + c);
      a1 = a1 + *(const float4*)(part_head + (chunk + q + GROUPS) * d + c);
    }
    if (q < np) {
      const float* s0 = q == 0 ? part_tail + chunk * d : part_head + (chunk + q) * d;
      a0 = a0 + *(const float4*)(s0 + c);
    }
    *(float4*)(red + g * d + c) = a0 + a1;
  }
  __syncthreads();
  if (g == 0) {
    for (int c = lane * 4; c < d; c += LPR * 4) {
      float4 t = *(const float4*)(red + c);
      for (int q = 1; q < GROUPS; ++q) t = t + *(const float4*)(red + q * d + c);
      float4* o = (float4*)(out + (long)key * d + c);
      *o = *o + t;
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
    v = v * make_float4(drop.mul(b), drop.mul(b + 1), drop.mul(b + 2), drop.mul(b + 3));
  }
  ((float4*)out)[i] = v;
}

// out[c] += T[c][0] for c < n  (T [n][4], the d = 4 segment sums of the (w_r, 0, 0, 0) rows)
__global__ void col0_add_kernel(const float* __restrict__ T, int n, float* __restrict__ out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < n) out[c] += T[4 * (long)c];
}

int lpr_for(int d) { return d / 4 >= 64 ? 64 : (d / 4 >= 32 ? 32 : (d / 4 >= 16 ? 16 : (d / 4 >= 8 ? 8 : 4))); }

struct SortWs {
  uint32_t *k0, *v0, *k1, *v1, *hist;
  float *ph, *pt;
  int nblocks;
};

size_t ws_layout(int n, int d, SortWs* w, char* base) {
  const int nblocks = c2::ceil_div(n, RS_TILE);
  const long nchunks = c2::ceil_div(n, SEG_CH);
  size_t off = 0;
  auto take = [&](size_t bytes) {
    size_t o = off;
    off += (bytes + 255) & ~size_t(255);
    return base ? base + o : nullptr;
  };
  char* k0 = take((size_t)n * 4);
  char* v0 = take((size_t)n * 4);
  char* k1 = take((size_t)n * 4);
  char* v1 = take((size_t)n * 4);
  char* hist = take((size_t)256 * nblocks * 4);
  char* ph = take((size_t)nchunks * d * 4);
  char* pt = take((size_t)nchunks * d * 4);
  if (w) {
    w->k0 = (uint32_t*)k0;
    w->v0 = (uint32_t*)v0;
    w->k1 = (uint32_t*)k1;
    w->v1 = (uint32_t*)v1;
    w->hist = (uint32_t*)hist;
    w->ph = (float*)ph;
    w->pt = (float*)pt;
    w->nblocks = nblocks;
  }
  return off;
}

// sort idx[0..n) (values < n_keys) → w.k0/w.v0 sorted (key, original row)
int radix_sort(const int64_t* idx, int n, int n_keys, SortWs& w, hipStream_t s) {
  prep_keys_kernel<<<c2::ceil_div(n, 256), 256, 0, s>>>(idx, n, w.k0, w.v0);
  int bits = 1;
  while ((1l << bits) < (long)n_keys) ++bits;
  uint32_t *ki = w.k0, *vi = w.v0, *ko = w.k1, *vo = w.v1;
  for (int shift = 0; shift < bits; shift += 8) {
    rs_hist_kernel<<<w.nblocks, RS_THREADS, 0, s>>>(ki, n, shift, w.nblocks, w.hist);
    rs_scan_kernel<<<1, 1024, 0, s>>>(w.hist, 256 * w.nblocks);
    rs_scatter_kernel<<<w.nblocks, RS_THREADS, 0, s>>>(ki, vi, n, shift, w.nblocks, w.hist, ko, vo);
    uint32_t* t = ki; ki = ko; ko = t;
    t = vi; vi = vo; vo = t;
  }
  if (ki != w.k0) {  // odd number of passes: copy back
    hipMemcpyAsync(w.k0, ki, (size_t)n * 4, hipMemcpyDeviceToDevice, s);
    hipMemcpyAsync(w.v0, vi, (size_t)n * 4, hipMemcpyDeviceToDevice, s);
  }
  C2_CHECK_LAUNCH();
  return 0;
}

template <int LPR>
void seg_launch(const SortWs& w, int n, const RowSrc& src, float* out, int skip_key, hipStream_t s) {
  constexpr int GROUPS = 256 / LPR;
  const int nchunks = c2::ceil_div(n, SEG_CH);
  dim3 grid(c2::ceil_div(nchunks, GROUPS));  // GROUPS chunks (GROUPS*SEG_CH entries) per block
  seg_reduce_a<LPR><<<grid, 256, 0, s>>>(w.k0, w.v0, n, src, out, w.ph, w.pt, skip_key);
  seg_reduce_b<LPR><<<nchunks, 1024, (size_t)(1024 / LPR) * src.d * 4, s>>>(w.k0, n, src.d, out, w.ph, w.pt, skip_key);
}

void seg_dispatch(const SortWs& w, int n, const RowSrc& src, float* out, int skip_key, hipStream_t s) {
  switch (lpr_for(src.d)) {
    case 64: seg_launch<64>(w, n, src, out, skip_key, s); break;
    case 32: seg_launch<32>(w, n, src, out, skip_key, s); break;
    case 16: seg_launch<16>(w, n, src, out, skip_key, s); break;
    case 8: seg_launch<8>(w, n, src, out, skip_key, s); break;
    default: seg_launch<4>(w, n, src, out, skip_key, s); break;
  }
}

}  // namespace

C2_API int c2dsr_embed_fwd(const int64_t* seq, const int64_t* pos, int n_rows, int d, const float* H, const float* E,
                           const float* Xin, const float* P, float scale, uint32_t k0, uint32_t k1, float p,
                           int64_t idx_base, float* X, void* stream) {
  if (d % 4 || n_rows <= 0) return n_rows == 0 ? 0 : (int)hipErrorInvalidValue;
  c2::Drop dr = c2::make_drop(k0, k1, p);
  hipStream_t s = (hipStream_t)stream;
  const int lpr = lpr_for(d);
  dim3 grid(c2::ceil_div(n_rows, 256 / lpr));
  const bool gather = Xin == nullptr;
#define C2_EMB(L)                                                                                                  \
  if (gather)                                                                                                      \
    embed_fwd_kernel<L, true><<<grid, 256, 0, s>>>(seq, pos, n_rows, d, H, E, Xin, P, scale, dr, idx_base, X);     \
  else                                                                                                             \
    embed_fwd_kernel<L, false><<<grid, 256, 0, s>>>(seq, pos, n_rows, d, H, E, Xin, P, scale, dr, idx_base, X);
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

C2_API size_t c2dsr_embed_bwd_workspace(int n_rows, int d) { return ws_layout(n_rows, d, nullptr, nullptr); }

// gX: grad w.r.t. the dropout output X [n_rows, d].
//   G[seq[r]]  += scale * drop(gX[r])            (G dense [n_items, d]; skipped if G null)
//   gP[pos[r]] += drop(gX[r])                     (gP dense [n_pos, d]; skipped if null)
//   gXin[r]     = drop(gX[r])                     (optional, for the non-gather mode)
C2_API int c2dsr_embed_bwd(const int64_t* seq, const int64_t* pos, int n_rows, int d, const float* gX, uint32_t k0,
                           uint32_t k1, float p, int64_t idx_base, float scale, float* G, int n_items, float* gP,
                           int n_pos, float* gXin, void* workspace, size_t ws_bytes, void* stream) {
  if (d % 4) return (int)hipErrorInvalidValue;
  if (n_rows == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  SortWs w;
  const size_t need = ws_layout(n_rows, d, &w, (char*)workspace);
  if (ws_bytes < need) return (int)hipErrorInvalidValue;
  c2::Drop dr = c2::make_drop(k0, k1, p);
  if (G) {
    int e = radix_sort(seq, n_rows, n_items, w, s);
    if (e) return e;
    RowSrc src{gX, d, dr, idx_base, scale, nullptr};
    seg_dispatch(w, n_rows, src, G, -1, s);
  }
  if (gP) {
    int e = radix_sort(pos, n_rows, n_pos, w, s);
    if (e) return e;
    RowSrc src{gX, d, dr, idx_base, 1.0f, nullptr};
    seg_dispatch(w, n_rows, src, gP, -1, s);
  }
  if (gXin) {
    long n4 = (long)n_rows * d / 4;
    drop_scale_kernel<<<c2::ceil_div(n4, 256), 256, 0, s>>>(gX, n4, d, dr, idx_base, gXin);
  }
  C2_CHECK_LAUNCH();
  return 0;
}

C2_API size_t c2dsr_ce_onehot_workspace(int M, int n, int D) {
  return ws_layout(M, D, nullptr, nullptr) + (((size_t)n * 16 + 255) & ~size_t(255));
}

// The one-hot part of the classifier-head gradient (trainer.py:131-154 via F.cross_entropy):
//   gW[t_r] -= rw_r·H[r],  gb[t_r] -= rw_r   for rows with 0 <= t_r < n (t_r = n is ignore_index)
// Rows are radix-sorted by target and each target's run is reduced in row order (deterministic);
// the bias part runs the same segment reduction over the rows (rw_r, 0, 0, 0).
C2_API int c2dsr_ce_onehot_dw(const int64_t* tgt, int M, int n, const float* H, int D, const float* rw, float* gW,
                              float* gb, void* workspace, size_t ws_bytes, void* stream) {
  if (D % 4) return (int)hipErrorInvalidValue;
  if (M == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  SortWs w;
  const size_t sort_bytes = ws_layout(M, D, &w, (char*)workspace);
  if (ws_bytes < c2dsr_ce_onehot_workspace(M, n, D)) return (int)hipErrorInvalidValue;
  int e = radix_sort(tgt, M, n + 1, w, s);
  if (e) return e;
  const c2::Drop nodrop = c2::make_drop(0, 0, 0.f);
  if (gW) {
    RowSrc src{H, D, nodrop, 0, -1.f, rw};
    seg_dispatch(w, M, src, gW, n, s);
  }
  if (gb) {
    float* T = (float*)((char*)workspace + sort_bytes);
    hipMemsetAsync(T, 0, (size_t)n * 16, s);
    RowSrc src{nullptr, 4, nodrop, 0, -1.f, rw};
    seg_dispatch(w, M, src, T, n, s);
    col0_add_kernel<<<c2::ceil_div(n, 256), 256, 0, s>>>(T, n, gb);
  }
  C2_CHECK_LAUNCH();
  return 0;
}
