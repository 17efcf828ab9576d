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

// ------------------------------------------------------------------ sort plan → work lists
// The sorted entries are cut into pieces: a piece starts at every run start (key change) and at
// every SEG_CH boundary, so a piece is a run, or the part of a long run inside one chunk.  One
// lane group sums one piece: a whole run goes to out[key] (+=), a cut run leaves its piece in the
// chunk's head/tail slot.  A "split" is a run that continues past the end of its first chunk:
// out[key] += tail[c] + head[c+1] + ... + head[last], summed in chunk order (deterministic).
// Building the lists depends on the indices only (part of the plan, off the critical path).
constexpr int SEG_CH = 32;
constexpr int PL_T = 256;         // plan kernels: threads per block
constexpr int PL_E = 4;           // entries per thread
constexpr int PL_B = PL_T * PL_E;  // entries per block

__device__ __forceinline__ bool piece_start(const uint32_t* K, int i) {
  return i == 0 || (i % SEG_CH) == 0 || K[i] != K[i - 1];
}
__device__ __forceinline__ bool split_start(const uint32_t* K, int n, int i) {
  if (!(i == 0 || K[i] != K[i - 1])) return false;
  const int ce = (i / SEG_CH + 1) * SEG_CH;
  return ce < n && K[ce] == K[i];
}

// per block: number of pieces and splits among its PL_B entries → cnt[2·b], cnt[2·b+1]
__global__ __launch_bounds__(PL_T) void plan_count_kernel(const uint32_t* __restrict__ K, int n,
                                                          uint32_t* __restrict__ cnt) {
  __shared__ uint32_t red[2][PL_T / 64];
  uint32_t p = 0, q = 0;
  for (int j = 0; j < PL_E; ++j) {
    const int i = blockIdx.x * PL_B + j * PL_T + threadIdx.x;
    if (i < n) {
      p += piece_start(K, i);
      q += split_start(K, n, i);
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    p += __shfl_xor(p, o, 64);
    q += __shfl_xor(q, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = p;
    red[1][threadIdx.x >> 6] = q;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    uint32_t t = 0;
    for (int w = 0; w < PL_T / 64; ++w) t += red[threadIdx.x][w];
    cnt[2 * blockIdx.x + threadIdx.x] = t;
  }
}

// exclusive scan of the block counts (single workgroup); totals → counts[0..1], starts[total] = n
__global__ __launch_bounds__(1024) void plan_scan_kernel(uint32_t* __restrict__ cnt, int nb, int n,
                                                         int* __restrict__ counts, int* __restrict__ starts) {
  __shared__ uint32_t part[2][1024];
  const int t = threadIdx.x;
  const int per = (nb + 1023) / 1024;
  const int lo = min(nb, t * per), hi = min(nb, lo + per);
  uint32_t s0 = 0, s1 = 0;
  for (int i = lo; i < hi; ++i) {
    s0 += cnt[2 * i];
    s1 += cnt[2 * i + 1];
  }
  part[0][t] = s0;
  part[1][t] = s1;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const uint32_t v0 = t >= o ? part[0][t - o] : 0, v1 = t >= o ? part[1][t - o] : 0;
    __syncthreads();
    part[0][t] += v0;
    part[1][t] += v1;
    __syncthreads();
  }
  uint32_t r0 = part[0][t] - s0, r1 = part[1][t] - s1;
  for (int i = lo; i < hi; ++i) {
    const uint32_t c0 = cnt[2 * i], c1 = cnt[2 * i + 1];
    cnt[2 * i] = r0;
    cnt[2 * i + 1] = r1;
    r0 += c0;
    r1 += c1;
  }
  if (t == 1023) {
    counts[0] = (int)part[0][1023];
    counts[1] = (int)part[1][1023];
    starts[part[0][1023]] = n;
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

// writes starts[piece] = first entry, splits[j] = {key, first chunk, chunks spanned, 0}
__global__ __launch_bounds__(PL_T) void plan_emit_kernel(const uint32_t* __restrict__ K, int n,
                                                         const uint32_t* __restrict__ cnt, int* __restrict__ starts,
                                                         int4* __restrict__ splits) {
  __shared__ uint32_t red[PL_T / 64];
  // thread t owns entries [base + t·PL_E, base + (t+1)·PL_E): contiguous, so the order is kept
  const int i0 = blockIdx.x * PL_B + threadIdx.x * PL_E;
  uint32_t fp = 0, fs = 0;
  for (int j = 0; j < PL_E; ++j) {
    const int i = i0 + j;
    if (i < n) {
      fp |= (uint32_t)piece_start(K, i) << j;
      fs |= (uint32_t)split_start(K, n, i) << j;
    }
  }
  uint32_t op = cnt[2 * blockIdx.x] + block_prefix(__popc(fp), red);
  uint32_t os = cnt[2 * blockIdx.x + 1] + block_prefix(__popc(fs), red);
  for (int j = 0; j < PL_E; ++j) {
    const int i = i0 + j;
    if (fp >> j & 1) starts[op++] = i;
    if (fs >> j & 1) {
      const uint32_t key = K[i];
      int lo = i, hi = n;  // first entry with a larger key (keys are sorted)
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (K[mid] <= key) lo = mid + 1; else hi = mid;
      }
      const int c = i / SEG_CH, last = (lo - 1) / SEG_CH;
      splits[os++] = make_int4((int)key, c, last - c + 1, 0);
    }
  }
}

// desc[w] = {first entry, end, key, kind}: kind 0 = whole run (out[key] +=), 1 = head slot of chunk
// first/SEG_CH, 2 = tail slot of chunk (end-1)/SEG_CH — everything pass A needs in one load.
__global__ __launch_bounds__(256) void plan_desc_kernel(const uint32_t* __restrict__ K, int n,
                                                        const int* __restrict__ starts, const int* __restrict__ counts,
                                                        int4* __restrict__ desc) {
  const int np = counts[0];
  for (int w = blockIdx.x * 256 + threadIdx.x; w < np; w += gridDim.x * 256) {
    const int s = starts[w], e = starts[w + 1];
    const uint32_t key = K[s];
    const bool head = (s % SEG_CH) == 0 && s > 0 && K[s - 1] == key;
    const bool tail = (e % SEG_CH) == 0 && e < n && K[e] == key;
    desc[w] = make_int4(s, e, (int)key, head ? 1 : (tail ? 2 : 0));
  }
}

// ------------------------------------------------------------------ segment sums
constexpr int SEG_U = 8;  // rows in flight per lane group

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

// pass A: one lane group per piece (grid-stride over the device-side piece count).  The chain per
// piece is descriptor → row ids → rows (+ the old out row, loaded alongside) → store; rows SEG_U at
// a time, summed in entry order.
// A plan that does not describe n entries over n_out output rows (a plan of other indices, or
// one read before it was complete) is never followed: the offending pieces are skipped and err
// is set (checked by the host in debug runs), so it cannot turn into a stray access.
template <int LPR>
__global__ __launch_bounds__(256) void seg_piece_kernel(const uint32_t* __restrict__ V, const int4* __restrict__ desc,
                                                        const int* __restrict__ counts, int n, int n_out, RowSrc src,
                                                        float* __restrict__ out, float* __restrict__ part_head,
                                                        float* __restrict__ part_tail, int skip_key,
                                                        int* __restrict__ err) {
  constexpr int GROUPS = 256 / LPR;
  const int lane = threadIdx.x % LPR;
  int npieces = counts[0];
  if (npieces < 0 || npieces > n) {
    if (threadIdx.x == 0) atomicOr(err, 1);
    return;
  }
  const int d = src.d;
  for (int w = blockIdx.x * GROUPS + threadIdx.x / LPR; w < npieces; w += gridDim.x * GROUPS) {
    const int4 ds = desc[w];
    const int s = ds.x, e = ds.y, key = ds.z, kind = ds.w;
    if (s < 0 || e > n || e <= s || e - s > SEG_CH || key < 0 || key >= n_out) {
      if (lane == 0) atomicOr(err, 2);
      continue;
    }
    if (key == skip_key) continue;
    float* dst = kind == 1 ? part_head + (long)(s / SEG_CH) * d
                           : (kind == 2 ? part_tail + (long)((e - 1) / SEG_CH) * d : out + (long)key * d);
    for (int c = lane * 4; c < d; c += LPR * 4) {
      float4 acc = kind == 0 ? *(const float4*)(dst + c) : c2::f4(0.f);
      for (int q0 = s; q0 < e; q0 += SEG_U) {
        uint32_t r[SEG_U];
#pragma unroll
        for (int u = 0; u < SEG_U; ++u) r[u] = q0 + u < e ? min(V[q0 + u], (uint32_t)(n - 1)) : 0u;
        float4 x[SEG_U];
#pragma unroll
        for (int u = 0; u < SEG_U; ++u) x[u] = q0 + u < e ? src.load(r[u], c) : c2::f4(0.f);
        float4 t = x[0];
#pragma unroll
        for (int u = 1; u < SEG_U; ++u) t = t + x[u];
        acc = acc + t;
      }
      *(float4*)(dst + c) = acc;
    }
  }
}

// pass B: one block per split (grid-stride): out[key] += tail[c] + head[c+1..c+np-1]; the pieces are
// dealt round-robin to the block's lane groups (four loads in flight per group), the group sums are
// added in group order.
template <int LPR>
__global__ __launch_bounds__(1024) void seg_split_kernel(const int4* __restrict__ splits,
                                                         const int* __restrict__ counts, int nchunks, int n_out,
                                                         int d, float* __restrict__ out,
                                                         const float* __restrict__ part_head,
                                                         const float* __restrict__ part_tail, int skip_key,
                                                         int* __restrict__ err) {
  constexpr int GROUPS = 1024 / LPR;
  extern __shared__ __attribute__((aligned(16))) float red[];  // [GROUPS][d]
  const int g = threadIdx.x / LPR;
  const int lane = threadIdx.x % LPR;
  const int nsplit = counts[1];
  if (nsplit < 0 || nsplit > nchunks) {
    if (threadIdx.x == 0) atomicOr(err, 4);
    return;
  }
  for (int j = blockIdx.x; j < nsplit; j += gridDim.x) {
    const int4 sp = splits[j];
    const int key = sp.x, chunk = sp.y, np = sp.z;
    if (key < 0 || key >= n_out || chunk < 0 || np < 2 || chunk + np > nchunks) {  // uniform over the block
      if (threadIdx.x == 0) atomicOr(err, 8);
      continue;
    }
    if (key == skip_key) continue;  // uniform over the block
    auto slot = [&](int q) -> const float* {
      return q == 0 ? part_tail + (long)chunk * d : part_head + (long)(chunk + q) * d;
    };
    for (int c = lane * 4; c < d; c += LPR * 4) {
      float4 a[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) a[u] = c2::f4(0.f);
      int q = g;
      for (; q + 7 * GROUPS < np; q += 8 * GROUPS) {
#pragma unroll
        for (int u = 0; u < 8; ++u) a[u] = a[u] + *(const float4*)(slot(q + u * GROUPS) + c);
      }
      for (; q < np; q += GROUPS) a[0] = a[0] + *(const float4*)(slot(q) + c);
      *(float4*)(red + g * d + c) = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
    }
    __syncthreads();
    for (int c = threadIdx.x * 4; c < d; c += 1024 * 4) {
      float4 t = *(const float4*)(red + c);
      for (int q = 1; q < GROUPS; ++q) t = t + *(const float4*)(red + q * d + c);
      float4* o = (float4*)(out + (long)key * d + c);
      *o = *o + t;
    }
    __syncthreads();
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

size_t align256(size_t b) { return (b + 255) & ~size_t(255); }

// A plan: keys[n] (sorted ids) | vals[n] (their rows) | starts[n+2] | splits[n/SEG_CH+1] int4 |
// counts[4] | desc[n] int4 | scratch (second LSD buffers, digit histograms, plan block counts).
struct Plan {
  uint32_t *k0, *v0;
  int* starts;
  int4* splits;
  int* counts;
  int4* desc;
  uint32_t *k1, *v1, *hist, *bcnt;
  int nblocks;
};

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
  char* st = take((size_t)(n + 2) * 4);
  char* sp = take((size_t)(n / SEG_CH + 1) * 16);
  char* ct = take(16);
  char* ds = take((size_t)n * 16);
  char* k1 = take((size_t)n * 4);
  char* v1 = take((size_t)n * 4);
  char* hist = take((size_t)256 * nblocks * 4);
  char* bc = take((size_t)2 * pb * 4);
  if (p)
    *p = Plan{(uint32_t*)k0, (uint32_t*)v0, (int*)st, (int4*)sp, (int*)ct, (int4*)ds,
              (uint32_t*)k1, (uint32_t*)v1, (uint32_t*)hist, (uint32_t*)bc, nblocks};
  return off;
}

Plan plan_view(const void* base, int n) {
  Plan p;
  plan_layout(n, &p, (char*)base);
  return p;
}

// head/tail partial slots of the segment sums, then the error word
size_t seg_slot_bytes(int n, int d) { return align256((size_t)c2::ceil_div(n, SEG_CH) * d * 4); }
size_t seg_ws_bytes(int n, int d) { return 2 * seg_slot_bytes(n, d) + 256; }

// sort idx[0..n) (values < n_keys) → k0/v0 sorted (key, original row), stable; then the work lists
int build_plan(const int64_t* idx, int n, int n_keys, const Plan& w, hipStream_t s) {
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
  const int pb = c2::ceil_div(n, PL_B);
  plan_count_kernel<<<pb, PL_T, 0, s>>>(w.k0, n, w.bcnt);
  plan_scan_kernel<<<1, 1024, 0, s>>>(w.bcnt, pb, n, w.counts, w.starts);
  plan_emit_kernel<<<pb, PL_T, 0, s>>>(w.k0, n, w.bcnt, w.starts, w.splits);
  plan_desc_kernel<<<std::min(c2::ceil_div(n, 256), 1024), 256, 0, s>>>(w.k0, n, w.starts, w.counts, w.desc);
  C2_CHECK_LAUNCH();
  return 0;
}

int g_ncu = 0;
int num_cus() {
  if (!g_ncu) {
    int dev = 0, v = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev);
    g_ncu = v > 0 ? v : 256;
  }
  return g_ncu;
}

template <int LPR>
void seg_launch(const Plan& p, int n, int n_out, const RowSrc& src, float* out, float* ph, float* pt, int skip_key,
                int* err, hipStream_t s) {
  constexpr int GROUPS = 256 / LPR;
  // pieces <= n; 8 blocks (32 waves) per CU, grid-stride over the device-side count
  const int grid = std::max(1, std::min(c2::ceil_div(n, GROUPS), 8 * num_cus()));
  seg_piece_kernel<LPR><<<grid, 256, 0, s>>>(p.v0, p.desc, p.counts, n, n_out, src, out, ph, pt, skip_key, err);
  if (n > SEG_CH) {
    const int nchunks = c2::ceil_div(n, SEG_CH);
    const int gs = std::max(1, std::min(n / SEG_CH, num_cus()));
    seg_split_kernel<LPR><<<gs, 1024, (size_t)(1024 / LPR) * src.d * 4, s>>>(p.splits, p.counts, nchunks, n_out,
                                                                             src.d, out, ph, pt, skip_key, err);
  }
}

// out[key] += Σ src rows of each run of the plan (keys < n_out), partial slots and the error word
// carved from ws
void seg_dispatch(const Plan& p, int n, int n_out, const RowSrc& src, float* out, char* ws, int skip_key,
                  hipStream_t s) {
  float* ph = (float*)ws;
  float* pt = (float*)(ws + seg_slot_bytes(n, src.d));
  int* err = (int*)(ws + 2 * seg_slot_bytes(n, src.d));
  switch (lpr_for(src.d)) {
    case 64: seg_launch<64>(p, n, n_out, src, out, ph, pt, skip_key, err, s); break;
    case 32: seg_launch<32>(p, n, n_out, src, out, ph, pt, skip_key, err, s); break;
    case 16: seg_launch<16>(p, n, n_out, src, out, ph, pt, skip_key, err, s); break;
    case 8: seg_launch<8>(p, n, n_out, src, out, ph, pt, skip_key, err, s); break;
    default: seg_launch<4>(p, n, n_out, src, out, ph, pt, skip_key, err, s); break;
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

C2_API size_t c2dsr_index_plan_bytes(int n) { return plan_layout(n, nullptr, nullptr); }

// Sort plan of an index array: plan = [keys u32 n | rows u32 n | scratch], keys ascending and
// rows ascending within equal keys (stable LSD radix sort).  Depends on the indices only, so
// the host builds it as soon as a batch's index tensors exist (on a side stream, under the
// forward pass) and the backward's segment sums consume it.
C2_API int c2dsr_index_plan(const int64_t* idx, int n, int n_keys, void* plan, size_t plan_bytes, void* stream) {
  if (n < 0 || n_keys <= 0) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  Plan p;
  if (plan_bytes < plan_layout(n, &p, (char*)plan)) return (int)hipErrorInvalidValue;
  return build_plan(idx, n, n_keys, p, (hipStream_t)stream);
}

C2_API size_t c2dsr_embed_bwd_planned_workspace(int n_rows, int d) { return seg_ws_bytes(n_rows, d); }

// gX: grad w.r.t. the dropout output X [n_rows, d]; seq_plan / pos_plan from c2dsr_index_plan.
//   G[seq[r]]  += scale * drop(gX[r])            (G dense [n_items, d]; skipped if G null)
//   gP[pos[r]] += drop(gX[r])                     (gP dense [n_pos, d]; skipped if null)
//   gXin[r]     = drop(gX[r])                     (optional, for the non-gather mode)
C2_API size_t c2dsr_seg_err_offset(int n_rows, int d) { return 2 * seg_slot_bytes(n_rows, d); }

C2_API int c2dsr_embed_bwd_planned(const void* seq_plan, const void* pos_plan, int n_rows, int d, const float* gX,
                                   uint32_t k0, uint32_t k1, float p, int64_t idx_base, float scale, float* G,
                                   int n_items, float* gP, int n_pos, float* gXin, void* workspace, size_t ws_bytes,
                                   void* stream) {
  if (d % 4) return (int)hipErrorInvalidValue;
  if (n_rows == 0) return 0;
  if (ws_bytes < seg_ws_bytes(n_rows, d) || (G && !seq_plan) || (gP && !pos_plan)) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  c2::Drop dr = c2::make_drop(k0, k1, p);
  hipMemsetAsync((char*)workspace + c2dsr_seg_err_offset(n_rows, d), 0, 4, s);
  if (G)
    seg_dispatch(plan_view(seq_plan, n_rows), n_rows, n_items, RowSrc{gX, d, dr, idx_base, scale, nullptr}, G,
                 (char*)workspace, -1, s);
  if (gP)
    seg_dispatch(plan_view(pos_plan, n_rows), n_rows, n_pos, RowSrc{gX, d, dr, idx_base, 1.0f, nullptr}, gP,
                 (char*)workspace, -1, s);
  if (gXin) {
    long n4 = (long)n_rows * d / 4;
    drop_scale_kernel<<<c2::ceil_div(n4, 256), 256, 0, s>>>(gX, n4, d, dr, idx_base, gXin);
  }
  C2_CHECK_LAUNCH();
  return 0;
}

C2_API size_t c2dsr_embed_bwd_workspace(int n_rows, int d) {
  return align256(plan_layout(n_rows, nullptr, nullptr)) + seg_ws_bytes(n_rows, d);
}

// unplanned form: sorts inside (one plan buffer reused for seq, then pos)
C2_API int c2dsr_embed_bwd(const int64_t* seq, const int64_t* pos, int n_rows, int d, const float* gX, uint32_t k0,
                           uint32_t k1, float p, int64_t idx_base, float scale, float* G, int n_items, float* gP,
                           int n_pos, float* gXin, void* workspace, size_t ws_bytes, void* stream) {
  if (d % 4) return (int)hipErrorInvalidValue;
  if (n_rows == 0) return 0;
  if (ws_bytes < c2dsr_embed_bwd_workspace(n_rows, d)) return (int)hipErrorInvalidValue;
  char* plan = (char*)workspace;
  const size_t pb = align256(plan_layout(n_rows, nullptr, nullptr));
  char* seg = plan + pb;
  const size_t sb = seg_ws_bytes(n_rows, d);
  int e;
  if (G) {
    if ((e = c2dsr_index_plan(seq, n_rows, n_items, plan, pb, stream))) return e;
    if ((e = c2dsr_embed_bwd_planned(plan, nullptr, n_rows, d, gX, k0, k1, p, idx_base, scale, G, n_items, nullptr,
                                     0, nullptr, seg, sb, stream)))
      return e;
  }
  if (gP) {
    if ((e = c2dsr_index_plan(pos, n_rows, n_pos, plan, pb, stream))) return e;
    if ((e = c2dsr_embed_bwd_planned(nullptr, plan, n_rows, d, gX, k0, k1, p, idx_base, 1.0f, nullptr, 0, gP, n_pos,
                                     nullptr, seg, sb, stream)))
      return e;
  }
  if (gXin) return c2dsr_embed_bwd_planned(nullptr, nullptr, n_rows, d, gX, k0, k1, p, idx_base, 1.0f, nullptr, 0,
                                           nullptr, 0, gXin, seg, sb, stream);
  return 0;
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
  hipMemsetAsync(seg + c2dsr_seg_err_offset(M, D), 0, 4, s);
  if (gW) seg_dispatch(p, M, n + 1, RowSrc{H, D, nodrop, 0, -1.f, rw}, gW, seg, n, s);
  if (gb) {
    float* T = (float*)(seg + seg_ws_bytes(M, D));
    hipMemsetAsync(T, 0, (size_t)n * 16, s);
    seg_dispatch(p, M, n + 1, RowSrc{nullptr, 4, nodrop, 0, -1.f, rw}, T, seg, n, s);
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
  int e = c2dsr_index_plan(tgt, M, n + 1, plan, pb, stream);
  if (e) return e;
  return c2dsr_ce_onehot_dw_planned(plan, M, n, H, D, rw, gW, gb, plan + pb, ws_bytes - pb, stream);
}
