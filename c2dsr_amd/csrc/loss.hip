// Loss head of Trainer.train_batch: masked mean pooling, bilinear infomax
// discriminators + BCE, classifier heads with a pad column + cross-entropy with
// ignore_index, and the scalar loss combination — forward and backward.
//
// Replaces trainer.py:85-156 (cal_mask, pooling, D_a/D_b, BCE-with-logits,
// torch.cat of the pad column, F.cross_entropy(ignore_index=n), count weighting).
#include "common.h"

namespace {

// w[b,l] = gm[b,l] / Σ_l gm[b,l]   (Trainer.cal_mask, trainer.py:85-89)
// one wave per sequence: lane l holds positions l, l + 64, ...; the mask counts are small integers, so the
// fp32 sum is exact in any order
__global__ __launch_bounds__(256) void pool_weights_kernel(const int64_t* __restrict__ gm, int B, int L,
                                                           float* __restrict__ w) {
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (b >= B) return;  // uniform over the wave
  const int64_t* g = gm + (long)b * L;
  float S = 0.f;
  for (int l = lane; l < L; l += 64) S += (float)g[l];
#pragma unroll
  for (int m = 32; m > 0; m >>= 1) S += __shfl_xor(S, m, 64);
  for (int l = lane; l < L; l += 64) w[(long)b * L + l] = (float)g[l] / S;
}

// out[b,c] = Σ_l h[b,l,c] * w[b,l]      (trainer.py:101-108)
__global__ void pool_fwd_kernel(const float* __restrict__ h, const float* __restrict__ w, int B, int L, int d,
                                float* __restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)B * d) return;
  const int b = (int)(i / d), c = (int)(i % d);
  float acc = 0.f;
  for (int l = 0; l < L; ++l) acc += h[((long)b * L + l) * d + c] * w[(long)b * L + l];
  out[i] = acc;
}

// dh[b,l,c] += dout[b,c] * w[b,l]   (float4 per thread)
__global__ void pool_bwd_kernel(const float* __restrict__ dout, const float* __restrict__ w, int B, int L, int d,
                                float* __restrict__ dh) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;  // float4 index
  if (i >= (long)B * L * d / 4) return;
  const long e = i * 4;
  const int c = (int)(e % d);
  const long bl = e / d;
  const long b = bl / L;
  const float wt = w[bl];
  const float4 g = *(const float4*)(dout + b * d + c);
  float4* o = (float4*)(dh + e);
  *o = c2::fma4(wt, g, *o);
}

// out1[b] = Σ_l h[b,l]·w1[b,l]  (and out2[b] = Σ_l h[b,l]·w2[b,l] when w2 is given: one read of h for
// both poolings of h_share).  One block per b: the four waves take rows l ≡ w (mod 4), float4 per
// lane (d <= 256 per pass over c), rows whose weights are all 0 (padding / non-target positions) are
// not read; the wave partials are added in wave order (deterministic).
__global__ __launch_bounds__(256) void pool2_fwd_kernel(const float* __restrict__ h, const int* __restrict__ hmap,
                                                        const float* __restrict__ w1,
                                                        const float* __restrict__ w2, int B, int L, int d,
                                                        float* __restrict__ out1, float* __restrict__ out2) {
  __shared__ float4 red[2][4][64];
  const int b = blockIdx.x;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float* wa = w1 + (long)b * L;
  const float* wb = w2 ? w2 + (long)b * L : nullptr;
  for (int c0 = 0; c0 < d; c0 += 256) {
    const int c = c0 + lane * 4;
    const bool cin = c < d;
    float4 a1 = c2::f4(0.f), a2 = c2::f4(0.f);
    for (int l0 = w; l0 < L; l0 += 16) {
      float x1[4], x2[4];
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int l = l0 + 4 * u;
        x1[u] = l < L ? wa[l] : 0.f;
        x2[u] = (wb && l < L) ? wb[l] : 0.f;
        const long bl = (long)b * L + l;
        v[u] = (cin && (x1[u] != 0.f || x2[u] != 0.f)) ? *(const float4*)(h + (hmap ? hmap[bl] : bl) * d + c)
                                                        : c2::f4(0.f);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a1 = c2::fma4(x1[u], v[u], a1);
        a2 = c2::fma4(x2[u], v[u], a2);
      }
    }
    red[0][w][lane] = a1;
    red[1][w][lane] = a2;
    __syncthreads();
    if (w < 2 && cin && (w == 0 || out2)) {
      float4 t = red[w][0][lane];
      for (int k = 1; k < 4; ++k) t = t + red[w][k][lane];
      *(float4*)((w ? out2 : out1) + (long)b * d + c) = t;
    }
    __syncthreads();
  }
}

// dh[k] = (accumulate ? dh[k] : 0) + d1[b]·w1[b,l] (+ d2[b]·w2[b,l]) for the row k of (b, l): k = b·L + l, or,
// with a compact dh, bl = idx[k] over its n_rows rows   (float4 per thread)
__global__ void pool2_bwd_kernel(const float* __restrict__ d1, const float* __restrict__ w1,
                                 const float* __restrict__ d2, const float* __restrict__ w2, int L, int d,
                                 long rows, const int* __restrict__ idx, int accumulate, float* __restrict__ dh) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;  // float4 index
  if (i >= rows * d / 4) return;
  const long e = i * 4;
  const int c = (int)(e % d);
  const long k = e / d;
  const long bl = idx ? idx[k] : k;
  const long b = bl / L;
  const float x1 = w1[bl], x2 = d2 ? w2[bl] : 0.f;
  float4 o = accumulate ? *(const float4*)(dh + e) : c2::f4(0.f);
  if (x1 != 0.f) o = c2::fma4(x1, *(const float4*)(d1 + b * d + c), o);
  if (x2 != 0.f) o = c2::fma4(x2, *(const float4*)(d2 + b * d + c), o);
  *(float4*)(dh + e) = o;
}

// Stable multi-set row compaction over M rows, two launches: block b covers rows [b·1024, (b+1)·1024)
// in four rounds of 256 (one row per lane, coalesced reads); membership of every set comes from one
// Op::mask(r) bit per set; a row's compact index is (rows of the set in earlier blocks) + (earlier
// waves and rounds of its block) + (lower lanes of its ballot).  The count pass writes per-block set
// sizes bc[b·NS + s]; the emit pass sums the earlier blocks' sizes and calls Op::put / Op::totals.
constexpr int CMP_TILE = 1024;

__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

template <class Op>
__global__ __launch_bounds__(256) void cmp_count_kernel(Op op, int M, int* __restrict__ bc) {
  constexpr int NS = Op::NS;
  __shared__ int wc[NS][4];
  const int th = threadIdx.x, w = th >> 6, ln = th & 63;
  int c[NS];
#pragma unroll
  for (int q = 0; q < NS; ++q) c[q] = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = blockIdx.x * CMP_TILE + j * 256 + th;
    const uint32_t m = r < M ? op.mask(r) : 0u;
#pragma unroll
    for (int q = 0; q < NS; ++q) c[q] += (int)__popcll(__ballot((m >> q) & 1u));
  }
  if (ln == 0)
#pragma unroll
    for (int q = 0; q < NS; ++q) wc[q][w] = c[q];
  __syncthreads();
  if (th < NS) bc[blockIdx.x * NS + th] = wc[th][0] + wc[th][1] + wc[th][2] + wc[th][3];
}

template <class Op>
__global__ __launch_bounds__(256) void cmp_emit_kernel(Op op, int M, const int* __restrict__ bc) {
  constexpr int NS = Op::NS;
  __shared__ int wc[NS][4];
  const int th = threadIdx.x, w = th >> 6, ln = th & 63;
  int base[NS];
#pragma unroll
  for (int q = 0; q < NS; ++q) base[q] = 0;
  for (int b = th; b < (int)blockIdx.x; b += 256)
#pragma unroll
    for (int q = 0; q < NS; ++q) base[q] += bc[b * NS + q];
#pragma unroll
  for (int q = 0; q < NS; ++q) base[q] = wave_sum_i(base[q]);
  if (ln == 0)
#pragma unroll
    for (int q = 0; q < NS; ++q) wc[q][w] = base[q];
  __syncthreads();
#pragma unroll
  for (int q = 0; q < NS; ++q) base[q] = wc[q][0] + wc[q][1] + wc[q][2] + wc[q][3];
  const uint64_t below = (1ull << ln) - 1ull;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = blockIdx.x * CMP_TILE + j * 256 + th;
    const uint32_t m = r < M ? op.mask(r) : 0u;
    uint64_t bal[NS];
#pragma unroll
    for (int q = 0; q < NS; ++q) bal[q] = __ballot((m >> q) & 1u);
    __syncthreads();  // wc free (previous round / the base reduction read it)
    if (ln == 0)
#pragma unroll
      for (int q = 0; q < NS; ++q) wc[q][w] = (int)__popcll(bal[q]);
    __syncthreads();
#pragma unroll
    for (int q = 0; q < NS; ++q) {
      int pre = base[q];
      for (int v = 0; v < w; ++v) pre += wc[q][v];
      if (r < M) op.put(q, r, (m >> q) & 1u, pre + (int)__popcll(bal[q] & below));
      base[q] += wc[q][0] + wc[q][1] + wc[q][2] + wc[q][3];
    }
  }
  if (blockIdx.x == gridDim.x - 1 && th == 0) op.totals(base);
}

// Valid-row compaction of a classifier head's targets (rows with t == ignore contribute nothing to the
// loss or to any gradient, trainer.py:131-154 / F.cross_entropy(ignore_index)).  Set 0 = valid rows
// (emitted: idx[k], inv[r], tc[k] = t[idx[k]]), set 1 = valid rows below split (counted only);
// counts = (valid rows in [0, split), valid rows in [split, M)).
struct ValidOp {
  static constexpr int NS = 2;
  const int64_t* t;
  int split;
  int64_t ignore;
  int *idx, *inv;
  int64_t* tc;
  int* counts;
  int* err;  // C2DSR_IDX_ERR_TARGET for a target outside [0, ignore] (F.cross_entropy's IndexError); not valid
  __device__ uint32_t mask(int r) const {
    const int64_t tv = t[r];
    const bool bad = tv < 0 || tv > ignore;
    if (bad && err) atomicOr(err, C2DSR_IDX_ERR_TARGET);
    const uint32_t v = tv != ignore && !bad;
    return v | ((v && r < split) ? 2u : 0u);
  }
  __device__ void put(int q, int r, uint32_t in, int k) const {
    if (q != 0) return;
    if (in) {
      idx[k] = r;
      tc[k] = t[r];
    }
    inv[r] = in ? k : -1;
  }
  __device__ void totals(const int* tot) const {
    counts[0] = tot[1];
    counts[1] = tot[0] - tot[1];
  }
};

// Rows of the encoder passes the loss reads: set q uses the 3-bit code (bits >> 3q) & 7 — 1 / 2 =
// positions with gm_a / gm_b nonzero (the pass's pooling weights), 4 = the last R positions of each
// sequence (classifier heads).  idx / inv of set q at offset q·M; count[q] = set size.
struct NeedOp {
  static constexpr int NS = 8;
  const int64_t *gm_a, *gm_b;
  int L, R, n_sets, bits;
  int *idx, *inv, *count, *off;  // off (may be null): [n_sets][B + 1] first compact row of each sequence
  long M;
  __device__ uint32_t mask(int r) const {
    const uint32_t a = gm_a[r] != 0, b = gm_b[r] != 0, tail = r % L >= L - R;
    const uint32_t have = a | (b << 1) | (tail << 2);
    uint32_t m = 0;
    for (int q = 0; q < n_sets; ++q) m |= ((bits >> (3 * q)) & 7u & have) ? (1u << q) : 0u;
    return m;
  }
  __device__ void put(int q, int r, uint32_t in, int k) const {
    if (q >= n_sets) return;
    if (in) idx[q * M + k] = r;
    inv[q * M + r] = in ? k : -1;
    if (off && r % L == 0) off[q * (M / L + 1) + r / L] = k;
  }
  __device__ void totals(const int* tot) const {
    for (int q = 0; q < n_sets; ++q) {
      count[q] = tot[q];
      if (off) off[q * (M / L + 1) + M / L] = tot[q];
    }
  }
};

// Padding rows of up to 8 encoder passes (the only admissible attention keys, Q1): set q = rows with
// seqs[q·M + r] == pad; idx / inv / count / off as NeedOp.
struct PadOp {
  static constexpr int NS = 8;
  const int64_t* seqs;
  int64_t pad;
  int L, n_sets;
  int *idx, *inv, *count, *off;
  long M;
  __device__ uint32_t mask(int r) const {
    uint32_t m = 0;
    for (int q = 0; q < n_sets; ++q) m |= (seqs[q * M + r] == pad) ? (1u << q) : 0u;
    return m;
  }
  __device__ void put(int q, int r, uint32_t in, int k) const {
    if (q >= n_sets) return;
    if (in) idx[q * M + k] = r;
    inv[q * M + r] = in ? k : -1;
    if (r % L == 0) off[q * (M / L + 1) + r / L] = k;
  }
  __device__ void totals(const int* tot) const {
    for (int q = 0; q < n_sets; ++q) {
      count[q] = tot[q];
      off[q * (M / L + 1) + M / L] = tot[q];
    }
  }
};

template <class Op>
int compact_rows(const Op& op, int M, int* ws, hipStream_t s) {
  const int nblk = c2::ceil_div(M, CMP_TILE);
  cmp_count_kernel<Op><<<nblk, 256, 0, s>>>(op, M, ws);
  cmp_emit_kernel<Op><<<nblk, 256, 0, s>>>(op, M, ws);
  C2_CHECK_LAUNCH();
  return 0;
}

// dst[k][c] = src[idx[k]·ld + c]   (k < n, c < d; float4 when d % 4 == 0 and ld % 4 == 0)
__global__ void gather_rows_kernel(const float* __restrict__ src, long ld, const int* __restrict__ idx, int n, int d,
                                   float* __restrict__ dst) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (d % 4 == 0 && ld % 4 == 0) {
    const int d4 = d / 4;
    if (i >= (long)n * d4) return;
    const long k = i / d4;
    const int c = (int)(i % d4) * 4;
    *(float4*)(dst + k * d + c) = *(const float4*)(src + (long)idx[k] * ld + c);
  } else {
    if (i >= (long)n * d) return;
    const long k = i / d;
    const int c = (int)(i % d);
    dst[k * d + c] = src[(long)idx[k] * ld + c];
  }
}

// dst[r][c] = (ia >= 0 ? a[ia·d + c] : 0) + (ib >= 0 ? b[ib·d + c] : 0), ia = inv_a[r], ib = inv_b[r]
__global__ void combine_rows_kernel(const float* __restrict__ a, const int* __restrict__ inv_a,
                                    const float* __restrict__ b, const int* __restrict__ inv_b, int M, int d4,
                                    float* __restrict__ dst) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)M * d4) return;
  const long r = i / d4;
  const int c = (int)(i % d4) * 4;
  const int ia = inv_a[r], ib = inv_b[r];
  const long d = 4l * d4;
  const float4 x = ia >= 0 ? *(const float4*)(a + ia * d + c) : c2::f4(0.f);
  const float4 y = ib >= 0 ? *(const float4*)(b + ib * d + c) : c2::f4(0.f);
  *(float4*)(dst + r * d + c) = make_float4(x.x + y.x, x.y + y.y, x.z + y.z, x.w + y.w);
}

// dst[r][c] = inv[r] >= 0 ? src[inv[r]·d + c] : 0   (r < M)
__global__ void expand_rows_kernel(const float* __restrict__ src, const int* __restrict__ inv, int M, int d,
                                   float* __restrict__ dst) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (d % 4 == 0) {
    const int d4 = d / 4;
    if (i >= (long)M * d4) return;
    const long r = i / d4;
    const int c = (int)(i % d4) * 4;
    const int k = inv[r];
    *(float4*)(dst + r * d + c) = k >= 0 ? *(const float4*)(src + (long)k * d + c) : c2::f4(0.f);
  } else {
    if (i >= (long)M * d) return;
    const long r = i / d;
    const int c = (int)(i % d);
    const int k = inv[r];
    dst[r * d + c] = k >= 0 ? src[(long)k * d + c] : 0.f;
  }
}

// out[r*ldo] = Σ_c x[r*ldx + c] * y[r*ldy + c] + (bias ? bias[0] : 0); one wave per row
__global__ __launch_bounds__(256) void rowdot_kernel(const float* __restrict__ x, long ldx, const float* __restrict__ y,
                                                     long ldy, int M, int d, const float* __restrict__ bias,
                                                     float* __restrict__ out, long ldo) {
  const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= M) return;
  float s = 0.f;
  for (int c = lane; c < d; c += 64) s += x[r * ldx + c] * y[r * ldy + c];
  s = c2::wave_sum(s);
  if (lane == 0) out[r * ldo] = s + (bias ? bias[0] : 0.f);
}

// the four discriminator scores in one launch (blockIdx.y = k): S[k][b] = x_k[b]·y_k[b] + bias_k with
// (x, y) = (x1a, Ua[0:B]), (x1a, Ua[B:2B]), (x1b, Ub[0:B]), (x1b, Ub[B:2B]) — rowdot_kernel's sum per row, the same bits
__global__ __launch_bounds__(256) void mi_scores_kernel(const float* __restrict__ x1a, const float* __restrict__ Ua,
                                                        const float* __restrict__ ba, const float* __restrict__ x1b,
                                                        const float* __restrict__ Ub, const float* __restrict__ bb,
                                                        int B, int d, float* __restrict__ S) {
  const int k = blockIdx.y;
  const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= B) return;
  const float* x = k < 2 ? x1a : x1b;
  const float* y = (k < 2 ? Ua : Ub) + (long)(k & 1) * B * d;
  const float* bias = k < 2 ? ba : bb;
  float s = 0.f;
  for (int c = lane; c < d; c += 64) s += x[r * d + c] * y[r * d + c];
  s = c2::wave_sum(s);
  if (lane == 0) S[(long)k * B + r] = s + (bias ? bias[0] : 0.f);
}

// s: [4][B] = sim_a_pos, sim_a_neg, sim_b_pos, sim_b_neg (labels 1,0,1,0).
// loss_mi = Σ_k Σ_b BCE(s_k, y_k) / Bn;  ds[k][b] = (σ(s) - y)/Bn  (Bn = global batch; = B on one device)
__global__ __launch_bounds__(1024) void mi_loss_kernel(const float* __restrict__ s, int B, float Bn,
                                                       float* __restrict__ loss_mi, float* __restrict__ ds) {
  __shared__ float red[1024];
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float x = s[k * B + b];
      const float y = (k & 1) ? 0.f : 1.f;
      acc[k] += fmaxf(x, 0.f) - x * y + log1pf(__expf(-fabsf(x)));
      const float sig = 1.f / (1.f + __expf(-x));
      ds[k * B + b] = (sig - y) / Bn;
    }
  }
  // fixed-order reduction: wave trees, then the wave sums in wave order (one barrier)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float v = c2::wave_sum(acc[k]);
    if (lane == 0) red[k * 16 + w] = v;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float tot = 0.f;
    for (int k = 0; k < 4; ++k) {
      float t = 0.f;
      for (int q = 0; q < nw; ++q) t += red[k * 16 + q];
      tot += t / Bn;
    }
    *loss_mi = tot;
  }
}

// Hcat = [hs_r ; hs_r + hx_r], Hpad = [hs_r ; hx_r] (rows (b, L-R+k)), tcat = [t_share_r ; t_spec_r]
// (row maps: a [B·L] → compact row index of hs / hx when they hold a row subset, else null)
__global__ void rec_gather_kernel(const float* __restrict__ hs, const int* __restrict__ hs_map,
                                  const float* __restrict__ hx, const int* __restrict__ hx_map, int B, int L, int d,
                                  int R, float* __restrict__ Hcat, float* __restrict__ Hpad) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long BR = (long)B * R;
  if (i >= BR * d) return;
  const long r = i / d;
  const int c = (int)(i % d);
  const long b = r / R, l = L - R + r % R;
  const long bl = b * L + l;
  const float a = hs[(hs_map ? hs_map[bl] : bl) * d + c], x = hx[(hx_map ? hx_map[bl] : bl) * d + c];
  Hcat[r * d + c] = a;
  Hcat[(BR + r) * d + c] = a + x;
  Hpad[r * d + c] = a;
  Hpad[(BR + r) * d + c] = x;
}

// The classifier head's operand rows in one pass: Hpad = [hs_r ; hx_r] over the 2BR stacked rows and, for the Mv valid
// rows (idx: compact → stacked row), Hc = Hcat[idx] (Hcat = [hs_r ; hs_r + hx_r]) and its MFMA image — split
// hi ‖ lo [M_pad][2d] (split) or bf16 [M_pad][d], rows Mv..M_pad zero.  The values of rec_gather → gather_rows →
// split_bf16 / to_bf16 (same additions, same RNE conversions) without the [2BR, d] Hcat round trip.  4 columns per
// thread: threads [0, BR·d/4) write Hpad, the rest the M_pad compact rows.
__global__ void rec_gather_c_kernel(const float* __restrict__ hs, const int* __restrict__ hs_map,
                                    const float* __restrict__ hx, const int* __restrict__ hx_map, int B, int L, int d,
                                    int R, const int* __restrict__ idx, int Mv, int M_pad, int split,
                                    float* __restrict__ Hpad, float* __restrict__ Hc, c2::tbf16* __restrict__ img) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int d4 = d >> 2;
  const long BR = (long)B * R;
  auto rows = [&](long r, float4& a, float4& x, int c) {  // the (b, L-R+k) rows of hs and hx for stacked row r < BR
    const long b = r / R, l = L - R + r % R, bl = b * L + l;
    a = *(const float4*)(hs + (hs_map ? hs_map[bl] : bl) * d + c);
    x = *(const float4*)(hx + (hx_map ? hx_map[bl] : bl) * d + c);
  };
  if (i < BR * d4) {
    const long r = i / d4;
    const int c = 4 * (int)(i % d4);
    float4 a, x;
    rows(r, a, x, c);
    *(float4*)(Hpad + r * d + c) = a;
    *(float4*)(Hpad + (BR + r) * d + c) = x;
    return;
  }
  const long j = i - BR * d4;
  if (j >= (long)M_pad * d4) return;
  const long m = j / d4;
  const int c = 4 * (int)(j % d4);
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  if (m < Mv) {
    const long rr = idx[m];
    float4 a, x;
    rows(rr % BR, a, x, c);
    v = rr < BR ? a : make_float4(a.x + x.x, a.y + x.y, a.z + x.z, a.w + x.w);
    *(float4*)(Hc + m * d + c) = v;
  }
  c2::tbf16 h[4] = {(c2::tbf16)v.x, (c2::tbf16)v.y, (c2::tbf16)v.z, (c2::tbf16)v.w};
  if (split) {
    c2::tbf16 lo[4] = {(c2::tbf16)(v.x - (float)h[0]), (c2::tbf16)(v.y - (float)h[1]), (c2::tbf16)(v.z - (float)h[2]),
                       (c2::tbf16)(v.w - (float)h[3])};
    c2::tbf16* o = img + m * 2 * d + c;
    for (int k = 0; k < 4; ++k) {
      o[k] = h[k];
      o[d + k] = lo[k];
    }
  } else {
    c2::tbf16* o = img + m * d + c;
    for (int k = 0; k < 4; ++k) o[k] = h[k];
  }
}

__global__ void rec_targets_kernel(const int64_t* __restrict__ ts, const int64_t* __restrict__ tx, int B, int L, int R,
                                   int64_t* __restrict__ tcat) {
  const long r = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long BR = (long)B * R;
  if (r >= BR) return;
  const long b = r / R, l = L - R + r % R;
  tcat[r] = ts[b * L + l];
  tcat[BR + r] = tx[b * L + l];
}

// dhs[b,l] += dHcat[r] + dHcat[BR+r] + pad[r]·wpad;  dhx[b,l] += dHcat[BR+r] + pad[BR+r]·wpad
// (pad = the pad column of dlogits, stride pad_ld: the classifier_pad input gradient is its outer product
// with wpad, folded in here instead of being materialised)
__global__ void rec_scatter_kernel(const float* __restrict__ dHcat, const float* __restrict__ pad, long pad_ld,
                                   const float* __restrict__ wpad, int B, int L,
                                   int d, int R, float* __restrict__ dhs, const int* __restrict__ dhs_map,
                                   float* __restrict__ dhx, const int* __restrict__ dhx_map) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long BR = (long)B * R;
  if (i >= BR * d) return;
  const long r = i / d;
  const int c = (int)(i % d);
  const long b = r / R, l = L - R + r % R;
  const long bl = b * L + l;
  const float g1 = dHcat[r * d + c], g2 = dHcat[(BR + r) * d + c], wp = wpad[c];
  dhs[(dhs_map ? dhs_map[bl] : bl) * d + c] += g1 + g2 + pad[r * pad_ld] * wp;
  dhx[(dhx_map ? dhx_map[bl] : bl) * d + c] += g2 + pad[(BR + r) * pad_ld] * wp;
}

// Per-row CE: lse over ncol logits, loss_row = valid ? lse - logit[t] : 0.  One wave per row.
__global__ __launch_bounds__(256) void ce_fwd_kernel(const float* __restrict__ lg, long ld, int M, int ncol,
                                                     const int64_t* __restrict__ tgt, int ignore,
                                                     float* __restrict__ lse_out, float* __restrict__ loss_row) {
  const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= M) return;
  const float* row = lg + r * ld;
  float m = -INFINITY, s = 0.f;
  for (int c = lane; c < ncol; c += 64) {
    const float v = row[c];
    if (v > m) {
      s = s * __expf(m - v) + 1.f;
      m = v;
    } else {
      s += __expf(v - m);
    }
  }
  // combine (m, s) across the wave
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    const float mm = fmaxf(m, m2);
    s = (m == -INFINITY ? 0.f : s * __expf(m - mm)) + (m2 == -INFINITY ? 0.f : s2 * __expf(m2 - mm));
    m = mm;
  }
  if (lane == 0) {
    const float lse = m + logf(s);
    lse_out[r] = lse;
    const long t = tgt[r];
    loss_row[r] = (t != ignore) ? lse - row[t] : 0.f;
  }
}

// dl[r,c] = (exp(l - lse) - [c==t]) * w_r,  w_r = valid ? gscale*lam*coef[r >= split] : 0.  In place allowed.
__global__ __launch_bounds__(256) void ce_bwd_kernel(float* __restrict__ lg, long ld, int M, int ncol,
                                                     const int64_t* __restrict__ tgt, int ignore,
                                                     const float* __restrict__ lse, const float* __restrict__ coef,
                                                     int split, const float* __restrict__ gscale, float lam) {
  const int ncb = (ncol + 255) / 256;
  const long r = blockIdx.x / ncb;
  const int c = (int)(blockIdx.x % ncb) * 256 + threadIdx.x;
  if (r >= M || c >= ncol) return;
  const long t = tgt[r];
  const float w = (t != ignore) ? gscale[0] * lam * coef[r >= split ? 1 : 0] : 0.f;
  float* p = lg + r * ld + c;
  const float e = __expf(*p - lse[r]);
  *p = (e - (c == t ? 1.f : 0.f)) * w;
}

// out[r, :] += a[r*sa] * v[:]
__global__ void outer_add_kernel(const float* __restrict__ a, long sa, const float* __restrict__ v, int M, int d,
                                 float* __restrict__ out, long ldo) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)M * d) return;
  const long r = i / d;
  const int c = (int)(i % d);
  out[r * ldo + c] += a[r * sa] * v[c];
}

// Per-head partial sums (trainer.py:143-152) of this rank's rows: vec[0..3] = Σ loss over
// valid rows of (share_a, spec_a, share_b, spec_b), vec[4..7] = their valid counts.
// rowsA/rowsB: per-row CE of the [share ; specific] stacks (2*BR rows each).
// stage 1: one row per thread, block partials part[blk][8] (wave trees, then wave order); stage 2: one wave
// adds the block partials in block order → vec[0..8).  Fixed orders: deterministic.
__global__ __launch_bounds__(256) void loss_partials_kernel(const float* __restrict__ rowsA,
                                                            const int64_t* __restrict__ tA, int n_a,
                                                            const float* __restrict__ rowsB,
                                                            const int64_t* __restrict__ tB, int n_b, int BR,
                                                            float* __restrict__ part) {
  __shared__ float red[8][4];
  const int r = blockIdx.x * 256 + threadIdx.x;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (r < 2 * BR) {
    const int h = r >= BR ? 1 : 0;
    if (tA[r] != n_a) {
      acc[h] = rowsA ? rowsA[r] : 0.f;
      acc[4 + h] = 1.f;
    }
    if (tB[r] != n_b) {
      acc[2 + h] = rowsB ? rowsB[r] : 0.f;
      acc[6 + h] = 1.f;
    }
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    float v = acc[k];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) red[k][w] = v;
  }
  __syncthreads();
  if (threadIdx.x < 8)
    part[blockIdx.x * 8 + threadIdx.x] = (red[threadIdx.x][0] + red[threadIdx.x][1]) +
                                         (red[threadIdx.x][2] + red[threadIdx.x][3]);
}

__global__ __launch_bounds__(64) void loss_partials_final_kernel(const float* __restrict__ part, int nblk,
                                                                 float* __restrict__ vec) {
  const int k = threadIdx.x & 7, g = threadIdx.x >> 3;  // 8 lane groups stride over the blocks
  float t = 0.f;
  for (int b = g; b < nblk; b += 8) t += part[b * 8 + k];
#pragma unroll
  for (int o = 8; o < 64; o <<= 1) t += __shfl_xor(t, o, 64);
  if (threadIdx.x < 8) vec[k] = t;
}


// scalar combination (trainer.py:143-156) from the (globally reduced) vec[0..8]
// (vec[8] = loss_mi).  out3 = (loss, loss_rec, loss_mi); coefA/coefB = per-row
// gradient weights (share, specific) of the two stacks.  cnt (nullable): the valid-target counts
// (cnt[4..7]) when they were reduced separately, ahead of the forward (data parallel).
__global__ void finalize_kernel(const float* __restrict__ vec, const float* __restrict__ cnt, float RB, float lam,
                                float* __restrict__ out3, float* __restrict__ coefA, float* __restrict__ coefB) {
  if (threadIdx.x != 0) return;
  const float* c = cnt ? cnt : vec;
  const float ce_sa = vec[0] / c[4], ce_a = vec[1] / c[5];
  const float ce_sb = vec[2] / c[6], ce_b = vec[3] / c[7];
  const float loss_share = ce_sa * c[4] / RB + ce_sb * c[6] / RB;
  const float loss_rec = loss_share + ce_a + ce_b;
  const float lmi = vec[8];
  out3[0] = lam * loss_rec + (1.f - lam) * lmi;
  out3[1] = loss_rec;
  out3[2] = lmi;
  coefA[0] = 1.f / RB;
  coefA[1] = 1.f / c[5];
  coefB[0] = 1.f / RB;
  coefB[1] = 1.f / c[7];
}

// acc[0..2] += w · (loss, loss_rec, loss_mi): the epoch's sample-weighted loss sums (trainer.py:50-52, run_epoch)
__global__ void loss_accumulate_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                       const float* __restrict__ c, float w, float* __restrict__ acc) {
  if (threadIdx.x == 0) {
    acc[0] += w * a[0];
    acc[1] += w * b[0];
    acc[2] += w * c[0];
  }
}

// ds[k][b] *= gscale * (1 - lam)
__global__ void scale_ds_kernel(float* __restrict__ ds, int n, const float* __restrict__ gscale, float f) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) ds[i] *= gscale[0] * f;
}

// out[i] = x[i] * s[i / d] (row scale; dx1 = ds ⊙ u)
__global__ void rowscale_kernel(const float* __restrict__ x, const float* __restrict__ s, long n, int d,
                                float* __restrict__ out, int accumulate) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float v = x[i] * s[i / d];
  out[i] = accumulate ? out[i] + v : v;
}

// The two bilinear discriminators' row-scale products of the MI-loss backward (trainer.py:104-119 through D_a / D_b)
// in ONE launch, blockIdx.y = discriminator j (replaces 4 c2dsr_rowscale launches per discriminator):
//   dx1_j = dS[2j] ⊙ U_j[0:B] + dS[2j+1] ⊙ U_j[B:2B],  dU_j[0:B] = dS[2j] ⊙ x1_j,  dU_j[B:2B] = dS[2j+1] ⊙ x1_j
// (dS [4][B] row scales; U_j, dU_j [2B][d]; x1_j, dx1_j [B][d]); the two products of dx1 are rounded before their sum
__global__ void bilinear_ds_kernel(const float* __restrict__ Ua, const float* __restrict__ Ub,
                                   const float* __restrict__ xa, const float* __restrict__ xb,
                                   const float* __restrict__ dS, int B, int d, float* __restrict__ dxa,
                                   float* __restrict__ dxb, float* __restrict__ dUa, float* __restrict__ dUb) {
  const long n4 = (long)B * d / 4;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  const int j = blockIdx.y;
  const float4* U = (const float4*)(j ? Ub : Ua);
  const float4* x = (const float4*)(j ? xb : xa);
  float4* dx = (float4*)(j ? dxb : dxa);
  float4* dU = (float4*)(j ? dUb : dUa);
  const int r = (int)(i * 4 / d);
  const float s0 = dS[(long)(2 * j) * B + r], s1 = dS[(long)(2 * j + 1) * B + r];
  const float4 u0 = U[i], u1 = U[n4 + i], xv = x[i];
  // explicitly rounded products and sum (no fma contraction: each product is rounded as rowscale's was)
  auto rsum = [&](float p, float q) {
    float a = s0 * p, b = s1 * q;
    asm volatile("" : "+v"(a), "+v"(b));  // rounded products: the sum below must not contract into an fma
    return a + b;
  };
  dx[i] = make_float4(rsum(u0.x, u1.x), rsum(u0.y, u1.y), rsum(u0.z, u1.z), rsum(u0.w, u1.w));
  dU[i] = make_float4(s0 * xv.x, s0 * xv.y, s0 * xv.z, s0 * xv.w);
  dU[n4 + i] = make_float4(s1 * xv.x, s1 * xv.y, s1 * xv.z, s1 * xv.w);
}

}  // namespace

C2_API int c2dsr_bilinear_ds(const float* Ua, const float* Ub, const float* x1a, const float* x1b, const float* dS,
                             int B, int d, float* dx1a, float* dx1b, float* dUa, float* dUb, void* stream) {
  if (B < 0 || d <= 0 || d % 4) return (int)hipErrorInvalidValue;
  if (B == 0) return 0;
  const long n4 = (long)B * d / 4;
  bilinear_ds_kernel<<<dim3((unsigned)c2::ceil_div(n4, 256), 2), 256, 0, (hipStream_t)stream>>>(Ua, Ub, x1a, x1b, dS, B,
                                                                                                d, dx1a, dx1b, dUa, dUb);
  C2_CHECK_LAUNCH();
  return 0;
}

C2_API int c2dsr_pool_weights(const int64_t* gm, int B, int L, float* w, void* stream) {
  if (B == 0) return 0;
  pool_weights_kernel<<<c2::ceil_div(B, 4), 256, 0, (hipStream_t)stream>>>(gm, B, L, w);
  C2_CHECK_LAUNCH();
  return 0;
}
C2_API int c2dsr_pool_fwd(const float* h, const float* w, int B, int L, int d, float* out, void* stream) {
  const long n = (long)B * d;
  if (n == 0) return 0;
  pool_fwd_kernel<<<c2::ceil_div(n, 256), 256, 0, (hipStream_t)stream>>>(h, w, B, L, d, out);
  C2_CHECK_LAUNCH();
  return 0;
}
C2_API int c2dsr_pool_bwd(const float* dout, const float* w, int B, int L, int d, float* dh, void* stream) {
  const long n = (long)B * L * d / 4;
  if (n == 0 || d % 4) return n == 0 ? 0 : (int)hipErrorInvalidValue;
  pool_bwd_kernel<<<c2::ceil_div(n, 256), 256, 0, (hipStream_t)stream>>>(dout, w, B, L, d, dh);
  C2_CHECK_LAUNCH();
  return 0;
}
C2_API int c2dsr_pool2_fwd(const float* h, const int* hmap, const float* w1, const float* w2, int B, int L, int d,
                           float* out1, float* out2, void* stream) {
  if (B == 0) return 0;
  if (d % 4 || (w2 && !out2)) return (int)hipErrorInvalidValue;
  pool2_fwd_kernel<<<B, 256, 0, (hipStream_t)stream>>>(h, hmap, w1, w2, B, L, d, out1, out2);
  C2_CHECK_LAUNCH();
  return 0;
}
C2_API int c2dsr_pool2_bwd(const float* d1, const float* w1, const float* d2, const float* w2, int B, int L, int d,
                           const int* idx, int n_rows, int accumulate, float* dh, void* stream) {
  const long rows = idx ? (long)n_rows : (long)B * L;
  const long n = rows * d / 4;
  if (n == 0 || d % 4) return n == 0 ? 0 : (int)hipErrorInvalidValue;
  pool2_bwd_kernel<<<c2::ceil_div(n, 256), 256, 0, (hipStream_t)stream>>>(d1, w1, d2, w2, L, d, rows, idx, accumulate,
                                                                          dh);
  C2_CHECK_LAUNCH();
  return 0;
}
C2_API size_t c2dsr_compact_workspace(int M, int n_sets) {
  return (size_t)c2::ceil_div(M, CMP_TILE) * (size_t)(n_sets < 2 ? 2 : 8) * sizeof(int);
}
C2_API int c2dsr_compact_valid(const int64_t* t, int M, int split, int ignore, int* idx, int* inv, int64_t* tc,
                               int* counts, int* ws, int* err, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (M < 0) return (int)hipErrorInvalidValue;
  if (M == 0) return (int)hipMemsetAsync(counts, 0, 2 * sizeof(int), s);
  return compact_rows(ValidOp{t, split, ignore, idx, inv, tc, counts, err}, M, ws, s);
}
C2_API int c2dsr_need_rows(const int64_t* gm_a, const int64_t* gm_b, int B, int L, int R, int n_sets, int bits,
                           int* idx, int* inv, int* count, int* off, int* ws, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (B < 0 || L <= 0 || n_sets < 1 || n_sets > 8) return (int)hipErrorInvalidValue;
  if (B == 0) {
    if (off) (void)hipMemsetAsync(off, 0, n_sets * sizeof(int), s);
    return (int)hipMemsetAsync(count, 0, n_sets * sizeof(int), s);
  }
  const int M = B * L;
  return compact_rows(NeedOp{gm_a, gm_b, L, R, n_sets, bits, idx, inv, count, off, (long)M}, M, ws, s);
}
C2_API int c2dsr_pad_rows(const int64_t* seqs, int64_t pad, int B, int L, int n_sets, int* idx, int* inv, int* count,
                          int* off, int* ws, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (B < 0 || L <= 0 || n_sets < 1 || n_sets > 8 || !off) return (int)hipErrorInvalidValue;
  if (B == 0) {
    (void)hipMemsetAsync(off, 0, n_sets * sizeof(int), s);
    return (int)hipMemsetAsync(count, 0, n_sets * sizeof(int), s);
  }
  const int M = B * L;
  return compact_rows(PadOp{seqs, pad, L, n_sets, idx, inv, count, off, (long)M}, M, ws, s);
}
C2_API int c2dsr_combine_rows(const float* a, const int* inv_a, const float* b, const int* inv_b, int M, int d,
                              float* dst, void* stream) {
  if (M <= 0) return 0;
  if (d <= 0 || d % 4) return (int)hipErrorInvalidValue;
  const long work = (long)M * d / 4;
  combine_rows_kernel<<<c2::ceil_div(work, 256), 256, 0, (hipStream_t)stream>>>(a, inv_a, b, inv_b, M, d / 4, dst);
  C2_CHECK_LAUNCH();
  return 0;
}
C2_API int c2dsr_gather_rows(const float* src, long ld, const int* idx, int n, int d, float* dst, void* stream) {
  if (n <= 0 || d <= 0) return 0;
  const long work = (d % 4 == 0 && ld % 4 == 0) ? (long)n * d / 4 : (long)n * d;
  gather_rows_kernel<<<c2::ceil_div(work, 256), 256, 0, (hipStream_t)stream>>>(src, ld, idx, n, d, dst);
  C2_CHECK_LAUNCH();
  return 0;
}
C2_API int c2dsr_expand_rows(const float* src, const int* inv, int M, int d, float* dst, void* stream) {
  if (M <= 0 || d <= 0) return 0;
  const long work = d % 4 == 0 ? (long)M * d / 4 : (long)M * d;
  expand_rows_kernel<<<c2::ceil_div(work, 256), 256, 0, (hipStream_t)stream>>>(src, inv, M, d, dst);
  C2_CHECK_LAUNCH();
  return 0;
}
C2_API int c2dsr_rowdot(const float* x, long ldx, const float* y, long ldy, int M, int d, const float* bias,
                        float* out, long ldo, void* stream) {
  if (M == 0) return 0;
  rowdot_kernel<<<c2::ceil_div(M, 4), 256, 0, (hipStream_t)stream>>>(x, ldx, y, ldy, M, d, bias, out, ldo);
  C2_CHECK_LAUNCH();
  return 0;
}
C2_API int c2dsr_mi_scores(const float* x1a, const float* Ua, const float* ba, const float* x1b, const float* Ub,
                           const float* bb, int B, int d, float* S, void* stream) {
  if (B < 0 || d <= 0) return (int)hipErrorInvalidValue;
  if (B == 0) return 0;
  mi_scores_kernel<<<dim3((unsigned)c2::ceil_div(B, 4), 4), 256, 0, (hipStream_t)stream>>>(x1a, Ua, ba, x1b, Ub, bb, B, d,
                                                                                       S);
  C2_CHECK_LAUNCH();
  return 0;
}
C2_API int c2dsr_mi_loss(const float* s, int B, int B_norm, float* loss_mi, float* ds, void* stream) {
  mi_loss_kernel<<<1, 1024, 0, (hipStream_t)stream>>>(s, B, (float)B_norm, loss_mi, ds);
  C2_CHECK_LAUNCH();
  return 0;
}
C2_API int c2dsr_rec_gather(const float* hs, const int* hs_map, const float* hx, const int* hx_map, int B, int L, int d,
                            int R, float* Hcat, float* Hpad, void* stream) {
  const long n = (long)B * R * d;
  if (n == 0) return 0;
  rec_gather_kernel<<<c2::ceil_div(n, 256), 256, 0, (hipStream_t)stream>>>(hs, hs_map, hx, hx_map, B, L, d, R, Hcat,
                                                                           Hpad);
  C2_CHECK_LAUNCH();
  return 0;
}
C2_API int c2dsr_rec_gather_compact(const float* hs, const int* hs_map, const float* hx, const int* hx_map, int B, int L,
                                     int d, int R, const int* idx, int Mv, int M_pad, int split, float* Hpad, float* Hc,
                                     void* img, void* stream) {
  if (d % 4 || Mv < 0 || M_pad < Mv || (Mv && (!idx || !Hc)) || !img) return (int)hipErrorInvalidValue;
  const long n = ((long)B * R + M_pad) * (d / 4);
  if (n == 0) return 0;
  rec_gather_c_kernel<<<c2::ceil_div(n, 256), 256, 0, (hipStream_t)stream>>>(hs, hs_map, hx, hx_map, B, L, d, R, idx, Mv,
                                                                             M_pad, split, Hpad, Hc, (c2::tbf16*)img);
  C2_CHECK_LAUNCH();
  return 0;
}
C2_API int c2dsr_rec_targets(const int64_t* ts, const int64_t* tx, int B, int L, int R, int64_t* tcat, void* stream) {
  const long n = (long)B * R;
  if (n == 0) return 0;
  rec_targets_kernel<<<c2::ceil_div(n, 256), 256, 0, (hipStream_t)stream>>>(ts, tx, B, L, R, tcat);
  C2_CHECK_LAUNCH();
  return 0;
}
C2_API int c2dsr_rec_scatter(const float* dHcat, const float* pad, long pad_ld, const float* wpad, int B, int L, int d,
                             int R, float* dhs, const int* dhs_map, float* dhx, const int* dhx_map, void* stream) {
  const long n = (long)B * R * d;
  if (n == 0) return 0;
  rec_scatter_kernel<<<c2::ceil_div(n, 256), 256, 0, (hipStream_t)stream>>>(dHcat, pad, pad_ld, wpad, B, L, d, R, dhs,
                                                                            dhs_map, dhx, dhx_map);
  C2_CHECK_LAUNCH();
  return 0;
}
C2_API int c2dsr_ce_fwd(const float* logits, long ld, int M, int ncol, const int64_t* tgt, int ignore, float* lse,
                        float* loss_row, void* stream) {
  if (M == 0) return 0;
  ce_fwd_kernel<<<c2::ceil_div(M, 4), 256, 0, (hipStream_t)stream>>>(logits, ld, M, ncol, tgt, ignore, lse, loss_row);
  C2_CHECK_LAUNCH();
  return 0;
}
C2_API int c2dsr_ce_bwd(float* logits, long ld, int M, int ncol, const int64_t* tgt, int ignore, const float* lse,
                        const float* coef, int split, const float* gscale, float lam, void* stream) {
  if (M == 0) return 0;
  dim3 grid((unsigned)((long)c2::ceil_div(ncol, 256) * M));
  ce_bwd_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(logits, ld, M, ncol, tgt, ignore, lse, coef, split, gscale, lam);
  C2_CHECK_LAUNCH();
  return 0;
}
C2_API int c2dsr_outer_add(const float* a, long sa, const float* v, int M, int d, float* out, long ldo, void* stream) {
  const long n = (long)M * d;
  if (n == 0) return 0;
  outer_add_kernel<<<c2::ceil_div(n, 256), 256, 0, (hipStream_t)stream>>>(a, sa, v, M, d, out, ldo);
  C2_CHECK_LAUNCH();
  return 0;
}
// the stage-1 partials of c2dsr_loss_partials (floats), allocated by the caller on the launch stream
C2_API size_t c2dsr_loss_partials_workspace(int BR) { return (size_t)c2::ceil_div(2 * BR, 256) * 8; }
C2_API int c2dsr_loss_partials(const float* rowsA, const int64_t* tA, int n_a, const float* rowsB, const int64_t* tB,
                               int n_b, int BR, float* vec, float* part, void* stream) {
  const int nblk = c2::ceil_div(2 * BR, 256);
  if (nblk == 0) return (int)hipMemsetAsync(vec, 0, 8 * sizeof(float), (hipStream_t)stream);
  if (!part) return (int)hipErrorInvalidValue;
  loss_partials_kernel<<<nblk, 256, 0, (hipStream_t)stream>>>(rowsA, tA, n_a, rowsB, tB, n_b, BR, part);
  loss_partials_final_kernel<<<1, 64, 0, (hipStream_t)stream>>>(part, nblk, vec);
  C2_CHECK_LAUNCH();
  return 0;
}
C2_API int c2dsr_loss_finalize(const float* vec, const float* cnt, int BR_global, float lam, float* out3, float* coefA,
                               float* coefB, void* stream) {
  finalize_kernel<<<1, 64, 0, (hipStream_t)stream>>>(vec, cnt, (float)BR_global, lam, out3, coefA, coefB);
  C2_CHECK_LAUNCH();
  return 0;
}
C2_API int c2dsr_loss_accumulate(const float* loss, const float* loss_rec, const float* loss_mi, float w, float* acc3,
                                  void* stream) {
  if (!loss || !loss_rec || !loss_mi || !acc3) return (int)hipErrorInvalidValue;
  loss_accumulate_kernel<<<1, 64, 0, (hipStream_t)stream>>>(loss, loss_rec, loss_mi, w, acc3);
  C2_CHECK_LAUNCH();
  return 0;
}
C2_API int c2dsr_scale_ds(float* ds, int n, const float* gscale, float f, void* stream) {
  if (n == 0) return 0;
  scale_ds_kernel<<<c2::ceil_div(n, 256), 256, 0, (hipStream_t)stream>>>(ds, n, gscale, f);
  C2_CHECK_LAUNCH();
  return 0;
}
C2_API int c2dsr_rowscale(const float* x, const float* s, long n, int d, float* out, int accumulate, void* stream) {
  if (n == 0) return 0;
  rowscale_kernel<<<c2::ceil_div(n, 256), 256, 0, (hipStream_t)stream>>>(x, s, n, d, out, accumulate);
  C2_CHECK_LAUNCH();
  return 0;
}
