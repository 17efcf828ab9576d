// Self-attention core for the sequence encoder: S = QKᵀ/√dh + mask, P = softmax(S),
// O = dropout(P)·V, one workgroup per (sequence, head), everything for a
// sequence staged in LDS (L <= 128).
//
// Replaces F.multi_head_attention_forward → scaled_dot_product_attention (math path)
// as reached from models/encoders.py:33 with attn_mask = causal (encoders.py:14) and
// key_padding_mask = (seq != pad) (encoders.py:33) merged additively — i.e. query i
// attends only to keys j <= i that ARE padding (Q1); a row with no admissible key
// yields 0 (Q2).  Keys that are masked for every query are skipped outright.
#include "common.h"

namespace {

// head-dim chunk staged in LDS for the QKᵀ-type products (smaller at L=128 to fit 160 KB)
template <int LMAX>
struct Ch {
  static constexpr int V = LMAX >= 128 ? 16 : 32;
};

// per-thread ownership of (i,j) pairs of an L x L tile: pair = t + 256*u
template <int LMAX>
struct Pairs {
  static constexpr int U = (LMAX * LMAX + 255) / 256;
};

// dot[i][j] = Σ_c X[i][c]·Y[j][c] over the head dim for admissible pairs, staged in CH-wide chunks.
template <int LMAX>
__device__ __forceinline__ void pair_dots(const float* __restrict__ Xg, long xs, const float* __restrict__ Yg, long ys,
                                          int L, int dh, const unsigned char* __restrict__ keyok, float* Xl, float* Yl,
                                          float (&acc)[Pairs<LMAX>::U]) {
  constexpr int CH = Ch<LMAX>::V;
  const int t = threadIdx.x;
#pragma unroll
  for (int u = 0; u < Pairs<LMAX>::U; ++u) acc[u] = 0.f;
  for (int c0 = 0; c0 < dh; c0 += CH) {
    __syncthreads();
    for (int e = t; e < L * CH; e += 256) {
      const int i = e / CH, c = e % CH;
      Xl[i * (CH + 1) + c] = (c0 + c < dh) ? Xg[i * xs + c0 + c] : 0.f;
      Yl[i * (CH + 1) + c] = (c0 + c < dh) ? Yg[i * ys + c0 + c] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < Pairs<LMAX>::U; ++u) {
      const int pr = t + 256 * u;
      const int i = pr / LMAX, j = pr % LMAX;
      if (i < L && j <= i && keyok[j]) {
        float s = acc[u];
#pragma unroll 8
        for (int c = 0; c < CH; ++c) s = fmaf(Xl[i * (CH + 1) + c], Yl[j * (CH + 1) + c], s);
        acc[u] = s;
      }
    }
  }
  __syncthreads();
}

template <int LMAX>
__global__ __launch_bounds__(256) void attn_fwd_kernel(const float* __restrict__ qkv, const int64_t* __restrict__ seq,
                                                       int64_t pad, int L, int d, int H, c2::Drop drop,
                                                       int64_t b_base, float* __restrict__ out,
                                                       float* __restrict__ Psave) {
  const int b = blockIdx.x / H, h = blockIdx.x % H;
  constexpr int CH = Ch<LMAX>::V;
  const int dh = d / H;
  const int t = threadIdx.x;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* Ps = sm;                         // [LMAX][LMAX+1]
  float* Xl = Ps + LMAX * (LMAX + 1);     // [LMAX][CH+1]
  float* Yl = Xl + LMAX * (CH + 1);       // [LMAX][CH+1]
  __shared__ unsigned char keyok[LMAX];
  for (int j = t; j < LMAX; j += 256) keyok[j] = (j < L) && (seq[(long)b * L + j] == pad);
  __syncthreads();
  const long rs = 3l * d;  // row stride of qkv
  const float* Q = qkv + (long)b * L * rs + h * dh;
  const float* K = Q + d;
  const float* V = Q + 2 * d;
  float acc[Pairs<LMAX>::U];
  pair_dots<LMAX>(Q, rs, K, rs, L, dh, keyok, Xl, Yl, acc);
  const float sc = 1.0f / sqrtf((float)dh);
#pragma unroll
  for (int u = 0; u < Pairs<LMAX>::U; ++u) {
    const int pr = t + 256 * u;
    const int i = pr / LMAX, j = pr % LMAX;
    if (i < L && j < L) Ps[i * (LMAX + 1) + j] = (j <= i && keyok[j]) ? acc[u] * sc : -INFINITY;
  }
  __syncthreads();
  // softmax per row: wave w rows w, w+4, ...
  const int w = t >> 6, lane = t & 63;
  for (int i = w; i < L; i += 4) {
    float m = -INFINITY;
    for (int j = lane; j < L; j += 64) m = fmaxf(m, Ps[i * (LMAX + 1) + j]);
    m = c2::wave_max(m);
    float s = 0.f;
    for (int j = lane; j < L; j += 64) {
      const float e = (m == -INFINITY) ? 0.f : __expf(Ps[i * (LMAX + 1) + j] - m);
      Ps[i * (LMAX + 1) + j] = e;
      s += e;
    }
    s = c2::wave_sum(s);
    const float inv = s > 0.f ? 1.0f / s : 0.f;
    const uint64_t rowidx = ((uint64_t)((b_base + b) * H + h) * L + i) * L;
    for (int j = lane; j < L; j += 64) {
      const float pv = Ps[i * (LMAX + 1) + j] * inv;
      Psave[((long)blockIdx.x * L + i) * L + j] = pv;
      Ps[i * (LMAX + 1) + j] = pv * drop.mul(rowidx + j);
    }
  }
  __syncthreads();
  // O[i][c] = Σ_{j<=i, key j admissible} Pd[i][j] V[j][c]; thread owns column c
  for (int c = t; c < dh; c += 256) {
    float o[LMAX];
#pragma unroll
    for (int i = 0; i < LMAX; ++i) o[i] = 0.f;
    for (int j = 0; j < L; ++j) {
      if (!keyok[j]) continue;
      const float v = V[(long)j * rs + c];
#pragma unroll
      for (int i = 0; i < LMAX; ++i)
        if (i >= j && i < L) o[i] = fmaf(Ps[i * (LMAX + 1) + j], v, o[i]);
    }
#pragma unroll
    for (int i = 0; i < LMAX; ++i)
      if (i < L) out[((long)b * L + i) * d + h * dh + c] = o[i];
  }
}

template <int LMAX>
__global__ __launch_bounds__(256) void attn_bwd_kernel(const float* __restrict__ qkv, const int64_t* __restrict__ seq,
                                                       int64_t pad, int L, int d, int H, c2::Drop drop,
                                                       int64_t b_base, const float* __restrict__ Psave,
                                                       const float* __restrict__ dout, float* __restrict__ dqkv) {
  const int b = blockIdx.x / H, h = blockIdx.x % H;
  constexpr int CH = Ch<LMAX>::V;
  const int dh = d / H;
  const int t = threadIdx.x;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* Pd = sm;                          // dropped probabilities [LMAX][LMAX+1]
  float* dS = Pd + LMAX * (LMAX + 1);      // [LMAX][LMAX+1]
  float* Xl = dS + LMAX * (LMAX + 1);
  float* Yl = Xl + LMAX * (CH + 1);
  __shared__ unsigned char keyok[LMAX];
  for (int j = t; j < LMAX; j += 256) keyok[j] = (j < L) && (seq[(long)b * L + j] == pad);
  const long rs = 3l * d;
  const float* Q = qkv + (long)b * L * rs + h * dh;
  const float* K = Q + d;
  const float* V = Q + 2 * d;
  const float* dO = dout + (long)b * L * d + h * dh;
  float* dQ = dqkv + (long)b * L * rs + h * dh;
  float* dK = dQ + d;
  float* dV = dQ + 2 * d;
  __syncthreads();
  // dPd[i][j] = dO_i · V_j
  float acc[Pairs<LMAX>::U];
  pair_dots<LMAX>(dO, d, V, rs, L, dh, keyok, Xl, Yl, acc);
  const float* Pg = Psave + (long)blockIdx.x * L * L;
#pragma unroll
  for (int u = 0; u < Pairs<LMAX>::U; ++u) {
    const int pr = t + 256 * u;
    const int i = pr / LMAX, j = pr % LMAX;
    if (i < L && j < L) {
      const uint64_t idx = ((uint64_t)((b_base + b) * H + h) * L + i) * L + j;
      const float mk = drop.mul(idx);
      const float p = Pg[(long)i * L + j];
      Pd[i * (LMAX + 1) + j] = p * mk;
      dS[i * (LMAX + 1) + j] = acc[u] * mk;  // dP (grad w.r.t. the softmax output)
    }
  }
  __syncthreads();
  // dS = P ⊙ (dP - Σ_j P·dP)
  const int w = t >> 6, lane = t & 63;
  for (int i = w; i < L; i += 4) {
    float s = 0.f;
    for (int j = lane; j < L; j += 64) s += Pg[(long)i * L + j] * dS[i * (LMAX + 1) + j];
    s = c2::wave_sum(s);
    for (int j = lane; j < L; j += 64) {
      const float p = Pg[(long)i * L + j];
      dS[i * (LMAX + 1) + j] = p * (dS[i * (LMAX + 1) + j] - s);
    }
  }
  __syncthreads();
  const float sc = 1.0f / sqrtf((float)dh);
  for (int c = t; c < dh; c += 256) {
    float a[LMAX];
    // dV[j] = Σ_{i>=j} Pd[i][j] dO[i]   and   dK[j] = sc Σ_{i>=j} dS[i][j] Q[i]
#pragma unroll
    for (int j = 0; j < LMAX; ++j) a[j] = 0.f;
    for (int i = 0; i < L; ++i) {
      const float go = dO[(long)i * d + c];
#pragma unroll
      for (int j = 0; j < LMAX; ++j)
        if (j <= i) a[j] = fmaf(Pd[i * (LMAX + 1) + j], go, a[j]);
    }
#pragma unroll
    for (int j = 0; j < LMAX; ++j)
      if (j < L) dV[(long)j * rs + c] = a[j];
#pragma unroll
    for (int j = 0; j < LMAX; ++j) a[j] = 0.f;
    for (int i = 0; i < L; ++i) {
      const float q = Q[(long)i * rs + c];
#pragma unroll
      for (int j = 0; j < LMAX; ++j)
        if (j <= i) a[j] = fmaf(dS[i * (LMAX + 1) + j], q, a[j]);
    }
#pragma unroll
    for (int j = 0; j < LMAX; ++j)
      if (j < L) dK[(long)j * rs + c] = a[j] * sc;
    // dQ[i] = sc Σ_{j<=i} dS[i][j] K[j]
#pragma unroll
    for (int i = 0; i < LMAX; ++i) a[i] = 0.f;
    for (int j = 0; j < L; ++j) {
      if (!keyok[j]) continue;
      const float k = K[(long)j * rs + c];
#pragma unroll
      for (int i = 0; i < LMAX; ++i)
        if (i >= j && i < L) a[i] = fmaf(dS[i * (LMAX + 1) + j], k, a[i]);
    }
#pragma unroll
    for (int i = 0; i < LMAX; ++i)
      if (i < L) dQ[(long)i * rs + c] = a[i] * sc;
  }
}

template <int LMAX>
size_t fwd_smem() { return sizeof(float) * (LMAX * (LMAX + 1) + 2 * LMAX * (Ch<LMAX>::V + 1)); }
template <int LMAX>
size_t bwd_smem() { return sizeof(float) * (2 * LMAX * (LMAX + 1) + 2 * LMAX * (Ch<LMAX>::V + 1)); }

template <int LMAX>
void launch_fwd(dim3 grid, hipStream_t s, const float* qkv, const int64_t* seq, int64_t pad, int L, int d, int H,
                c2::Drop dr, int64_t b_base, float* out, float* Psave) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)attn_fwd_kernel<LMAX>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)fwd_smem<LMAX>());
    attr = true;
  }
  attn_fwd_kernel<LMAX><<<grid, 256, fwd_smem<LMAX>(), s>>>(qkv, seq, pad, L, d, H, dr, b_base, out, Psave);
}

template <int LMAX>
void launch_bwd(dim3 grid, hipStream_t s, const float* qkv, const int64_t* seq, int64_t pad, int L, int d, int H,
                c2::Drop dr, int64_t b_base, const float* Psave, const float* dout, float* dqkv) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)attn_bwd_kernel<LMAX>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)bwd_smem<LMAX>());
    attr = true;
  }
  attn_bwd_kernel<LMAX><<<grid, 256, bwd_smem<LMAX>(), s>>>(qkv, seq, pad, L, d, H, dr, b_base, Psave, dout, dqkv);
}

}  // namespace

// qkv [B, L, 3d] (q | k | v per row, heads contiguous inside each), out [B, L, d],
// Psave [B, H, L, L] softmax probabilities (pre-dropout).  Dropout index:
// (((b_base + b)*H + h)*L + i)*L + j.
C2_API int c2dsr_attn_fwd(const float* qkv, const int64_t* seq, int64_t pad, int B, int L, int d, int H, uint32_t k0,
                          uint32_t k1, float p, int64_t b_base, float* out, float* Psave, void* stream) {
  if (L > 128 || d % H) return (int)hipErrorInvalidValue;
  if (B == 0) return 0;
  c2::Drop dr = c2::make_drop(k0, k1, p);
  hipStream_t s = (hipStream_t)stream;
  dim3 grid(B * H);
  if (L <= 16)
    launch_fwd<16>(grid, s, qkv, seq, pad, L, d, H, dr, b_base, out, Psave);
  else if (L <= 32)
    launch_fwd<32>(grid, s, qkv, seq, pad, L, d, H, dr, b_base, out, Psave);
  else if (L <= 64)
    launch_fwd<64>(grid, s, qkv, seq, pad, L, d, H, dr, b_base, out, Psave);
  else
    launch_fwd<128>(grid, s, qkv, seq, pad, L, d, H, dr, b_base, out, Psave);
  C2_CHECK_LAUNCH();
  return 0;
}

C2_API int c2dsr_attn_bwd(const float* qkv, const int64_t* seq, int64_t pad, int B, int L, int d, int H, uint32_t k0,
                          uint32_t k1, float p, int64_t b_base, const float* Psave, const float* dout, float* dqkv,
                          void* stream) {
  if (L > 128 || d % H) return (int)hipErrorInvalidValue;
  if (B == 0) return 0;
  c2::Drop dr = c2::make_drop(k0, k1, p);
  hipStream_t s = (hipStream_t)stream;
  dim3 grid(B * H);
  if (L <= 16)
    launch_bwd<16>(grid, s, qkv, seq, pad, L, d, H, dr, b_base, Psave, dout, dqkv);
  else if (L <= 32)
    launch_bwd<32>(grid, s, qkv, seq, pad, L, d, H, dr, b_base, Psave, dout, dqkv);
  else if (L <= 64)
    launch_bwd<64>(grid, s, qkv, seq, pad, L, d, H, dr, b_base, Psave, dout, dqkv);
  else
    launch_bwd<128>(grid, s, qkv, seq, pad, L, d, H, dr, b_base, Psave, dout, dqkv);
  C2_CHECK_LAUNCH();
  return 0;
}
