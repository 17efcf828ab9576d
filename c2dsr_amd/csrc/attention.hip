// Self-attention core of the sequence encoder on the matrix cores (exact fp32:
// v_mfma_f32_32x32x2_f32), one workgroup (4 waves) per (sequence, head), the sequence
// padded to LP = 32/64/128 rows and the head dim streamed through LDS in chunks.
//
//   S = Q·Kᵀ/√dh + mask,  P = softmax(S),  O = drop(P)·V           (forward)
//   dPd = dO·Vᵀ, dS = P ⊙ (dP - Σ_j P·dP), dQ = dS·K/√dh, dK = dSᵀ·Q/√dh, dV = Pdᵀ·dO
//
// Replaces F.multi_head_attention_forward → scaled_dot_product_attention (math path)
// reached from models/encoders.py:33 with attn_mask = causal (encoders.py:14) and
// key_padding_mask = (seq != pad) merged additively — query i attends only to keys
// j <= i that ARE padding (Q1); a row with no admissible key yields 0 (Q2).  The
// attention FLOPs are small (L <= 128), so the exact-fp32 MFMA keeps both precision
// modes bit-identical here while staying far off the critical path.
#include "common.h"

#include <type_traits>

typedef __bf16 bf16;

#define WMFMA(a, b, c, x, y, z) __builtin_amdgcn_mfma_f32_32x32x2f32((a), (b), (c), (x), (y), (z))

#include <cstdlib>

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int creg(int reg, int lane) { return (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5); }

// KC: head-dim chunk for the Q·Kᵀ-type products; CC: output-column chunk for the P·V-type
// products (smaller at LP = 128 so the backward's two score tiles + staging fit 160 KB).
template <int LP>
struct Smem {
  static constexpr int KC = LP >= 128 ? 16 : 32;
  static constexpr int CC = LP >= 128 ? 32 : 128;
  static constexpr int SLD = LP + 1;
  static constexpr int XLD = KC + 1;
  static constexpr int VLD = CC + 1;
  static constexpr int STAGE = 2 * LP * XLD > LP * VLD ? 2 * LP * XLD : LP * VLD;
};

// acc (32x32 tile (ti, tj) of X·Yᵀ over the head dim, X/Y rows = sequence positions) —
// each wave owns tiles w, w+4, ... of the (LP/32)^2 grid.  X, Y: global rows of stride xs/ys.
template <int LP>
__device__ __forceinline__ void xyT(const float* __restrict__ X, long xs, const float* __restrict__ Y, long ys, int L, int dh,
                    float* Xs, float* Ys, f32x16 (&acc)[(LP / 32) * (LP / 32) / 4 > 0 ? (LP / 32) * (LP / 32) / 4 : 1]) {
  constexpr int NT = LP / 32;
  constexpr int XLD = Smem<LP>::XLD;
  constexpr int KC = Smem<LP>::KC;
  constexpr int PER = (NT * NT + 3) / 4;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
#pragma unroll
  for (int u = 0; u < PER; ++u)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[u][i] = 0.f;
  for (int k0 = 0; k0 < dh; k0 += KC) {
    __syncthreads();
    for (int e = t; e < LP * KC; e += 256) {
      const int i = e / KC, c = e % KC;
      const bool ok = i < L && k0 + c < dh;
      Xs[i * XLD + c] = ok ? X[i * xs + k0 + c] : 0.f;
      Ys[i * XLD + c] = ok ? Y[i * ys + k0 + c] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int tile = w + 4 * u;
      if (tile >= NT * NT) break;
      const int ti = tile / NT, tj = tile % NT;
      if (tj > ti) continue;  // causal: j > i never admissible
#pragma unroll 4
      for (int ks = 0; ks < KC / 2; ++ks) {
        const float a = Xs[(ti * 32 + (lane & 31)) * XLD + ks * 2 + (lane >> 5)];
        const float b = Ys[(tj * 32 + (lane & 31)) * XLD + ks * 2 + (lane >> 5)];
        acc[u] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[u], 0, 0, 0);
      }
    }
  }
}

// out[i][c] (+)= scale * Σ_j A[i][j] * Y[j][c] for i < L, c < dh.  A in LDS ([LP][SLD], or
// transposed: A[i][j] = As[j][i]); Y global rows (stride ys).  Each wave: 32 output columns of
// a CC-wide chunk, all LP rows.
template <int LP, bool TRANS_A>
__device__ __forceinline__ void pv(const float* As, const float* __restrict__ Y, long ys, int L, int dh, float* Vs,
                   float* __restrict__ out, long os, float scale, int jmax) {
  constexpr int NT = LP / 32;
  constexpr int SLD = Smem<LP>::SLD;
  constexpr int VLD = Smem<LP>::VLD;
  constexpr int CC = Smem<LP>::CC;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  for (int c0 = 0; c0 < dh; c0 += CC) {
    __syncthreads();
    for (int e = t; e < LP * CC; e += 256) {
      const int j = e / CC, c = e % CC;
      Vs[j * VLD + c] = (j < L && c0 + c < dh) ? Y[j * ys + c0 + c] : 0.f;
    }
    __syncthreads();
    const int cw = w * 32;
    if (cw < CC && c0 + cw < dh) {
      f32x16 acc[NT];
#pragma unroll
      for (int ti = 0; ti < NT; ++ti)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[ti][i] = 0.f;
      for (int ks = 0; ks < jmax / 2; ++ks) {
        const int j = ks * 2 + (lane >> 5);
        const float b = Vs[j * VLD + cw + (lane & 31)];
#pragma unroll
        for (int ti = 0; ti < NT; ++ti) {
          const int i = ti * 32 + (lane & 31);
          const float a = TRANS_A ? As[j * SLD + i] : As[i * SLD + j];
          acc[ti] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[ti], 0, 0, 0);
        }
      }
      const int c = c0 + cw + (lane & 31);
      if (c < dh) {
#pragma unroll
        for (int ti = 0; ti < NT; ++ti)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int i = ti * 32 + creg(r, lane);
            if (i < L) out[i * os + c] = scale * acc[ti][r];
          }
      }
    }
  }
}

template <int LP>
__global__ __launch_bounds__(256) void attn_fwd_kernel(const float* __restrict__ qkv, const int64_t* __restrict__ seq,
                                                       int64_t pad, int L, int d, int H, c2::Drop drop,
                                                       int64_t b_base, float* __restrict__ out,
                                                       float* __restrict__ Psave) {
  constexpr int NT = LP / 32;
  constexpr int SLD = Smem<LP>::SLD;
  constexpr int XLD = Smem<LP>::XLD;
  constexpr int PER = (NT * NT + 3) / 4;
  const int b = blockIdx.x / H, h = blockIdx.x % H;
  const int dh = d / H;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* Ss = sm;                      // [LP][SLD]  scores → dropped probabilities
  float* Xs = Ss + LP * SLD;           // [LP][XLD]
  float* Ys = Xs + LP * XLD;           // [LP][XLD]
  float* Vs = Xs;                      // the P·V staging reuses the X/Y staging area (Smem::STAGE)
  __shared__ unsigned char keyok[LP];
  for (int j = t; j < LP; j += 256) keyok[j] = (j < L) && (seq[(long)b * L + j] == pad);
  const long rs = 3l * d;
  const float* Q = qkv + (long)b * L * rs + h * dh;
  const float* K = Q + d;
  const float* V = Q + 2 * d;
  f32x16 acc[PER];
  xyT<LP>(Q, rs, K, rs, L, dh, Xs, Ys, acc);
  const float sc = 1.0f / sqrtf((float)dh);
  __syncthreads();
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int tile = w + 4 * u;
    if (tile >= NT * NT) break;
    const int ti = tile / NT, tj = tile % NT;
    const int j = tj * 32 + (lane & 31);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int i = ti * 32 + creg(r, lane);
      Ss[i * SLD + j] = (j <= i && keyok[j]) ? acc[u][r] * sc : -INFINITY;
    }
  }
  __syncthreads();
  for (int i = w; i < LP; i += 4) {
    if (i >= L) {
      for (int j = lane; j < LP; j += 64) Ss[i * SLD + j] = 0.f;
      continue;
    }
    float m = -INFINITY;
    for (int j = lane; j < L; j += 64) m = fmaxf(m, Ss[i * SLD + j]);
    m = c2::wave_max(m);
    float s = 0.f;
    for (int j = lane; j < L; j += 64) {
      const float e = (m == -INFINITY) ? 0.f : __expf(Ss[i * SLD + j] - m);
      Ss[i * SLD + j] = e;
      s += e;
    }
    s = c2::wave_sum(s);
    const float inv = s > 0.f ? 1.0f / s : 0.f;
    const uint64_t rowidx = ((uint64_t)((b_base + b) * H + h) * L + i) * L;
    for (int j = lane; j < LP; j += 64) {
      if (j < L) {
        const float pv_ = Ss[i * SLD + j] * inv;
        Psave[((long)blockIdx.x * L + i) * L + j] = pv_;
        Ss[i * SLD + j] = pv_ * drop.mul(rowidx + j);
      } else {
        Ss[i * SLD + j] = 0.f;
      }
    }
  }
  pv<LP, false>(Ss, V, rs, L, dh, Vs, out + (long)b * L * d + h * dh, d, 1.0f, LP);
}

template <int LP>
__global__ __launch_bounds__(256) void attn_bwd_kernel(const float* __restrict__ qkv, const int64_t* __restrict__ seq,
                                                       int64_t pad, int L, int d, int H, c2::Drop drop,
                                                       int64_t b_base, const float* __restrict__ Psave,
                                                       const float* __restrict__ dout, float* __restrict__ dqkv) {
  constexpr int NT = LP / 32;
  constexpr int SLD = Smem<LP>::SLD;
  constexpr int XLD = Smem<LP>::XLD;
  constexpr int PER = (NT * NT + 3) / 4;
  const int b = blockIdx.x / H, h = blockIdx.x % H;
  const int dh = d / H;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* Pd = sm;                      // dropped probabilities [LP][SLD]
  float* dS = Pd + LP * SLD;           // dP → dS [LP][SLD]
  float* Xs = dS + LP * SLD;
  float* Ys = Xs + LP * XLD;
  float* Vs = Xs;
  __shared__ unsigned char keyok[LP];
  for (int j = t; j < LP; j += 256) keyok[j] = (j < L) && (seq[(long)b * L + j] == pad);
  const long rs = 3l * d;
  const float* Q = qkv + (long)b * L * rs + h * dh;
  const float* K = Q + d;
  const float* V = Q + 2 * d;
  const float* dO = dout + (long)b * L * d + h * dh;
  float* dQ = dqkv + (long)b * L * rs + h * dh;
  float* dK = dQ + d;
  float* dV = dQ + 2 * d;
  const float* Pg = Psave + (long)blockIdx.x * L * L;
  f32x16 acc[PER];
  xyT<LP>(dO, d, V, rs, L, dh, Xs, Ys, acc);  // dPd = dO·Vᵀ
  __syncthreads();
  // dP = dPd ⊙ mask/(1-p); Pd = P ⊙ mask/(1-p)
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int tile = w + 4 * u;
    if (tile >= NT * NT) break;
    const int ti = tile / NT, tj = tile % NT;
    const int j = tj * 32 + (lane & 31);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int i = ti * 32 + creg(r, lane);
      float p = 0.f, dp = 0.f;
      if (i < L && j < L) {
        const float mk = drop.mul(((uint64_t)((b_base + b) * H + h) * L + i) * L + j);
        p = Pg[(long)i * L + j];
        dp = (j <= i) ? acc[u][r] * mk : 0.f;
        p *= mk;
      }
      Pd[i * SLD + j] = p;
      dS[i * SLD + j] = dp;
    }
  }
  __syncthreads();
  for (int i = w; i < LP; i += 4) {
    if (i >= L) {
      for (int j = lane; j < LP; j += 64) dS[i * SLD + j] = 0.f;
      continue;
    }
    float s = 0.f;
    for (int j = lane; j < L; j += 64) s += Pg[(long)i * L + j] * dS[i * SLD + j];
    s = c2::wave_sum(s);
    for (int j = lane; j < LP; j += 64) dS[i * SLD + j] = j < L ? Pg[(long)i * L + j] * (dS[i * SLD + j] - s) : 0.f;
  }
  const float sc = 1.0f / sqrtf((float)dh);
  pv<LP, false>(dS, K, rs, L, dh, Vs, dQ, rs, sc, LP);  // dQ = dS·K/√dh
  pv<LP, true>(dS, Q, rs, L, dh, Vs, dK, rs, sc, LP);   // dK = dSᵀ·Q/√dh
  pv<LP, true>(Pd, dO, d, L, dh, Vs, dV, rs, 1.0f, LP);  // dV = Pdᵀ·dO
}

// ---------------------------------------------------------------------------------------
// Register-streamed variant (LP = 32/64, dh % 4 == 0): no LDS staging of Q/K/V/dO at all.
//  * score tiles (Q·Kᵀ, dO·Vᵀ): each wave owns one causal 32x32 tile (LP = 64: 3 tiles on
//    waves 0-2) or a quarter of the head dim of the single tile (LP = 32, partials summed
//    in LDS in a fixed order).  Operands come straight from HBM as float4 per lane: lane
//    (r, hi) holds row r, columns 8c + 4hi .. +3, and MFMA step (c, e) consumes element e of
//    both operands — any k-permutation works as long as A and B share it.  Chunks of 8
//    c-steps are double-buffered in registers.
//  * P·V-type products: each wave owns 32-column tiles of the output; the B operand
//    (V / K / Q / dO rows, 128 contiguous bytes per half-wave) is preloaded for every k-step
//    before the MFMA chain; A (probabilities / dS) is read from LDS.
//  * key range: every column j >= jmax (one past the last padding key) is masked for every
//    query, so the k-loops of the P·V and dS·K products stop at jmax (exact: those P are 0).
// ---------------------------------------------------------------------------------------
template <int LP>
struct Fast {
  static constexpr int NT = LP / 32;
  static constexpr int T = NT * (NT + 1) / 2;  // causal tiles
  static constexpr int KS = 4 / T;             // head-dim split per tile
  static constexpr int SLD = LP + 1;
};

__device__ __forceinline__ void tile_of(int t, int& ti, int& tj) {
  // causal tiles in order (0,0), (1,0), (1,1)
  ti = t == 0 ? 0 : 1;
  tj = t == 2 ? 1 : 0;
}

// buffer descriptor over rows [0, rows) x columns [0, width) of a row-major fp32 matrix (row stride
// `stride` floats): the range ends with the last row's `width` columns, so a load past the head of
// the last row (the end of qkv for the last sequence) reads 0 instead of running off the buffer.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rows_rsrc(const float* base, int rows, long stride, int width) {
  const int bytes = __builtin_amdgcn_readfirstlane(rows > 0 ? ((rows - 1) * (int)stride + width) * 4 : 0);
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, bytes, 0x00020000);
}
__device__ __forceinline__ float4 ld_b128(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}

// Raw (unscaled, unmasked) X·Yᵀ tiles into S[LP][SLD]; tiles never computed are left untouched.
// part: LDS scratch of 4*1024 floats (used only when KS > 1).
template <int LP>
__device__ __forceinline__ void scores_fast(const float* __restrict__ X, long xs, const float* __restrict__ Y, long ys, int L, int dh,
                            int jmax, float* S, float* part) {
  using F = Fast<LP>;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63, r = lane & 31, hi = lane >> 5;
  const int tile = w / F::KS, kp = w % F::KS;
  int ti = 0, tj = 0;
  tile_of(tile, ti, tj);
  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  const bool active = tile < F::T && tj * 32 < jmax;
  if (active) {
    const int CS = (dh + 7) >> 3;  // c-steps of 8 columns
    const int cb = kp * CS / F::KS, ce = (kp + 1) * CS / F::KS;
    // buffer loads: rows past L (X) or jmax (Y) fall outside the descriptor and read 0
    const auto xsrc = rows_rsrc(X, L, xs, dh);
    const auto ysrc = rows_rsrc(Y, jmax, ys, dh);
    const int xo = ((ti * 32 + r) * (int)xs + 4 * hi) * 4;
    const int yo = ((tj * 32 + r) * (int)ys + 4 * hi) * 4;
    const int cmax = (dh - 4 * hi - 4) >> 3;  // last c-step whose columns are inside the head
    float4 xa[8], ya[8], xb[8], yb[8];
    auto load = [&](float4 (&xv)[8], float4 (&yv)[8], int c0) {
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const bool cok = c0 + c < ce && c0 + c <= cmax;
        // the whole offset in voffset: the descriptor's range check does not cover soffset, so a
        // scalar part could carry a load of the last sequence past the end of the buffer
        const float4 xv_ = ld_b128(xsrc, xo + 32 * (c0 + c), 0);
        const float4 yv_ = ld_b128(ysrc, yo + 32 * (c0 + c), 0);
        xv[c] = cok ? xv_ : make_float4(0.f, 0.f, 0.f, 0.f);
        yv[c] = cok ? yv_ : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    };
    auto mma = [&](const float4 (&xv)[8], const float4 (&yv)[8]) {
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(xv[c].x, yv[c].x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(xv[c].y, yv[c].y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(xv[c].z, yv[c].z, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(xv[c].w, yv[c].w, acc, 0, 0, 0);
      }
    };
    load(xa, ya, cb);
    for (int c0 = cb; c0 < ce; c0 += 16) {
      if (c0 + 8 < ce) load(xb, yb, c0 + 8);
      mma(xa, ya);
      if (c0 + 8 >= ce) break;
      if (c0 + 16 < ce) load(xa, ya, c0 + 16);
      mma(xb, yb);
    }
  }
  if constexpr (F::KS == 1) {
    if (active) {
#pragma unroll
      for (int q = 0; q < 16; ++q) S[(ti * 32 + creg(q, lane)) * F::SLD + tj * 32 + r] = acc[q];
    }
  } else {
#pragma unroll
    for (int q = 0; q < 16; ++q) part[w * 1024 + q * 64 + lane] = acc[q];
    __syncthreads();
    for (int e = t; e < 1024; e += 256) {
      const int q = e >> 6, ln = e & 63;
      const float v = (part[e] + part[1024 + e]) + (part[2048 + e] + part[3072 + e]);
      S[creg(q, ln) * F::SLD + (ln & 31)] = v;
      (void)q;
    }
  }
}

// out[i][c] = scale * Σ_{k < kend} A[i][k] * Y[k][c]  for i < rows, c < dh (all of them written).
// A in LDS: A[i][k] = As[i*SLD + k], or As[k*SLD + i] when TRANS.  Y: global rows of stride ys.
template <int LP, bool TRANS>
__device__ __forceinline__ void pv_fast(const float* As, const float* __restrict__ Y, long ys, int rows, int dh, int kend,
                        float* __restrict__ out, long os, float scale) {
  using F = Fast<LP>;
  constexpr int KMAX = LP / 2;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63, r = lane & 31, hi = lane >> 5;
  const int CT = (dh + 31) >> 5;
  const int ksteps = (kend + 1) >> 1;
  for (int ct = w; ct < CT; ct += 4) {
    const int c = ct * 32 + r;
    const bool cok = c < dh;
    float bv[KMAX];
    const auto ysrc = rows_rsrc(Y, kend, ys, dh);  // rows >= kend read 0
    const int yo = (hi * (int)ys + c) * 4;
#pragma unroll
    for (int ks = 0; ks < KMAX; ++ks) {
      const float v = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ysrc, yo + 8 * ks * (int)ys, 0, 0));
      bv[ks] = cok ? v : 0.f;
    }
    f32x16 acc[F::NT];
#pragma unroll
    for (int ti = 0; ti < F::NT; ++ti)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[ti][i] = 0.f;
#pragma unroll
    for (int ks = 0; ks < KMAX; ++ks) {
      if (ks < ksteps) {
        const int k = 2 * ks + hi;
#pragma unroll
        for (int ti = 0; ti < F::NT; ++ti) {
          const int i = ti * 32 + r;
          const float a = TRANS ? As[k * F::SLD + i] : As[i * F::SLD + k];
          acc[ti] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bv[ks], acc[ti], 0, 0, 0);
        }
      }
    }
    if (cok) {
#pragma unroll
      for (int ti = 0; ti < F::NT; ++ti)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int i = ti * 32 + creg(q, lane);
          if (i < rows) out[(long)i * os + c] = scale * acc[ti][q];
        }
    }
  }
}

// padding keys of sequence b: keyok[j], and jmax = 1 + last padding position (0 if none)
template <int LP>
__device__ __forceinline__ int key_setup(const int64_t* __restrict__ seq, int64_t pad, int b, int L, unsigned char* keyok) {
  const int t = threadIdx.x;
  __shared__ int jm;
  if (t == 0) jm = 0;
  __syncthreads();
  if (t < LP) {
    const bool ok = t < L && seq[(long)b * L + t] == pad;
    keyok[t] = ok;
    if (ok) atomicMax(&jm, t + 1);
  }
  __syncthreads();
  return jm;
}

template <int LP>
__global__ __launch_bounds__(256, 2) void attn_fwd_fast(const float* __restrict__ qkv,
                                                        const int64_t* __restrict__ seq, int64_t pad, int L, int d,
                                                        int H, c2::Drop drop, int64_t b_base,
                                                        float* __restrict__ out, float* __restrict__ Psave) {
  using F = Fast<LP>;
  const int b = blockIdx.x / H, h = blockIdx.x % H;
  const int dh = d / H;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  __shared__ float Ss[LP * F::SLD];
  __shared__ float part[F::KS > 1 ? 4 * 1024 : 1];
  __shared__ unsigned char keyok[LP];
  const int jmax = key_setup<LP>(seq, pad, b, L, keyok);
  const long rs = 3l * d;
  const float* Q = qkv + (long)b * L * rs + h * dh;
  const float* K = Q + d;
  const float* V = Q + 2 * d;
  scores_fast<LP>(Q, rs, K, rs, L, dh, jmax, Ss, part);
  __syncthreads();
  const float sc = 1.0f / sqrtf((float)dh);
  for (int i = w; i < LP; i += 4) {
    const int j = lane;
    const bool adm = i < L && j < LP && j <= i && j < jmax && keyok[j];
    const float sv = adm ? Ss[i * F::SLD + j] * sc : -INFINITY;
    const float m = c2::wave_max(sv);
    const float e = (adm && m != -INFINITY) ? __expf(sv - m) : 0.f;
    const float s = c2::wave_sum(e);
    const float pv_ = s > 0.f ? e * (1.0f / s) : 0.f;
    if (i < L && j < L) {
      Psave[((long)blockIdx.x * L + i) * L + j] = pv_;
      const uint64_t idx = ((uint64_t)((b_base + b) * H + h) * L + i) * L + j;
      if (j < LP) Ss[i * F::SLD + j] = pv_ * drop.mul(idx);
    } else if (j < LP) {
      Ss[i * F::SLD + j] = 0.f;
    }
  }
  __syncthreads();
  pv_fast<LP, false>(Ss, V, rs, L, dh, jmax, out + (long)b * L * d + h * dh, d, 1.0f);
}

template <int LP>
__global__ __launch_bounds__(256, 2) void attn_bwd_fast(const float* __restrict__ qkv,
                                                        const int64_t* __restrict__ seq, int64_t pad, int L, int d,
                                                        int H, c2::Drop drop, int64_t b_base,
                                                        const float* __restrict__ Psave,
                                                        const float* __restrict__ dout, float* __restrict__ dqkv) {
  using F = Fast<LP>;
  const int b = blockIdx.x / H, h = blockIdx.x % H;
  const int dh = d / H;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  __shared__ float Pd[LP * F::SLD];
  __shared__ float dS[LP * F::SLD];
  __shared__ float part[F::KS > 1 ? 4 * 1024 : 1];
  __shared__ unsigned char keyok[LP];
  const int jmax = key_setup<LP>(seq, pad, b, L, keyok);
  const long rs = 3l * d;
  const float* Q = qkv + (long)b * L * rs + h * dh;
  const float* K = Q + d;
  const float* V = Q + 2 * d;
  const float* dO = dout + (long)b * L * d + h * dh;
  float* dQ = dqkv + (long)b * L * rs + h * dh;
  float* dK = dQ + d;
  float* dV = dQ + 2 * d;
  const float* Pg = Psave + (long)blockIdx.x * L * L;
  scores_fast<LP>(dO, d, V, rs, L, dh, jmax, dS, part);  // dPd = dO·Vᵀ (admissible tiles)
  __syncthreads();
  // dP = dPd ⊙ mask/(1-p); Pd = P ⊙ mask/(1-p); dS = P ⊙ (dP - Σ_j P·dP)
  for (int i = w; i < LP; i += 4) {
    const int j = lane;
    float p = 0.f, dp = 0.f, pd = 0.f;
    if (i < L && j < L) {
      p = Pg[(long)i * L + j];
      const float mk = drop.mul(((uint64_t)((b_base + b) * H + h) * L + i) * L + j);
      pd = p * mk;
      if (j <= i && j < jmax && keyok[j]) dp = dS[i * F::SLD + j] * mk;
    }
    const float s = c2::wave_sum(p * dp);
    if (j < LP) {
      Pd[i * F::SLD + j] = pd;
      dS[i * F::SLD + j] = p * (dp - s);
    }
  }
  __syncthreads();
  const float sc = 1.0f / sqrtf((float)dh);
  pv_fast<LP, false>(dS, K, rs, L, dh, jmax, dQ, rs, sc);  // dQ = dS·K/√dh
  pv_fast<LP, true>(dS, Q, rs, L, dh, L, dK, rs, sc);      // dK = dSᵀ·Q/√dh
  pv_fast<LP, true>(Pd, dO, d, L, dh, L, dV, rs, 1.0f);    // dV = Pdᵀ·dO
}

// ---------------------------------------------------------------------------------------
// Wave-per-sequence forward (L <= 64, dh % 32 == 0): no LDS, no barriers.  The score tiles are
// computed TRANSPOSED, Sᵀ = K·Qᵀ, so the lane of a query holds its whole row of scores in
// registers (keys j = 32tj + creg(r, lane)): the softmax is in-register plus one lane^32 exchange.
// P·V then takes the probabilities straight from those registers as the MFMA A operand: step r of
// a key tile consumes register r, i.e. key (r&3) + 8(r>>2) + 4·(lane>>5) — a permutation of the
// reduction index that the B operand (V rows, one float per lane, loaded in the same permuted
// order) shares, so the sum is exact.  Output tiles come out lane = column: coalesced stores.
// Keys past the last padding key are inadmissible for every query (Q1), so only jmax rows of K/V
// are read (buffer descriptors zero the rest).
// softmax of one query tile of transposed scores held by lane = query (tiles a: keys 0..31 and, when
// TWO, b: keys 32..63) → probabilities to the wave's save area in REGISTER layout (tile t of query tile
// ti at pw[(2·ti + t)·1024 + 64·q + lane]: every store instruction writes 256 contiguous bytes, and the
// backward reloads them in the same layout) and the dropped probabilities back into a / b.
// Masks: see WMask (masked entries are stored as 0).
constexpr int WAVE_PSAVE = 4096;  // floats of probability save per (sequence, head) on the wave path

// Which (query, key) pairs of one wave's sequence are admissible, and where they sit in the dropout index.
// Full layout (ROWS = false): query i and key j are sequence positions; admissible iff i < L, j <= i and
// position j is padding (bit j of kb, Q1).  Row-subset layout (ROWS = true, c2dsr_attn_fwd_rows): queries
// are the rows of the pass the loss reads and keys the padding rows, both compact in position order, so
// the keys admissible to a query are a prefix of the key list: j < cq (cq = padding positions <= the
// query's position); query / key positions (qp per lane, key j's held by lane j in kposv) give the
// full-layout dropout index, so both layouts drop the same entries.
struct WMask {
  uint64_t kb;  // full: padding positions of the sequence
  int L;        // positions per sequence (dropout index stride; full: query rows)
  int qp[2];    // ROWS: positions of this lane's queries 32t + (lane & 31), t = 0, 1
  int cq[2];    // ROWS: admissible key prefix of those queries (0 past the last query)
  int kposv;    // ROWS: lane j holds the position of key j
};

template <bool ROWS>
__device__ __forceinline__ bool wm_adm(const WMask& mk, int t, int j) {
  if constexpr (ROWS) return j < mk.cq[t];
  const int i = 32 * t + (threadIdx.x & 31);
  return i < mk.L && j <= i && ((mk.kb >> j) & 1);
}
template <bool ROWS>
__device__ __forceinline__ int wm_kpos(const WMask& mk, int j) {
  if constexpr (ROWS) return __shfl(mk.kposv, j, 64);
  return j;
}
template <bool ROWS>
__device__ __forceinline__ int wm_qpos(const WMask& mk, int t) {
  if constexpr (ROWS) return mk.qp[t];
  return 32 * t + (threadIdx.x & 31);
}

template <bool TWO, bool ROWS>
__device__ __forceinline__ void wave_softmax(f32x16& a, f32x16& b, int ti, const WMask& mk, float sc,
                                             const c2::Drop& drop, uint64_t pbase, float* __restrict__ prow0) {
  const int lane = threadIdx.x & 63;
  // admissible keys of this lane's 16 (or 32) registers as bit masks
  uint32_t m0 = 0, m1 = 0;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int j = creg(q, lane);
    m0 |= (uint32_t)wm_adm<ROWS>(mk, ti, j) << q;
    if constexpr (TWO) m1 |= (uint32_t)wm_adm<ROWS>(mk, ti, 32 + j) << q;
  }
  float m = -INFINITY;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    if ((m0 >> q) & 1) m = fmaxf(m, a[q] * sc);
    if constexpr (TWO) if ((m1 >> q) & 1) m = fmaxf(m, b[q] * sc);
  }
  m = fmaxf(m, __shfl_xor(m, 32, 64));
  float sum = 0.f;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    a[q] = ((m0 >> q) & 1) ? __expf(a[q] * sc - m) : 0.f;
    sum += a[q];
    if constexpr (TWO) {
      b[q] = ((m1 >> q) & 1) ? __expf(b[q] * sc - m) : 0.f;
      sum += b[q];
    }
  }
  sum += __shfl_xor(sum, 32, 64);
  const float inv = sum > 0.f ? 1.0f / sum : 0.f;
  float* pw = prow0 + 2 * ti * 1024 + lane;
  const uint64_t rb = pbase + (uint64_t)wm_qpos<ROWS>(mk, ti) * mk.L;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int j = creg(q, lane);
    const float p0 = a[q] * inv;
    pw[64 * q] = p0;
    a[q] = p0 * drop.mul(rb + wm_kpos<ROWS>(mk, j));
    if constexpr (TWO) {
      const float p1 = b[q] * inv;
      pw[1024 + 64 * q] = p1;
      b[q] = p1 * drop.mul(rb + wm_kpos<ROWS>(mk, 32 + j));
    }
  }
}

// Q rows of stride qs (nq of them), K / V rows of stride ks (nk), O rows of stride os.  Score tiles (tj, ti):
// t0 = (0,0), t1 = (0,1), t2 = (1,1) and, in the row-subset layout only, t3 = (1,0) (in the full layout
// it lies above the causal diagonal; compact queries can see keys of higher index).
template <int TJ, int TI, bool ROWS>
__device__ __forceinline__ void fwd_wave_body(const float* __restrict__ Q, long qs, const float* __restrict__ K,
                                              const float* __restrict__ V, long ks, int nq, int dh, int nk,
                                              const WMask& mk, const c2::Drop& drop, uint64_t pbase,
                                              float* __restrict__ o_row0, long os, float* __restrict__ prow0) {
  constexpr bool T3 = ROWS && TJ > 1;
  const int lane = threadIdx.x & 63, r = lane & 31, hi = lane >> 5;
  f32x16 t0, t1, t2, t3;
#pragma unroll
  for (int q = 0; q < 16; ++q) t0[q] = t1[q] = t2[q] = t3[q] = 0.f;
  {
    const auto qsrc = rows_rsrc(Q, nq, qs, dh);
    const auto ksrc = rows_rsrc(K, nk, ks, dh);
    const int q0o = (r * (int)qs + 4 * hi) * 4, q1o = ((32 + r) * (int)qs + 4 * hi) * 4;
    const int k0o = (r * (int)ks + 4 * hi) * 4, k1o = ((32 + r) * (int)ks + 4 * hi) * 4;
    const int CS = dh >> 3;
    constexpr int SU = 2;  // c-steps per register buffer, two buffers in flight
    float4 ba[SU][4], bb[SU][4];  // [c-step][k0, k1, q0, q1]
    auto load = [&](float4 (&kq)[SU][4], int c0) {
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const int co = 32 * (c0 + u);  // past the head: outside the descriptors → 0
        kq[u][0] = ld_b128(ksrc, k0o + co, 0);
        kq[u][1] = TJ > 1 ? ld_b128(ksrc, k1o + co, 0) : make_float4(0.f, 0.f, 0.f, 0.f);
        kq[u][2] = ld_b128(qsrc, q0o + co, 0);
        kq[u][3] = TI > 1 ? ld_b128(qsrc, q1o + co, 0) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    };
    auto mma = [&](const float4 (&kq)[SU][4]) {
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const float ka[4] = {kq[u][0].x, kq[u][0].y, kq[u][0].z, kq[u][0].w};
        const float kc[4] = {kq[u][1].x, kq[u][1].y, kq[u][1].z, kq[u][1].w};
        const float qa[4] = {kq[u][2].x, kq[u][2].y, kq[u][2].z, kq[u][2].w};
        const float qc[4] = {kq[u][3].x, kq[u][3].y, kq[u][3].z, kq[u][3].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          t0 = WMFMA(ka[e], qa[e], t0, 0, 0, 0);
          if constexpr (T3) t3 = WMFMA(kc[e], qa[e], t3, 0, 0, 0);
          if constexpr (TI > 1) t1 = WMFMA(ka[e], qc[e], t1, 0, 0, 0);
          if constexpr (TI > 1 && TJ > 1) t2 = WMFMA(kc[e], qc[e], t2, 0, 0, 0);
        }
      }
    };
    load(ba, 0);
#pragma unroll 1
    for (int c0 = 0; c0 < CS; c0 += 2 * SU) {
      if (c0 + SU < CS) load(bb, c0 + SU);
      mma(ba);
      if (c0 + SU >= CS) break;
      if (c0 + 2 * SU < CS) load(ba, c0 + 2 * SU);
      mma(bb);
    }
  }
  const float sc = 1.0f / sqrtf((float)dh);
  wave_softmax<T3, ROWS>(t0, t3, 0, mk, sc, drop, pbase, prow0);
  if constexpr (TI > 1) wave_softmax<(TJ > 1), ROWS>(t1, t2, 1, mk, sc, drop, pbase, prow0);
  // O = Pd·V per 32-column tile of the head (two waves per SIMD hide each other's V loads)
  const auto vsrc = rows_rsrc(V, nk, ks, dh);
  auto vload = [&](float (&v)[2][16], int ct) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int key = (q & 3) + 8 * (q >> 2) + 4 * hi;  // the key of register q (lane half hi)
      v[0][q] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(vsrc, (key * (int)ks + 32 * ct + r) * 4, 0, 0));
      v[1][q] = TJ > 1 ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                             vsrc, ((32 + key) * (int)ks + 32 * ct + r) * 4, 0, 0))
                       : 0.f;
    }
  };
  auto otile = [&](const float (&v)[2][16], int ct) {
    f32x16 o0, o1;
#pragma unroll
    for (int q = 0; q < 16; ++q) o0[q] = o1[q] = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      o0 = WMFMA(t0[q], v[0][q], o0, 0, 0, 0);
      if constexpr (T3) o0 = WMFMA(t3[q], v[1][q], o0, 0, 0, 0);
      if constexpr (TI > 1) {
        o1 = WMFMA(t1[q], v[0][q], o1, 0, 0, 0);
        if constexpr (TJ > 1) o1 = WMFMA(t2[q], v[1][q], o1, 0, 0, 0);
      }
    }
    const int c = 32 * ct + r;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int i0 = creg(q, lane), i1 = 32 + i0;
      if (i0 < nq) o_row0[(long)i0 * os + c] = o0[q];
      if (TI > 1 && i1 < nq) o_row0[(long)i1 * os + c] = o1[q];
    }
  };
  const int CT = dh >> 5;
#pragma unroll 1
  for (int ct = 0; ct < CT; ++ct) {
    float va[2][16];
    vload(va, ct);
    otile(va, ct);
  }
}

// the wave's sequence in the full layout: padding bits and key extent (one past the last padding key)
__device__ __forceinline__ WMask full_mask(const int64_t* __restrict__ seq, int64_t pad, int b, int L, int& jmax) {
  const int lane = threadIdx.x & 63;
  const bool ok = lane < L && seq[(long)b * L + lane] == pad;
  WMask mk;
  mk.kb = __ballot(ok);
  mk.L = L;
  jmax = mk.kb ? 64 - __clzll((long long)mk.kb) : 0;
  return mk;
}

__global__ __launch_bounds__(256) void attn_fwd_wave(const float* __restrict__ qkv, const int64_t* __restrict__ seq,
                                                     int64_t pad, int B, int L, int d, int H, c2::Drop drop,
                                                     int64_t b_base, float* __restrict__ out,
                                                     float* __restrict__ Psave) {
  // (the wave index stays a vector value here: as a scalar the full-layout kernels measured slower — fwd 117 → 127 µs,
  // bwd 238 → 335 µs at the bench shape — while attn_fwd_rows gains)
  const int bh = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (bh >= B * H) return;  // uniform over the wave
  const int b = bh / H, h = bh % H, dh = d / H;
  int jmax;
  const WMask mk = full_mask(seq, pad, b, L, jmax);
  const long rs = 3l * d;
  const float* Q = qkv + (long)b * L * rs + h * dh;
  const uint64_t pbase = (uint64_t)((b_base + b) * H + h) * L * L;
  float* orow = out + (long)b * L * d + h * dh;
  float* prow = Psave + (long)bh * WAVE_PSAVE;
  const int TJ = jmax > 32 ? 2 : 1, TI = L > 32 ? 2 : 1;
  if (TI == 1)
    fwd_wave_body<1, 1, false>(Q, rs, Q + d, Q + 2 * d, rs, L, dh, jmax, mk, drop, pbase, orow, d, prow);
  else if (TJ == 1)
    fwd_wave_body<1, 2, false>(Q, rs, Q + d, Q + 2 * d, rs, L, dh, jmax, mk, drop, pbase, orow, d, prow);
  else
    fwd_wave_body<2, 2, false>(Q, rs, Q + d, Q + 2 * d, rs, L, dh, jmax, mk, drop, pbase, orow, d, prow);
}

// the wave's sequence in the row-subset layout: compact query rows [q0, q0 + nq) and key rows [k0, k0 + nk)
// (q_off / k_off per sequence; q_idx / k_idx hold global rows b·L + position)
__device__ __forceinline__ WMask rows_mask(const int64_t* __restrict__ seq, int64_t pad, int b, int L,
                                           const int* __restrict__ q_idx, const int* __restrict__ q_off,
                                           const int* __restrict__ k_idx, const int* __restrict__ k_off, int& q0,
                                           int& nq, int& k0, int& nk) {
  const int lane = threadIdx.x & 63;
  q0 = __builtin_amdgcn_readfirstlane(q_off[b]);
  nq = __builtin_amdgcn_readfirstlane(q_off[b + 1]) - q0;
  k0 = __builtin_amdgcn_readfirstlane(k_off[b]);
  nk = __builtin_amdgcn_readfirstlane(k_off[b + 1]) - k0;
  nq = min(max(nq, 0), L);
  nk = min(max(nk, 0), L);
  const bool ok = lane < L && seq[(long)b * L + lane] == pad;
  const uint64_t kb = __ballot(ok);
  WMask mk;
  mk.kb = kb;
  mk.L = L;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int i = 32 * t + (lane & 31);
    const int qp = i < nq ? q_idx[q0 + i] - b * L : 0;
    const uint64_t upto = qp >= 63 ? ~0ull : ((2ull << qp) - 1ull);  // positions 0..qp
    mk.qp[t] = qp;
    mk.cq[t] = i < nq ? min((int)__popcll(kb & upto), nk) : 0;
  }
  mk.kposv = lane < nk ? k_idx[k0 + lane] - b * L : 0;
  return mk;
}

#ifndef ATTN_ROWS_OCC
#define ATTN_ROWS_OCC 2
#endif
#ifndef ATTN_PD_EARLY
#define ATTN_PD_EARLY 1
#endif
#ifndef ATTN_ROWS_OCC_F
#define ATTN_ROWS_OCC_F ATTN_ROWS_OCC
#endif
__global__ __launch_bounds__(256, ATTN_ROWS_OCC_F) void attn_fwd_rows(const float* __restrict__ q, const float* __restrict__ kv,
                                                     const int64_t* __restrict__ seq, int64_t pad,
                                                     const int* __restrict__ q_idx, const int* __restrict__ q_off,
                                                     const int* __restrict__ k_idx, const int* __restrict__ k_off,
                                                     int B, int L, int d, int H, c2::Drop drop, int64_t b_base,
                                                     float* __restrict__ out, float* __restrict__ Psave) {
  // the wave index as a scalar: everything derived from it (sequence, row ranges, buffer descriptors) stays uniform,
  // so each buffer load takes its descriptor from SGPRs instead of a readfirstlane waterfall loop
  const int bh = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  if (bh >= B * H) return;  // uniform over the wave
  const int b = bh / H, h = bh % H, dh = d / H;
  int q0, nq, k0, nk;
  const WMask mk = rows_mask(seq, pad, b, L, q_idx, q_off, k_idx, k_off, q0, nq, k0, nk);
  if (nq == 0) return;  // uniform
  const float* Q = q + (long)q0 * d + h * dh;
  const float* K = kv + (long)k0 * 2 * d + h * dh;
  const uint64_t pbase = (uint64_t)((b_base + b) * H + h) * L * L;
  float* orow = out + (long)q0 * d + h * dh;
  float* prow = Psave + (long)bh * WAVE_PSAVE;
  const int TJ = nk > 32 ? 2 : 1, TI = nq > 32 ? 2 : 1;
  if (TI == 1 && TJ == 1)
    fwd_wave_body<1, 1, true>(Q, d, K, K + d, 2l * d, nq, dh, nk, mk, drop, pbase, orow, d, prow);
  else if (TI == 1)
    fwd_wave_body<2, 1, true>(Q, d, K, K + d, 2l * d, nq, dh, nk, mk, drop, pbase, orow, d, prow);
  else if (TJ == 1)
    fwd_wave_body<1, 2, true>(Q, d, K, K + d, 2l * d, nq, dh, nk, mk, drop, pbase, orow, d, prow);
  else
    fwd_wave_body<2, 2, true>(Q, d, K, K + d, 2l * d, nq, dh, nk, mk, drop, pbase, orow, d, prow);
}

// ---------------------------------------------------------------------------------------
// Wave-per-sequence backward (L <= 64, dh % 32 == 0), the forward's transposed layout:
//   dPᵀ = V·dOᵀ (lane = query i, registers = keys j), P reloaded in the same layout;
//   dP⊙mask, Pd = P⊙mask, dS = P⊙(dPm − Σ_j P·dPm) in registers (+ one lane^32 exchange);
//   dQ = dS·K/√dh straight from the registers (key permutation as in the forward);
//   dV = Pdᵀ·dO and dK = dSᵀ·Q/√dh need keys in lanes: Pd and dS go through a per-wave LDS
//   transpose ([64][65] floats) and are read back with lane = key, register r = query
//   (r&3) + 8(r>>2) + 4·(lane>>5) — the same permutation trick over the query index.
// Rows of dK / dV past the last padding key are written as zeros (those keys are inadmissible).
// order this wave's LDS writes before its later reads (and reads before later writes)
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ void zero16(f32x16& a) {
#pragma unroll
  for (int q = 0; q < 16; ++q) a[q] = 0.f;
}

// OT: element type of dQ / dK / dV (float, or bf16 when their only consumers — the in_proj backward GEMMs —
// read them as a bf16 MFMA operand anyway: c2dsr_attn_bwd_b16).  Strides: Q qs, K / V ks, dO ds, dQ dqs,
// dK / dV dks; nkw: key rows of dK / dV to write (rows past the key tiles get zeros).  Tiles as in
// fwd_wave_body (g3 = (1,0) in the row-subset layout only).
template <int TJ, int TI, typename OT, bool ROWS>
__device__ __forceinline__ void bwd_wave_body(const float* __restrict__ Q, long qs, const float* __restrict__ K,
                                              const float* __restrict__ V, long ks, const float* __restrict__ dO,
                                              long ds, int nq, int dh, int nk, const WMask& mk,
                                              const c2::Drop& drop, uint64_t pbase, const float* __restrict__ prow0,
                                              OT* __restrict__ dQ, long dqs, OT* __restrict__ dK,
                                              OT* __restrict__ dV, long dks, int nkw, float* T) {
  constexpr bool T3 = ROWS && TJ > 1;
  const int lane = threadIdx.x & 63, r = lane & 31, hi = lane >> 5;
  // ---- dPᵀ tiles (tj, ti): 0 = (0,0), 1 = (0,1), 2 = (1,1), 3 = (1,0)
  f32x16 g0, g1, g2, g3;
  zero16(g0); zero16(g1); zero16(g2); zero16(g3);
  {
    const auto vsrc = rows_rsrc(V, nk, ks, dh);
    const auto osrc = rows_rsrc(dO, nq, ds, dh);
    const int v0o = (r * (int)ks + 4 * hi) * 4, v1o = ((32 + r) * (int)ks + 4 * hi) * 4;
    const int o0o = (r * (int)ds + 4 * hi) * 4, o1o = ((32 + r) * (int)ds + 4 * hi) * 4;
    const int CS = dh >> 3;
#pragma unroll 1
    for (int c0 = 0; c0 < CS; c0 += 2) {
      float4 kq[2][4];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int co = 32 * (c0 + u);
        kq[u][0] = ld_b128(vsrc, v0o + co, 0);
        kq[u][1] = TJ > 1 ? ld_b128(vsrc, v1o + co, 0) : make_float4(0.f, 0.f, 0.f, 0.f);
        kq[u][2] = ld_b128(osrc, o0o + co, 0);
        kq[u][3] = TI > 1 ? ld_b128(osrc, o1o + co, 0) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const float ka[4] = {kq[u][0].x, kq[u][0].y, kq[u][0].z, kq[u][0].w};
        const float kc[4] = {kq[u][1].x, kq[u][1].y, kq[u][1].z, kq[u][1].w};
        const float qa[4] = {kq[u][2].x, kq[u][2].y, kq[u][2].z, kq[u][2].w};
        const float qc[4] = {kq[u][3].x, kq[u][3].y, kq[u][3].z, kq[u][3].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          g0 = WMFMA(ka[e], qa[e], g0, 0, 0, 0);
          if constexpr (T3) g3 = WMFMA(kc[e], qa[e], g3, 0, 0, 0);
          if constexpr (TI > 1) g1 = WMFMA(ka[e], qc[e], g1, 0, 0, 0);
          if constexpr (TI > 1 && TJ > 1) g2 = WMFMA(kc[e], qc[e], g2, 0, 0, 0);
        }
      }
    }
  }
  // ---- softmax gradient per query (lane): P reloaded, dS into g*, Pd into p*
  f32x16 p0, p1, p2, p3;
  auto sgrad = [&](f32x16& g_a, f32x16& g_b, f32x16& p_a, f32x16& p_b, bool two, int ti) {
    // rows past the queries were saved as 0 (every register of a computed tile is stored)
    const bool row = ROWS || 32 * ti + r < mk.L;
    const float* pw = prow0 + 2 * ti * 1024 + lane;  // the forward's register-layout save (wave_softmax)
    const uint64_t rb = pbase + (uint64_t)wm_qpos<ROWS>(mk, ti) * mk.L;
    float acc = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int j0 = creg(q, lane), j1 = 32 + j0;
      const float pa = row ? pw[64 * q] : 0.f;
      const float pb = two && row ? pw[1024 + 64 * q] : 0.f;
      const float ma = drop.mul(rb + wm_kpos<ROWS>(mk, j0)), mb = two ? drop.mul(rb + wm_kpos<ROWS>(mk, j1)) : 0.f;
      const bool ada = wm_adm<ROWS>(mk, ti, j0), adb = two && wm_adm<ROWS>(mk, ti, j1);
      g_a[q] = ada ? g_a[q] * ma : 0.f;
      g_b[q] = adb ? g_b[q] * mb : 0.f;
      acc += pa * g_a[q] + pb * g_b[q];
      p_a[q] = pa;
      p_b[q] = pb;
    }
    acc += __shfl_xor(acc, 32, 64);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int j0 = creg(q, lane), j1 = 32 + j0;
      g_a[q] = p_a[q] * (g_a[q] - acc);
      g_b[q] = two ? p_b[q] * (g_b[q] - acc) : 0.f;
      p_a[q] = p_a[q] * drop.mul(rb + wm_kpos<ROWS>(mk, j0));
      p_b[q] = two ? p_b[q] * drop.mul(rb + wm_kpos<ROWS>(mk, j1)) : 0.f;
    }
  };
  {
    f32x16 zg, zp;
    zero16(zg); zero16(zp);
    zero16(p1); zero16(p2); zero16(p3);
    if constexpr (T3)
      sgrad(g0, g3, p0, p3, true, 0);
    else
      sgrad(g0, zg, p0, zp, false, 0);
    if constexpr (TI > 1) sgrad(g1, g2, p1, p2, TJ > 1, 1);
  }
  const float sc = 1.0f / sqrtf((float)dh);
  const int CT = dh >> 5;
  // ---- dV = Pdᵀ·dO, dK = dSᵀ·Q/√dh: transpose through this wave's LDS tile T[i][j] (stride 65)
  constexpr int TLD = 65;
  auto put = [&](const f32x16& a, const f32x16& b, bool two, int ti) {
    const int i = 32 * ti + r;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int j0 = creg(q, lane);
      T[i * TLD + j0] = a[q];
      if (two) T[i * TLD + 32 + j0] = b[q];
    }
  };
  // T starts as garbage: every entry the products read ([0, 32·TI) x [0, 32·TJ)) is written first.  Pd goes to LDS
  // before the dQ product (ATTN_PD_EARLY, round 6): its 64 registers are dead through dQ, which then holds only dS —
  // the row kernel's spills 294 → 115 (fp32 out) / 133 → 86 (bf16 out); rows bwd fp32 out 139.8 → 134.7 µs, domain-pass
  // shape 158.0 → 151.0 µs (tools/attn_micro.py), main line +0.4 % (same-box A/B)
  auto put_pd = [&] {
    put(p0, p3, T3, 0);
    if constexpr (TI > 1) put(p1, p2, TJ > 1, 1);
    if constexpr (!ROWS && TJ > 1) {  // full layout: tile (tj = 1, ti = 0) is above the diagonal: zero
#pragma unroll
      for (int q = 0; q < 16; ++q) T[r * TLD + 32 + creg(q, lane)] = 0.f;
    }
  };
  if constexpr (ATTN_PD_EARLY) put_pd();
  // ---- dQ = dS·K/√dh (lane = column, rows = queries)
  {
    const auto ksrc = rows_rsrc(K, nk, ks, dh);
#pragma unroll 1
    for (int ct = 0; ct < CT; ++ct) {
      float k0v[16], k1v[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int key = (q & 3) + 8 * (q >> 2) + 4 * hi;
        k0v[q] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ksrc, (key * (int)ks + 32 * ct + r) * 4, 0, 0));
        k1v[q] = TJ > 1 ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                              ksrc, ((32 + key) * (int)ks + 32 * ct + r) * 4, 0, 0))
                        : 0.f;
      }
      f32x16 o0, o1;
      zero16(o0); zero16(o1);
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        o0 = WMFMA(g0[q], k0v[q], o0, 0, 0, 0);
        if constexpr (T3) o0 = WMFMA(g3[q], k1v[q], o0, 0, 0, 0);
        if constexpr (TI > 1) {
          o1 = WMFMA(g1[q], k0v[q], o1, 0, 0, 0);
          if constexpr (TJ > 1) o1 = WMFMA(g2[q], k1v[q], o1, 0, 0, 0);
        }
      }
      const int c = 32 * ct + r;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int i0 = creg(q, lane), i1 = 32 + i0;
        if (i0 < nq) dQ[(long)i0 * dqs + c] = (OT)(sc * o0[q]);
        if (TI > 1 && i1 < nq) dQ[(long)i1 * dqs + c] = (OT)(sc * o1[q]);
      }
    }
  }
  auto keys_out = [&](const float* __restrict__ Src, long ss, float scale, OT* __restrict__ Dst) {
    const auto src = rows_rsrc(Src, nq, ss, dh);
#pragma unroll 1
    for (int ct = 0; ct < CT; ++ct) {
      float b0v[16], b1v[16];  // Src rows (queries) of register q: (q&3) + 8(q>>2) + 4hi (+32)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int qi = (q & 3) + 8 * (q >> 2) + 4 * hi;
        b0v[q] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(src, (qi * (int)ss + 32 * ct + r) * 4, 0, 0));
        b1v[q] = TI > 1 ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                              src, ((32 + qi) * (int)ss + 32 * ct + r) * 4, 0, 0))
                        : 0.f;
      }
      const int c = 32 * ct + r;
#pragma unroll
      for (int tj = 0; tj < TJ; ++tj) {
        f32x16 o;
        zero16(o);
#pragma unroll
        for (int ti = ROWS ? 0 : tj; ti < TI; ++ti) {
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            const int qi = 32 * ti + (q & 3) + 8 * (q >> 2) + 4 * hi;
            const float a = T[qi * TLD + 32 * tj + r];
            o = WMFMA(a, ti ? b1v[q] : b0v[q], o, 0, 0, 0);
          }
        }
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int j = 32 * tj + creg(q, lane);
          if (j < nkw) Dst[(long)j * dks + c] = (OT)(scale * o[q]);
        }
      }
      for (int j = 32 * TJ + hi; j < nkw; j += 2) Dst[(long)j * dks + c] = (OT)0.f;  // keys past the tiles
    }
  };
  if constexpr (!ATTN_PD_EARLY) put_pd();
  wave_lds_sync();
  keys_out(dO, ds, 1.0f, dV);
  wave_lds_sync();
  put(g0, g3, T3, 0);
  if constexpr (TI > 1) put(g1, g2, TJ > 1, 1);
  wave_lds_sync();
  keys_out(Q, qs, sc, dK);
}

template <typename OT>
__global__ __launch_bounds__(256) void attn_bwd_wave(const float* __restrict__ qkv, const int64_t* __restrict__ seq,
                                                     int64_t pad, int B, int L, int d, int H, c2::Drop drop,
                                                     int64_t b_base, const float* __restrict__ Psave,
                                                     const float* __restrict__ dout, OT* __restrict__ dqkv) {
  __shared__ float tbuf[4][64 * 65];
  const int w = threadIdx.x >> 6;  // (vector, as in attn_fwd_wave)
  const int bh = blockIdx.x * 4 + w;
  if (bh >= B * H) return;  // uniform over the wave (no block-level barriers below)
  const int b = bh / H, h = bh % H, dh = d / H;
  int jmax;
  const WMask mk = full_mask(seq, pad, b, L, jmax);
  const long rs = 3l * d;
  const float* Q = qkv + (long)b * L * rs + h * dh;
  const float* dO = dout + (long)b * L * d + h * dh;
  OT* dQ = dqkv + (long)b * L * rs + h * dh;
  const uint64_t pbase = (uint64_t)((b_base + b) * H + h) * L * L;
  const float* prow = Psave + (long)bh * WAVE_PSAVE;
  const int TJ = jmax > 32 ? 2 : 1, TI = L > 32 ? 2 : 1;
#define BWD_FULL(TJ_, TI_)                                                                                     \
  bwd_wave_body<TJ_, TI_, OT, false>(Q, rs, Q + d, Q + 2 * d, rs, dO, d, L, dh, jmax, mk, drop, pbase, prow, dQ, rs, \
                                     dQ + d, dQ + 2 * d, rs, L, tbuf[w])
  if (TI == 1)
    BWD_FULL(1, 1);
  else if (TJ == 1)
    BWD_FULL(1, 2);
  else
    BWD_FULL(2, 2);
#undef BWD_FULL
}

template <typename OT>
__global__ __launch_bounds__(256, ATTN_ROWS_OCC) void attn_bwd_rows(const float* __restrict__ q, const float* __restrict__ kv,
                                                     const int64_t* __restrict__ seq, int64_t pad,
                                                     const int* __restrict__ q_idx, const int* __restrict__ q_off,
                                                     const int* __restrict__ k_idx, const int* __restrict__ k_off,
                                                     int B, int L, int d, int H, c2::Drop drop, int64_t b_base,
                                                     const float* __restrict__ Psave, const float* __restrict__ dout,
                                                     OT* __restrict__ dq, OT* __restrict__ dkv) {
  __shared__ float tbuf[4][64 * 65];
  // The wave index as a scalar (uniform descriptors, no waterfall loops, as attn_fwd_rows) for the bf16-output
  // instantiation only: 130 → 109 µs (tools/attn_micro.py); the fp32-output one (the fp32 mode) measured slower that
  // way, 138 → 191 µs (and 148 → 218 µs in the step), with or without its two-tile path split out as a call.
  const int w = std::is_same_v<OT, float> ? (int)(threadIdx.x >> 6) : __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int lane = threadIdx.x & 63;
  const int bh = blockIdx.x * 4 + w;
  if (bh >= B * H) return;  // uniform over the wave (no block-level barriers below)
  const int b = bh / H, h = bh % H, dh = d / H;
  int q0, nq, k0, nk;
  const WMask mk = rows_mask(seq, pad, b, L, q_idx, q_off, k_idx, k_off, q0, nq, k0, nk);
  OT* dK = dkv + (long)k0 * 2 * d + h * dh;
  if (nq == 0) {  // no query of this sequence is read: its keys get no gradient
    for (int e = lane; e < nk * dh; e += 64) {
      const int j = e / dh, c = e % dh;
      dK[(long)j * 2 * d + c] = (OT)0.f;
      dK[(long)j * 2 * d + d + c] = (OT)0.f;
    }
    return;
  }
  const float* Q = q + (long)q0 * d + h * dh;
  const float* K = kv + (long)k0 * 2 * d + h * dh;
  const float* dO = dout + (long)q0 * d + h * dh;
  OT* dQ = dq + (long)q0 * d + h * dh;
  const uint64_t pbase = (uint64_t)((b_base + b) * H + h) * L * L;
  const float* prow = Psave + (long)bh * WAVE_PSAVE;
  const int TJ = nk > 32 ? 2 : 1, TI = nq > 32 ? 2 : 1;
#define BWD_ROWS(TJ_, TI_)                                                                                     \
  bwd_wave_body<TJ_, TI_, OT, true>(Q, d, K, K + d, 2l * d, dO, d, nq, dh, nk, mk, drop, pbase, prow, dQ, d, dK,  \
                                    dK + d, 2l * d, nk, tbuf[w])
  if (TI == 1 && TJ == 1)
    BWD_ROWS(1, 1);
  else if (TI == 1)
    BWD_ROWS(2, 1);
  else if (TJ == 1)
    BWD_ROWS(1, 2);
  else
    BWD_ROWS(2, 2);
#undef BWD_ROWS
}

template <int LP>
size_t fwd_smem() { return sizeof(float) * ((size_t)LP * Smem<LP>::SLD + Smem<LP>::STAGE); }
template <int LP>
size_t bwd_smem() { return sizeof(float) * ((size_t)2 * LP * Smem<LP>::SLD + Smem<LP>::STAGE); }

template <int LP>
void launch_fwd(dim3 grid, hipStream_t s, const float* qkv, const int64_t* seq, int64_t pad, int L, int d, int H,
                c2::Drop dr, int64_t b_base, float* out, float* Psave) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)attn_fwd_kernel<LP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)fwd_smem<LP>());
    attr = true;
  }
  attn_fwd_kernel<LP><<<grid, 256, fwd_smem<LP>(), s>>>(qkv, seq, pad, L, d, H, dr, b_base, out, Psave);
}

template <int LP>
void launch_bwd(dim3 grid, hipStream_t s, const float* qkv, const int64_t* seq, int64_t pad, int L, int d, int H,
                c2::Drop dr, int64_t b_base, const float* Psave, const float* dout, float* dqkv) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)attn_bwd_kernel<LP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)bwd_smem<LP>());
    attr = true;
  }
  attn_bwd_kernel<LP><<<grid, 256, bwd_smem<LP>(), s>>>(qkv, seq, pad, L, d, H, dr, b_base, Psave, dout, dqkv);
}

bool wave_path(int L, int d, int H) { return L <= 64 && (d / H) % 32 == 0 && !getenv("C2DSR_ATTN_TILED"); }

}  // namespace

// floats of Psave c2dsr_attn_fwd / _bwd need: B·H·L·L on the tiled paths, B·H·4096 on the wave path
// (probabilities kept in the kernels' register layout)
C2_API size_t c2dsr_attn_psave_floats(int B, int L, int d, int H) {
  if (H <= 0 || d % H) return 0;
  return (size_t)B * H * (wave_path(L, d, H) ? WAVE_PSAVE : (size_t)L * L);
}

// qkv [B, L, 3d] (q | k | v per row, heads contiguous inside each), out [B, L, d],
// Psave c2dsr_attn_psave_floats(B, L, d, H) floats: softmax probabilities (pre-dropout), [B, H, L, L]
// on the tiled paths, the wave kernels' register layout on the wave path.  Dropout index:
// (((b_base + b)*H + h)*L + i)*L + j.
C2_API int c2dsr_attn_fwd(const float* qkv, const int64_t* seq, int64_t pad, int B, int L, int d, int H, uint32_t k0,
                          uint32_t k1, float p, int64_t b_base, float* out, float* Psave, void* stream) {
  if (L > 128 || d % H) return (int)hipErrorInvalidValue;
  if (B == 0) return 0;
  c2::Drop dr = c2::make_drop(k0, k1, p);
  hipStream_t s = (hipStream_t)stream;
  dim3 grid(B * H);
  const bool fast = (d / H) % 4 == 0 && d % 4 == 0;
  if (wave_path(L, d, H))
    attn_fwd_wave<<<c2::ceil_div((long)B * H, 4), 256, 0, s>>>(qkv, seq, pad, B, L, d, H, dr, b_base, out, Psave);
  else if (fast && L <= 32)
    attn_fwd_fast<32><<<grid, 256, 0, s>>>(qkv, seq, pad, L, d, H, dr, b_base, out, Psave);
  else if (fast && L <= 64)
    attn_fwd_fast<64><<<grid, 256, 0, s>>>(qkv, seq, pad, L, d, H, dr, b_base, out, Psave);
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
  const bool fast = (d / H) % 4 == 0 && d % 4 == 0;
  if (wave_path(L, d, H))
    attn_bwd_wave<float><<<c2::ceil_div((long)B * H, 4), 256, 0, s>>>(qkv, seq, pad, B, L, d, H, dr, b_base, Psave,
                                                                      dout, dqkv);
  else if (fast && L <= 32)
    attn_bwd_fast<32><<<grid, 256, 0, s>>>(qkv, seq, pad, L, d, H, dr, b_base, Psave, dout, dqkv);
  else if (fast && L <= 64)
    attn_bwd_fast<64><<<grid, 256, 0, s>>>(qkv, seq, pad, L, d, H, dr, b_base, Psave, dout, dqkv);
  else if (L <= 32)
    launch_bwd<32>(grid, s, qkv, seq, pad, L, d, H, dr, b_base, Psave, dout, dqkv);
  else if (L <= 64)
    launch_bwd<64>(grid, s, qkv, seq, pad, L, d, H, dr, b_base, Psave, dout, dqkv);
  else
    launch_bwd<128>(grid, s, qkv, seq, pad, L, d, H, dr, b_base, Psave, dout, dqkv);
  C2_CHECK_LAUNCH();
  return 0;
}

// 1 when c2dsr_attn_bwd_b16 takes the shape (the wave kernels: L <= 64, d/H a multiple of 32)
C2_API int c2dsr_attn_bwd_b16_supported(int L, int d, int H) { return H > 0 && d % H == 0 && wave_path(L, d, H); }

// c2dsr_attn_bwd with dqkv written in bf16 (its consumers, the in_proj backward GEMMs c2dsr_rgemm_aux_b16a /
// c2dsr_wgemm_b16y, use it as a bf16 MFMA operand: the same values they would round it to)
C2_API int c2dsr_attn_bwd_b16(const float* qkv, const int64_t* seq, int64_t pad, int B, int L, int d, int H,
                              uint32_t k0, uint32_t k1, float p, int64_t b_base, const float* Psave, const float* dout,
                              void* dqkv, void* stream) {
  if (!c2dsr_attn_bwd_b16_supported(L, d, H)) return (int)hipErrorInvalidValue;
  if (B == 0) return 0;
  c2::Drop dr = c2::make_drop(k0, k1, p);
  attn_bwd_wave<bf16><<<c2::ceil_div((long)B * H, 4), 256, 0, (hipStream_t)stream>>>(
      qkv, seq, pad, B, L, d, H, dr, b_base, Psave, dout, (bf16*)dqkv);
  C2_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------------------
// Row-subset attention (the last post-norm encoder layer of a training pass, whose output the loss reads
// only at the rows of a RowSet): queries are those rows, keys the padding rows (the only admissible ones,
// Q1), both compact in position order per sequence — q [nq_total, d] (row q_off[b] + i = query i of
// sequence b, global row q_idx[...]), kv [nk_total, 2d] (K | V, row k_off[b] + j), out [nq_total, d].
// Same masks, dropout indices and Psave layout (B·H·4096 floats) as c2dsr_attn_fwd's wave path; the
// outputs at the query rows equal the full-layout ones up to the order of the key sums.
C2_API int c2dsr_attn_rows_supported(int L, int d, int H) { return c2dsr_attn_bwd_b16_supported(L, d, H); }

C2_API int c2dsr_attn_fwd_rows(const float* q, const float* kv, const int64_t* seq, int64_t pad, const int* q_idx,
                               const int* q_off, const int* k_idx, const int* k_off, int B, int L, int d, int H,
                               uint32_t k0, uint32_t k1, float p, int64_t b_base, float* out, float* Psave,
                               void* stream) {
  if (!c2dsr_attn_rows_supported(L, d, H)) return (int)hipErrorInvalidValue;
  if (B == 0) return 0;
  attn_fwd_rows<<<c2::ceil_div((long)B * H, 4), 256, 0, (hipStream_t)stream>>>(
      q, kv, seq, pad, q_idx, q_off, k_idx, k_off, B, L, d, H, c2::make_drop(k0, k1, p), b_base, out, Psave);
  C2_CHECK_LAUNCH();
  return 0;
}

// dq [nq_total, d], dkv [nk_total, 2d]: fp32 (out_bf16 = 0) or bf16 (1; their consumers, the in_proj
// backward GEMMs, read them as a bf16 MFMA operand)
C2_API int c2dsr_attn_bwd_rows(const float* q, const float* kv, const int64_t* seq, int64_t pad, const int* q_idx,
                               const int* q_off, const int* k_idx, const int* k_off, int B, int L, int d, int H,
                               uint32_t k0, uint32_t k1, float p, int64_t b_base, const float* Psave,
                               const float* dout, void* dq, void* dkv, int out_bf16, void* stream) {
  if (!c2dsr_attn_rows_supported(L, d, H)) return (int)hipErrorInvalidValue;
  if (B == 0) return 0;
  const c2::Drop dr = c2::make_drop(k0, k1, p);
  const dim3 grid(c2::ceil_div((long)B * H, 4));
  hipStream_t s = (hipStream_t)stream;
  if (out_bf16)
    attn_bwd_rows<bf16><<<grid, 256, 0, s>>>(q, kv, seq, pad, q_idx, q_off, k_idx, k_off, B, L, d, H, dr, b_base,
                                             Psave, dout, (bf16*)dq, (bf16*)dkv);
  else
    attn_bwd_rows<float><<<grid, 256, 0, s>>>(q, kv, seq, pad, q_idx, q_off, k_idx, k_off, B, L, d, H, dr, b_base,
                                              Psave, dout, (float*)dq, (float*)dkv);
  C2_CHECK_LAUNCH();
  return 0;
}
