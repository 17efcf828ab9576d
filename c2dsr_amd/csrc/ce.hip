// K5: fused classifier-head linear + cross-entropy (the one real dense contraction of
// the path), bf16 MFMA with fp32 accumulation, logits never materialised.
//
// Replaces trainer.py:131-154: logits = h·Wᵀ + b (classifier_a/b, C2DSR.py:36-44) over
// all n items, concatenated with the pad column, F.cross_entropy(ignore_index = n)
// forward and backward.  Rows are the stacked [share ; specific] heads that share W
// (M = 2·B·R), K = D = d_latent.
//
//   lse kernel  (S^T = W·Hᵀ): per row tile, online log-sum-exp over a column range
//   dH kernel   (S^T again):   P'ᵀ = (softmax - onehot)·w_r, dHᵀ += Wᵀ·P'ᵀ
//   dW kernel   (S = H·Wᵀ):    P'  likewise,                 dWᵀ += Hᵀ·P',  db += Σ_r P'
// The accumulator of the first product is fed straight back as the B operand of the
// second (gfx950 32x32 C/D layout = B layout up to a k permutation), and the other
// operand is read TRANSPOSED from the same LDS image with ds_read_b64_tr_b16: one
// XOR-swizzled image per tile serves both the row reads (ds_read_b128) and the
// transposed reads, conflict-free (cdna_hip_programming.md §5.5 T10, image (b)).
// Each lane keeps its rows' (or columns') operand fragments in registers for the
// whole sweep; the swept operand is double-buffered through LDS with register-staged
// prefetch.  Work is split over column (lse, dH) or row (dW) ranges for occupancy and
// the partials are combined in a fixed order (deterministic).
#include "common.h"

namespace {

typedef __bf16 bf16;
typedef bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
typedef __attribute__((address_space(3))) i16x4 lds_i16x4;

constexpr float LOG2E = 1.4426950408889634f;
constexpr int TILE = 64;  // rows of the swept operand per LDS tile

// ---------------------------------------------------------------- LDS image
// A [TILE][D] bf16 tile is stored as D/128 half-tiles of [TILE][128] bf16 (256-byte
// rows); 16-byte chunk `ch` of row `row` sits at swz(row, ch).
__device__ __forceinline__ int swz(int row, int ch) {
  return row * 256 + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}
// byte offset of element (row, k) (k multiple of 8 for a 16-byte read)
__device__ __forceinline__ int img_off(int row, int k) { return (k >> 7) * (TILE * 256) + swz(row, (k & 127) >> 3) + 2 * (k & 7); }

// A-operand fragment for v_mfma_f32_32x32x16_bf16 whose rows are TILE rows r0..r0+31 and
// whose k-slice is k0..k0+15 (k0 multiple of 16): lane (i = l&31, h = l>>5) gets (row r0+i, k0+8h..+7).
__device__ __forceinline__ bf16x8 row_frag(const char* img, int r0, int k0, int lane) {
  const int row = r0 + (lane & 31), k = k0 + 8 * (lane >> 5);
  return *(const bf16x8*)(img + img_off(row, k));
}

// Transposed fragment: the MFMA operand whose row index is the image's k (kb0..kb0+31 ↔ lane&31)
// and whose reduction index runs over image rows in the permuted order of an accumulator
// fed back as B: element j of lane half h ↔ image row rr0 + 8*(j>>2) + 4*h + (j&3).
__device__ __forceinline__ bf16x8 tr_frag(const char* img, int rr0, int kb0, int lane) {
  const int g = lane >> 4, h = lane >> 5, q = (lane & 15) >> 2, p = lane & 3;
  const int kcol = kb0 + 16 * (g & 1);  // this 16-lane group's 16 image columns
  const int row = rr0 + 4 * h + q;
  const int ch = ((kcol & 127) >> 3) + (p >> 1);
  const int base = (kcol >> 7) * (TILE * 256);
  const char* a0 = img + base + swz(row, ch) + 8 * (p & 1);
  const char* a1 = img + base + swz(row + 8, ch) + 8 * (p & 1);
  bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)a0);
  bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)a1);
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

// accumulator registers 8s..8s+7 → bf16 B operand of k-step s
__device__ __forceinline__ bf16x8 acc_frag(const f32x16& a, int s) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (bf16)a[8 * s + j];
  return r;
}

// Register-staged tile loader: rows g0..g0+TILE-1 of a row-major bf16 [rows][D] matrix
template <int D>
struct TileLoad {
  static constexpr int CHUNKS = TILE * D / 8;  // 16-byte chunks per tile
  static constexpr int PER = CHUNKS / 256;
  uint4 v[PER];
  __device__ __forceinline__ void load(const bf16* __restrict__ X, long nrows, long g0) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int q = threadIdx.x + 256 * i;
      const int row = q / (D / 8), ch = q % (D / 8);
      const long gr = g0 + row;
      v[i] = gr < nrows ? *(const uint4*)(X + gr * D + ch * 8) : make_uint4(0, 0, 0, 0);
    }
  }
  __device__ __forceinline__ void store(char* img) const {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int q = threadIdx.x + 256 * i;
      const int row = q / (D / 8), ch = q % (D / 8);
      *(uint4*)(img + (ch >> 4) * (TILE * 256) + swz(row, ch & 15)) = v[i];
    }
  }
};

__device__ __forceinline__ int creg(int reg, int lane) { return (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5); }

// ---------------------------------------------------------------- forward: partial LSE
// grid (ceil(M/256), n_split); 4 waves x 64 rows.  part_m/part_s [n_split][M]: log2-domain
// running max and sum of 2^(s·log2e) over the split's columns.
template <int D>
__global__ __launch_bounds__(256, 1) void ce_lse_kernel(const bf16* __restrict__ Hb, const bf16* __restrict__ Wb,
                                                        const float* __restrict__ bias, int M, int n,
                                                        int cols_per_split, float* __restrict__ part_m,
                                                        float* __restrict__ part_s) {
  constexpr int KS = D / 16;
  __shared__ __attribute__((aligned(16))) char img[2][TILE * D * 2];
  __shared__ float b2s[2][TILE];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int rbase = blockIdx.x * 256 + w * 64;
  const int c_beg = blockIdx.y * cols_per_split;
  const int c_end = min(n, c_beg + cols_per_split);
  bf16x8 hf[2][KS];
#pragma unroll
  for (int rb = 0; rb < 2; ++rb) {
    const int r = rbase + rb * 32 + (lane & 31);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (r < M)
        hf[rb][ks] = *(const bf16x8*)(Hb + (long)r * D + ks * 16 + 8 * (lane >> 5));
      else
        for (int j = 0; j < 8; ++j) hf[rb][ks][j] = (bf16)0.f;
    }
  }
  float mrun[2] = {-INFINITY, -INFINITY}, srun[2] = {0.f, 0.f};
  const int ntiles = c_end > c_beg ? (c_end - c_beg + TILE - 1) / TILE : 0;
  TileLoad<D> ld;
  if (ntiles > 0) {
    ld.load(Wb, n, c_beg);
    ld.store(img[0]);
    if (threadIdx.x < TILE) {
      const int c = c_beg + threadIdx.x;
      b2s[0][threadIdx.x] = c < n ? bias[c] * LOG2E : -INFINITY;
    }
  }
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1;
    const int c0 = c_beg + t * TILE;
    if (t + 1 < ntiles) ld.load(Wb, n, c0 + TILE);
    f32x16 acc[2][2];
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[cb][rb][i] = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        const bf16x8 a = row_frag(img[cur], cb * 32, ks * 16, lane);
#pragma unroll
        for (int rb = 0; rb < 2; ++rb)
          acc[cb][rb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, hf[rb][ks], acc[cb][rb], 0, 0, 0);
      }
    }
    // online log2-sum-exp2 per lane row (lanes l and l^32 share a row, different columns)
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      float tmax = -INFINITY;
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float v = fmaf(acc[cb][rb][i], LOG2E, b2s[cur][cb * 32 + creg(i, lane)]);
          acc[cb][rb][i] = v;
          tmax = fmaxf(tmax, v);
        }
      const float mnew = fmaxf(mrun[rb], tmax);
      float s = (mrun[rb] == -INFINITY) ? 0.f : srun[rb] * exp2f(mrun[rb] - mnew);
      if (mnew != -INFINITY) {
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
          for (int i = 0; i < 16; ++i) s += exp2f(acc[cb][rb][i] - mnew);
      }
      mrun[rb] = mnew;
      srun[rb] = s;
    }
    if (t + 1 < ntiles) {
      ld.store(img[cur ^ 1]);
      if (threadIdx.x < TILE) {
        const int c = c0 + TILE + threadIdx.x;
        b2s[cur ^ 1][threadIdx.x] = c < n ? bias[c] * LOG2E : -INFINITY;
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int rb = 0; rb < 2; ++rb) {
    const float m2 = __shfl_xor(mrun[rb], 32, 64), s2 = __shfl_xor(srun[rb], 32, 64);
    const float mm = fmaxf(mrun[rb], m2);
    const float s = (mrun[rb] == -INFINITY ? 0.f : srun[rb] * exp2f(mrun[rb] - mm)) +
                    (m2 == -INFINITY ? 0.f : s2 * exp2f(m2 - mm));
    const int r = rbase + rb * 32 + (lane & 31);
    if (lane < 32 && r < M) {
      part_m[(long)blockIdx.y * M + r] = mm;
      part_s[(long)blockIdx.y * M + r] = s;
    }
  }
}

// per row: lse over the splits and the pad column, target logit (fp32), loss.  One wave per row.
__global__ __launch_bounds__(256) void ce_rows_kernel(const float* __restrict__ part_m,
                                                      const float* __restrict__ part_s, int n_split, int M,
                                                      const float* __restrict__ padlogit,
                                                      const int64_t* __restrict__ tgt, int n,
                                                      const float* __restrict__ H, const float* __restrict__ W,
                                                      const float* __restrict__ bias, int D,
                                                      float* __restrict__ lse_out, float* __restrict__ lse2_out,
                                                      float* __restrict__ loss_row) {
  const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= M) return;
  const long t = tgt[r];
  float dot = 0.f;
  if (t >= 0 && t < n)
    for (int k = lane; k < D; k += 64) dot += H[r * D + k] * W[t * D + k];
  dot = c2::wave_sum(dot);
  if (lane == 0) {
    float mm = -INFINITY;
    for (int s = 0; s < n_split; ++s) mm = fmaxf(mm, part_m[(long)s * M + r]);
    float ss = 0.f;
    for (int s = 0; s < n_split; ++s) {
      const float m = part_m[(long)s * M + r];
      if (m != -INFINITY) ss += part_s[(long)s * M + r] * exp2f(m - mm);
    }
    const float lse_items = (mm + log2f(ss)) / LOG2E;
    const float pl = padlogit[r];
    const float hi = fmaxf(lse_items, pl);
    const float lse = hi + logf(expf(lse_items - hi) + expf(pl - hi));
    lse_out[r] = lse;
    lse2_out[r] = lse * LOG2E;
    loss_row[r] = (t != n) ? lse - (t < n ? dot + bias[t] : pl) : 0.f;
  }
}

// ---------------------------------------------------------------- backward: dH
// grid (ceil(M/128), n_split); 4 waves x 32 rows; sweeps the split's columns.
// dHp [n_split][M][D] (fp32 partials, combined by ce_sum_parts_kernel).
template <int D>
__global__ __launch_bounds__(256, 1) void ce_dh_kernel(const bf16* __restrict__ Hb, const bf16* __restrict__ Wb,
                                                       const float* __restrict__ bias, int M, int n,
                                                       int cols_per_split, const float* __restrict__ lse2,
                                                       const int64_t* __restrict__ tgt,
                                                       const float* __restrict__ roww, float* __restrict__ dHp) {
  constexpr int KS = D / 16;
  constexpr int KB = D / 32;
  __shared__ __attribute__((aligned(16))) char img[2][TILE * D * 2];
  __shared__ float b2s[2][TILE];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = blockIdx.x * 128 + w * 32 + (lane & 31);
  const int c_beg = blockIdx.y * cols_per_split;
  const int c_end = min(n, c_beg + cols_per_split);
  bf16x8 hf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    if (r < M)
      hf[ks] = *(const bf16x8*)(Hb + (long)r * D + ks * 16 + 8 * (lane >> 5));
    else
      for (int j = 0; j < 8; ++j) hf[ks][j] = (bf16)0.f;
  }
  const float lr = r < M ? lse2[r] : 0.f;
  const float rw = r < M ? roww[r] : 0.f;
  const long tr = r < M ? tgt[r] : -1;
  f32x16 dacc[KB];
#pragma unroll
  for (int kb = 0; kb < KB; ++kb)
#pragma unroll
    for (int i = 0; i < 16; ++i) dacc[kb][i] = 0.f;
  const int ntiles = c_end > c_beg ? (c_end - c_beg + TILE - 1) / TILE : 0;
  TileLoad<D> ld;
  if (ntiles > 0) {
    ld.load(Wb, n, c_beg);
    ld.store(img[0]);
    if (threadIdx.x < TILE) {
      const int c = c_beg + threadIdx.x;
      b2s[0][threadIdx.x] = c < n ? bias[c] * LOG2E : -INFINITY;
    }
  }
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1;
    const int c0 = c_beg + t * TILE;
    if (t + 1 < ntiles) ld.load(Wb, n, c0 + TILE);
    f32x16 s[2];
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int i = 0; i < 16; ++i) s[cb][i] = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
        s[cb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag(img[cur], cb * 32, ks * 16, lane), hf[ks], s[cb], 0,
                                                        0, 0);
    // P'ᵀ[c][r] = (2^(s·log2e + b2 - lse2) - [c == t]) * w_r
    bf16x8 x[2][2];
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int cl = cb * 32 + creg(i, lane);
        const float e = exp2f(fmaf(s[cb][i], LOG2E, b2s[cur][cl]) - lr);
        s[cb][i] = (e - ((long)(c0 + cl) == tr ? 1.f : 0.f)) * rw;
      }
      x[cb][0] = acc_frag(s[cb], 0);
      x[cb][1] = acc_frag(s[cb], 1);
    }
    // dHᵀ[k][r] += Σ_c W[c][k] P'ᵀ[c][r]
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int st = 0; st < 2; ++st)
          dacc[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_frag(img[cur], cb * 32 + 16 * st, kb * 32, lane),
                                                             x[cb][st], dacc[kb], 0, 0, 0);
    if (t + 1 < ntiles) {
      ld.store(img[cur ^ 1]);
      if (threadIdx.x < TILE) {
        const int c = c0 + TILE + threadIdx.x;
        b2s[cur ^ 1][threadIdx.x] = c < n ? bias[c] * LOG2E : -INFINITY;
      }
    }
    __syncthreads();
  }
  if (r < M) {
    float* out = dHp + ((long)blockIdx.y * M + r) * D;
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
      for (int i = 0; i < 16; ++i) out[kb * 32 + creg(i, lane)] = dacc[kb][i];
  }
}

// ---------------------------------------------------------------- backward: dW, db
// grid (ceil(n/128), n_rsplit); 4 waves x 32 columns; sweeps the split's rows.
// dWp [n_rsplit][n][D], dbp [n_rsplit][n] fp32 partials.
template <int D>
__global__ __launch_bounds__(256, 1) void ce_dw_kernel(const bf16* __restrict__ Hb, const bf16* __restrict__ Wb,
                                                       const float* __restrict__ bias, int M, int n,
                                                       int rows_per_split, const float* __restrict__ lse2,
                                                       const int64_t* __restrict__ tgt,
                                                       const float* __restrict__ roww, float* __restrict__ dWp,
                                                       float* __restrict__ dbp) {
  constexpr int KS = D / 16;
  constexpr int KB = D / 32;
  __shared__ __attribute__((aligned(16))) char img[2][TILE * D * 2];
  __shared__ float rl[2][TILE], rwv[2][TILE];
  __shared__ long rt[2][TILE];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 128 + w * 32 + (lane & 31);
  const int r_beg = blockIdx.y * rows_per_split;
  const int r_end = min(M, r_beg + rows_per_split);
  bf16x8 wf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    if (c < n)
      wf[ks] = *(const bf16x8*)(Wb + (long)c * D + ks * 16 + 8 * (lane >> 5));
    else
      for (int j = 0; j < 8; ++j) wf[ks][j] = (bf16)0.f;
  }
  const float b2 = c < n ? bias[c] * LOG2E : 0.f;
  f32x16 dacc[KB];
#pragma unroll
  for (int kb = 0; kb < KB; ++kb)
#pragma unroll
    for (int i = 0; i < 16; ++i) dacc[kb][i] = 0.f;
  float db = 0.f;
  const int ntiles = r_end > r_beg ? (r_end - r_beg + TILE - 1) / TILE : 0;
  TileLoad<D> ld;
  auto rowinfo = [&](int buf, int r0) {
    if (threadIdx.x < TILE) {
      const int r = r0 + threadIdx.x;
      const bool ok = r < r_end;
      rl[buf][threadIdx.x] = ok ? lse2[r] : 0.f;
      rwv[buf][threadIdx.x] = ok ? roww[r] : 0.f;
      rt[buf][threadIdx.x] = ok ? tgt[r] : -1;
    }
  };
  if (ntiles > 0) {
    ld.load(Hb, r_end, r_beg);
    ld.store(img[0]);
    rowinfo(0, r_beg);
  }
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1;
    const int r0 = r_beg + t * TILE;
    if (t + 1 < ntiles) ld.load(Hb, r_end, r0 + TILE);
    f32x16 s[2];
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int i = 0; i < 16; ++i) s[rb][i] = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
        s[rb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag(img[cur], rb * 32, ks * 16, lane), wf[ks], s[rb], 0,
                                                        0, 0);
    bf16x8 x[2][2];
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int rl_ = rb * 32 + creg(i, lane);
        const float e = exp2f(fmaf(s[rb][i], LOG2E, b2) - rl[cur][rl_]);
        const float v = c < n ? (e - ((long)c == rt[cur][rl_] ? 1.f : 0.f)) * rwv[cur][rl_] : 0.f;
        s[rb][i] = v;
        db += v;
      }
      x[rb][0] = acc_frag(s[rb], 0);
      x[rb][1] = acc_frag(s[rb], 1);
    }
    // dWᵀ[k][c] += Σ_r H[r][k] P'[r][c]
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int st = 0; st < 2; ++st)
          dacc[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_frag(img[cur], rb * 32 + 16 * st, kb * 32, lane),
                                                             x[rb][st], dacc[kb], 0, 0, 0);
    if (t + 1 < ntiles) {
      ld.store(img[cur ^ 1]);
      rowinfo(cur ^ 1, r0 + TILE);
    }
    __syncthreads();
  }
  db += __shfl_xor(db, 32, 64);
  if (c < n) {
    if (lane < 32) dbp[(long)blockIdx.y * n + c] = db;
    float* out = dWp + ((long)blockIdx.y * n + c) * D;
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
      for (int i = 0; i < 16; ++i) out[kb * 32 + creg(i, lane)] = dacc[kb][i];
  }
}

// out[i] = beta*out[i] + Σ_s part[s][i]   (fixed order)
__global__ void sum_parts_kernel(const float* __restrict__ part, int nparts, long n, float beta,
                                 float* __restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float t = 0.f;
  for (int s = 0; s < nparts; ++s) t += part[(long)s * n + i];
  out[i] = (beta == 0.f ? 0.f : beta * out[i]) + t;
}

__global__ void f32_to_bf16_kernel(const float* __restrict__ x, long n, bf16* __restrict__ y) {
  const long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i >= n) return;
  if (i + 3 < n) {
    const float4 v = *(const float4*)(x + i);
    y[i] = (bf16)v.x;
    y[i + 1] = (bf16)v.y;
    y[i + 2] = (bf16)v.z;
    y[i + 3] = (bf16)v.w;
  } else {
    for (long j = i; j < n; ++j) y[j] = (bf16)x[j];
  }
}

// rw[r] = valid ? gscale * lam * coef[r >= split] : 0
__global__ void ce_roww_kernel(const int64_t* __restrict__ tgt, int M, int ignore, const float* __restrict__ coef,
                               int split, const float* __restrict__ gscale, float lam, float* __restrict__ rw) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= M) return;
  rw[r] = tgt[r] != ignore ? gscale[0] * lam * coef[r >= split ? 1 : 0] : 0.f;
}

// dpad[r] = exp(pl[r] - lse[r]) * rw[r]  (pad column of the softmax; its target is ignored)
__global__ void ce_padgrad_kernel(const float* __restrict__ pl, const float* __restrict__ lse,
                                  const float* __restrict__ rw, int M, float* __restrict__ dpad) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= M) return;
  dpad[r] = expf(pl[r] - lse[r]) * rw[r];
}

// self-test of the transposed fragment addressing: image row = rr, col = k holds rr*256+k (int16)
__global__ void selftest_tr_kernel(int rr0, int kb0, short* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) char img[TILE * 256 * 2];
  for (int q = threadIdx.x; q < TILE * 256; q += blockDim.x) {
    const int row = q / 256, k = q % 256;
    *(short*)(img + img_off(row, k)) = (short)(row * 256 + k);
  }
  __syncthreads();
  const int lane = threadIdx.x;
  const int g = lane >> 4, h = lane >> 5, q = (lane & 15) >> 2, p = lane & 3;
  const int kcol = kb0 + 16 * (g & 1);
  const int row = rr0 + 4 * h + q;
  const int ch = ((kcol & 127) >> 3) + (p >> 1);
  const int base = (kcol >> 7) * (TILE * 256);
  i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(img + base + swz(row, ch) + 8 * (p & 1)));
  i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(img + base + swz(row + 8, ch) + 8 * (p & 1)));
  for (int j = 0; j < 4; ++j) {
    out[lane * 8 + j] = lo[j];
    out[lane * 8 + 4 + j] = hi[j];
  }
  // row fragment check (rows rr0.., k-slice kb0..)
  const bf16x8 rf = row_frag(img, rr0, kb0, lane);
  const short* rs = (const short*)&rf;
  for (int j = 0; j < 8; ++j) out[512 + lane * 8 + j] = rs[j];
}

template <int D>
void launch_all(int which, dim3 grid, hipStream_t s, const bf16* Hb, const bf16* Wb, const float* bias, int M, int n,
                int per, float* a0, float* a1, const float* lse2, const int64_t* tgt, const float* rw) {
  if (which == 0) ce_lse_kernel<D><<<grid, 256, 0, s>>>(Hb, Wb, bias, M, n, per, a0, a1);
  if (which == 1) ce_dh_kernel<D><<<grid, 256, 0, s>>>(Hb, Wb, bias, M, n, per, lse2, tgt, rw, a0);
  if (which == 2) ce_dw_kernel<D><<<grid, 256, 0, s>>>(Hb, Wb, bias, M, n, per, lse2, tgt, rw, a0, a1);
}

int launch_d(int D, int which, dim3 grid, hipStream_t s, const bf16* Hb, const bf16* Wb, const float* bias, int M,
             int n, int per, float* a0, float* a1, const float* lse2, const int64_t* tgt, const float* rw) {
  if (D == 128)
    launch_all<128>(which, grid, s, Hb, Wb, bias, M, n, per, a0, a1, lse2, tgt, rw);
  else if (D == 256)
    launch_all<256>(which, grid, s, Hb, Wb, bias, M, n, per, a0, a1, lse2, tgt, rw);
  else
    return (int)hipErrorInvalidValue;
  C2_CHECK_LAUNCH();
  return 0;
}

int per_split(int total, int nsplit, int gran) {
  int tiles = c2::ceil_div(total, gran);
  return c2::ceil_div(tiles, nsplit) * gran;
}

}  // namespace

C2_API int c2dsr_ce_supported(int D) { return D == 128 || D == 256; }

C2_API int c2dsr_f32_to_bf16(const float* x, long n, void* y, void* stream) {
  if (n == 0) return 0;
  f32_to_bf16_kernel<<<c2::ceil_div((n + 3) / 4, 256), 256, 0, (hipStream_t)stream>>>(x, n, (bf16*)y);
  C2_CHECK_LAUNCH();
  return 0;
}

// forward: part_m/part_s [n_split][M] → (with pad logits, targets, fp32 H/W for the target logit)
// lse, lse2 (= lse·log2e), loss_row [M].
C2_API int c2dsr_ce_fused_fwd(const void* Hb, const void* Wb, const float* bias, int M, int n, int D, int n_split,
                              float* part_m, float* part_s, const float* padlogit, const int64_t* tgt,
                              const float* H, const float* W, float* lse, float* lse2, float* loss_row,
                              void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (M == 0) return 0;
  const int per = per_split(n, n_split, TILE);
  dim3 grid(c2::ceil_div(M, 256), n_split);
  int e = launch_d(D, 0, grid, s, (const bf16*)Hb, (const bf16*)Wb, bias, M, n, per, part_m, part_s, nullptr, nullptr,
                   nullptr);
  if (e) return e;
  ce_rows_kernel<<<c2::ceil_div(M, 4), 256, 0, s>>>(part_m, part_s, n_split, M, padlogit, tgt, n, H, W, bias, D, lse,
                                                    lse2, loss_row);
  C2_CHECK_LAUNCH();
  return 0;
}

C2_API int c2dsr_ce_row_weights(const int64_t* tgt, int M, int ignore, const float* coef, int split,
                                const float* gscale, float lam, const float* padlogit, const float* lse, float* rw,
                                float* dpad, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (M == 0) return 0;
  ce_roww_kernel<<<c2::ceil_div(M, 256), 256, 0, s>>>(tgt, M, ignore, coef, split, gscale, lam, rw);
  ce_padgrad_kernel<<<c2::ceil_div(M, 256), 256, 0, s>>>(padlogit, lse, rw, M, dpad);
  C2_CHECK_LAUNCH();
  return 0;
}

// dH = Σ_c P'[r][c] W[c]  → dH [M][D] (overwritten); dHp: [n_split][M][D] scratch
C2_API int c2dsr_ce_fused_dh(const void* Hb, const void* Wb, const float* bias, int M, int n, int D, int n_split,
                             const float* lse2, const int64_t* tgt, const float* rw, float* dHp, float* dH,
                             void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (M == 0) return 0;
  const int per = per_split(n, n_split, TILE);
  dim3 grid(c2::ceil_div(M, 128), n_split);
  int e = launch_d(D, 1, grid, s, (const bf16*)Hb, (const bf16*)Wb, bias, M, n, per, dHp, nullptr, lse2, tgt, rw);
  if (e) return e;
  const long tot = (long)M * D;
  sum_parts_kernel<<<c2::ceil_div(tot, 256), 256, 0, s>>>(dHp, n_split, tot, 0.f, dH);
  C2_CHECK_LAUNCH();
  return 0;
}

// dWp[s][c] = Σ_{r in split s} P'[r][c] H[r];  dbp[s][c] = Σ_r P'[r][c]  (combine with c2dsr_sum_parts).
C2_API int c2dsr_ce_fused_dw(const void* Hb, const void* Wb, const float* bias, int M, int n, int D, int n_rsplit,
                             const float* lse2, const int64_t* tgt, const float* rw, float* dWp, float* dbp,
                             float* gW, float* gb, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (n == 0) return 0;
  const int per = per_split(M, n_rsplit, TILE);
  dim3 grid(c2::ceil_div(n, 128), n_rsplit);
  int e = launch_d(D, 2, grid, s, (const bf16*)Hb, (const bf16*)Wb, bias, M, n, per, dWp, dbp, lse2, tgt, rw);
  if (e) return e;
  (void)gW;
  (void)gb;
  return 0;
}

// out[i] = beta*out[i] + Σ_s part[s][i]  (fixed order) — combines the split partials
C2_API int c2dsr_sum_parts(const float* part, int nparts, long n, float beta, float* out, void* stream) {
  if (n == 0) return 0;
  sum_parts_kernel<<<c2::ceil_div(n, 256), 256, 0, (hipStream_t)stream>>>(part, nparts, n, beta, out);
  C2_CHECK_LAUNCH();
  return 0;
}

C2_API int c2dsr_selftest_tr(int rr0, int kb0, short* out, void* stream) {
  selftest_tr_kernel<<<1, 64, 0, (hipStream_t)stream>>>(rr0, kb0, out);
  C2_CHECK_LAUNCH();
  return 0;
}
