// Dense GEMM on the matrix cores for the encoder projections, the bilinear
// discriminators and (with logits materialised) the classifier heads.
//
//   C[M,N] = alpha * op(A)[M,K] * op(B)[K,N] + beta * C + bias[N]   (+ relu·dropout epilogue)
//   op(A): transA=0 → A[m*lda+k], 1 → A[k*lda+m];  op(B): transB=0 → B[k*ldb+n], 1 → B[n*ldb+k]
//
// Replaces the nn.Linear / F.linear / nn.Bilinear addmm calls reached from
// models/encoders.py:33 (TransformerEncoderLayer in_proj/out_proj/linear1/linear2),
// trainer.py:104-108 (D_a/D_b) and trainer.py:131-140 (classifier_{a,b,pad}) and their
// autograd backward (dX = dY·W, dW = dYᵀ·X with split-K over the long row axis).
//
// fp32 storage; compute either on v_mfma_f32_32x32x16_bf16 (bf16 operands, fp32
// accumulate: the performance mode) or v_mfma_f32_32x32x2_f32 (exact fp32: the
// 1e-4 parity mode).  Tile 128x128x32, 4 waves (2x2), each wave 64x64 = 2x2 MFMA
// 32x32 tiles; operands staged global→registers→LDS (the register pass converts
// to bf16 and transposes M-contiguous operands), next tile prefetched into
// registers while the current one is consumed.
#include "common.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BM = 128, BN = 128, BK = 32;
constexpr int THREADS = 256;

template <bool BF16>
struct Lds;
template <>
struct Lds<true> {
  static constexpr int LD = BK + 8;  // bf16 elements per LDS row (80 B)
  typedef __bf16 T;
};
template <>
struct Lds<false> {
  static constexpr int LD = BK + 1;  // fp32 elements per LDS row
  typedef float T;
};

struct Epi {
  float alpha, beta;
  const float* bias;
  int relu;
  c2::Drop drop;
  int64_t row_base;
  const int* rowmap;  // dropout row index = row_base + (rowmap ? rowmap[row] : row)
};

// Operand tile loader: fills S[r][k] (r over BM or BN rows, k over BK) from a global
// operand stored either "row-major along k" (KCONT: X[r*ld + k]) or "k-major" (X[k*ld + r]).
template <bool KCONT, bool VEC, typename T, int LD>
struct TileLoader {
  float v[4][4];
  __device__ __forceinline__ void load(const float* __restrict__ X, int ld, int R, int K, int r0, int k0) {
    const int t = threadIdx.x;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int f = t + THREADS * q;
      int r, k;
      if (KCONT) {
        r = f >> 3;
        k = (f & 7) * 4;
      } else {
        k = f >> 5;
        r = (f & 31) * 4;
      }
      const int gr = r0 + r, gk = k0 + k;
      if (VEC) {
        bool ok = KCONT ? (gr < R && gk < K) : (gk < K && gr < R);
        float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
        if (ok) x = KCONT ? *(const float4*)(X + (long)gr * ld + gk) : *(const float4*)(X + (long)gk * ld + gr);
        v[q][0] = x.x;
        v[q][1] = x.y;
        v[q][2] = x.z;
        v[q][3] = x.w;
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int rr = KCONT ? gr : gr + i;
          const int kk = KCONT ? gk + i : gk;
          v[q][i] = (rr < R && kk < K) ? (KCONT ? X[(long)rr * ld + kk] : X[(long)kk * ld + rr]) : 0.f;
        }
      }
    }
  }
  __device__ __forceinline__ void store(T* S) const {
    const int t = threadIdx.x;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int f = t + THREADS * q;
      if (KCONT) {
        const int r = f >> 3, k = (f & 7) * 4;
#pragma unroll
        for (int i = 0; i < 4; ++i) S[r * LD + k + i] = (T)v[q][i];
      } else {
        const int k = f >> 5, r = (f & 31) * 4;
#pragma unroll
        for (int i = 0; i < 4; ++i) S[(r + i) * LD + k] = (T)v[q][i];
      }
    }
  }
};

template <bool BF16, bool TA, bool TB, bool VEC>
__global__ __launch_bounds__(THREADS) void gemm_kernel(int M, int N, int K, const float* __restrict__ A, int lda,
                                                       const float* __restrict__ B, int ldb, float* __restrict__ C,
                                                       int ldc, Epi ep, int k_per_split, int partial) {
  typedef typename Lds<BF16>::T T;
  constexpr int LD = Lds<BF16>::LD;
  __shared__ __attribute__((aligned(16))) T As[BM * LD];
  __shared__ __attribute__((aligned(16))) T Bs[BN * LD];

  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int kbeg = blockIdx.z * k_per_split;
  const int kend = min(K, kbeg + k_per_split);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = w >> 1, wn = w & 1;

  // A is "k-contiguous" when not transposed; B is k-contiguous when transposed.
  TileLoader<!TA, VEC, T, LD> la;
  TileLoader<TB, VEC, T, LD> lb;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  if (kbeg < kend) {
    la.load(A, lda, M, kend, m0, kbeg);
    lb.load(B, ldb, N, kend, n0, kbeg);
  }
  for (int k0 = kbeg; k0 < kend; k0 += BK) {
    la.store(As);
    lb.store(Bs);
    __syncthreads();
    if (k0 + BK < kend) {
      la.load(A, lda, M, kend, m0, k0 + BK);
      lb.load(B, ldb, N, kend, n0, k0 + BK);
    }
    const int r = lane & 31, h = lane >> 5;
    if constexpr (BF16) {
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) {
        bf16x8 af[2], bfr[2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
          af[i] = *(const bf16x8*)(&As[(wm * 64 + i * 32 + r) * LD + ks * 16 + 8 * h]);
#pragma unroll
        for (int j = 0; j < 2; ++j)
          bfr[j] = *(const bf16x8*)(&Bs[(wn * 64 + j * 32 + r) * LD + ks * 16 + 8 * h]);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    } else {
#pragma unroll 4
      for (int ks = 0; ks < BK / 2; ++ks) {
        float af[2], bfr[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) af[i] = As[(wm * 64 + i * 32 + r) * LD + ks * 2 + h];
#pragma unroll
        for (int j = 0; j < 2; ++j) bfr[j] = Bs[(wn * 64 + j * 32 + r) * LD + ks * 2 + h];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
    __syncthreads();
  }

  // epilogue: C/D layout col = lane&31, row = (reg&3) + 8*(reg>>2) + 4*(lane>>5)
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = n0 + wn * 64 + j * 32 + (lane & 31);
      if (col >= N) continue;
      const float bcol = (ep.bias && !partial) ? ep.bias[col] : 0.f;
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int row = m0 + wm * 64 + i * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5);
        if (row >= M) continue;
        float v = ep.alpha * acc[i][j][reg];
        if (partial) {  // split-K: this split's partial slab [M][N] (summed in split order afterwards)
          C[(long)blockIdx.z * M * N + (long)row * N + col] = v;
        } else {
          float* cp = C + (long)row * ldc + col;
          if (ep.beta != 0.f) v = fmaf(ep.beta, *cp, v);
          v += bcol;
          if (ep.relu) {
            v = fmaxf(v, 0.f);
            v *= ep.drop.mul((uint64_t)(ep.row_base + (ep.rowmap ? ep.rowmap[row] : row)) * N + col);
          }
          *cp = v;
        }
      }
    }
}

// C[r][c] = beta·C[r][c] + Σ_s part[s][r][c], s in order (deterministic split-K combine)
__global__ void splitk_sum_kernel(const float* __restrict__ part, int splits, int M, int N, float beta,
                                  float* __restrict__ C, int ldc) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)M * N) return;
  const int r = (int)(i / N), c = (int)(i % N);
  float t = 0.f;
  const long sl = (long)M * N;
  int s = 0;
  for (; s + 8 <= splits; s += 8) {  // eight slabs' loads in flight, added in split order
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = part[(s + u) * sl + i];
#pragma unroll
    for (int u = 0; u < 8; ++u) t += v[u];
  }
  for (; s < splits; ++s) t += part[s * sl + i];
  float* cp = C + (long)r * ldc + c;
  *cp = beta == 0.f ? t : fmaf(beta, *cp, t);
}

// split-K partial slabs: one scratch buffer per device, grown on demand (never inside a captured graph)
float* splitk_scratch(size_t floats) {
  static float* buf[64] = {nullptr};
  static size_t cap[64] = {0};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 64) return nullptr;
  if (cap[dev] < floats) {
    if (buf[dev]) {
      (void)hipDeviceSynchronize();
      (void)hipFree(buf[dev]);
    }
    buf[dev] = nullptr;
    cap[dev] = 0;
    if (hipMalloc((void**)&buf[dev], floats * sizeof(float)) != hipSuccess) return nullptr;
    cap[dev] = floats;
  }
  return buf[dev];
}

__global__ void scale_kernel(float* __restrict__ C, int M, int N, int ldc, float beta) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)M * N) return;
  const int r = (int)(i / N), c = (int)(i % N);
  C[(long)r * ldc + c] = beta == 0.f ? 0.f : beta * C[(long)r * ldc + c];
}

// colsum: out[n] = beta*out[n] + alpha * Σ_m X[m*ldx + n]  (bias gradients).
// Stage 1: a 64-column x CS_ROWS-row block per workgroup (4 waves interleaved over rows,
// each wave reading 256 contiguous bytes per row) → part[chunk][n]; stage 2: 16 wave groups
// per 64 columns sum the chunks, combined in a fixed order (deterministic).
constexpr int CS_ROWS = 256;
// w (may be null): per-row weights w[r·ldw] (c2dsr_wcolsum)
__global__ __launch_bounds__(256) void colsum_part_kernel(const float* __restrict__ X, int M, int N, long ldx,
                                                          float* __restrict__ part, const float* __restrict__ w = nullptr,
                                                          long ldw = 0) {
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const int chunk = blockIdx.y;
  const int r0 = chunk * CS_ROWS, r1 = min(M, r0 + CS_ROWS);
  float s0 = 0.f, s1 = 0.f;
  if (c < N) {
    int r = r0 + q;
    if (w) {
      for (; r + 4 < r1; r += 8) {
        s0 = fmaf(w[(long)r * ldw], X[(long)r * ldx + c], s0);
        s1 = fmaf(w[(long)(r + 4) * ldw], X[(long)(r + 4) * ldx + c], s1);
      }
      if (r < r1) s0 = fmaf(w[(long)r * ldw], X[(long)r * ldx + c], s0);
    } else {
      for (; r + 4 < r1; r += 8) {
        s0 += X[(long)r * ldx + c];
        s1 += X[(long)(r + 4) * ldx + c];
      }
      if (r < r1) s0 += X[(long)r * ldx + c];
    }
  }
  red[q][cl] = s0 + s1;
  __syncthreads();
  if (q == 0 && c < N) part[(long)chunk * N + c] = (red[0][cl] + red[1][cl]) + (red[2][cl] + red[3][cl]);
}

__global__ __launch_bounds__(1024) void colsum_final_kernel(const float* __restrict__ part, int chunks, int N,
                                                            float alpha, float beta, float* __restrict__ out) {
  __shared__ float red[16][64];
  const int cl = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  float t = 0.f;
  if (c < N)
    for (int k = q; k < chunks; k += 16) t += part[(long)k * N + c];
  red[q][cl] = t;
  __syncthreads();
  if (q == 0 && c < N) {
    float s = 0.f;
    for (int k = 0; k < 16; ++k) s += red[k][cl];
    out[c] = (beta == 0.f ? 0.f : beta * out[c]) + alpha * s;
  }
}

template <bool BF16, bool TA, bool TB>
void launch_t(dim3 grid, hipStream_t s, bool vec, int M, int N, int K, const float* A, int lda, const float* B, int ldb,
              float* C, int ldc, Epi ep, int kps, int partial) {
  if (vec)
    gemm_kernel<BF16, TA, TB, true><<<grid, THREADS, 0, s>>>(M, N, K, A, lda, B, ldb, C, ldc, ep, kps, partial);
  else
    gemm_kernel<BF16, TA, TB, false><<<grid, THREADS, 0, s>>>(M, N, K, A, lda, B, ldb, C, ldc, ep, kps, partial);
}

template <bool BF16>
void launch_p(int ta, int tb, dim3 grid, hipStream_t s, bool vec, int M, int N, int K, const float* A, int lda,
              const float* B, int ldb, float* C, int ldc, Epi ep, int kps, int partial) {
  if (!ta && !tb) launch_t<BF16, false, false>(grid, s, vec, M, N, K, A, lda, B, ldb, C, ldc, ep, kps, partial);
  if (!ta && tb) launch_t<BF16, false, true>(grid, s, vec, M, N, K, A, lda, B, ldb, C, ldc, ep, kps, partial);
  if (ta && !tb) launch_t<BF16, true, false>(grid, s, vec, M, N, K, A, lda, B, ldb, C, ldc, ep, kps, partial);
  if (ta && tb) launch_t<BF16, true, true>(grid, s, vec, M, N, K, A, lda, B, ldb, C, ldc, ep, kps, partial);
}

inline bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

// precision: 0 = exact fp32 MFMA, 1 = bf16 MFMA (fp32 accumulate).
// split_k: 0 = auto (split the K axis when the output has too few tiles), 1 = none, >1 = given.
// epilogue 1 = relu then dropout(p) with index (row_base+row)*N + col.
C2_API int c2dsr_gemm(int transA, int transB, int M, int N, int K, const float* A, int lda, const float* B, int ldb,
                      float* C, int ldc, float alpha, float beta, const float* bias, int epilogue, uint32_t k0,
                      uint32_t k1, float p, int64_t row_base, const int* rowmap, int precision, int split_k,
                      void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (M <= 0 || N <= 0) return 0;
  if (K <= 0) {
    // C = beta*C + bias
    Epi ep{0.f, beta, bias, 0, c2::make_drop(0, 0, 0.f), 0, nullptr};
    (void)ep;
    scale_kernel<<<c2::ceil_div((long)M * N, 256), 256, 0, s>>>(C, M, N, ldc, beta);
    if (bias) return (int)hipErrorInvalidValue;
    C2_CHECK_LAUNCH();
    return 0;
  }
  const int tiles = c2::ceil_div(M, BM) * c2::ceil_div(N, BN);
  int splits = split_k;
  if (splits <= 0) {
    splits = 1;
    const int ktiles = c2::ceil_div(K, BK);
    while (tiles * splits < 512 && ktiles / (splits * 2) >= 4) splits *= 2;
  }
  if (splits > 1 && (bias || epilogue)) splits = 1;
  int kps = c2::ceil_div(K, splits);
  kps = c2::ceil_div(kps, BK) * BK;
  splits = c2::ceil_div(K, kps);
  // float4 path: contiguous dims multiple of 4 and 16-byte aligned bases / strides
  const bool a_ok = al16(A) && lda % 4 == 0 && (transA ? M % 4 == 0 : K % 4 == 0);
  const bool b_ok = al16(B) && ldb % 4 == 0 && (transB ? K % 4 == 0 : N % 4 == 0);
  const bool vec = a_ok && b_ok;
  Epi ep{alpha, beta, bias, epilogue == 1, c2::make_drop(k0, k1, epilogue == 1 ? p : 0.f), row_base, rowmap};
  // split-K: each split writes its partial product to a slab, summed in split order afterwards
  // (deterministic: no float atomics)
  int partial = 0;
  float* out = C;
  if (splits > 1) {
    out = splitk_scratch((size_t)splits * M * N);
    if (!out) return (int)hipErrorOutOfMemory;
    partial = 1;
  }
  dim3 grid(c2::ceil_div(N, BN), c2::ceil_div(M, BM), splits);
  if (precision == 1)
    launch_p<true>(transA, transB, grid, s, vec, M, N, K, A, lda, B, ldb, out, ldc, ep, kps, partial);
  else
    launch_p<false>(transA, transB, grid, s, vec, M, N, K, A, lda, B, ldb, out, ldc, ep, kps, partial);
  if (partial)
    splitk_sum_kernel<<<c2::ceil_div((long)M * N, 256), 256, 0, s>>>(out, splits, M, N, beta, C, ldc);
  C2_CHECK_LAUNCH();
  return 0;
}

C2_API size_t c2dsr_colsum_workspace(int M, int N) { return (size_t)c2::ceil_div(M, CS_ROWS) * (size_t)N * 4 + 256; }

C2_API int c2dsr_wcolsum(const float* X, int M, int N, int ldx, const float* w, long ldw, float alpha, float beta,
                         float* out, void* workspace, void* stream);
C2_API int c2dsr_colsum(const float* X, int M, int N, int ldx, float alpha, float beta, float* out, void* workspace,
                        void* stream) {
  return c2dsr_wcolsum(X, M, N, ldx, nullptr, 0, alpha, beta, out, workspace, stream);
}

// out[n] = beta·out[n] + alpha·Σ_m w[m·ldw]·X[m·ldx + n]  (w null: 1) — the classifier_pad weight gradient
// (a 1 × d product over the 2·B·R stacked rows), without a split-K GEMM
C2_API int c2dsr_wcolsum(const float* X, int M, int N, int ldx, const float* w, long ldw, float alpha, float beta,
                         float* out, void* workspace, void* stream) {
  if (N <= 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const int chunks = c2::ceil_div(M, CS_ROWS);
  float* part = (float*)workspace;
  if (chunks > 0) {
    dim3 g1(c2::ceil_div(N, 64), chunks);
    colsum_part_kernel<<<g1, 256, 0, s>>>(X, M, N, ldx, part, w, ldw);
  }
  colsum_final_kernel<<<c2::ceil_div(N, 64), 1024, 0, s>>>(part, chunks, N, alpha, beta, out);
  C2_CHECK_LAUNCH();
  return 0;
}
