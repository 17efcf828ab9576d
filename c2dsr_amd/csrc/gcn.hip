// K1: item-graph propagation (GCN) — CSR SpMM with fused dropout and fused mean.
//
// Replaces models/encoders.py:42-48 (F.dropout + torch.spmm + stack/mean) as called
// by models/C2DSR.py:59-62, and its autograd backward.
//
//   Y[i] = alpha * Σ_e val[e] * (Min ⊙ X)[col[e]]   (mask on the gathered row:  forward)
//   Y[i] = alpha * Mout_i ⊙ Σ_e val[e] * X[col[e]]  (mask on the output row: backward, A^T CSR)
//        + (beta + (i != pad_row ? delta : 0)) * Z[i] + gamma * Y[i]
//   Y2[i] = Σ_e ...   (raw propagation, optional: next GCN layer's input)
//
// Layout: one row of d fp32 per "row group" of LPR lanes, each lane a float4
// column slice (d <= 4*LPR per pass, looped for larger d).  Rows are dealt to
// row groups in order; the gather of neighbour rows is the HBM/Infinity-cache
// bound part (bytes per row: (2 + nnz_i) * d * 4 + 8 nnz_i).
#include "common.h"

namespace {

template <int LPR, bool MASK_OUT>
__global__ __launch_bounds__(256) void spmm_kernel(const int* __restrict__ rowptr, const int* __restrict__ col,
                                                   const float* __restrict__ val, int n_rows, int d,
                                                   const float* __restrict__ X, c2::Drop drop, float alpha,
                                                   const float* __restrict__ Z, float beta, float delta,
                                                   int pad_row, float gamma, float* __restrict__ Y,
                                                   float* __restrict__ Y2) {
  constexpr int GROUPS = 256 / LPR;
  const int g = threadIdx.x / LPR;
  const int lane = threadIdx.x % LPR;
  const long row = (long)blockIdx.x * GROUPS + g;
  if (row >= n_rows) return;
  const int e0 = rowptr[row], e1 = rowptr[row + 1];
  for (int c = lane * 4; c < d; c += LPR * 4) {
    float4 acc = c2::f4(0.f);
    int e = e0;
    for (; e + 3 < e1; e += 4) {
      int j0 = col[e], j1 = col[e + 1], j2 = col[e + 2], j3 = col[e + 3];
      float v0 = val[e], v1 = val[e + 1], v2 = val[e + 2], v3 = val[e + 3];
      float4 x0 = *(const float4*)(X + (long)j0 * d + c);
      float4 x1 = *(const float4*)(X + (long)j1 * d + c);
      float4 x2 = *(const float4*)(X + (long)j2 * d + c);
      float4 x3 = *(const float4*)(X + (long)j3 * d + c);
      if (!MASK_OUT && drop.active()) {
        const uint64_t b0 = (uint64_t)j0 * d + c, b1 = (uint64_t)j1 * d + c;
        const uint64_t b2 = (uint64_t)j2 * d + c, b3 = (uint64_t)j3 * d + c;
        x0 = x0 * make_float4(drop.mul(b0), drop.mul(b0 + 1), drop.mul(b0 + 2), drop.mul(b0 + 3));
        x1 = x1 * make_float4(drop.mul(b1), drop.mul(b1 + 1), drop.mul(b1 + 2), drop.mul(b1 + 3));
        x2 = x2 * make_float4(drop.mul(b2), drop.mul(b2 + 1), drop.mul(b2 + 2), drop.mul(b2 + 3));
        x3 = x3 * make_float4(drop.mul(b3), drop.mul(b3 + 1), drop.mul(b3 + 2), drop.mul(b3 + 3));
      }
      acc = c2::fma4(v0, x0, acc);
      acc = c2::fma4(v1, x1, acc);
      acc = c2::fma4(v2, x2, acc);
      acc = c2::fma4(v3, x3, acc);
    }
    for (; e < e1; ++e) {
      int j = col[e];
      float4 x = *(const float4*)(X + (long)j * d + c);
      if (!MASK_OUT && drop.active()) {
        const uint64_t b = (uint64_t)j * d + c;
        x = x * make_float4(drop.mul(b), drop.mul(b + 1), drop.mul(b + 2), drop.mul(b + 3));
      }
      acc = c2::fma4(val[e], x, acc);
    }
    if (MASK_OUT && drop.active()) {
      const uint64_t b = (uint64_t)row * d + c;
      acc = acc * make_float4(drop.mul(b), drop.mul(b + 1), drop.mul(b + 2), drop.mul(b + 3));
    }
    if (Y2) *(float4*)(Y2 + row * d + c) = acc;
    float4 y = alpha * acc;
    if (Z) {
      const float zc = beta + (row != pad_row ? delta : 0.f);
      y = c2::fma4(zc, *(const float4*)(Z + row * d + c), y);
    }
    if (gamma != 0.f) y = c2::fma4(gamma, *(const float4*)(Y + row * d + c), y);
    *(float4*)(Y + row * d + c) = y;
  }
}

template <bool MASK_OUT>
int launch_spmm(const int* rowptr, const int* col, const float* val, int n_rows, int d, const float* X, c2::Drop dr,
                float alpha, const float* Z, float beta, float delta, int pad_row, float gamma, float* Y, float* Y2,
                hipStream_t s) {
  if (d % 4) return (int)hipErrorInvalidValue;
  int lpr = d / 4 >= 64 ? 64 : (d / 4 >= 32 ? 32 : (d / 4 >= 16 ? 16 : (d / 4 >= 8 ? 8 : 4)));
  int groups = 256 / lpr;
  dim3 grid(c2::ceil_div(n_rows, groups));
  switch (lpr) {
    case 64: spmm_kernel<64, MASK_OUT><<<grid, 256, 0, s>>>(rowptr, col, val, n_rows, d, X, dr, alpha, Z, beta, delta, pad_row, gamma, Y, Y2); break;
    case 32: spmm_kernel<32, MASK_OUT><<<grid, 256, 0, s>>>(rowptr, col, val, n_rows, d, X, dr, alpha, Z, beta, delta, pad_row, gamma, Y, Y2); break;
    case 16: spmm_kernel<16, MASK_OUT><<<grid, 256, 0, s>>>(rowptr, col, val, n_rows, d, X, dr, alpha, Z, beta, delta, pad_row, gamma, Y, Y2); break;
    case 8: spmm_kernel<8, MASK_OUT><<<grid, 256, 0, s>>>(rowptr, col, val, n_rows, d, X, dr, alpha, Z, beta, delta, pad_row, gamma, Y, Y2); break;
    default: spmm_kernel<4, MASK_OUT><<<grid, 256, 0, s>>>(rowptr, col, val, n_rows, d, X, dr, alpha, Z, beta, delta, pad_row, gamma, Y, Y2); break;
  }
  C2_CHECK_LAUNCH();
  return 0;
}

}  // namespace

C2_API int c2dsr_gcn_spmm(const int* rowptr, const int* col, const float* val, int n_rows, int d, const float* X,
                          uint32_t k0, uint32_t k1, float p, int mask_on_output, float alpha, const float* Z,
                          float beta, float delta, int pad_row, float gamma, float* Y, float* Y2, void* stream) {
  c2::Drop dr = c2::make_drop(k0, k1, p);
  hipStream_t s = (hipStream_t)stream;
  if (mask_on_output)
    return launch_spmm<true>(rowptr, col, val, n_rows, d, X, dr, alpha, Z, beta, delta, pad_row, gamma, Y, Y2, s);
  return launch_spmm<false>(rowptr, col, val, n_rows, d, X, dr, alpha, Z, beta, delta, pad_row, gamma, Y, Y2, s);
}
