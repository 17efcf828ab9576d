// Residual + dropout + LayerNorm (eps 1e-8) forward/backward, and the plain
// residual/dropout element-wise ops used by the pre-norm variant.
//
// Replaces TransformerEncoderLayer's `norm1(x + dropout1(sa))`, `norm2(x + dropout2(ff))`
// (post-norm, models/encoders.py:23-27 → torch transformer.py) and the final
// `encoder.norm` (Q16: two LayerNorms back to back), plus their backward.
// One row per group of LPR lanes, float4 per lane, the row kept in registers.
#include "common.h"

namespace {

constexpr int MAXC = 4;  // float4 chunks per lane → d <= 16*LPR

// NC = float4 chunks per lane (a compile-time count, so the row lives in exactly NC float4s)
template <int LPR, int NC>
__global__ __launch_bounds__(256) void add_ln_fwd_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                         int rows, int d, c2::Drop drop, int64_t idx_base,
                                                         const int* __restrict__ rowmap,
                                                         const float* __restrict__ gw, const float* __restrict__ gb,
                                                         float eps, float* __restrict__ xsave, float* __restrict__ y,
                                                         float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  constexpr int GROUPS = 256 / LPR;
  const int g = threadIdx.x / LPR, lane = threadIdx.x % LPR;
  const long r = (long)blockIdx.x * GROUPS + g;
  if (r >= rows) return;
  float4 x[NC];
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < NC; ++q) {
    const int c = (lane + q * LPR) * 4;
    x[q] = c2::f4(0.f);
    if (c < d) {
      float4 v = c2::f4(0.f);
      if (a) v = *(const float4*)(a + r * d + c);
      if (b) {
        float4 u = *(const float4*)(b + r * d + c);
        if (drop.active()) {
          const uint64_t bi = (uint64_t)(idx_base + (rowmap ? rowmap[r] : r)) * d + c;
          u = u * drop.mul4(bi);
        }
        v = v + u;
      }
      x[q] = v;
      if (xsave) *(float4*)(xsave + r * d + c) = v;
      s += v.x + v.y + v.z + v.w;
    }
  }
  const float mean = c2::group_sum<LPR>(s) / d;
  float ss = 0.f;
#pragma unroll
  for (int q = 0; q < NC; ++q) {
    const int c = (lane + q * LPR) * 4;
    if (c < d) {
      const float4 t = x[q] + c2::f4(-mean);
      ss += t.x * t.x + t.y * t.y + t.z * t.z + t.w * t.w;
    }
  }
  const float var = c2::group_sum<LPR>(ss) / d;
  const float rstd = 1.0f / sqrtf(var + eps);
#pragma unroll
  for (int q = 0; q < NC; ++q) {
    const int c = (lane + q * LPR) * 4;
    if (c < d) {
      const float4 w4 = *(const float4*)(gw + c), b4 = *(const float4*)(gb + c);
      float4 o;
      o.x = (x[q].x - mean) * rstd * w4.x + b4.x;
      o.y = (x[q].y - mean) * rstd * w4.y + b4.y;
      o.z = (x[q].z - mean) * rstd * w4.z + b4.z;
      o.w = (x[q].w - mean) * rstd * w4.w + b4.w;
      *(float4*)(y + r * d + c) = o;
    }
  }
  if (lane == 0) {
    mean_out[r] = mean;
    rstd_out[r] = rstd;
  }
}

// backward; grid-stride over rows with a fixed grid so dgamma/dbeta partials are per block.
// Each lane group works on RB rows per step (all their loads issued before the reductions).
template <int LPR, int NC>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const float* __restrict__ x, const float* __restrict__ mean_in,
                                                     const float* __restrict__ rstd_in, const float* __restrict__ gw,
                                                     const float* __restrict__ dy, int rows, int d,
                                                     float* __restrict__ dx, int dx_accumulate,
                                                     float* __restrict__ db_out, c2::Drop drop, int64_t idx_base,
                                                     const int* __restrict__ rowmap, float* __restrict__ part) {
  constexpr int GROUPS = 256 / LPR;
  constexpr int RB = 2;
  const int g = threadIdx.x / LPR, lane = threadIdx.x % LPR;
  float4 pg[NC], pb[NC], w4[NC];
#pragma unroll
  for (int q = 0; q < NC; ++q) {
    pg[q] = pb[q] = c2::f4(0.f);
    const int c = (lane + q * LPR) * 4;
    w4[q] = c < d ? *(const float4*)(gw + c) : c2::f4(0.f);
  }
  const long stride = (long)gridDim.x * GROUPS;
  for (long r0 = (long)blockIdx.x * GROUPS + g; r0 < rows; r0 += RB * stride) {
    float4 xv[RB][NC], dv[RB][NC];
    float mean[RB], rstd[RB];
#pragma unroll
    for (int k = 0; k < RB; ++k) {
      const long r = r0 + k * stride;
      const bool ok = r < rows;
      mean[k] = ok ? mean_in[r] : 0.f;
      rstd[k] = ok ? rstd_in[r] : 0.f;
#pragma unroll
      for (int q = 0; q < NC; ++q) {
        const int c = (lane + q * LPR) * 4;
        const bool in = ok && c < d;
        xv[k][q] = in ? *(const float4*)(x + r * d + c) : c2::f4(0.f);
        dv[k][q] = in ? *(const float4*)(dy + r * d + c) : c2::f4(0.f);
      }
    }
#pragma unroll
    for (int k = 0; k < RB; ++k) {
      const long r = r0 + k * stride;
      if (r >= rows) break;  // uniform over the group
      float4 xh[NC], gg[NC];
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int q = 0; q < NC; ++q) {
        xh[q] = make_float4((xv[k][q].x - mean[k]) * rstd[k], (xv[k][q].y - mean[k]) * rstd[k],
                            (xv[k][q].z - mean[k]) * rstd[k], (xv[k][q].w - mean[k]) * rstd[k]);
        gg[q] = dv[k][q] * w4[q];
        s1 += gg[q].x + gg[q].y + gg[q].z + gg[q].w;
        s2 += gg[q].x * xh[q].x + gg[q].y * xh[q].y + gg[q].z * xh[q].z + gg[q].w * xh[q].w;
        pg[q] = pg[q] + dv[k][q] * xh[q];
        pb[q] = pb[q] + dv[k][q];
      }
      const float m1 = c2::group_sum<LPR>(s1) / d, m2 = c2::group_sum<LPR>(s2) / d;
#pragma unroll
      for (int q = 0; q < NC; ++q) {
        const int c = (lane + q * LPR) * 4;
        if (c < d) {
          float4 o;
          o.x = rstd[k] * (gg[q].x - m1 - xh[q].x * m2);
          o.y = rstd[k] * (gg[q].y - m1 - xh[q].y * m2);
          o.z = rstd[k] * (gg[q].z - m1 - xh[q].z * m2);
          o.w = rstd[k] * (gg[q].w - m1 - xh[q].w * m2);
          if (dx) {
            float4 prev = dx_accumulate ? *(const float4*)(dx + r * d + c) : c2::f4(0.f);
            *(float4*)(dx + r * d + c) = prev + o;
          }
          if (db_out) {
            if (drop.active()) {
              const uint64_t bi = (uint64_t)(idx_base + (rowmap ? rowmap[r] : r)) * d + c;
              o = o * drop.mul4(bi);
            }
            *(float4*)(db_out + r * d + c) = o;
          }
        }
      }
    }
  }
  // block reduce of the per-group partials → part[block][2][d]
  __shared__ float red[256 * 4];
#pragma unroll
  for (int q = 0; q < NC; ++q) {
    const int c = (lane + q * LPR) * 4;
    for (int which = 0; which < 2; ++which) {
      const float4 v = which ? pb[q] : pg[q];
      // each group writes its float4; then groups are summed by the first group
      __syncthreads();
      *(float4*)(&red[threadIdx.x * 4]) = v;
      __syncthreads();
      if (g == 0 && c < d) {
        float4 t = c2::f4(0.f);
        for (int gg2 = 0; gg2 < GROUPS; ++gg2) t = t + *(const float4*)(&red[(gg2 * LPR + lane) * 4]);
        *(float4*)(part + ((long)blockIdx.x * 2 + which) * d + c) = t;
      }
    }
  }
}

// dgw/dgb += Σ_blocks part: 64 columns x 16 block-groups per workgroup, fixed-order combine (bx: the workgroup's
// column block)
__device__ __forceinline__ void reduce_parts_body(const float* __restrict__ part, int nblk, int d,
                                                  float* __restrict__ dgw, float* __restrict__ dgb, int bx) {
  __shared__ float red[16][64];
  const int cl = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int c = bx * 64 + cl;
  float s = 0.f;
  if (c < 2 * d) {
    const int which = c / d, cc = c % d;
    const float* pp = part + (long)which * d + cc;
    const long st = 2l * d;
    float s1 = 0.f, s2 = 0.f, s3 = 0.f, s4 = 0.f, s5 = 0.f, s6 = 0.f, s7 = 0.f;
    int b = q;
    for (; b + 7 * 16 < nblk; b += 8 * 16) {  // eight independent loads in flight per lane
      s += pp[b * st];
      s1 += pp[(b + 16) * st];
      s2 += pp[(b + 32) * st];
      s3 += pp[(b + 48) * st];
      s4 += pp[(b + 64) * st];
      s5 += pp[(b + 80) * st];
      s6 += pp[(b + 96) * st];
      s7 += pp[(b + 112) * st];
    }
    for (; b < nblk; b += 16) s += pp[b * st];
    s = ((s + s1) + (s2 + s3)) + ((s4 + s5) + (s6 + s7));
  }
  red[q][cl] = s;
  __syncthreads();
  if (q == 0 && c < 2 * d) {
    float t = 0.f;
    for (int k = 0; k < 16; ++k) t += red[k][cl];
    const int which = c / d, cc = c % d;
    float* o = which ? dgb : dgw;
    if (o) o[cc] += t;
  }
}
__global__ __launch_bounds__(1024) void reduce_parts_kernel(const float* __restrict__ part, int nblk, int d,
                                                            float* __restrict__ dgw, float* __restrict__ dgb) {
  reduce_parts_body(part, nblk, d, dgw, dgb, blockIdx.x);
}

// ---- Two LayerNorms back to back (the last post-norm layer's norm2 and the encoder's final norm, Q16):
//   x = a + drop(b),  x2 = LN2(x)·w2 + b2,  y = LNF(x2)·wF + bF
// in one pass; x2 is never stored (the backward recomputes it from x and LN2's statistics).
template <int LPR, int NC>
__global__ __launch_bounds__(256) void add_ln2_fwd_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                          int rows, int d, c2::Drop drop, int64_t idx_base,
                                                          const int* __restrict__ rowmap, const float* __restrict__ w2,
                                                          const float* __restrict__ b2, float eps2,
                                                          const float* __restrict__ wF, const float* __restrict__ bF,
                                                          float epsF, float* __restrict__ xsave, float* __restrict__ y,
                                                          float* __restrict__ st) {
  constexpr int GROUPS = 256 / LPR;
  const int g = threadIdx.x / LPR, lane = threadIdx.x % LPR;
  const long r = (long)blockIdx.x * GROUPS + g;
  if (r >= rows) return;
  float4 x[NC];
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < NC; ++q) {
    const int c = (lane + q * LPR) * 4;
    x[q] = c2::f4(0.f);
    if (c < d) {
      float4 u = *(const float4*)(b + r * d + c);
      if (drop.active()) u = u * drop.mul4((uint64_t)(idx_base + (rowmap ? rowmap[r] : r)) * d + c);
      const float4 v = *(const float4*)(a + r * d + c) + u;
      x[q] = v;
      *(float4*)(xsave + r * d + c) = v;
      s += v.x + v.y + v.z + v.w;
    }
  }
  float mean[2], rstd[2];
  const float* ws[2] = {w2, wF};
  const float* bs[2] = {b2, bF};
  const float eps[2] = {eps2, epsF};
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    if (k) {
      s = 0.f;
#pragma unroll
      for (int q = 0; q < NC; ++q) {
        const int c = (lane + q * LPR) * 4;
        if (c < d) s += x[q].x + x[q].y + x[q].z + x[q].w;
      }
    }
    mean[k] = c2::group_sum<LPR>(s) / d;
    float ss = 0.f;
#pragma unroll
    for (int q = 0; q < NC; ++q) {
      const int c = (lane + q * LPR) * 4;
      if (c < d) {
        const float4 t = x[q] + c2::f4(-mean[k]);
        ss += t.x * t.x + t.y * t.y + t.z * t.z + t.w * t.w;
      }
    }
    rstd[k] = 1.0f / sqrtf(c2::group_sum<LPR>(ss) / d + eps[k]);
#pragma unroll
    for (int q = 0; q < NC; ++q) {
      const int c = (lane + q * LPR) * 4;
      if (c < d) {
        const float4 w4 = *(const float4*)(ws[k] + c), b4 = *(const float4*)(bs[k] + c);
        float4 o;
        o.x = (x[q].x - mean[k]) * rstd[k] * w4.x + b4.x;
        o.y = (x[q].y - mean[k]) * rstd[k] * w4.y + b4.y;
        o.z = (x[q].z - mean[k]) * rstd[k] * w4.z + b4.z;
        o.w = (x[q].w - mean[k]) * rstd[k] * w4.w + b4.w;
        x[q] = o;
      }
    }
  }
#pragma unroll
  for (int q = 0; q < NC; ++q) {
    const int c = (lane + q * LPR) * 4;
    if (c < d) *(float4*)(y + r * d + c) = x[q];
  }
  if (lane == 0) {
    st[r] = mean[0];
    st[rows + r] = rstd[0];
    st[2l * rows + r] = mean[1];
    st[3l * rows + r] = rstd[1];
  }
}

// backward of add_ln2_fwd: dxF → dx2 (final norm) → dx (norm2) in registers; dx = the residual gradient,
// db_out = dx ⊙ drop mask; the four weight/bias gradients as per-block partials part[blk][4][d]
// (norm2 weight, norm2 bias, final weight, final bias).  x2 is recomputed from x and LN2's statistics.
template <int LPR, int NC>
__global__ __launch_bounds__(256) void ln2_bwd_kernel(const float* __restrict__ x, const float* __restrict__ st,
                                                      const float* __restrict__ w2, const float* __restrict__ b2,
                                                      const float* __restrict__ wF, const float* __restrict__ dy,
                                                      int rows, int d, float* __restrict__ dx,
                                                      float* __restrict__ db_out, c2::Drop drop, int64_t idx_base,
                                                      const int* __restrict__ rowmap, float* __restrict__ part) {
  constexpr int GROUPS = 256 / LPR;
  const int g = threadIdx.x / LPR, lane = threadIdx.x % LPR;
  float4 p2w[NC], p2b[NC], pFw[NC], pFb[NC], w24[NC], b24[NC], wF4[NC];
#pragma unroll
  for (int q = 0; q < NC; ++q) {
    p2w[q] = p2b[q] = pFw[q] = pFb[q] = c2::f4(0.f);
    const int c = (lane + q * LPR) * 4;
    w24[q] = c < d ? *(const float4*)(w2 + c) : c2::f4(0.f);
    b24[q] = c < d ? *(const float4*)(b2 + c) : c2::f4(0.f);
    wF4[q] = c < d ? *(const float4*)(wF + c) : c2::f4(0.f);
  }
  const long stride = (long)gridDim.x * GROUPS;
  constexpr int RB = 2;  // rows per step per lane group: both rows' loads issued before the reductions
  for (long r0 = (long)blockIdx.x * GROUPS + g; r0 < rows; r0 += RB * stride) {
    float4 xin[RB][NC], din[RB][NC];
    float stv[RB][4];
#pragma unroll
    for (int k = 0; k < RB; ++k) {
      const long rk = r0 + k * stride;
      const bool ok = rk < rows;
#pragma unroll
      for (int j = 0; j < 4; ++j) stv[k][j] = ok ? st[j * (long)rows + rk] : 0.f;
#pragma unroll
      for (int q = 0; q < NC; ++q) {
        const int c = (lane + q * LPR) * 4;
        const bool in = ok && c < d;
        xin[k][q] = in ? *(const float4*)(x + rk * d + c) : c2::f4(0.f);
        din[k][q] = in ? *(const float4*)(dy + rk * d + c) : c2::f4(0.f);
      }
    }
#pragma unroll
    for (int k = 0; k < RB; ++k) {
    const long r = r0 + k * stride;
    if (r >= rows) break;  // uniform over the group
    const float m2 = stv[k][0], r2 = stv[k][1], mF = stv[k][2], rF = stv[k][3];
    float4 xh2[NC], xhF[NC], gv[NC], dv[NC];
#pragma unroll
    for (int q = 0; q < NC; ++q) {
      const float4 xv = xin[k][q];
      dv[q] = din[k][q];
      xh2[q] = make_float4((xv.x - m2) * r2, (xv.y - m2) * r2, (xv.z - m2) * r2, (xv.w - m2) * r2);
      // x2 exactly as the forward computed it: (x - m2)·r2·w2 + b2
      const float4 x2 = make_float4((xv.x - m2) * r2 * w24[q].x + b24[q].x, (xv.y - m2) * r2 * w24[q].y + b24[q].y,
                                    (xv.z - m2) * r2 * w24[q].z + b24[q].z, (xv.w - m2) * r2 * w24[q].w + b24[q].w);
      xhF[q] = make_float4((x2.x - mF) * rF, (x2.y - mF) * rF, (x2.z - mF) * rF, (x2.w - mF) * rF);
    }
    // final norm: dx2 = rF·(g − mean(g) − x̂F·mean(g·x̂F)),  g = dy·wF
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int q = 0; q < NC; ++q) {
      gv[q] = dv[q] * wF4[q];
      s1 += gv[q].x + gv[q].y + gv[q].z + gv[q].w;
      s2 += gv[q].x * xhF[q].x + gv[q].y * xhF[q].y + gv[q].z * xhF[q].z + gv[q].w * xhF[q].w;
      pFw[q] = pFw[q] + dv[q] * xhF[q];
      pFb[q] = pFb[q] + dv[q];
    }
    float a1 = c2::group_sum<LPR>(s1) / d, a2 = c2::group_sum<LPR>(s2) / d;
#pragma unroll
    for (int q = 0; q < NC; ++q)
      dv[q] = make_float4(rF * (gv[q].x - a1 - xhF[q].x * a2), rF * (gv[q].y - a1 - xhF[q].y * a2),
                          rF * (gv[q].z - a1 - xhF[q].z * a2), rF * (gv[q].w - a1 - xhF[q].w * a2));
    // norm2 with dy2 = dx2
    s1 = s2 = 0.f;
#pragma unroll
    for (int q = 0; q < NC; ++q) {
      gv[q] = dv[q] * w24[q];
      s1 += gv[q].x + gv[q].y + gv[q].z + gv[q].w;
      s2 += gv[q].x * xh2[q].x + gv[q].y * xh2[q].y + gv[q].z * xh2[q].z + gv[q].w * xh2[q].w;
      p2w[q] = p2w[q] + dv[q] * xh2[q];
      p2b[q] = p2b[q] + dv[q];
    }
    a1 = c2::group_sum<LPR>(s1) / d;
    a2 = c2::group_sum<LPR>(s2) / d;
#pragma unroll
    for (int q = 0; q < NC; ++q) {
      const int c = (lane + q * LPR) * 4;
      if (c < d) {
        float4 o = make_float4(r2 * (gv[q].x - a1 - xh2[q].x * a2), r2 * (gv[q].y - a1 - xh2[q].y * a2),
                               r2 * (gv[q].z - a1 - xh2[q].z * a2), r2 * (gv[q].w - a1 - xh2[q].w * a2));
        *(float4*)(dx + r * d + c) = o;
        if (drop.active()) o = o * drop.mul4((uint64_t)(idx_base + (rowmap ? rowmap[r] : r)) * d + c);
        *(float4*)(db_out + r * d + c) = o;
      }
    }
    }
  }
  // block reduce of the per-group partials → part[block][4][d]
  __shared__ float red[256 * 4];
#pragma unroll
  for (int q = 0; q < NC; ++q) {
    const int c = (lane + q * LPR) * 4;
    for (int which = 0; which < 4; ++which) {
      const float4 v = which == 0 ? p2w[q] : which == 1 ? p2b[q] : which == 2 ? pFw[q] : pFb[q];
      __syncthreads();
      *(float4*)(&red[threadIdx.x * 4]) = v;
      __syncthreads();
      if (g == 0 && c < d) {
        float4 t = c2::f4(0.f);
        for (int gg2 = 0; gg2 < GROUPS; ++gg2) t = t + *(const float4*)(&red[(gg2 * LPR + lane) * 4]);
        *(float4*)(part + ((long)blockIdx.x * 4 + which) * d + c) = t;
      }
    }
  }
}

// out_k[c] += Σ_blocks part[blk][k][c] for k < 4 (null outputs skipped): as reduce_parts_kernel over 4 sets
__device__ __forceinline__ void reduce_parts4_body(const float* __restrict__ part, int nblk, int d,
                                                   float* __restrict__ o0, float* __restrict__ o1,
                                                   float* __restrict__ o2, float* __restrict__ o3, int bx) {
  __shared__ float red[16][64];
  const int cl = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int c = bx * 64 + cl;
  float s = 0.f;
  if (c < 4 * d) {
    const float* pp = part + c;
    const long st = 4l * d;
    float s1 = 0.f, s2 = 0.f, s3 = 0.f;
    int b = q;
    for (; b + 3 * 16 < nblk; b += 4 * 16) {
      s += pp[b * st];
      s1 += pp[(b + 16) * st];
      s2 += pp[(b + 32) * st];
      s3 += pp[(b + 48) * st];
    }
    for (; b < nblk; b += 16) s += pp[b * st];
    s = (s + s1) + (s2 + s3);
  }
  red[q][cl] = s;
  __syncthreads();
  if (q == 0 && c < 4 * d) {
    float t = 0.f;
    for (int k = 0; k < 16; ++k) t += red[k][cl];
    const int which = c / d, cc = c % d;
    float* o = which == 0 ? o0 : which == 1 ? o1 : which == 2 ? o2 : o3;
    if (o) o[cc] += t;
  }
}
__global__ __launch_bounds__(1024) void reduce_parts4_kernel(const float* __restrict__ part, int nblk, int d,
                                                             float* __restrict__ o0, float* __restrict__ o1,
                                                             float* __restrict__ o2, float* __restrict__ o3) {
  reduce_parts4_body(part, nblk, d, o0, o1, o2, o3, blockIdx.x);
}
// both reductions of an encoder layer's two LayerNorm backwards in one launch (c2dsr_ln_reduce2): blocks
// [0, nb4) the four sets of c2dsr_ln2_bwd's partials, the rest the two of c2dsr_ln_bwd's — each block the same sums
__global__ __launch_bounds__(1024) void ln_reduce2_kernel(const float* __restrict__ part2, int nblk2,
                                                          const float* __restrict__ part1, int nblk1, int d, int nb4,
                                                          float* __restrict__ o0, float* __restrict__ o1,
                                                          float* __restrict__ o2, float* __restrict__ o3,
                                                          float* __restrict__ w1, float* __restrict__ b1) {
  if ((int)blockIdx.x < nb4)
    reduce_parts4_body(part2, nblk2, d, o0, o1, o2, o3, blockIdx.x);
  else
    reduce_parts_body(part1, nblk1, d, w1, b1, (int)blockIdx.x - nb4);
}

__global__ void add_drop_kernel(const float* __restrict__ a, const float* __restrict__ b, long n4, int d,
                                c2::Drop drop, int64_t idx_base, float* __restrict__ y) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  float4 u = ((const float4*)b)[i];
  if (drop.active()) {
    const uint64_t bi = (uint64_t)idx_base * d + (uint64_t)i * 4;
    u = u * drop.mul4(bi);
  }
  if (a) u = u + ((const float4*)a)[i];
  ((float4*)y)[i] = u;
}

// dx = (y > 0) ? dy * scale : 0   — backward of drop(relu(.)) given its output y
__global__ void relu_drop_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ y, long n, float scale,
                                     float* __restrict__ dx) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  dx[i] = y[i] > 0.f ? dy[i] * scale : 0.f;
}

int lpr_for(int d) {
  // one float4 per lane up to d = 256, then up to MAXC float4 per lane (d <= 1024)
  int l = 4;
  while (l < d / 4 && l < 64) l *= 2;
  return l;
}

#ifndef LN_BWD_BLOCKS_CFG
#define LN_BWD_BLOCKS_CFG 1024
#endif
constexpr int LN_BWD_BLOCKS = LN_BWD_BLOCKS_CFG;  // grid-stride over rows; 1024: half the partials of 2048 (LN bwd + reduce 88 -> 77 us per pass)

}  // namespace

C2_API size_t c2dsr_ln_bwd_workspace(int d) { return (size_t)LN_BWD_BLOCKS * 2 * d * 4; }

// y = LN(a + drop(b)) * w + bias; a or b may be null.  xsave (LN input) optional.
C2_API int c2dsr_add_ln_fwd(const float* a, const float* b, int rows, int d, uint32_t k0, uint32_t k1, float p,
                            int64_t idx_base, const int* rowmap, const float* w, const float* bias, float eps,
                            float* xsave, float* y, float* mean, float* rstd, void* stream) {
  if (d % 4 || d > 1024) return (int)hipErrorInvalidValue;
  if (rows == 0) return 0;
  c2::Drop dr = c2::make_drop(k0, k1, p);
  hipStream_t s = (hipStream_t)stream;
  const int lpr = lpr_for(d);
  dim3 grid(c2::ceil_div(rows, 256 / lpr));
#define C2_LN(L, NC) add_ln_fwd_kernel<L, NC><<<grid, 256, 0, s>>>(a, b, rows, d, dr, idx_base, rowmap, w, bias, eps, xsave, y, mean, rstd)
#define C2_LNC(L)                                   \
  switch (c2::ceil_div(d, 4 * L)) {                 \
    case 1: C2_LN(L, 1); break;                     \
    case 2: C2_LN(L, 2); break;                     \
    case 3: C2_LN(L, 3); break;                     \
    default: C2_LN(L, 4); break;                    \
  }
  switch (lpr) {
    case 64: C2_LNC(64); break;
    case 32: C2_LNC(32); break;
    case 16: C2_LNC(16); break;
    case 8: C2_LNC(8); break;
    default: C2_LNC(4); break;
  }
#undef C2_LNC
#undef C2_LN
  C2_CHECK_LAUNCH();
  return 0;
}

// dx (+)= LN backward; db_out = dx ⊙ dropout mask (grad of the dropped residual branch);
// dgw/dgb += Σ_rows (accumulated; may be null).
C2_API int c2dsr_ln_bwd(const float* x, const float* mean, const float* rstd, const float* w, const float* dy, int rows,
                        int d, float* dx, int dx_accumulate, float* db_out, uint32_t k0, uint32_t k1, float p,
                        int64_t idx_base, const int* rowmap, float* dgw, float* dgb, void* workspace, void* stream) {
  if (d % 4 || d > 1024) return (int)hipErrorInvalidValue;
  if (rows == 0) return 0;
  c2::Drop dr = c2::make_drop(k0, k1, p);
  hipStream_t s = (hipStream_t)stream;
  const int lpr = lpr_for(d);
  const int groups = 256 / lpr;
  int nblk = c2::ceil_div(rows, groups);
  if (nblk > LN_BWD_BLOCKS) nblk = LN_BWD_BLOCKS;
  float* part = (float*)workspace;
#define C2_LNB(L, NC) \
  ln_bwd_kernel<L, NC><<<nblk, 256, 0, s>>>(x, mean, rstd, w, dy, rows, d, dx, dx_accumulate, db_out, dr, idx_base, rowmap, part)
#define C2_LNBC(L)                                  \
  switch (c2::ceil_div(d, 4 * L)) {                 \
    case 1: C2_LNB(L, 1); break;                    \
    case 2: C2_LNB(L, 2); break;                    \
    case 3: C2_LNB(L, 3); break;                    \
    default: C2_LNB(L, 4); break;                   \
  }
  switch (lpr) {
    case 64: C2_LNBC(64); break;
    case 32: C2_LNBC(32); break;
    case 16: C2_LNBC(16); break;
    case 8: C2_LNBC(8); break;
    default: C2_LNBC(4); break;
  }
#undef C2_LNBC
#undef C2_LNB
  if (dgw || dgb) reduce_parts_kernel<<<c2::ceil_div(2 * d, 64), 1024, 0, s>>>(part, nblk, d, dgw, dgb);
  C2_CHECK_LAUNCH();
  return 0;
}

// y = LNF(LN2(a + drop(b))·w2 + b2)·wF + bF (post-norm norm2 + the encoder's final norm); xsave = a + drop(b);
// st [4][rows] = (mean2, rstd2, meanF, rstdF)
C2_API int c2dsr_add_ln2_fwd(const float* a, const float* b, int rows, int d, uint32_t k0, uint32_t k1, float p,
                             int64_t idx_base, const int* rowmap, const float* w2, const float* b2, float eps2,
                             const float* wF, const float* bF, float epsF, float* xsave, float* y, float* st,
                             void* stream) {
  if (d % 4 || d > 1024 || !a || !b) return (int)hipErrorInvalidValue;
  if (rows == 0) return 0;
  c2::Drop dr = c2::make_drop(k0, k1, p);
  hipStream_t s = (hipStream_t)stream;
  const int lpr = lpr_for(d);
  dim3 grid(c2::ceil_div(rows, 256 / lpr));
#define C2_LN(L, NC) add_ln2_fwd_kernel<L, NC><<<grid, 256, 0, s>>>(a, b, rows, d, dr, idx_base, rowmap, w2, b2, eps2, wF, bF, epsF, xsave, y, st)
#define C2_LNC(L)                                   \
  switch (c2::ceil_div(d, 4 * L)) {                 \
    case 1: C2_LN(L, 1); break;                     \
    case 2: C2_LN(L, 2); break;                     \
    case 3: C2_LN(L, 3); break;                     \
    default: C2_LN(L, 4); break;                    \
  }
  switch (lpr) {
    case 64: C2_LNC(64); break;
    case 32: C2_LNC(32); break;
    case 16: C2_LNC(16); break;
    case 8: C2_LNC(8); break;
    default: C2_LNC(4); break;
  }
#undef C2_LNC
#undef C2_LN
  C2_CHECK_LAUNCH();
  return 0;
}

C2_API size_t c2dsr_ln2_bwd_workspace(int d) { return (size_t)LN_BWD_BLOCKS * 4 * d * 4; }

// partial blocks the LayerNorm backwards write for `rows` rows (both kernels: one lane group per row)
static int ln_bwd_nblk(int rows, int d) { return std::min(c2::ceil_div(rows, 256 / lpr_for(d)), LN_BWD_BLOCKS); }

// the LayerNorm parameter gradients of one encoder layer's two backwards in ONE launch: c2dsr_ln2_bwd and c2dsr_ln_bwd
// called with null parameter-gradient outputs leave their partials in their workspaces; this adds them (rows2 / rows1:
// the rows each backward ran on; the same fixed-order sums as their own reductions)
C2_API int c2dsr_ln_reduce2(const void* ws2, int rows2, const void* ws1, int rows1, int d, float* dgw2, float* dgb2,
                            float* dgwF, float* dgbF, float* dgw1, float* dgb1, void* stream) {
  if (d % 4 || d > 1024 || rows2 < 0 || rows1 < 0) return (int)hipErrorInvalidValue;
  const int nb4 = rows2 ? c2::ceil_div(4 * d, 64) : 0, nb2 = rows1 ? c2::ceil_div(2 * d, 64) : 0;
  if (nb4 + nb2 == 0) return 0;
  ln_reduce2_kernel<<<nb4 + nb2, 1024, 0, (hipStream_t)stream>>>((const float*)ws2, rows2 ? ln_bwd_nblk(rows2, d) : 0,
                                                                  (const float*)ws1, rows1 ? ln_bwd_nblk(rows1, d) : 0,
                                                                  d, nb4, dgw2, dgb2, dgwF, dgbF, dgw1, dgb1);
  C2_CHECK_LAUNCH();
  return 0;
}

// backward of c2dsr_add_ln2_fwd: dx = the gradient w.r.t. a, db_out = dx ⊙ drop mask (w.r.t. b); the four
// LayerNorm parameter gradients accumulated (null ones skipped)
C2_API int c2dsr_ln2_bwd(const float* xsave, const float* st, const float* w2, const float* b2, const float* wF,
                         const float* dy, int rows, int d, float* dx, float* db_out, uint32_t k0, uint32_t k1, float p,
                         int64_t idx_base, const int* rowmap, float* dgw2, float* dgb2, float* dgwF, float* dgbF,
                         void* workspace, void* stream) {
  if (d % 4 || d > 1024 || !dx || !db_out) return (int)hipErrorInvalidValue;
  if (rows == 0) return 0;
  c2::Drop dr = c2::make_drop(k0, k1, p);
  hipStream_t s = (hipStream_t)stream;
  const int lpr = lpr_for(d);
  int nblk = c2::ceil_div(rows, 256 / lpr);
  if (nblk > LN_BWD_BLOCKS) nblk = LN_BWD_BLOCKS;
  float* part = (float*)workspace;
#define C2_LNB(L, NC) \
  ln2_bwd_kernel<L, NC><<<nblk, 256, 0, s>>>(xsave, st, w2, b2, wF, dy, rows, d, dx, db_out, dr, idx_base, rowmap, part)
#define C2_LNBC(L)                                  \
  switch (c2::ceil_div(d, 4 * L)) {                 \
    case 1: C2_LNB(L, 1); break;                    \
    case 2: C2_LNB(L, 2); break;                    \
    case 3: C2_LNB(L, 3); break;                    \
    default: C2_LNB(L, 4); break;                   \
  }
  switch (lpr) {
    case 64: C2_LNBC(64); break;
    case 32: C2_LNBC(32); break;
    case 16: C2_LNBC(16); break;
    case 8: C2_LNBC(8); break;
    default: C2_LNBC(4); break;
  }
#undef C2_LNBC
#undef C2_LNB
  if (dgw2 || dgb2 || dgwF || dgbF)
    reduce_parts4_kernel<<<c2::ceil_div(4 * d, 64), 1024, 0, s>>>(part, nblk, d, dgw2, dgb2, dgwF, dgbF);
  C2_CHECK_LAUNCH();
  return 0;
}

// y = (a ? a : 0) + drop(b)      (element-wise, n multiple of 4; row index = flat/d)
C2_API int c2dsr_add_dropout(const float* a, const float* b, long n, int d, uint32_t k0, uint32_t k1, float p,
                             int64_t idx_base, float* y, void* stream) {
  if (n % 4 || d % 4) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  c2::Drop dr = c2::make_drop(k0, k1, p);
  const long n4 = n / 4;
  add_drop_kernel<<<c2::ceil_div(n4, 256), 256, 0, (hipStream_t)stream>>>(a, b, n4, d, dr, idx_base, y);
  C2_CHECK_LAUNCH();
  return 0;
}

C2_API int c2dsr_relu_drop_bwd(const float* dy, const float* y, long n, float p, float* dx, void* stream) {
  if (n == 0) return 0;
  const float scale = p > 0.f ? (float)(1.0 / (1.0 - (double)p)) : 1.f;
  relu_drop_bwd_kernel<<<c2::ceil_div(n, 256), 256, 0, (hipStream_t)stream>>>(dy, y, n, scale, dx);
  C2_CHECK_LAUNCH();
  return 0;
}
