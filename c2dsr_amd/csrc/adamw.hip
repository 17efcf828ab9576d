// K6: fused AdamW(amsgrad) over the flat parameter buffer.
//
// Replaces torch.optim.AdamW(lr, weight_decay=l2, amsgrad=True).step() (trainer.py:21-22,158)
// together with the reference's "zero_grad once per epoch" accumulation (trainer.py:42, Q3):
// the backward of a step writes a fresh gradient buffer F (all-reduced across ranks
// under data parallelism); this kernel folds it into the epoch accumulator A (g = A + F),
// clears F for the next step and applies the update — one pass, 48 B/param.  On one device the
// backward accumulates straight into A (fresh == accum: KEEP), and the pass reads g = A only:
// 36 B/param.
#include "common.h"

// ADAMW_NT: non-temporal (streaming) loads and stores — every byte is touched once per step
#ifndef ADAMW_NT
#define ADAMW_NT 1
#endif

namespace {

typedef float f32x4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ld_s(const float4* p) {
#if ADAMW_NT
  const f32x4v v = __builtin_nontemporal_load((const f32x4v*)p);
  return make_float4(v[0], v[1], v[2], v[3]);
#else
  return *p;
#endif
}
__device__ __forceinline__ void st_s(float4* p, float4 v) {
#if ADAMW_NT
  f32x4v x;
  x[0] = v.x; x[1] = v.y; x[2] = v.z; x[3] = v.w;
  __builtin_nontemporal_store(x, (f32x4v*)p);
#else
  *p = v;
#endif
}

template <bool KEEP>
__global__ __launch_bounds__(256) void adamw_kernel(float4* __restrict__ p, float4* __restrict__ fresh,
                                                    float4* __restrict__ accum, float4* __restrict__ m,
                                                    float4* __restrict__ v, float4* __restrict__ vmax, long n4,
                                                    float lr, float wd_factor, float b1, float b2, float eps,
                                                    float step_size, float inv_bc2_sqrt,
                                                    const int* __restrict__ err) {
  // a step whose indices were out of range changes nothing (the reference raises before optimizer.step(),
  // trainer.py:97-158); the host raises IndexError at its next sync
  if (err && *err) return;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    float4 g = ld_s(fresh + i);
    if constexpr (!KEEP) {
      if (accum) {
        g = g + ld_s(accum + i);
        st_s(accum + i, g);
      }
      st_s(fresh + i, make_float4(0.f, 0.f, 0.f, 0.f));
    }
    float4 pp = ld_s(p + i), mm = ld_s(m + i), vv = ld_s(v + i), vx = ld_s(vmax + i);
    float* P = (float*)&pp;
    float* G = (float*)&g;
    float* Mm = (float*)&mm;
    float* Vv = (float*)&vv;
    float* Vx = (float*)&vx;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      P[k] *= wd_factor;
      Mm[k] = Mm[k] + (1.f - b1) * (G[k] - Mm[k]);  // lerp
      Vv[k] = Vv[k] * b2 + (1.f - b2) * G[k] * G[k];
      Vx[k] = fmaxf(Vx[k], Vv[k]);
      const float denom = sqrtf(Vx[k]) * inv_bc2_sqrt + eps;
      P[k] = P[k] - step_size * (Mm[k] / denom);
    }
    st_s(p + i, pp);
    st_s(m + i, mm);
    st_s(v + i, vv);
    st_s(vmax + i, vx);
  }
}

}  // namespace

// All buffers fp32 [n], n % 4 == 0, 16-byte aligned.  accum may be null (no epoch accumulation);
// accum == fresh: the gradient buffer is the epoch accumulation itself (read only).
C2_API int c2dsr_adamw(float* p, float* fresh, float* accum, float* m, float* v, float* vmax, long n, float lr, float wd,
                       float b1, float b2, float eps, int step, const int* err, void* stream) {
  if (n % 4) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  const double bc1 = 1.0 - pow((double)b1, (double)step);
  const double bc2 = 1.0 - pow((double)b2, (double)step);
  const float step_size = (float)(lr / bc1);
  const float inv_bc2_sqrt = (float)(1.0 / sqrt(bc2));
  const long n4 = n / 4;
  int blocks = c2::ceil_div(n4, 256);
// one float4 per thread (no grid-stride loop): every load of the pass in flight at once — measured
// 841 → 700 µs (36 B/param) and 1109 → 939 µs (48 B/param) over 105.8 M parameters against a
// 4096-block grid-stride loop (tools/adamw_micro.py)
#ifndef ADAMW_BLOCK_CAP
#define ADAMW_BLOCK_CAP 0
#endif
  if (ADAMW_BLOCK_CAP > 0 && blocks > ADAMW_BLOCK_CAP) blocks = ADAMW_BLOCK_CAP;
  if (accum && accum == fresh)
    adamw_kernel<true><<<blocks, 256, 0, (hipStream_t)stream>>>((float4*)p, (float4*)fresh, nullptr, (float4*)m,
                                                                (float4*)v, (float4*)vmax, n4, lr, 1.f - lr * wd, b1,
                                                                b2, eps, step_size, inv_bc2_sqrt, err);
  else
    adamw_kernel<false><<<blocks, 256, 0, (hipStream_t)stream>>>((float4*)p, (float4*)fresh, (float4*)accum,
                                                                 (float4*)m, (float4*)v, (float4*)vmax, n4, lr,
                                                                 1.f - lr * wd, b1, b2, eps, step_size, inv_bc2_sqrt, err);
  C2_CHECK_LAUNCH();
  return 0;
}
