// Isolates the cost of K5's S-phase step (csrc/ce3.hip) on this MI355X: one wave per SIMD (256 threads, one
// workgroup per CU), each step = 6 v_mfma_f32_16x16x32_bf16 as two dependent chains of three (the split product
// a_hi·b_hi + a_lo·b_hi + a_hi·b_lo for two stationary row blocks, B in AGPRs) plus, by variant,
//   R: the step's two ds_read_b128 A fragments (issued 2 steps ahead, as ce3's ring)
//   V: its epilogue element (v_sub, v_exp, v_add)
//   C: every 8th step, the hi/lo conversion burst of 8 values
//   I: the same 6 MFMAs as independent single-MFMA chains (6 accumulators) instead of 2×3 dependent
// prints cycles per step (clock from hipDeviceProp) and the MFMA share.  usage: ./s_phase [iters]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void tri(f32x4& acc, const bf16x8& ah, const bf16x8& al, const bf16x8& bh,
                                    const bf16x8& bl) {
  asm volatile(
      "v_mfma_f32_16x16x32_bf16 %0, %1, %3, %0\n\t"
      "v_mfma_f32_16x16x32_bf16 %0, %2, %3, %0\n\t"
      "v_mfma_f32_16x16x32_bf16 %0, %1, %4, %0"
      : "+v"(acc)
      : "v"(ah), "v"(al), "a"(bh), "a"(bl));
}
__device__ __forceinline__ void tri_a(f32x4& acc, const bf16x8& ah, const bf16x8& al, const bf16x8& bh,
                                      const bf16x8& bl) {  // accumulator in AGPRs (VGPR ports free for VALU / DS)
  asm volatile(
      "v_mfma_f32_16x16x32_bf16 %0, %1, %3, %0\n\t"
      "v_mfma_f32_16x16x32_bf16 %0, %2, %3, %0\n\t"
      "v_mfma_f32_16x16x32_bf16 %0, %1, %4, %0"
      : "+a"(acc)
      : "v"(ah), "v"(al), "a"(bh), "a"(bl));
}
__device__ __forceinline__ void one(f32x4& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "a"(b));
}

#define MFB(a, b, c) __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0)
// PD: prefetch distance of the reads (steps); BI: compiler-visible MFMAs, one read / VALU group per MFMA gap
template <bool R, bool V, bool C, bool I, int PD = 2, bool BI = false, bool ACCA = false>
__global__ __launch_bounds__(256, 1) void s_phase(int iters, float* out, unsigned long long* cyc) {
  __shared__ __attribute__((aligned(16))) char img[65536];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 65536 / 16; i += 256)
    ((float4*)img)[i] = make_float4(1e-3f * (i & 7), 2e-3f, -1e-3f, 1.f);
  __syncthreads();
  bf16x8 bh0, bl0, bh1, bl1, ah, al;
  for (int i = 0; i < 8; ++i) {
    bh0[i] = (__bf16)(0.01f * ((lane + i) & 7));
    bl0[i] = (__bf16)(0.001f * i);
    bh1[i] = (__bf16)(0.02f * i);
    bl1[i] = (__bf16)(0.002f * ((lane + i) & 3));
    ah[i] = (__bf16)(0.5f + 0.01f * i);
    al[i] = (__bf16)(0.003f * i);
  }
  f32x4 s0 = {}, s1 = {}, s2 = {}, s3 = {}, s4 = {}, s5 = {};
  float z = 0.f, sc = 0.1f * lane, m = 0.5f;
  bf16x8 fr[8][2];
  const int base = (lane * 16) & 0x3ff0;
  for (int k = 0; k < 8; ++k) {
    fr[k][0] = ah;
    fr[k][1] = al;
  }
  const unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      if constexpr (R) {
        const int o = (k * 2048 + (it & 7) * 4096) & 0x7fff;  // varies with it: not hoisted
        fr[(k + PD) & 7][0] = *(const bf16x8*)(img + base + o);
        fr[(k + PD) & 7][1] = *(const bf16x8*)(img + base + o + 32768);
      }
      const bf16x8& a = fr[k & 7][0];
      const bf16x8& b = fr[k & 7][1];
      if constexpr (BI) {
        s0 = MFB(a, bh0, s0);
        s0 = MFB(b, bh0, s0);
        s0 = MFB(a, bl0, s0);
        if constexpr (V) {
          const float p = __builtin_amdgcn_exp2f(sc - m);
          sc = p * 0.999f;
          z += p;
        }
        s1 = MFB(a, bh1, s1);
        s1 = MFB(b, bh1, s1);
        s1 = MFB(a, bl1, s1);
#pragma unroll
        for (int q = 0; q < 6; ++q) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
        }
      } else if constexpr (I) {
        one(s0, a, bh0);
        one(s1, b, bh0);
        one(s2, a, bl0);
        one(s3, a, bh1);
        one(s4, b, bh1);
        one(s5, a, bl1);
      } else {
        if constexpr (ACCA) tri_a(s0, a, b, bh0, bl0); else tri(s0, a, b, bh0, bl0);
        if constexpr (V) {
          __builtin_amdgcn_sched_barrier(0);
          const float p = __builtin_amdgcn_exp2f(sc - m);
          sc = p * 0.999f;
          z += p;
          __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (C) {
          if ((k & 7) == 7) {
            bf16x8 h, l;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const float x = sc + 0.01f * j;
              h[j] = (__bf16)x;
              l[j] = (__bf16)(x - (float)h[j]);
            }
            ah = h;
            al = l;
            __builtin_amdgcn_sched_barrier(0);
          }
        }
        if constexpr (ACCA) tri_a(s1, a, b, bh1, bl1); else tri(s1, a, b, bh1, bl1);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  const unsigned long long t1 = __builtin_readcyclecounter();
  float r = z + (float)ah[0] + (float)al[1];
  for (int i = 0; i < 4; ++i) r += s0[i] + s1[i] + s2[i] + s3[i] + s4[i] + s5[i];
  out[blockIdx.x * 256 + threadIdx.x] = r;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <bool R, bool V, bool C, bool I, int PD = 2, bool BI = false, bool ACCA = false>
void run(const char* name, int iters, float* out, unsigned long long* cyc, int ncu) {
  s_phase<R, V, C, I, PD, BI, ACCA><<<ncu, 256>>>(iters, out, cyc);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  s_phase<R, V, C, I, PD, BI, ACCA><<<ncu, 256>>>(iters, out, cyc);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  unsigned long long c[1024];
  hipMemcpy(c, cyc, sizeof(unsigned long long) * ncu, hipMemcpyDeviceToHost);
  double avg = 0;
  for (int i = 0; i < ncu; ++i) avg += (double)c[i];
  avg /= ncu;
  const double steps = 16.0 * iters;
  printf("%-24s %7.1f cycles/step (s_memtime)  %7.3f ms  %6.1f ns/step  MFMA %.0f TFLOP/s\n", name, avg / steps, ms,
         ms * 1e6 / steps, 6.0 * 16 * 16 * 32 * 2 * 4 * ncu * steps / (ms * 1e-3) / 1e12);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20000;
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int ncu = p.multiProcessorCount;
  float* out;
  unsigned long long* cyc;
  hipMalloc(&out, sizeof(float) * 256 * ncu);
  hipMalloc(&cyc, sizeof(unsigned long long) * ncu);
  run<false, false, false, false>("mfma 2x3 dep", iters, out, cyc, ncu);
  run<false, false, false, true>("mfma 6 indep", iters, out, cyc, ncu);
  run<true, false, false, false>("+reads", iters, out, cyc, ncu);
  run<false, true, false, false>("+valu", iters, out, cyc, ncu);
  run<true, true, false, false>("+reads+valu", iters, out, cyc, ncu);
  run<true, true, true, false>("+reads+valu+burst", iters, out, cyc, ncu);
  run<false, false, true, false>("+burst", iters, out, cyc, ncu);
  run<true, false, false, false, 4>("+reads pd4", iters, out, cyc, ncu);
  run<true, true, false, false, 4>("+reads+valu pd4", iters, out, cyc, ncu);
  run<true, false, false, false, 2, true>("BI +reads", iters, out, cyc, ncu);
  run<true, true, false, false, 2, true>("BI +reads+valu", iters, out, cyc, ncu);
  run<true, true, false, false, 4, true>("BI +reads+valu pd4", iters, out, cyc, ncu);
  run<true, false, false, false, 2, false, true>("accA +reads", iters, out, cyc, ncu);
  run<false, true, false, false, 2, false, true>("accA +valu", iters, out, cyc, ncu);
  run<true, true, false, false, 2, false, true>("accA +reads+valu", iters, out, cyc, ncu);
  run<true, true, true, false, 2, false, true>("accA +reads+valu+burst", iters, out, cyc, ncu);
  return 0;
}
