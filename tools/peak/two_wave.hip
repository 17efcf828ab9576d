// Feasibility micro for K5 at two waves per SIMD (csrc/ce3.hip runs one): the S-phase step of one wave as
// NSB stationary 16-row blocks × one split product (3 v_mfma_f32_16x16x32_bf16 each) on the swept fragment it
// reads from LDS (2 ds_read_b128 per step: hi, lo), plus one exp element per 16 stationary rows and step.
//   NSB = 2 at 4 waves per CU (today's shape: 6 MFMAs per 2 reads)
//   NSB = 1 at 8 waves per CU (two per SIMD: 3 MFMAs per 2 reads — twice the LDS bytes per MFMA)
// and the U-phase analogue (TR: 4 ds_read_b64_tr_b16 per step).  Prints cycles per MFMA per SIMD (the matrix
// pipe's share: 16 = saturated).  usage: ./two_wave [iters]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

__device__ __forceinline__ void tri(f32x4& acc, const bf16x8& ah, const bf16x8& al, const bf16x8& bh,
                                    const bf16x8& bl) {
  asm volatile(
      "v_mfma_f32_16x16x32_bf16 %0, %1, %3, %0\n\t"
      "v_mfma_f32_16x16x32_bf16 %0, %2, %3, %0\n\t"
      "v_mfma_f32_16x16x32_bf16 %0, %1, %4, %0"
      : "+v"(acc)
      : "v"(ah), "v"(al), "a"(bh), "a"(bl));
}

template <int NSB, bool TR>
__global__ __launch_bounds__(NSB == 2 ? 256 : 512, 1) void step_kernel(int iters, float* out,
                                                                        unsigned long long* cyc) {
  __shared__ __attribute__((aligned(16))) char img[65536];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 65536 / 16; i += blockDim.x)
    ((float4*)img)[i] = make_float4(1e-3f * (i & 7), 2e-3f, -1e-3f, 1.f);
  __syncthreads();
  bf16x8 bh[2], bl[2], ah, al;
  for (int i = 0; i < 8; ++i) {
    bh[0][i] = (__bf16)(0.01f * ((lane + i) & 7));
    bl[0][i] = (__bf16)(0.001f * i);
    bh[1][i] = (__bf16)(0.02f * i);
    bl[1][i] = (__bf16)(0.002f * ((lane + i) & 3));
    ah[i] = (__bf16)(0.5f + 0.01f * i);
    al[i] = (__bf16)(0.003f * i);
  }
  f32x4 s[2] = {};
  float z = 0.f, sc = 0.1f * lane, m = 0.5f;
  bf16x8 fr[4][2];
  for (int k = 0; k < 4; ++k) {
    fr[k][0] = ah;
    fr[k][1] = al;
  }
  const int base = (lane * 16) & 0x3ff0;
  const unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int o = (k * 2048 + (it & 7) * 4096) & 0x7fff;
      if constexpr (TR) {
        bf16x8 v[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const bf16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
              (lds_bf16x4*)(size_t)(base / 2 + o + 16384 * h));
          const bf16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
              (lds_bf16x4*)(size_t)(base / 2 + o + 16384 * h + 4096));
          v[h][0] = a[0]; v[h][1] = a[1]; v[h][2] = a[2]; v[h][3] = a[3];
          v[h][4] = b[0]; v[h][5] = b[1]; v[h][6] = b[2]; v[h][7] = b[3];
        }
        fr[(k + 2) & 3][0] = v[0];
        fr[(k + 2) & 3][1] = v[1];
      } else {
        fr[(k + 2) & 3][0] = *(const bf16x8*)(img + base + o);
        fr[(k + 2) & 3][1] = *(const bf16x8*)(img + base + o + 32768);
      }
#pragma unroll
      for (int sb = 0; sb < NSB; ++sb) {
        tri(s[sb], fr[k & 3][0], fr[k & 3][1], bh[sb], bl[sb]);
        if ((k & 1) == 0 || NSB == 2) {
          __builtin_amdgcn_sched_barrier(0);
          const float p = __builtin_amdgcn_exp2f(sc - m);
          sc = p * 0.999f;
          z += p;
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  const unsigned long long t1 = __builtin_readcyclecounter();
  float r = z;
  for (int i = 0; i < 4; ++i) r += s[0][i] + s[1][i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int NSB, bool TR>
void run(const char* name, int iters, float* out, unsigned long long* cyc, int ncu) {
  const int nt = NSB == 2 ? 256 : 512;
  step_kernel<NSB, TR><<<ncu, nt>>>(iters, out, cyc);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  step_kernel<NSB, TR><<<ncu, nt>>>(iters, out, cyc);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  unsigned long long c[1024];
  hipMemcpy(c, cyc, sizeof(unsigned long long) * ncu, hipMemcpyDeviceToHost);
  double avg = 0;
  for (int i = 0; i < ncu; ++i) avg += (double)c[i];
  avg /= ncu;
  const double mf_per_simd = 16.0 * iters * NSB * 3 * (nt / 256);
  printf("%-28s %6.2f cycles per MFMA per SIMD  %7.3f ms  MFMA %.0f TFLOP/s\n", name, avg / mf_per_simd, ms,
         16.0 * 16 * 32 * 2 * mf_per_simd * 4 * ncu / (ms * 1e-3) / 1e12);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20000;
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int ncu = p.multiProcessorCount;
  float* out;
  unsigned long long* cyc;
  hipMalloc(&out, sizeof(float) * 512 * ncu);
  hipMalloc(&cyc, sizeof(unsigned long long) * ncu);
  run<2, false>("S: 1 wave/SIMD, 2 blocks", iters, out, cyc, ncu);
  run<1, false>("S: 2 waves/SIMD, 1 block", iters, out, cyc, ncu);
  run<2, true>("U: 1 wave/SIMD, 2 blocks", iters, out, cyc, ncu);
  run<1, true>("U: 2 waves/SIMD, 1 block", iters, out, cyc, ncu);
  return 0;
}
