// Sustained bf16 MFMA rate on this MI355X (the practical ceiling for K5's roofline): every wave issues
// v_mfma_f32_32x32x16_bf16 back to back on 4 independent accumulators, no memory traffic in the loop.
// usage: ./mfma_peak [waves_per_simd=1] [iters=200000]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void mfma_loop(int iters, float* out) {
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = (__bf16)(0.001f * (threadIdx.x + i));
    b[i] = (__bf16)(0.002f * (threadIdx.x - i));
  }
  f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  for (int it = 0; it < iters; ++it) {
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c3, 0, 0, 0);
  }
  float s = 0.f;
  for (int i = 0; i < 16; ++i) s += c0[i] + c1[i] + c2[i] + c3[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main(int argc, char** argv) {
  const int wps = argc > 1 ? atoi(argv[1]) : 1;
  const int iters = argc > 2 ? atoi(argv[2]) : 200000;
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int blocks = p.multiProcessorCount;  // one workgroup of 4·wps waves per CU
  const int threads = 256 * wps;
  float* out;
  hipMalloc(&out, (size_t)blocks * threads * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  mfma_loop<<<blocks, threads>>>(1000, out);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  mfma_loop<<<blocks, threads>>>(iters, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double flops = 2.0 * 32 * 32 * 16 * 4.0 * iters * (blocks * threads / 64);
  printf("mfma_peak: %d CUs, %d waves/SIMD, %.3f ms, %.1f TFLOP/s bf16 dense (32x32x16)\n", blocks, wps, ms,
         flops / ms / 1e9);
  hipFree(out);
  return 0;
}
