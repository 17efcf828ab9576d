// Sustained bf16 MFMA rate on this MI355X (the practical ceiling for K5's roofline): every wave issues
// bf16 MFMAs back to back on 4 independent accumulators, no memory traffic in the loop; operands are
// per-lane pseudo-random values (the clock the chip holds depends on the data).
// usage: ./mfma_peak [waves_per_simd=1] [iters=200000] [shape=32 (32x32x16) | 16 (16x16x32)]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ float rnd(unsigned x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return (float)(x & 0xffff) * (1.f / 32768.f) - 1.f;
}

template <int SHAPE>
__global__ void mfma_loop(int iters, float* out) {
  bf16x8 a, b;
  const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
  for (int i = 0; i < 8; ++i) {
    a[i] = (__bf16)rnd(t * 16 + i);
    b[i] = (__bf16)rnd(t * 16 + 8 + i);
  }
  float s = 0.f;
  if constexpr (SHAPE == 32) {
    f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
    for (int it = 0; it < iters; ++it) {
      c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c3, 0, 0, 0);
    }
    for (int i = 0; i < 16; ++i) s += c0[i] + c1[i] + c2[i] + c3[i];
  } else {
    f32x4 c[8] = {};
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int k = 0; k < 8; ++k) c[k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c[k], 0, 0, 0);
    for (int k = 0; k < 8; ++k)
      for (int i = 0; i < 4; ++i) s += c[k][i];
  }
  out[t] = s;
}

int main(int argc, char** argv) {
  const int wps = argc > 1 ? atoi(argv[1]) : 1;
  const int iters = argc > 2 ? atoi(argv[2]) : 200000;
  const int shape = argc > 3 ? atoi(argv[3]) : 32;
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int blocks = p.multiProcessorCount;  // one workgroup of 4·wps waves per CU
  const int threads = 256 * wps;
  float* out;
  hipMalloc(&out, (size_t)blocks * threads * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto run = [&](int n) {
    if (shape == 32)
      mfma_loop<32><<<blocks, threads>>>(n, out);
    else
      mfma_loop<16><<<blocks, threads>>>(n, out);
  };
  run(1000);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  run(iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  // flops per iteration per wave: 4 × 32x32x16 or 8 × 16x16x32 — both 131,072·... (2·M·N·K each)
  const double per_it = shape == 32 ? 4.0 * 2 * 32 * 32 * 16 : 8.0 * 2 * 16 * 16 * 32;
  const double flops = per_it * iters * (blocks * threads / 64);
  printf("mfma_peak: %d CUs, %d waves/SIMD, shape %d, %.3f ms, %.1f TFLOP/s bf16 dense\n", blocks, wps, shape, ms,
         flops / ms / 1e9);
  hipFree(out);
  return 0;
}
