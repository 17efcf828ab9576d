// Kernel-boundary cost behind a kernel that leaves its output in L2 (tools/boundary_micro.py): a streaming kernel
// writes B bytes with default-policy or non-temporal float4 stores, a one-workgroup kernel follows on the stream.
// Build: hipcc -O3 --offload-arch=gfx950 -shared -fPIC tools/boundary_micro.hip -o tools/_boundary_micro.so
#include <hip/hip_runtime.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void write_kernel(const f32x4* __restrict__ x, f32x4* __restrict__ y, long n4, int nt) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  const f32x4 v = __builtin_nontemporal_load(x + i) * 1.0001f;
  if (nt)
    __builtin_nontemporal_store(v, y + i);
  else
    y[i] = v;
}

__global__ void tiny_kernel(float* p) {
  if (threadIdx.x == 0) p[0] += 1.f;
}

extern "C" float boundary_run(const float* x, float* y, long n, int nt, int pairs, int tiny, float* scratch) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const long n4 = n / 4;
  const int blocks = (int)((n4 + 255) / 256);
  for (int w = 0; w < 2; ++w) write_kernel<<<blocks, 256>>>((const f32x4*)x, (f32x4*)y, n4, nt);
  (void)hipEventRecord(e0, 0);
  for (int i = 0; i < pairs; ++i) {
    write_kernel<<<blocks, 256>>>((const f32x4*)x, (f32x4*)y, n4, nt);
    if (tiny) tiny_kernel<<<1, 64>>>(scratch);
  }
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return ms * 1e3f / pairs;  // µs per (write [+ tiny]) pair
}
