// Shader clock under fp64 load: s_memtime (core clock) vs s_memrealtime (100 MHz) over a
// dependent fp64 FMA loop, one wave per SIMD on every CU (the MPPI phase-1 shape) and one wave alone.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void spin(double* out, unsigned long long* t, int iters) {
  double a = threadIdx.x * 1e-3, b = 1.0000001;
  const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; i++) {
    a = __builtin_fma(a, b, 1e-9);
    b = __builtin_fma(b, a, -1e-9);
  }
  const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) { t[2 * blockIdx.x] = c1 - c0; t[2 * blockIdx.x + 1] = r1 - r0; }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a + b;
}

int main() {
  double* out; unsigned long long* t;
  hipMalloc(&out, 8 * 4096 * 256); hipMalloc(&t, 16 * 4096);
  for (int blocks : {1, 1024, 2048}) {
    for (int rep = 0; rep < 2; rep++) {
      hipLaunchKernelGGL(spin, dim3(blocks), dim3(64), 0, 0, out, t, 200000);
      hipDeviceSynchronize();
    }
    unsigned long long h[2];
    hipMemcpy(h, t, 16, hipMemcpyDeviceToHost);
    printf("blocks %d: core cycles %llu real ticks %llu -> %.0f MHz; %.2f cycles per dependent fma\n", blocks, h[0], h[1],
           h[0] / (h[1] / 100.0), (double)h[0] / (2.0 * 200000));
  }
  return 0;
}
