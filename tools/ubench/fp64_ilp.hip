// Micro-benchmark: fp64 FMA dependent-chain latency vs ILP vs waves per SIMD on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int CH>
__global__ void chains(double* out, long long* cyc, int iters, double a, double b) {
  double x[CH];
  for (int c = 0; c < CH; c++) x[c] = threadIdx.x * 1e-3 + c;
  __syncthreads();
  long long t0 = clock64();
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int c = 0; c < CH; c++) x[c] = __builtin_fma(x[c], a, b);
  }
  long long t1 = clock64();
  double s = 0;
  for (int c = 0; c < CH; c++) s += x[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}
__global__ void divchain(double* out, long long* cyc, int iters, double a) {
  double x = threadIdx.x + 1.0;
  long long t0 = clock64();
  for (int i = 0; i < iters; i++) x = a / x + 1.0;
  long long t1 = clock64();
  out[threadIdx.x] = x;
  if ((threadIdx.x & 63) == 0) cyc[threadIdx.x / 64] = t1 - t0;
}
template <int CH>
void run(const char* name, int threads, int iters) {
  double* out; long long* cyc;
  hipMalloc(&out, threads * 8 * 4); hipMalloc(&cyc, 64 * 8);
  chains<CH><<<1, threads>>>(out, cyc, iters, 0.999999, 1e-7);
  hipDeviceSynchronize();
  chains<CH><<<1, threads>>>(out, cyc, iters, 0.999999, 1e-7);
  long long h[16]; hipMemcpy(h, cyc, 8 * (threads / 64), hipMemcpyDeviceToHost);
  double per = (double)h[0] / ((double)iters * CH);
  printf("%-28s waves/block=%d  cycles per fma per chain-step: %.2f  (per iter all chains %.2f)\n", name, threads / 64, per, (double)h[0] / iters);
  hipFree(out); hipFree(cyc);
}
int main() {
  run<1>("1 chain, 1 wave", 64, 20000);
  run<2>("2 chains, 1 wave", 64, 20000);
  run<4>("4 chains, 1 wave", 64, 20000);
  run<8>("8 chains, 1 wave", 64, 20000);
  run<1>("1 chain, 4 waves (1/SIMD)", 256, 20000);
  run<1>("1 chain, 8 waves (2/SIMD)", 512, 20000);
  run<1>("1 chain, 16 waves (4/SIMD)", 1024, 20000);
  run<4>("4 chains, 8 waves (2/SIMD)", 512, 20000);
  double* out; long long* cyc; hipMalloc(&out, 4096); hipMalloc(&cyc, 64);
  divchain<<<1, 64>>>(out, cyc, 2000, 3.0); hipDeviceSynchronize();
  divchain<<<1, 64>>>(out, cyc, 2000, 3.0);
  long long h; hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
  printf("dependent fp64 div+add: %.1f cycles per iteration\n", (double)h / 2000);
  return 0;
}
