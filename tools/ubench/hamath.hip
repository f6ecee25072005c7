// Lane-safe libm latency on one wavefront (the Hybrid A* build), lanes spread over ranges.
#include <hip/hip_runtime.h>
#include <cstdio>
#define MPJ_LANE_SAFE 1
#include "../../include/mp_jlmath.h"
#define ITERS 200
template <int F>
__global__ void lat(double* out, long long* cyc, double seed) {
  double x = seed + threadIdx.x * 0.013;
  long long t0 = clock64();
  for (int i = 0; i < ITERS; i++) {
    if (F == 0) x = mpj_acos(x * 0.5) * 0.3;
    if (F == 1) x = mpj_asin(x * 0.5) * 0.9;
    if (F == 2) x = mpj_atan2_bl(x, 1.3 - x) * 0.5;
    if (F == 3) x = mpj_modpi_bl(x * 3.0 + 2.0) * 0.3;
    if (F == 4) x = mpj_sqrt(x + 1.0) - 0.9;
    if (F == 5) { double s, c; mpj_sincos_bl(x, &s, &c); x = s + c * 0.1; }
    if (F == 6) x = mpj_sin(x * 3.0) * 0.5;
    if (F == 7) x = mpj_atan2(x, 1.3 - x) * 0.5;
  }
  long long t1 = clock64();
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}
template <int F>
void run(const char* name) {
  double* out; long long* cyc; long long h;
  hipMalloc(&out, 64 * 8); hipMalloc(&cyc, 8);
  lat<F><<<1, 64>>>(out, cyc, 0.1); hipDeviceSynchronize();
  lat<F><<<1, 64>>>(out, cyc, 0.1); hipDeviceSynchronize();
  hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
  printf("%-28s %8.1f cycles/call\n", name, (double)h / ITERS);
}
int main() {
  run<0>("acos (lane-safe)");
  run<1>("asin");
  run<2>("atan2_bl");
  run<3>("modpi_bl");
  run<4>("sqrt");
  run<5>("sincos_bl (lane-safe)");
  run<6>("sin (exact, branchy)");
  run<7>("atan2 (exact atan)");
  return 0;
}
