// Latency of the hot math on one wavefront (cycles per dependent call), gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../include/mp_jlmath.h"
#include "../../motionplanning_amd/csrc/mppi_device.hpp"
using namespace mpk;
#define ITERS 400
template <int F>
__global__ void lat(double* out, long long* cyc, double seed) {
  double x = seed + threadIdx.x * 1e-4;
  double st[7] = {x, 0.1, 0.2, 0.05, 0.1, 5.0, 0.01}, d[7];
  long long t0 = clock64();
  for (int i = 0; i < ITERS; i++) {
    if (F == 0) x = mpj_atan(x) + 0.7;
    if (F == 1) x = mpj_atan_bl(x) + 0.7;
    if (F == 2) x = mpj_sin(x) + 1.3;
    if (F == 3) x = mpj_sin_bl(x) + 1.3;
    if (F == 4) { double s, c; mpj_sincos_bl(x, &s, &c); x = s + c; }
    if (F == 5) x = 1.0 / (x + 0.01) + 0.5;
    if (F == 6) x = mpj_exp(-x) + 0.5;
    if (F == 7) x = mpj_log(x) + 2.0;
    if (F == 8) { dyn_pair(st, 0.01, 0.2, d, threadIdx.x & 1); for (int k = 0; k < 7; k++) st[k] = st[k] + d[k] * 1e-3; }
    if (F == 9) { double z[2]; MppiDev P{}; P.offset = i; philox_normal2(P, 0, threadIdx.x, i, z); x = x + z[0] + z[1]; }
  }
  long long t1 = clock64();
  out[threadIdx.x] = x + st[0] + st[4];
  if (threadIdx.x == 0) *cyc = t1 - t0;
}
template <int F>
void run(const char* name) {
  double* out; long long* cyc; long long h;
  hipMalloc(&out, 64 * 8); hipMalloc(&cyc, 8);
  lat<F><<<1, 64>>>(out, cyc, 0.3); hipDeviceSynchronize();
  lat<F><<<1, 64>>>(out, cyc, 0.3); hipDeviceSynchronize();
  hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
  printf("%-34s %8.1f cycles/call\n", name, (double)h / ITERS);
  hipFree(out); hipFree(cyc);
}
int main() {
  run<0>("atan (FDLIBM, branchy)");
  run<1>("atan_bl");
  run<2>("sin (FDLIBM, branchy)");
  run<3>("sin_bl");
  run<4>("sincos_bl");
  run<5>("fp64 reciprocal-div + add");
  run<6>("exp");
  run<7>("log");
  run<8>("dyn_pair (one VehicleDynamics)");
  run<9>("philox_normal2 (Philox+Box-Muller)");
  return 0;
}
