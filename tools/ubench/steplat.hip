// Cycles per MPPI horizon step on one wavefront (gfx950), by variant.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../motionplanning_amd/csrc/mppi_device.hpp"
using namespace mpk;
#define HH 50
template <int V>
__global__ void steps(double* out, long long* cyc, const unsigned char* grid_g) {
  __shared__ unsigned char grid[10000];
  __shared__ double unom[2 * HH];
  for (int i = threadIdx.x; i < 10000; i += 64) grid[i] = grid_g[i];
  for (int i = threadIdx.x; i < 2 * HH; i += 64) unom[i] = 0.0;
  __syncthreads();
  MppiDev P{};
  P.H = HH; P.dt = 0.15; P.lambda = 25; P.Si[0] = 20; P.Si[3] = 10; P.ctrl_cost = 1;
  const double XL[7] = {-10, -20, -2, -1.5707963267948966, -1.5707963267948966, 1, -0.3490658503988659};
  const double XU[7] = {130, 20, 2, 1.5707963267948966, 1.5707963267948966, 10, 0.3490658503988659};
  for (int i = 0; i < 7; i++) { P.XL[i] = XL[i]; P.XU[i] = XU[i]; }
  P.slack = 1e5; P.obs_pen = 71250; P.gnx = 100; P.gny = 100; P.gx0 = -10; P.gy0 = -20; P.gdx = 1.4; P.gdy = 0.4;
  const int side = threadIdx.x & 1;
  const double X0[7] = {0, 0, 0, 0, 0, 5, 0}, goal[2] = {110, 0};
  double x[7];
  for (int i = 0; i < 7; i++) x[i] = X0[i];
  double sum = 0;
  int ok = 1;
  long long t0 = clock64();
  for (int j = 0; j < HH; j++) {
    const double u[2] = {0.01 * ((threadIdx.x >> 1) % 7) - 0.03, 0.1 * ((threadIdx.x >> 1) % 5)};
    double k1[7], k2[7], x2[7];
    double cc = 0, cb = 0, pc = 0;
    int okc = 1, okb = 1;
    if (V == 0 || V == 2) {
      if (j > 0) { cc = obstacle_cost(P, x, nullptr, grid, &okc); cb = bound_cost(P, x, &okb); }
      pc = run_cost(x, u[0], u[1]);
    }
    dyn_pair(x, u[0], u[1], k1, side);
    for (int i = 0; i < 7; i++) x2[i] = x[i] + k1[i] * P.dt;
    if (V != 3) dyn_pair(x2, u[0], u[1], k2, side);
    else for (int i = 0; i < 7; i++) k2[i] = k1[i];
    for (int i = 0; i < 7; i++) x[i] = x[i] + P.dt * (k1[i] + k2[i]) / 2;
    if (V == 2) { cc += 0; }
    sum = sum + (pc + cb + cc);
    ok &= okc & okb;
  }
  long long t1 = clock64();
  out[threadIdx.x] = sum + x[0] + x[4] + ok + goal[0];
  if (threadIdx.x == 0) *cyc = t1 - t0;
}
template <int V>
void run(const char* name, const unsigned char* g) {
  double* out; long long* cyc; long long h;
  hipMalloc(&out, 64 * 8); hipMalloc(&cyc, 8);
  steps<V><<<1, 64>>>(out, cyc, g); hipDeviceSynchronize();
  steps<V><<<1, 64>>>(out, cyc, g); hipDeviceSynchronize();
  hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
  printf("%-40s %8.1f cycles/step\n", name, (double)h / HH);
}
int main() {
  unsigned char* g; hipMalloc(&g, 10000); hipMemset(g, 0, 10000);
  run<0>("full step (costs + 2x dyn)", g);
  run<1>("2x dyn + RK2 update only", g);
  run<3>("1x dyn + update", g);
  return 0;
}
