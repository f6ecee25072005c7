// Micro-benchmark: dependent-chain latency of one 2x2 pinv on gfx950 (a lone wave):
// mpj_pinv2 (Julia pinv = LAPACK dgesdd 2x2 path) vs the round-1/2 closed-form SVD, and a plain
// fp64 division and sqrt chain for scale.  Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../include/mp_jlmath.h"
__device__ void pinv_closed(const double* M, double* Pm) {
  const double E = (M[0] + M[3]) / 2, F = (M[0] - M[3]) / 2, G = (M[2] + M[1]) / 2, H = (M[2] - M[1]) / 2;
  const double Q = mpj_sqrt(E * E + H * H), R = mpj_sqrt(F * F + G * G);
  const double sx = Q + R, sy = Q - R;
  const double a1 = mpj_atan2(G, F), a2 = mpj_atan2(H, E);
  const double th = (a2 - a1) / 2, ph = (a2 + a1) / 2;
  double st, ct, sp, cp;
  mpj_sincos(th, &st, &ct);
  mpj_sincos(ph, &sp, &cp);
  const double smax = __builtin_fabs(sx) > __builtin_fabs(sy) ? __builtin_fabs(sx) : __builtin_fabs(sy);
  const double tol = 4.440892098500626e-16 * smax;
  const double i1 = __builtin_fabs(sx) > tol ? 1.0 / sx : 0.0, i2 = __builtin_fabs(sy) > tol ? 1.0 / sy : 0.0;
  Pm[0] = ct * i1 * cp - st * i2 * sp; Pm[1] = ct * i1 * sp + st * i2 * cp;
  Pm[2] = -st * i1 * cp - ct * i2 * sp; Pm[3] = -st * i1 * sp + ct * i2 * cp;
}
template <int V>
__global__ void chain(double* out, long long* cyc, int iters) {
  double M[4] = {3.0 + threadIdx.x * 1e-3, 0.7, -0.4, 2.0};
  long long t0 = clock64();
  for (int i = 0; i < iters; i++) {
    double P[4];
    if (V == 0) mpj_pinv2(M, P);
    else if (V == 4) mpj_pinv2_bl(M, P);
    else if (V == 1) pinv_closed(M, P);
    else if (V == 2) { P[0] = 1.0 / M[0]; P[1] = P[2] = P[3] = 0.0; }
    else { P[0] = mpj_sqrt(M[0]); P[1] = P[2] = P[3] = 0.0; }
    M[0] = M[0] + 1e-9 * P[0]; M[1] = M[1] + 1e-9 * P[1]; M[2] = M[2] + 1e-9 * P[2]; M[3] = M[3] + 1e-9 * P[3];
  }
  long long t1 = clock64();
  out[threadIdx.x] = M[0] + M[1] + M[2] + M[3];
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
template <int V>
void run(const char* name) {
  double* out; long long* cyc;
  hipMalloc(&out, 64 * 8); hipMalloc(&cyc, 8);
  chain<V><<<1, 64>>>(out, cyc, 200); hipDeviceSynchronize();
  chain<V><<<1, 64>>>(out, cyc, 2000); hipDeviceSynchronize();
  long long h; hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
  printf("%-36s %.0f cycles per dependent step\n", name, (double)h / 2000);
  hipFree(out); hipFree(cyc);
}
int main() {
  run<0>("pinv2 (LAPACK dgesdd path)");
  run<4>("pinv2_bl (straight-line + fallback)");
  run<1>("pinv closed form (atan2+sincos)");
  run<2>("fp64 division (+ fma)");
  run<3>("fp64 sqrt (+ fma)");
  return 0;
}
