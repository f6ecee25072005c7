// diag.hip — device evaluation of the shared FDLIBM restatement (include/mp_jlmath.h).
#include "../../include/mp_jlmath.h"
#include "runtime.hpp"

namespace {
__global__ void math_kernel(int fn, long long n, const double* x, const double* y, double* out) {
  __shared__ double atab[20];
  if (threadIdx.x == 0) mpj_atan_tab_init(atab);
  __syncthreads();
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double a = x[i];
  double r = 0.0;
  switch (fn) {
    case 0: r = mpj_sin(a); break;
    case 1: r = mpj_cos(a); break;
    case 2: r = mpj_tan(a); break;
    case 3: r = mpj_atan(a); break;
    case 4: r = mpj_atan2(a, y[i]); break;
    case 5: r = mpj_asin(a); break;
    case 6: r = mpj_acos(a); break;
    case 7: r = mpj_exp(a); break;
    case 8: r = mpj_log(a); break;
    case 9: r = mpj_modpi(a); break;
    case 10: r = mpj_sqrt(a); break;
    // branch-free device variants used by the hot kernels (must equal the exact routines)
    case 11: r = mpj_modpi_bl(a); break;
    case 12: r = mpj_atan_bl(a); break;
    case 13: r = mpj_atan_tab(a, atab); break;
    case 14: { double s, c; mpj_sincos_bl(a, &s, &c); r = s; break; }
    case 15: { double s, c; mpj_sincos_bl(a, &s, &c); r = c; break; }
    case 16: r = mpj_exp_fdlibm(a); break;
    case 17: r = mpj_tan_bl(a); break;
    case 18: r = mpj_atan2_sel(a, y[i]); break;
    case 19: { double s, c; int b = 0; mpj_sincos_wide(a, &s, &c, &b); r = b ? mpj_sin(a) : s; break; }
    case 20: { double s, c; int b = 0; mpj_sincos_wide(a, &s, &c, &b); r = b ? mpj_cos(a) : c; break; }
    case 21: { int b = 0; r = mpj_tan_wide(a, &b); r = b ? mpj_tan(a) : r; break; }
    case 22: r = mpj_sin_34(a); break;
    case 23: r = mpj_log_bl(a); break;
  }
  out[i] = r;
}
}  // namespace

extern "C" int mp_math_eval(mp_ctx* ctx, int32_t fn, int64_t n, const double* x, const double* y, double* out) {
  if (!ctx) return MP_ERR_INVALID;
  MP_CHECK(ctx, fn >= 0 && fn <= 23 && n >= 0 && x && out && ((fn != 4 && fn != 18) || y), "bad mp_math_eval arguments");
  if (n == 0) return MP_OK;
  MP_HIP(ctx, hipSetDevice(ctx->device));
  int st = MP_OK;
  const double* dx = mp_upload(ctx, WS_IO0, x, (size_t)n, &st);
  const double* dy = mp_upload(ctx, WS_IO1, (fn == 4 || fn == 18) ? y : nullptr, (size_t)n, &st);
  double* dout = mp_alloc_out(ctx, WS_IO2, out, (size_t)n, &st);
  if (st) return st;
  hipLaunchKernelGGL(math_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream, fn, (long long)n, dx,
                     dy, dout);
  MP_HIP(ctx, hipGetLastError());
  if ((st = mp_download(ctx, out, (const double*)dout, (size_t)n))) return st;
  MP_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return MP_OK;
}
