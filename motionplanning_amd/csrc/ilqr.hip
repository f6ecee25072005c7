// ilqr.hip — placeholder entry points (implemented in a later milestone).
#include "runtime.hpp"
extern "C" {
int mp_ilqr_rollout(mp_ctx* c, const mp_ilqr_params*, int32_t, const double*, const double*, double*, double*) {
  return mp_fail(c, MP_ERR_UNSUPPORTED, "iLQR not built yet");
}
int mp_ilqr_backward(mp_ctx* c, const mp_ilqr_params*, int32_t, const double*, const double*, double*, double*) {
  return mp_fail(c, MP_ERR_UNSUPPORTED, "iLQR not built yet");
}
int mp_ilqr_forward(mp_ctx* c, const mp_ilqr_params*, int32_t, const double*, const double*, const double*,
                    const double*, const double*, double*, double*, double*) {
  return mp_fail(c, MP_ERR_UNSUPPORTED, "iLQR not built yet");
}
int mp_ilqr_solve(mp_ctx* c, const mp_ilqr_params*, int32_t, double*, double*, double*, int32_t*) {
  return mp_fail(c, MP_ERR_UNSUPPORTED, "iLQR not built yet");
}
}
