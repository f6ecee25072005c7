// hastar.hip — placeholder entry points (implemented in a later milestone).
#include "runtime.hpp"
extern "C" {
int mp_ha_set_primitives(mp_ctx* c, const mp_ha_params*, const double*, const double*) {
  return mp_fail(c, MP_ERR_UNSUPPORTED, "Hybrid A* not built yet");
}
int mp_ha_expand(mp_ctx* c, const mp_ha_params*, int32_t, const double*, const double*, const double*, double*,
                 int64_t*, uint8_t*, double*) {
  return mp_fail(c, MP_ERR_UNSUPPORTED, "Hybrid A* not built yet");
}
int mp_ha_rs_connect(mp_ctx* c, const mp_ha_params*, int32_t, const double*, const double*, const double*, uint8_t*,
                     double*, int32_t*) {
  return mp_fail(c, MP_ERR_UNSUPPORTED, "Hybrid A* not built yet");
}
int mp_ha_allpath(mp_ctx* c, int32_t, const double*, double*, double*, int32_t*) {
  return mp_fail(c, MP_ERR_UNSUPPORTED, "Hybrid A* not built yet");
}
int mp_ha_plan(mp_ctx* c, const mp_ha_params*, int32_t, const double*, const double*, const double*, int32_t*,
               int32_t*, int32_t*, int64_t*, int32_t*, double*, int32_t*, double*) {
  return mp_fail(c, MP_ERR_UNSUPPORTED, "Hybrid A* not built yet");
}
}
