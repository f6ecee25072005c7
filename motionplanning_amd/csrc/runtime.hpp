// runtime.hpp — context, error reporting and cached device workspaces for libmpgpu.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include "../../include/mpgpu.h"

// Snapshot buffers of the deferred final rollout.  A call waits (on the host) for the final
// rollout MP_FIN_RING calls back; with 4 that one finished long before, so the host stays
// ahead of the GPU and the context stream never idles between plan kernels.
#define MP_FIN_RING 4

struct mp_comm_group;  // RCCL communicators of the contexts joined by mp_comm_init (comm.cpp)

struct mp_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  // growable device scratch buffers, keyed by slot
  std::vector<void*> ws_ptr;
  std::vector<size_t> ws_size;
  // pinned host staging
  void* pinned = nullptr;
  size_t pinned_size = 0;
  // a few words of fine-grained (coherent) host memory the device writes while a plan runs (mp_mapped)
  unsigned long long* mapped = nullptr;
  unsigned long long* mapped_dev = nullptr;
  // Hybrid A* primitive table (device)
  double* ha_states_candi = nullptr;
  double* ha_paths_candi = nullptr;
  int ha_n_prim = 0, ha_n_col = 0;
  double ha_prim_ext = 0;  // max |x|, |y| of the installed primitive poses (the SAT culls' coordinate guard)
  // mp_ha_neighbor_origin's inputs for the installed table (empty: installed by mp_ha_set_primitives) and
  // its host copies, so a repeat call with the same settings neither recomputes nor re-uploads
  std::vector<double> ha_prim_key, ha_sc_host, ha_pc_host;
  // per-scene arrival counters for the MPPI last-block combine (zero at rest)
  unsigned int* tickets = nullptr;
  int n_tickets = 0;
  int* flags = nullptr;  // device status flags (NaN seen, ...)
  // optional HIP-event timing of the dominant kernel
  bool timing = false;
  std::vector<hipEvent_t> ev_pool;
  size_t ev_used = 0;
  // side stream of the deferred MPPI final rollout (mp_mppi_params.final_stream = 1):
  // plan-done / final-done events per snapshot buffer (a ring of MP_FIN_RING, by call count)
  hipStream_t side = nullptr;
  hipEvent_t ev_plan[MP_FIN_RING] = {}, ev_fin[MP_FIN_RING] = {}, ev_join = nullptr;
  int fin_par = 0;
  // cap on any one workspace slot (mp_ctx_set_workspace_limit), 0 = none
  size_t ws_limit = 0;
  // kernel attributes (150 KiB dynamic LDS) are per device: set once per context, on its device
  // (a context is used by one thread at a time, so the flags need no lock)
  bool mppi_lds_attr = false, fin_lds_attr = false;
  bool ilqr_fused_attr = false;  // the fused iLQR backward kernel's dynamic-LDS attribute is set
  int ha_pcap[3] = {-1, -1, -1};  // co-resident blocks of each ha_persist_kernel shape on this device (0: none)
  // multi-GPU in one process (mp_comm_init): the group and this context's rank in it
  mp_comm_group* comm = nullptr;
  int comm_rank = -1;
};

// Create the side stream and its events on first use.
int mp_side_init(mp_ctx* ctx);
// Wait for the context stream and (if created) the side stream.
void mp_sync_all(mp_ctx* ctx);

// Bracket a kernel launch with timing events when ctx->timing is on.
void mp_time_begin(mp_ctx* ctx);
void mp_time_end(mp_ctx* ctx);
// Timing event pair for hipExtLaunchKernel (recorded by the dispatch itself, no marker
// packets between kernels); both nullptr when timing is off.
void mp_time_pair(mp_ctx* ctx, hipEvent_t* start, hipEvent_t* stop);

// workspace slots
enum {
  WS_MPPI_PART = 0,
  WS_MPPI_COST,
  WS_MPPI_FEAS,
  WS_IO0,
  WS_IO1,
  WS_IO2,
  WS_IO3,
  WS_IO4,
  WS_IO5,
  WS_IO6,
  WS_IO7,
  WS_IO8,
  WS_IO9,
  WS_IO10,
  WS_IO11,
  WS_IO12,
  WS_IO13,
  WS_IO14,
  WS_IO15,
  WS_IO16,
  WS_NOISE,
  WS_ILQR0,
  WS_ILQR1,
  WS_ILQR2,
  WS_HA0,
  WS_HA1,
  WS_HA2,
  WS_HA3,  // Hybrid A* diagnostics (MPGPU_HA_STAMPS)
  WS_HA4,  // Hybrid A* neighbour groups' Dict records (IterArgs::drec)
  WS_FIN0,  // MPPI final-rollout snapshots, MP_FIN_RING slots
  WS_FIN_END = WS_FIN0 + MP_FIN_RING - 1,
  WS_SHARD_SEND,  // mp_mppi_plan_sharded: this rank's packed per-scene results
  WS_SHARD_RECV,  // ... and every rank's, after the all-gather
  WS_COUNT
};

int mp_fail(mp_ctx* ctx, int code, const char* fmt, ...);
// ctxs[0..n) are ranks 0..n-1 of one mp_comm_init group (error on ctxs[0] otherwise)
int mp_comm_check(mp_ctx** ctxs, int n);
// ncclAllGather of `bytes` per rank, ctxs[i]'s send[i] -> recv[i] ([n][bytes]) on each context stream
int mp_comm_allgather(mp_ctx** ctxs, int n, void* const* send, void* const* recv, size_t bytes);
void* mp_ws(mp_ctx* ctx, int slot, size_t bytes);  // nullptr on failure (error set)
// bytes currently held by a workspace slot (0 if none)
size_t mp_ws_size(mp_ctx* ctx, int slot);
// whether a slot of `bytes` may be allocated now: within the context limit and, if the slot must
// grow, within `frac` of the device's free memory (optional speed-up buffers only)
bool mp_ws_affordable(mp_ctx* ctx, int slot, size_t bytes, double frac);
int mp_ticket_reserve(mp_ctx* ctx, int n);
void* mp_pinned(mp_ctx* ctx, size_t bytes);
// 8 words of coherent host memory (host pointer; *dev = the device's address of it), nullptr on failure
unsigned long long* mp_mapped(mp_ctx* ctx, unsigned long long** dev);

#define MP_HIP(ctx, call)                                                                \
  do {                                                                                   \
    hipError_t e_ = (call);                                                              \
    if (e_ != hipSuccess)                                                                \
      return mp_fail((ctx), MP_ERR_HIP, "%s failed: %s (%s:%d)", #call, hipGetErrorString(e_), \
                     __FILE__, __LINE__);                                                \
  } while (0)

#define MP_CHECK(ctx, cond, ...)                              \
  do {                                                        \
    if (!(cond)) return mp_fail((ctx), MP_ERR_INVALID, __VA_ARGS__); \
  } while (0)

// Copy host -> device scratch slot (nullptr-safe); returns device pointer or nullptr.
template <typename T>
static inline T* mp_upload(mp_ctx* ctx, int slot, const T* host, size_t n, int* st) {
  if (!host || n == 0) return nullptr;
  T* d = (T*)mp_ws(ctx, slot, n * sizeof(T));
  if (!d) { *st = MP_ERR_NOMEM; return nullptr; }
  hipError_t e = hipMemcpyAsync(d, host, n * sizeof(T), hipMemcpyHostToDevice, ctx->stream);
  if (e != hipSuccess) { *st = mp_fail(ctx, MP_ERR_HIP, "H2D copy failed: %s", hipGetErrorString(e)); return nullptr; }
  return d;
}
template <typename T>
static inline T* mp_alloc_out(mp_ctx* ctx, int slot, const T* host, size_t n, int* st) {
  if (!host || n == 0) return nullptr;
  T* d = (T*)mp_ws(ctx, slot, n * sizeof(T));
  if (!d) *st = MP_ERR_NOMEM;
  return d;
}
template <typename T>
static inline int mp_download(mp_ctx* ctx, T* host, const T* dev, size_t n) {
  if (!host || !dev || n == 0) return MP_OK;
  MP_HIP(ctx, hipMemcpyAsync(host, dev, n * sizeof(T), hipMemcpyDeviceToHost, ctx->stream));
  return MP_OK;
}
