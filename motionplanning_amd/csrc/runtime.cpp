// runtime.cpp — libmpgpu context lifecycle, error strings, workspaces.
#include "runtime.hpp"

#include <cstdlib>
#include <cstring>

static thread_local std::string g_noctx_err;

int mp_fail(mp_ctx* ctx, int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (ctx) ctx->err = buf;
  else g_noctx_err = buf;
  return code;
}

void* mp_ws(mp_ctx* ctx, int slot, size_t bytes) {
  if (slot < 0) return nullptr;
  if ((int)ctx->ws_ptr.size() <= slot) {
    ctx->ws_ptr.resize(slot + 1, nullptr);
    ctx->ws_size.resize(slot + 1, 0);
  }
  if (bytes == 0) bytes = 16;
  if (ctx->ws_size[slot] >= bytes) return ctx->ws_ptr[slot];
  if (ctx->ws_limit && bytes > ctx->ws_limit) {
    mp_fail(ctx, MP_ERR_NOMEM, "workspace slot %d needs %zu B, above the context limit of %zu B", slot, bytes,
            ctx->ws_limit);
    return nullptr;
  }
  if (ctx->ws_ptr[slot]) {
    mp_sync_all(ctx);
    hipFree(ctx->ws_ptr[slot]);
    ctx->ws_ptr[slot] = nullptr;
    ctx->ws_size[slot] = 0;
  }
  size_t cap = bytes + bytes / 4;  // grow with headroom
  if (ctx->ws_limit && cap > ctx->ws_limit) cap = ctx->ws_limit;
  void* p = nullptr;
  if (hipMalloc(&p, cap) != hipSuccess) {
    // an out-of-memory hipMalloc is not sticky, but it stays the thread's last error: clear it so
    // the next launch check does not report it; then try without the headroom
    (void)hipGetLastError();
    p = nullptr;
    if (cap == bytes || hipMalloc(&p, bytes) != hipSuccess) {
      (void)hipGetLastError();
      mp_fail(ctx, MP_ERR_NOMEM, "hipMalloc(%zu) failed for workspace slot %d", bytes, slot);
      return nullptr;
    }
    cap = bytes;
  }
  ctx->ws_ptr[slot] = p;
  ctx->ws_size[slot] = cap;
  return p;
}

size_t mp_ws_size(mp_ctx* ctx, int slot) {
  return slot >= 0 && slot < (int)ctx->ws_size.size() ? ctx->ws_size[slot] : 0;
}

bool mp_ws_affordable(mp_ctx* ctx, int slot, size_t bytes, double frac) {
  if (mp_ws_size(ctx, slot) >= bytes) return true;
  if (ctx->ws_limit && bytes > ctx->ws_limit) return false;
  size_t fr = 0, tot = 0;
  if (hipMemGetInfo(&fr, &tot) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return (double)(bytes - mp_ws_size(ctx, slot)) <= frac * (double)fr;
}

int mp_ticket_reserve(mp_ctx* ctx, int n) {
  if (ctx->n_tickets >= n) return MP_OK;
  if (ctx->tickets) {
    mp_sync_all(ctx);
    hipFree(ctx->tickets);
    ctx->tickets = nullptr;
  }
  int cap = n < 64 ? 64 : n;
  MP_HIP(ctx, hipMalloc(&ctx->tickets, cap * sizeof(unsigned int)));
  MP_HIP(ctx, hipMemset(ctx->tickets, 0, cap * sizeof(unsigned int)));
  ctx->n_tickets = cap;
  return MP_OK;
}

void* mp_pinned(mp_ctx* ctx, size_t bytes) {
  if (ctx->pinned_size >= bytes) return ctx->pinned;
  if (ctx->pinned) hipHostFree(ctx->pinned);
  ctx->pinned = nullptr;
  ctx->pinned_size = 0;
  if (hipHostMalloc(&ctx->pinned, bytes, 0) != hipSuccess) return nullptr;
  ctx->pinned_size = bytes;
  return ctx->pinned;
}

unsigned long long* mp_mapped(mp_ctx* ctx, unsigned long long** dev) {
  if (!ctx->mapped) {
    void* h = nullptr;
    void* d = nullptr;
    if (hipHostMalloc(&h, 64, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) return nullptr;
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
      hipHostFree(h);
      return nullptr;
    }
    ctx->mapped = static_cast<unsigned long long*>(h);
    ctx->mapped_dev = static_cast<unsigned long long*>(d);
  }
  *dev = ctx->mapped_dev;
  return ctx->mapped;
}

void mp_sync_all(mp_ctx* ctx) {
  hipStreamSynchronize(ctx->stream);
  if (ctx->side) hipStreamSynchronize(ctx->side);
}

int mp_side_init(mp_ctx* ctx) {
  if (ctx->side) return MP_OK;
  MP_HIP(ctx, hipStreamCreateWithFlags(&ctx->side, hipStreamNonBlocking));
  for (int i = 0; i < MP_FIN_RING; i++) {
    MP_HIP(ctx, hipEventCreateWithFlags(&ctx->ev_plan[i], hipEventDisableTiming));
    MP_HIP(ctx, hipEventCreateWithFlags(&ctx->ev_fin[i], hipEventDisableTiming));
    MP_HIP(ctx, hipEventRecord(ctx->ev_fin[i], ctx->side));  // "buffer free" from the start
  }
  MP_HIP(ctx, hipEventCreateWithFlags(&ctx->ev_join, hipEventDisableTiming));
  return MP_OK;
}

static hipEvent_t next_event(mp_ctx* ctx) {
  if (ctx->ev_used == ctx->ev_pool.size()) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    ctx->ev_pool.push_back(e);
  }
  return ctx->ev_pool[ctx->ev_used++];
}

void mp_time_begin(mp_ctx* ctx) {
  if (!ctx->timing) return;
  hipEvent_t e = next_event(ctx);
  if (e) hipEventRecord(e, ctx->stream);
}

void mp_time_end(mp_ctx* ctx) {
  if (!ctx->timing) return;
  hipEvent_t e = next_event(ctx);
  if (e) hipEventRecord(e, ctx->stream);
}

void mp_time_pair(mp_ctx* ctx, hipEvent_t* start, hipEvent_t* stop) {
  *start = *stop = nullptr;
  if (!ctx->timing) return;
  hipEvent_t a = next_event(ctx);
  hipEvent_t b = a ? next_event(ctx) : nullptr;
  if (!a || !b) return;
  *start = a;
  *stop = b;
}

extern "C" {

int mp_ctx_kernel_timing(mp_ctx* ctx, int enable) {
  if (!ctx) return MP_ERR_INVALID;
  ctx->timing = enable != 0;
  // the event pool made up front (two per timed launch, reused after each mp_ctx_kernel_ms): creating events
  // on demand would put hipEventCreate calls between the launches being timed
  while (ctx->timing && ctx->ev_pool.size() < 512) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) break;
    ctx->ev_pool.push_back(e);
  }
  return MP_OK;
}

int mp_ctx_kernel_ms(mp_ctx* ctx, double* ms_sum, int32_t* count) {
  if (!ctx || !ms_sum || !count) return MP_ERR_INVALID;
  MP_HIP(ctx, hipStreamSynchronize(ctx->stream));
  double t = 0.0;
  int n = 0;
  for (size_t i = 0; i + 1 < ctx->ev_used; i += 2) {
    float ms = 0.f;
    MP_HIP(ctx, hipEventElapsedTime(&ms, ctx->ev_pool[i], ctx->ev_pool[i + 1]));
    t += ms;
    n++;
  }
  ctx->ev_used = 0;
  *ms_sum = t;
  *count = n;
  return MP_OK;
}

const char* mp_version(void) { return MPGPU_VERSION " (gfx950)"; }

int mp_device_count(int* n) {
  if (!n) return MP_ERR_INVALID;
  hipError_t e = hipGetDeviceCount(n);
  if (e != hipSuccess) {
    *n = 0;
    return mp_fail(nullptr, MP_ERR_HIP, "hipGetDeviceCount: %s", hipGetErrorString(e));
  }
  return MP_OK;
}

int mp_ctx_create(int device, mp_ctx** out) {
  if (!out) return MP_ERR_INVALID;
  *out = nullptr;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n == 0)
    return mp_fail(nullptr, MP_ERR_HIP, "no HIP device available (%s)", hipGetErrorString(e));
  if (device < 0 || device >= n) return mp_fail(nullptr, MP_ERR_INVALID, "device %d out of range [0,%d)", device, n);
  e = hipSetDevice(device);
  if (e != hipSuccess) return mp_fail(nullptr, MP_ERR_HIP, "hipSetDevice: %s", hipGetErrorString(e));
  mp_ctx* c = new mp_ctx();
  c->device = device;
  e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete c;
    return mp_fail(nullptr, MP_ERR_HIP, "hipStreamCreate: %s", hipGetErrorString(e));
  }
  if (hipMalloc(&c->flags, 64 * sizeof(int)) != hipSuccess) {
    hipStreamDestroy(c->stream);
    delete c;
    return mp_fail(nullptr, MP_ERR_NOMEM, "flag buffer allocation failed");
  }
  hipMemset(c->flags, 0, 64 * sizeof(int));
  *out = c;
  return MP_OK;
}

int mp_ctx_destroy(mp_ctx* ctx) {
  if (!ctx) return MP_OK;
  // a context still joined to an RCCL communicator would leave the group's other ranks with a
  // dangling rank: the caller must run mp_comm_destroy over the whole group first
  MP_CHECK(ctx, ctx->comm == nullptr, "context is rank %d of a communicator: call mp_comm_destroy first",
           ctx->comm_rank);
  hipSetDevice(ctx->device);
  mp_sync_all(ctx);
  for (void* p : ctx->ws_ptr)
    if (p) hipFree(p);
  if (ctx->pinned) hipHostFree(ctx->pinned);
  if (ctx->mapped) hipHostFree(ctx->mapped);
  if (ctx->tickets) hipFree(ctx->tickets);
  if (ctx->flags) hipFree(ctx->flags);
  for (hipEvent_t e : ctx->ev_pool) hipEventDestroy(e);
  if (ctx->ha_states_candi) hipFree(ctx->ha_states_candi);
  if (ctx->ha_paths_candi) hipFree(ctx->ha_paths_candi);
  for (int i = 0; i < MP_FIN_RING; i++) {
    if (ctx->ev_plan[i]) hipEventDestroy(ctx->ev_plan[i]);
    if (ctx->ev_fin[i]) hipEventDestroy(ctx->ev_fin[i]);
  }
  if (ctx->ev_join) hipEventDestroy(ctx->ev_join);
  if (ctx->side) hipStreamDestroy(ctx->side);
  hipStreamDestroy(ctx->stream);
  delete ctx;
  return MP_OK;
}

const char* mp_last_error(mp_ctx* ctx) {
  if (!ctx) return g_noctx_err.c_str();
  return ctx->err.c_str();
}

int mp_ctx_synchronize(mp_ctx* ctx) {
  if (!ctx) return MP_ERR_INVALID;
  MP_HIP(ctx, hipStreamSynchronize(ctx->stream));
  if (ctx->side) MP_HIP(ctx, hipStreamSynchronize(ctx->side));
  return MP_OK;
}

int mp_ctx_join(mp_ctx* ctx) {
  if (!ctx) return MP_ERR_INVALID;
  if (!ctx->side) return MP_OK;
  MP_HIP(ctx, hipEventRecord(ctx->ev_join, ctx->side));
  MP_HIP(ctx, hipStreamWaitEvent(ctx->stream, ctx->ev_join, 0));
  return MP_OK;
}

void* mp_ctx_stream(mp_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

int mp_ctx_trim(mp_ctx* ctx, size_t keep_bytes) {
  if (!ctx) return MP_ERR_INVALID;
  MP_HIP(ctx, hipSetDevice(ctx->device));
  mp_sync_all(ctx);  // in-flight work (incl. the side stream's final rollouts) may still read them
  for (size_t i = 0; i < ctx->ws_ptr.size(); i++)
    if (ctx->ws_ptr[i] && (keep_bytes == 0 || ctx->ws_size[i] > keep_bytes)) {
      MP_HIP(ctx, hipFree(ctx->ws_ptr[i]));
      ctx->ws_ptr[i] = nullptr;
      ctx->ws_size[i] = 0;
    }
  return MP_OK;
}

int mp_ctx_set_workspace_limit(mp_ctx* ctx, size_t bytes) {
  if (!ctx) return MP_ERR_INVALID;
  ctx->ws_limit = bytes;
  return MP_OK;
}

}  // extern "C"
