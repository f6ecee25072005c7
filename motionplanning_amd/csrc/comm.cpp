// comm.cpp — RCCL over xGMI for a single host process that drives several GPUs (the Julia host of
// north_star: one process, one mp_ctx per GPU).  mp_comm_init builds one communicator per context
// with ncclCommInitAll; collectives are enqueued on each context's own stream inside
// ncclGroupStart/End (one thread, several devices).  RCCL is loaded with dlopen on first use, so
// libmpgpu has no link-time dependency on it and a host without librccl gets MP_ERR_UNSUPPORTED
// from mp_comm_init instead of a load failure of the whole library.  The few RCCL types and entry
// points used here are declared locally (the stable NCCL 2.x C ABI), so building libmpgpu does not
// need the RCCL headers either.
#include <dlfcn.h>

#include <mutex>
#include <vector>

#include "runtime.hpp"

// NCCL 2.x ABI (rccl.h): ncclComm_t is an opaque pointer, ncclResult_t / ncclDataType_t are C enums
typedef struct ncclComm* ncclComm_t;
typedef int ncclResult_t;
static constexpr ncclResult_t ncclSuccess = 0;
static constexpr int ncclUint8 = 1;

namespace {

struct Rccl {
  ncclResult_t (*init_all)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  const char* (*err)(ncclResult_t) = nullptr;
  bool ok = false;
  std::string why;
};

const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      const char* e = dlerror();
      r.why = e ? e : "librccl not found";
      return;
    }
    r.init_all = (decltype(r.init_all))dlsym(h, "ncclCommInitAll");
    r.destroy = (decltype(r.destroy))dlsym(h, "ncclCommDestroy");
    r.all_gather = (decltype(r.all_gather))dlsym(h, "ncclAllGather");
    r.group_start = (decltype(r.group_start))dlsym(h, "ncclGroupStart");
    r.group_end = (decltype(r.group_end))dlsym(h, "ncclGroupEnd");
    r.err = (decltype(r.err))dlsym(h, "ncclGetErrorString");
    r.ok = r.init_all && r.destroy && r.all_gather && r.group_start && r.group_end && r.err;
    if (!r.ok) r.why = "librccl lacks a required symbol";
  });
  return r;
}

}  // namespace

struct mp_comm_group {
  std::vector<mp_ctx*> ctxs;
  std::vector<ncclComm_t> comms;
};

int mp_comm_check(mp_ctx** ctxs, int n) {
  MP_CHECK(ctxs[0], ctxs[0]->comm != nullptr, "no communicator: call mp_comm_init on these contexts first");
  mp_comm_group* g = ctxs[0]->comm;
  MP_CHECK(ctxs[0], (int)g->ctxs.size() == n, "communicator spans %d contexts, call passes %d",
           (int)g->ctxs.size(), n);
  for (int i = 0; i < n; i++)
    MP_CHECK(ctxs[0], ctxs[i] == g->ctxs[i], "context %d is not rank %d of the communicator (same order as mp_comm_init)",
             i, i);
  return MP_OK;
}

int mp_comm_allgather(mp_ctx** ctxs, int n, void* const* send, void* const* recv, size_t bytes) {
  int st = mp_comm_check(ctxs, n);
  if (st) return st;
  const Rccl& R = rccl();
  mp_comm_group* g = ctxs[0]->comm;
  int dev0 = 0;
  hipGetDevice(&dev0);
  ncclResult_t e = R.group_start();
  bool dev_ok = true;
  for (int i = 0; i < n && e == ncclSuccess; i++) {
    if (hipSetDevice(ctxs[i]->device) != hipSuccess) {
      dev_ok = false;  // leave the loop, but still close the group below
      break;
    }
    e = R.all_gather(send[i], recv[i], bytes, ncclUint8, g->comms[i], ctxs[i]->stream);
  }
  const ncclResult_t e2 = R.group_end();  // always: a group left open would poison the next RCCL call
  hipSetDevice(dev0);
  if (!dev_ok) return mp_fail(ctxs[0], MP_ERR_HIP, "hipSetDevice failed inside the all-gather group");
  if (e == ncclSuccess) e = e2;
  if (e != ncclSuccess) return mp_fail(ctxs[0], MP_ERR_HIP, "ncclAllGather: %s", R.err(e));
  return MP_OK;
}

extern "C" {

int mp_comm_init(mp_ctx** ctxs, int32_t n) {
  if (!ctxs || n < 1) return mp_fail(nullptr, MP_ERR_INVALID, "mp_comm_init: need n >= 1 contexts");
  for (int i = 0; i < n; i++)
    if (!ctxs[i]) return mp_fail(nullptr, MP_ERR_INVALID, "mp_comm_init: context %d is NULL", i);
  for (int i = 0; i < n; i++) {
    MP_CHECK(ctxs[0], ctxs[i]->comm == nullptr, "context %d already belongs to a communicator", i);
    for (int j = 0; j < i; j++)
      MP_CHECK(ctxs[0], ctxs[i]->device != ctxs[j]->device, "contexts %d and %d share device %d (one context per GPU)",
               j, i, ctxs[i]->device);
  }
  const Rccl& R = rccl();
  if (!R.ok) return mp_fail(ctxs[0], MP_ERR_UNSUPPORTED, "RCCL unavailable: %s", R.why.c_str());
  mp_comm_group* g = new mp_comm_group();
  g->ctxs.assign(ctxs, ctxs + n);
  g->comms.assign(n, nullptr);
  std::vector<int> devs(n);
  for (int i = 0; i < n; i++) devs[i] = ctxs[i]->device;
  const ncclResult_t e = R.init_all(g->comms.data(), n, devs.data());
  if (e != ncclSuccess) {
    delete g;
    return mp_fail(ctxs[0], MP_ERR_HIP, "ncclCommInitAll(%d devices): %s", n, R.err(e));
  }
  for (int i = 0; i < n; i++) {
    ctxs[i]->comm = g;
    ctxs[i]->comm_rank = i;
  }
  return MP_OK;
}

int mp_comm_destroy(mp_ctx** ctxs, int32_t n) {
  if (!ctxs || n < 1 || !ctxs[0]) return MP_ERR_INVALID;
  int st = mp_comm_check(ctxs, n);
  if (st) return st;
  mp_comm_group* g = ctxs[0]->comm;
  for (int i = 0; i < n; i++) {
    hipSetDevice(ctxs[i]->device);
    mp_sync_all(ctxs[i]);
    rccl().destroy(g->comms[i]);
    ctxs[i]->comm = nullptr;
    ctxs[i]->comm_rank = -1;
  }
  delete g;
  return MP_OK;
}

int mp_comm_allgather_dev(mp_ctx** ctxs, int32_t n, void* const* send, void* const* recv, size_t bytes) {
  if (!ctxs || n < 1 || !ctxs[0] || !send || !recv) return MP_ERR_INVALID;
  for (int i = 0; i < n; i++) MP_CHECK(ctxs[0], send[i] && recv[i], "buffer %d is NULL", i);
  return mp_comm_allgather(ctxs, n, send, recv, bytes);
}

}  // extern "C"
