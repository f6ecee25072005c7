// Back-to-back dispatch gap on one stream for launch shapes like mppi_plan_kernel's
// (2,048 workgroups x 512 threads, ~100 KB dynamic LDS): run under
//   rocprofv3 --kernel-trace --stats -d DIR -o run --output-format csv -- ./gap
// and take Start(i+1) - End(i) per kernel name (tools/ubench/gap_stats.py).
// Each kernel spins ~spin_ns per wave so the launch is long enough to be "real".
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <chrono>

__global__ void k_spin(int spin, double* out) {
  extern __shared__ double lds[];
  double a = threadIdx.x;
  for (int i = 0; i < spin; i++) a = a * 0.999999 + 1e-9;
  if (a == -1.0) out[0] = a + lds[0];  // never true: keeps the loop
}
__global__ void k_spin_store(int spin, double* out, size_t n) {
  double a = threadIdx.x;
  for (int i = 0; i < spin; i++) a = a * 0.999999 + 1e-9;
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x, nt = (size_t)gridDim.x * blockDim.x;
  for (size_t i = t; i < n; i += nt) out[i] = a;
}

// plan-shaped kernel whose last block publishes a sequence number in signal memory (the side
// stream's hipStreamWaitValue64 dependency instead of an event packet on the main stream)
__global__ void k_spin_sig(int spin, double* out, unsigned* cnt, unsigned long long* sig) {
  extern __shared__ double lds[];
  double a = threadIdx.x;
  for (int i = 0; i < spin; i++) a = a * 0.999999 + 1e-9;
  if (a == -1.0) out[0] = a + lds[0];
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    if (atomicAdd(cnt, 1u) == gridDim.x - 1) {
      *cnt = 0;
      __hip_atomic_fetch_add(sig, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

#define CK(x)                                                             \
  do {                                                                    \
    hipError_t e_ = (x);                                                  \
    if (e_ != hipSuccess) {                                               \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                            \
    }                                                                     \
  } while (0)

int main() {
  double* buf;
  const size_t n = (size_t)64 << 20 >> 3;  // 64 MB of doubles
  CK(hipMalloc(&buf, n * 8));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  CK(hipFuncSetAttribute((const void*)k_spin, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  const int reps = 100;
  // 1: small grid, no LDS
  for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k_spin, dim3(256), dim3(64), 0, s, 20000, buf);
  // 2: plan-shaped grid, no LDS
  for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k_spin, dim3(2048), dim3(512), 0, s, 20000, buf);
  // 3: plan-shaped grid, 70 KB dynamic LDS (two blocks per CU)
  for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k_spin, dim3(2048), dim3(512), 70 * 1024, s, 20000, buf);
  // 4: plan-shaped grid writing 64 MB (dirty lines at kernel end)
  for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k_spin_store, dim3(2048), dim3(512), 0, s, 20000, buf, n);
  CK(hipStreamSynchronize(s));
  // the plan loop's pattern (mppi.hip mp_mppi_plan_dev, final_stream = 1): a plan-shaped kernel
  // (256 x 512, one block per CU) launched with timing events on the dispatch packet, then on a
  // side stream: wait on the stop event, a small kernel, an event in a ring of 4 the host syncs
  hipStream_t s2;
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t evf[4], evp[4], t0[reps], t1[reps];
  for (int i = 0; i < 4; i++) {
    CK(hipEventCreateWithFlags(&evf[i], hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&evp[i], hipEventDisableTiming));
    CK(hipEventRecord(evf[i], s2));
  }
  for (int i = 0; i < reps; i++) {
    CK(hipEventCreate(&t0[i]));
    CK(hipEventCreate(&t1[i]));
  }
  const int spin = 16000, side_spin = 3000;
  unsigned* cnt;
  unsigned long long* sig;
  CK(hipMalloc(&cnt, 4));
  CK(hipMemset(cnt, 0, 4));
  CK(hipExtMallocWithFlags((void**)&sig, 8, hipMallocSignalMemory));
  CK(hipMemset(sig, 0, 8));
  CK(hipDeviceSynchronize());
  unsigned long long seq = 0;
  CK(hipFuncSetAttribute((const void*)k_spin_sig, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  // 0: events on the dispatch + side wait on stop   1: plain + event record + side wait
  // 2: events on the dispatch only                  3: plain
  // 4: plain, last block bumps a signal, side hipStreamWaitValue64   5: events on every 8th launch only
  for (int mode = 0; mode < 6; mode++) {
    const auto w0 = std::chrono::steady_clock::now();
    for (int r = 0; r < reps; r++) {
      const int par = r & 3;
      const bool side = mode < 2 || mode == 4;
      if (side) CK(hipEventSynchronize(evf[par]));
      int sp = spin;
      const bool ev = mode == 0 || mode == 2 || (mode == 5 && r % 8 == 0);
      hipEvent_t a = ev ? t0[r] : nullptr, b = ev ? t1[r] : nullptr;
      if (mode == 4) {
        void* args[] = {(void*)&sp, (void*)&buf, (void*)&cnt, (void*)&sig};
        CK(hipExtLaunchKernel((const void*)k_spin_sig, dim3(256 - mode), dim3(512), args, 70 * 1024, s, a, b, 0));
      } else {
        void* args[] = {(void*)&sp, (void*)&buf};
        CK(hipExtLaunchKernel((const void*)k_spin, dim3(256 - mode), dim3(512), args, 70 * 1024, s, a, b, 0));
      }
      if (side) {
        if (mode == 4) {
          CK(hipStreamWaitValue64(s2, sig, ++seq, hipStreamWaitValueGte, ~0ull));
        } else {
          hipEvent_t done = b;
          if (!done) {
            done = evp[par];
            CK(hipEventRecord(done, s));
          }
          CK(hipStreamWaitEvent(s2, done, 0));
        }
        hipLaunchKernelGGL(k_spin_store, dim3(8), dim3(64), 0, s2, side_spin, buf, (size_t)4096);
        CK(hipEventRecord(evf[par], s2));
      }
    }
    CK(hipStreamSynchronize(s));
    CK(hipStreamSynchronize(s2));
    const double wall = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - w0).count() / reps;
    float ms = 0;
    if (mode != 1 && mode != 3 && mode != 4) CK(hipEventElapsedTime(&ms, t0[mode == 5 ? 8 : 1], t1[mode == 5 ? 8 : 1]));
    printf("mode %d: %.1f us per launch (wall), sampled kernel %.1f us\n", mode, wall, ms * 1e3);
  }
  CK(hipGetLastError());
  printf("done\n");
  return 0;
}
