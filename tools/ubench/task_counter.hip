// a reduced kernel of the dynamic task protocol the first ilqr_backward_fused_kernel used
// (and that hung): 7 worker waves of a 512-thread block fetch tasks from a shared LDS counter -- lane 0's LDS
// atomic, broadcast to the wave -- and run them in order; wave 0 consumes them through per-slot LDS ready
// counts, as the fused kernel's sweep does.  Every task records how often it ran (global atomics) and each
// worker loop is capped (4x the task count), so a miscompiled fetch shows up as a task run twice / never, not
// as a hang.  Variants: the broadcast by v_readfirstlane (0) or by __shfl (1); the fetch after a divergent
// branch inside the loop body (2).  Build: hipcc --offload-arch=gfx950 -O3 task_counter.hip -o task_counter;
// ISA: add --save-temps (the worker loop: ds_add_rtn_u32, s_waitcnt lgkmcnt(0), v_readfirstlane_b32).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

constexpr int NW = 7, NTASK = 200, RG = 4;

template <int V>
__global__ __launch_bounds__(64 * (1 + NW)) void tasks(int* runs, int* order, int* fails) {
  __shared__ int ctr, ready[RG], consumed;
  __shared__ double ring[RG][64];
  __shared__ double scratch[NW + 1][64];  // variant 2's divergent branch writes only its own wave's row
  const int tid = threadIdx.x, lane = tid & 63;
  if (tid == 0) { ctr = 0; consumed = 0; }
  if (tid < 64 * (NW + 1)) scratch[tid >> 6][tid & 63] = 0.0;
  if (tid < RG) ready[tid] = 0;
  __syncthreads();
  if (tid >= 64) {
    for (int it = 0; it < 4 * NTASK; it++) {  // capped: a rerun shows up in runs[], not as a hang
      if (V == 2 && (lane & 1)) {  // a divergent branch before the fetch (reconverges at its end)
        scratch[tid >> 6][lane] += 1.0;
      }
      int t = 0;
      if (lane == 0) t = __hip_atomic_fetch_add(&ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      t = V == 1 ? __shfl(t, 0) : __builtin_amdgcn_readfirstlane(t);
      if (t >= NTASK) break;
      const int slot = t % RG;
      if (t >= RG)  // the slot's previous task consumed
        while (__hip_atomic_load(&consumed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < t - RG + 1)
          __builtin_amdgcn_s_sleep(1);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      double v = t;
      for (int k = 0; k < 20; k++) v = v * 1.0000001 + lane;  // some work
      ring[slot][lane] = v;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      if (lane == 0) {
        atomicAdd(runs + t, 1);
        __hip_atomic_fetch_add(ready + slot, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
    return;
  }
  // consumer (wave 0): task t in order, from slot t % RG once written (t / RG + 1 writes into the slot)
  for (int t = 0; t < NTASK; t++) {
    const int slot = t % RG;
    int spins = 0;
    while (__hip_atomic_load(ready + slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < t / RG + 1) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1 << 22)) {  // bounded: report instead of hanging
        if (lane == 0) atomicAdd(fails, 1);
        return;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    double v = t;
    for (int k = 0; k < 20; k++) v = v * 1.0000001 + lane;
    if (ring[slot][lane] != v) atomicAdd(fails + 1, 1);  // the consumed record is task t's
    if (lane == 0) order[t] = t;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_store(&consumed, t + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
}

template <int V>
int run(const char* name) {
  int *runs, *order, *fails;
  hipMalloc(&runs, NTASK * 4);
  hipMalloc(&order, NTASK * 4);
  hipMalloc(&fails, 8);
  int bad = 0;
  for (int rep = 0; rep < 200; rep++) {
    hipMemset(runs, 0, NTASK * 4);
    hipMemset(order, 0xff, NTASK * 4);
    hipMemset(fails, 0, 8);
    tasks<V><<<256, 64 * (1 + NW)>>>(runs, order, fails);  // 256 blocks: one per CU
    hipDeviceSynchronize();
    std::vector<int> r(NTASK), o(NTASK), f(2);
    hipMemcpy(r.data(), runs, NTASK * 4, hipMemcpyDeviceToHost);
    hipMemcpy(o.data(), order, NTASK * 4, hipMemcpyDeviceToHost);
    hipMemcpy(f.data(), fails, 8, hipMemcpyDeviceToHost);
    // runs[] sums over the 256 blocks: each task exactly once per block
    for (int t = 0; t < NTASK; t++) bad += (r[t] != 256) + (o[t] != t);
    bad += f[0] + f[1];
  }
  printf("%-34s 200 launches x 256 blocks x %d tasks: %s (%d mismatches)\n", name, NTASK, bad ? "FAIL" : "ok", bad);
  hipFree(runs);
  hipFree(order);
  hipFree(fails);
  return bad;
}

int main() {
  int bad = run<0>("lane-0 LDS atomic + readfirstlane");
  bad += run<1>("lane-0 LDS atomic + __shfl");
  bad += run<2>("fetch after a divergent branch");
  return bad ? 1 : 0;
}
