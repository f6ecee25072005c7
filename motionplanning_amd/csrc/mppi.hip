// mppi.hip — MPPIPlan / TrajectoryRollout / plant kernels for gfx950 and their C-ABI
// entry points (include/mpgpu.h).
//
// mp_mppi_plan is ONE kernel launch per call (no memset, no host round trip):
//   phase 1  every block: NT/2 rollouts (lane pairs) — noise draw, clamp, RK2
//            dynamics and all step costs fused; per-rollout cost/flag and the
//            control list go to HBM (the TrajectoryCollection contract);
//            the two waves sharing a SIMD pace each other by issue priority
//            (MPPI_PRIO 3).  Then the block's online-softmax partial (ρ_b, η_b,
//            Σ e·u; the latter per wave over its own rollouts, from registers
//            prefetched when the wave ends) is published with agent-coherent
//            stores (sc1), every thread's stores acknowledged, then an arrival
//            ticket (round 4: no agent-scope release / acquire fences).
//   phase 2  the last block to arrive for a scene applies the
//            FeasibilityCount prefix (MPPIUtils.jl:175), combines the partials
//            with a log-sum-exp rescale into MPPICtrl (:186-190) and runs the
//            final TrajectoryRollout (:192-198).  It resets the ticket.
#include "mppi_device.hpp"
#include "runtime.hpp"

#include <hip/hip_ext.h>

#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include <vector>

using namespace mpk;

namespace {

constexpr int NT = 256;     // threads per block (4 waves)
constexpr int RPB = NT / 2; // rollouts per block
#ifndef MPPI_PRIO
#define MPPI_PRIO 3  // issue-priority scheme of the rollout loop (see ctrl()); 0 = quarters (round 2)
#endif
constexpr size_t kMaxLds = 148 * 1024;  // dynamic LDS budget per block (160 KiB per CU on gfx950)
constexpr size_t kCoLds = 72 * 1024;    // budget that keeps two blocks co-resident per CU

__device__ __forceinline__ double block_reduce_min(double v, double* sh) {
  for (int o = 32; o >= 1; o >>= 1) v = nanmin(v, __shfl_xor(v, o));
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[w] = v;
  __syncthreads();
  double r = sh[0];
  for (int i = 1; i < (int)(blockDim.x >> 6); i++) r = nanmin(r, sh[i]);
  __syncthreads();
  return r;
}

// deterministic block sum: fixed shuffle tree per wave, then waves in order
__device__ __forceinline__ double block_reduce_sum(double v, double* sh) {
  for (int o = 32; o >= 1; o >>= 1) v = v + __shfl_xor(v, o);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[w] = v;
  __syncthreads();
  double r = sh[0];
  for (int i = 1; i < (int)(blockDim.x >> 6); i++) r = r + sh[i];
  __syncthreads();
  return r;
}

struct PlanArgs {
  const double* X0;
  const double* goal;
  const double* unom;
  const double* obs;
  const unsigned char* grid;
  const double* noise;
  double* ctrl_all;    // [S][H][K][2]  (rollout index fastest: coalesced per-step stores)
  double* cost_all;    // [S][K]
  unsigned char* feas_all;  // [S][K]
  double* part;        // [S][nb][pstride]
  double* coll_traj;   // [S][H+1][7][K] or null
  unsigned* tickets;
  int* flags;
  double* U_out;
  double* traj_out;
  double* cost_out;
  int* feas_out;
  int* rc_out;
  int* fc_out;
  int nb;
  int pstride;
  int lds_unom, lds_obs, lds_grid;  // offsets (in doubles) into dynamic LDS; lds_grid < 0: grid stays in HBM
  int lds_cq;                       // control-cost rows [H][2] (ctrl_cost_row)
  int lds_ctrl, lds_part;           // control lists [RPB][2H+1] / staged partials (< 0: use HBM)
  unsigned long long* stamps;       // diagnostic build only (MPGPU_STAMPS=1): [grid][8] s_memrealtime
  int inline_noise;                 // 1: Philox draws inside the rollout loop (no noise_prep pass)
  double* fin;                      // deferred final rollout: per-scene input snapshot (FinRec), or null
  int fin_stride;                   // doubles per scene record
  const int* live;                  // closed loop: scenes with live[s] == 0 are skipped (null: all run)
};

#ifndef MPPI_NT_CTRL
#define MPPI_NT_CTRL 0
#endif

// Snapshot record of one scene for the deferred final rollout (final_stream = 1), in doubles:
// [0, 2H) MPPICtrl | [2H, 4H) U_nom | X0[7] | goal[2] | obstacles[3 n_obs] | grid bytes | ran
// `ran` (1.0 / 0.0) is written by the plan kernel of the same call: whether it planned the scene.
// The final rollout reads it, not the closed loop's live flags, which the plant kernel on the
// context stream may already have cleared for a later replan when the side stream gets there.
struct FinRec {
  int u, unom, x0, goal, obs, grid, ran, stride;
  __host__ __device__ FinRec(int H, int n_obs, int gbytes) {
    u = 0;
    unom = 2 * H;
    x0 = 4 * H;
    goal = x0 + 7;
    obs = goal + 2;
    grid = obs + 3 * n_obs;
    ran = grid + (gbytes + 7) / 8;
    stride = (ran + 2) & ~1;
  }
};

#define MP_STAMP(i)                                                                  \
  do {                                                                               \
    if (A.stamps && threadIdx.x == 0) {                                              \
      A.stamps[blockIdx.x * 32 + (i)] = __builtin_amdgcn_s_memrealtime();            \
      if ((i) == 0) {                                                                \
        unsigned xcc;                                                                \
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));           \
        A.stamps[blockIdx.x * 32 + 30] = xcc;                                        \
      }                                                                              \
    }                                                                                \
  } while (0)
// per-wave phase-1 end time [8 + w] and HW_ID (SIMD placement) [20 + w], diagnostic build only
#define MP_STAMP_WAVE()                                                              \
  do {                                                                               \
    if (A.stamps && (threadIdx.x & 63) == 0) {                                       \
      unsigned hwid;                                                                 \
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));             \
      A.stamps[blockIdx.x * 32 + 8 + (threadIdx.x >> 6)] = __builtin_amdgcn_s_memrealtime(); \
      A.stamps[blockIdx.x * 32 + 20 + (threadIdx.x >> 6)] = hwid;                    \
    }                                                                                \
  } while (0)

// Noise for every (scene, step, rollout), h-major [S][H][K][2] so the rollout's
// per-step read is one coalesced 16-B load per lane pair.  Philox draws are
// generated here by the whole GPU (409,600 independent Box–Muller pairs at
// cfg2) instead of sitting on the rollouts' serial per-step critical path;
// MP_NOISE_EXTERNAL input [S][K][H][2] is transposed into the same layout.
__global__ __launch_bounds__(256) void noise_prep_kernel(MppiDev P, int S, const double* ext, double* zh) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long n = (long long)S * P.H * P.K;
  if (i >= n) return;
  const int k = (int)(i % P.K);
  const long long t = i / P.K;
  const int h = (int)(t % P.H), s = (int)(t / P.H);
  double z[2];
  if (P.noise_mode == 0) {
    const double2 e = *reinterpret_cast<const double2*>(ext + (((size_t)s * P.K + k) * P.H + h) * 2);
    z[0] = e.x;
    z[1] = e.y;
  } else {
    philox_normal2(P, (unsigned)s, (unsigned)k, (unsigned)h, z);
  }
  reinterpret_cast<double2*>(zh)[i] = make_double2(z[0], z[1]);
}

// Agent-coherent relaxed stores / loads (global_store / global_load with the sc1 policy): the records
// one block hands to the scene's last block (block partials, per-rollout costs and feasibility flags)
// reach the device coherence point directly, so the arrival needs no agent-scope release fence (an L2
// write-back of the whole XCD) and the last block no acquire (L1/L2 invalidate).
template <class T>
__device__ __forceinline__ void st_ag(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T>
__device__ __forceinline__ T ld_ag(const T* p) {
  return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// The arrival of a block's records at the scene's last block.  0 (default): each thread's records
// acknowledged (vmcnt), then an agent-scope release fence before the relaxed ticket and an acquire fence in
// the last block -- ordered within the HIP/HSA memory model.  1 (A/B): the records are agent-coherent stores
// and the ticket relaxed, ordered by the per-thread vmcnt wait alone (sound on gfx94x/95x hardware, but
// outside the language model); round 4 measured no gain from it (profiles/r04w_mppi_coherent_ha_scan_ab.txt),
// so the fenced form is the default.
#ifndef MPPI_COHERENT_PARTS
#define MPPI_COHERENT_PARTS 0
#endif

// BT threads per block (4 or 8 waves); LPR lanes per rollout: 2 = lane pair (dyn_pair, the
// two tire chains on the two lanes), 1 = one rollout per lane (dyn_lane) when the launch has a
// rollout per lane for every SIMD.  BT/LPR rollouts per block.
// INL: device Philox noise drawn inside the rollout loop (else the caller's noise, transposed
// by noise_prep_kernel): a compile-time mode, so the rollout loop carries neither the other
// mode's registers nor its branch (measured 318 -> 306 us per 8-scene launch, 224 -> 212 us single scene).
template <int BT, int LPR, bool INL>
__global__ __launch_bounds__(BT) void mppi_plan_kernel(MppiDev P, PlanArgs A) {
  constexpr int NT = BT, RPB = BT / LPR, NQ = BT / 128;
  // WPART: the block partial Σ e·u is formed per wave over the wave's own 32 rollouts (lane pair
  // layout, H <= 64), with the HBM control lists prefetched into registers as soon as the wave's
  // rollouts end -- their latency then hides behind the block's slower waves and the reductions.
  constexpr bool WPART = LPR == 2;
  __shared__ double sh_red[NT / 64];
  __shared__ double sh_e[RPB];
  __shared__ double sh_q[WPART ? NT / 64 : NQ][128];  // per-wave (WPART) or per-quarter control sums
  __shared__ int sh_last, sh_m, sh_bstar, sh_fc;
  __shared__ double sh_eta;
  __shared__ double atab[20];  // mpj_atan_tab range constants
  extern __shared__ double dyn[];
  const int H = P.H, H2 = 2 * H, K = P.K;
  const int s = blockIdx.x / A.nb, b = blockIdx.x % A.nb;
  const int tid = threadIdx.x, pair = LPR == 2 ? tid >> 1 : tid, side = LPR == 2 ? tid & 1 : 0;
  const int k = b * RPB + pair;
  const bool active = k < K;
  const int kk = active ? k : K - 1;
  if (A.live && A.live[s] == 0) {  // closed loop: this scene has reached its goal (block-uniform)
    if (A.fin && b == 0 && tid == 0) A.fin[(size_t)s * A.fin_stride + FinRec(H, P.n_obs, P.gnx * P.gny).ran] = 0.0;
    return;
  }
  MP_STAMP(0);
  __builtin_amdgcn_s_setprio(3);

  const double* X0 = A.X0 + 7 * s;
  const double* goal = A.goal + 2 * s;
  const double* noise = A.noise ? A.noise + (size_t)K * H2 * s : nullptr;  // h-major [H][K][2] (noise_prep_kernel)
  // Stage the scene's read-only inputs in LDS: the rollout loop then issues no
  // global loads but the prefetched noise, so no s_waitcnt vmcnt ever waits on
  // the (uncoalesced) TrajectoryCollection stores (CDNA4 vmcnt counts stores).
  double* unom = dyn + A.lds_unom;
  double* obs = A.obs ? dyn + A.lds_obs : nullptr;
  double* ush = A.lds_ctrl >= 0 ? dyn + A.lds_ctrl : nullptr;  // [RPB][H2+1] this block's control lists
  const int ustr = H2 + 1;
  const unsigned char* grid = nullptr;
  {
    const double* gu = A.unom + (size_t)H2 * s;
    if (tid == 0) mpj_atan_tab_init(atab);
    for (int i = tid; i < H2; i += NT) unom[i] = gu[i];
    if (P.ctrl_cost)
      for (int i = tid; i < H; i += NT) ctrl_cost_row(P, gu[2 * i], gu[2 * i + 1], dyn + A.lds_cq + 2 * i);
    if (A.obs) {
      const double* go = A.obs + (size_t)3 * P.n_obs * s;
      for (int i = tid; i < 3 * P.n_obs; i += NT) obs[i] = go[i];
    }
    if (A.grid) {
      const int gb = P.gnx * P.gny;
      const unsigned char* gg = A.grid + (size_t)gb * s;
      if (A.lds_grid >= 0) {
        unsigned char* lg = reinterpret_cast<unsigned char*>(dyn + A.lds_grid);
        for (int i = tid; i < gb; i += NT) lg[i] = gg[i];
        grid = lg;
      } else {
        grid = gg;
      }
    }
    __syncthreads();
  }
  double* ctrl_g = A.ctrl_all ? A.ctrl_all + ((size_t)s * H * K + kk) * 2 + side : nullptr;  // LPR 1: + 0

#if MPPI_PRIO == 3
  // Sibling-paced issue priority: each wave publishes its step in LDS and finds the other wave of the
  // block on its SIMD (HW_ID.SIMD_ID); per step it drops below the sibling when ahead of it and rises
  // above it when behind, so the pair ends together instead of one wave finishing the horizon alone.
  __shared__ int sh_simd[NT / 64];
  __shared__ volatile int sh_prog[NT / 64];
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  int sib = -1;
  {
    unsigned hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    if ((tid & 63) == 0) {
      sh_simd[wv] = (int)((hw >> 4) & 3u);
      sh_prog[wv] = 0;
    }
    __syncthreads();
    const int me = sh_simd[wv];
    for (int w = 0; w < NT / 64; w++)
      if (w != wv && sh_simd[w] == me) sib = w;
    sib = __builtin_amdgcn_readfirstlane(sib);
  }
  int sib_j = 0;
#endif
  // ---------------- phase 1: the rollout of this lane pair
  int feas;
  double c;
  {
    // z for step j+1 is loaded at the top of step j: the wait for it never covers
    // the TrajectoryCollection stores issued later in the step.
    // Inline Philox (device noise): the pair draws two steps at once, the even lane step j and
    // the odd lane step j+1 (one instruction stream, lane-varying counter), and swaps: one
    // Box–Muller per lane per two steps, issued into the dynamics chain's latency bubbles.
    const double2* zrow = noise ? reinterpret_cast<const double2*>(noise) + kk : nullptr;
    double2 zc = zrow ? zrow[0] : make_double2(0.0, 0.0), zn = zc;
    auto ctrl = [&](int j, double* u) {
      double2 zj;
      if (INL && LPR == 1) {
        double zz[2];
        philox_normal2(P, (unsigned)s, (unsigned)kk, (unsigned)j, zz);
        zj = make_double2(zz[0], zz[1]);
      } else if (INL) {
        if ((j & 1) == 0) {
          double zz[2];
          philox_normal2(P, (unsigned)s, (unsigned)kk, (unsigned)(j + side), zz);
          const double o0 = pair_swap(zz[0]), o1 = pair_swap(zz[1]);
          zj = side ? make_double2(o0, o1) : make_double2(zz[0], zz[1]);
          zn = side ? make_double2(zz[0], zz[1]) : make_double2(o0, o1);
        } else {
          zj = zn;
        }
      } else {
        zj = zc;
        if (j + 1 < H) zc = zrow[(size_t)(j + 1) * K];
      }
      const double z[2] = {zj.x, zj.y};
      sample_ctrl(P, z, unom + 2 * j, u);
      // Self-balancing issue priority: a wave's priority drops by one per quarter of the
      // horizon it has completed, so the waves sharing a SIMD (oldest-first arbitration
      // otherwise lets one run ahead and leaves the other to finish alone) end together.
#if MPPI_PRIO == 0
      if ((4 * j) % H < 4 && j > 0) {
        const int q = (4 * j) / H;
        if (q == 1) __builtin_amdgcn_s_setprio(2);
        else if (q == 2) __builtin_amdgcn_s_setprio(1);
        else if (q == 3) __builtin_amdgcn_s_setprio(0);
      }
#elif MPPI_PRIO == 3
      if (sib >= 0) {
        // sib_j was read one step ago (its LDS latency hidden behind the step)
        const int o = __builtin_amdgcn_readfirstlane(sib_j);
        if (j > o) __builtin_amdgcn_s_setprio(0);
        else if (j < o) __builtin_amdgcn_s_setprio(2);
        else __builtin_amdgcn_s_setprio(1);
        sh_prog[wv] = j;
        sib_j = sh_prog[sib];
      } else if ((4 * j) % H < 4 && j > 0) {  // no sibling in the block on this SIMD: quarter levels
        const int q = (4 * j) / H;
        if (q == 1) __builtin_amdgcn_s_setprio(2);
        else if (q == 2) __builtin_amdgcn_s_setprio(1);
        else if (q == 3) __builtin_amdgcn_s_setprio(0);
      }
#else
      // (A/B) levels crowded towards the end of the horizon, where a lag turns into lone-wave time:
      // 1: H/2, 3H/4, 7H/8;  2: H-12, H-6, H-3
      if (j > 0) {
        const int t1 = MPPI_PRIO == 1 ? H / 2 : H - 12, t2 = MPPI_PRIO == 1 ? 3 * H / 4 : H - 6,
                  t3 = MPPI_PRIO == 1 ? 7 * H / 8 : H - 3;
        if (j == t1) __builtin_amdgcn_s_setprio(2);
        else if (j == t2) __builtin_amdgcn_s_setprio(1);
        else if (j == t3) __builtin_amdgcn_s_setprio(0);
      }
#endif
    };
    auto store = [&](int j, const double* u) {
      if (LPR == 2) {
        if (ush) ush[pair * ustr + 2 * j + side] = u[side];
        if (ctrl_g) {
#if MPPI_NT_CTRL
          __builtin_nontemporal_store(u[side], ctrl_g + (size_t)j * K * 2);
#else
          ctrl_g[(size_t)j * K * 2] = u[side];
#endif
        }
      } else {
        if (ush) {
          ush[pair * ustr + 2 * j] = u[0];
          ush[pair * ustr + 2 * j + 1] = u[1];
        }
        if (ctrl_g) *reinterpret_cast<double2*>(ctrl_g + (size_t)j * K * 2) = make_double2(u[0], u[1]);
      }
    };
    // inactive pairs (k >= K) recompute rollout K-1 and write identical values
    const TrajOut traj{A.coll_traj ? A.coll_traj + (size_t)s * (H + 1) * 7 * K + kk : nullptr, 7LL * K, (long long)K};
    c = rollout_pair<LPR>(P, X0, goal, obs, grid, unom, side, ctrl, store, traj, &feas, atab, dyn + A.lds_cq);
  }
  MP_STAMP(1);
  MP_STAMP_WAVE();
  if (active && side == 0) {
    st_ag(A.cost_all + (size_t)s * K + k, c);
    st_ag(A.feas_all + (size_t)s * K + k, (unsigned char)feas);
    if (c != c) atomicOr(A.flags, 1);
  }
  // ---------------- block partial (online softmax), MPPIUtils.jl:154-167
  // WPART: lane l of wave w sums outputs t = l and l + 64 (t = 2h + side) over the wave's rollouts
  // [32w, 32w + nr) of the block in rollout order; the block value is then the wave sums added in
  // wave order.  Single- and multi-scene launches share this order (scene batching invariance).
  const int wid = tid >> 6, lane = tid & 63;
  const bool wp = WPART && H2 <= 128;  // block-uniform
  const int nr = wp ? max(0, min(32, K - b * RPB - 32 * wid)) : 0;  // wave-uniform
  // The register prefetch only in the 8-wave (multi-scene) kernels: it holds 128 VGPRs across the
  // reductions, which slowed the 4-wave single-scene kernel's rollout loop (LDS path anyway).
  constexpr bool PREF = BT == 512;
  double v0[32], v1[32];
  if (PREF && wp && !ush) {
    // this wave's own control-list stores -> its own loads (same wave, same CU): wait for the stores
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const double* cb = A.ctrl_all + (((size_t)s * H + (lane >> 1)) * K + (size_t)b * RPB + 32 * wid) * 2 + (lane & 1);
    const size_t up = (size_t)64 * K;  // t + 64 is step h + 32, same side
#pragma unroll
    for (int r = 0; r < 32; r++) v0[r] = (r < nr && lane < H2) ? cb[2 * r] : 0.0;
    if (H2 > 64) {
#pragma unroll
      for (int r = 0; r < 32; r++) v1[r] = (r < nr && lane + 64 < H2) ? cb[up + 2 * r] : 0.0;
    }
  }
  const double cm = active ? c : __builtin_inf();
  const double rho_b = block_reduce_min(cm, sh_red);
  const double e = active ? mpj_exp(P.nil * (c - rho_b)) : 0.0;
  if (side == 0) sh_e[pair] = e;
  const double eta_b = block_reduce_sum(side == 0 ? e : 0.0, sh_red);
  const double fc_b = block_reduce_sum((side == 0 && active && feas) ? 1.0 : 0.0, sh_red);
  __syncthreads();  // control-list stores of this block -> visible to its own loads below (same CU)
  double* part = A.part + ((size_t)s * A.nb + b) * A.pstride;
  if (wp) {
    const double* ew = sh_e + 32 * wid;
    double a0 = 0.0, a1 = 0.0;
    if (ush) {
      const double* uw = ush + (size_t)(32 * wid) * ustr + lane;
      for (int r = 0; r < nr; r++) {
        const double er = ew[r];
        if (lane < H2) a0 = a0 + er * uw[r * ustr];
        if (lane + 64 < H2) a1 = a1 + er * uw[r * ustr + 64];
      }
    } else if (PREF) {
#pragma unroll
      for (int r = 0; r < 32; r++) {
        if (r < nr) {
          const double er = ew[r];
          a0 = a0 + er * v0[r];
          if (H2 > 64) a1 = a1 + er * v1[r];
        }
      }
    } else {  // the same sums, loads issued here
      const double* cb = A.ctrl_all + (((size_t)s * H + (lane >> 1)) * K + (size_t)b * RPB + 32 * wid) * 2 + (lane & 1);
      const size_t up = (size_t)64 * K;
      for (int r = 0; r < nr; r++) {
        const double er = ew[r];
        if (lane < H2) a0 = a0 + er * cb[2 * r];
        if (lane + 64 < H2) a1 = a1 + er * cb[up + 2 * r];
      }
    }
    sh_q[wid][lane] = a0;
    sh_q[wid][lane + 64] = a1;
    __syncthreads();
    if (tid < H2) {
      double v = sh_q[0][tid];
#pragma unroll
      for (int w = 1; w < NT / 64; w++) v = v + sh_q[w][tid];
      st_ag(part + 4 + tid, v);
    }
  } else {
    // Σ_i e_i u_i[t] over this block's rollouts; fixed quarters per output, summed in order
    const int t = tid % 128, q = tid / 128;
    const int r0 = q * (RPB / NQ), r1 = r0 + RPB / NQ;
    for (int t0 = 0; t0 < H2; t0 += 128) {  // block-uniform trip count: barriers are safe
      const int tt = t0 + t;
      double acc = 0.0;
      if (tt < H2) {
        if (ush) {
          for (int r = r0; r < r1; r++) acc = acc + sh_e[r] * ush[r * ustr + tt];
        } else {
          // independent loads: issue 16 before consuming (L2 latency, not a serial chain)
          const double* cb = A.ctrl_all + (((size_t)s * H + (tt >> 1)) * K + (size_t)b * RPB) * 2 + (tt & 1);
          const int rmax = min(r1, K - b * RPB);
#pragma unroll 16
          for (int r = r0; r < rmax; r++) acc = acc + sh_e[r] * cb[(size_t)r * 2];
        }
      }
      sh_q[q][t] = acc;
      __syncthreads();
      if (q == 0 && tt < H2) {
        double v = sh_q[0][t];
#pragma unroll
        for (int i = 1; i < NQ; i++) v = v + sh_q[i][t];
        st_ag(part + 4 + tt, v);
      }
      __syncthreads();
    }
  }
  if (tid == 0) {
    st_ag(part + 0, rho_b);
    st_ag(part + 1, eta_b);
    st_ag(part + 2, fc_b);
  }
  // ---------------- arrival: every thread's records acknowledged, then the ticket
  MP_STAMP(2);
  // (__syncthreads() on gfx950 waits for LDS only: each thread waits for its own stores first, so the
  // partial written by waves 1.. is complete before wave 0 takes the ticket)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    if (!MPPI_COHERENT_PARTS) {
      __threadfence();  // agent-scope release: write back this XCD's L2
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const unsigned t = __hip_atomic_fetch_add(A.tickets + s, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sh_last = (t == (unsigned)(A.nb - 1));
    // the last block reads the partials agent-coherently while it stages them in LDS; without the
    // stage (too little LDS) it reads them with plain loads, after an acquire
    if (sh_last && (!MPPI_COHERENT_PARTS || A.lds_part < 0)) {
      __threadfence();  // agent-scope acquire: invalidate this CU's L1
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  MP_STAMP(3);
  if (!sh_last) return;

  // ---------------- phase 2: combine + final rollout (last block of scene s)
  double* Ush = dyn;         // [H2]
  double* scale = dyn + H2;  // [nb]
  // every partial record of the scene, staged with independent coalesced loads
  const double* partG = A.part + (size_t)s * A.nb * A.pstride;
  const double* partS = partG;
  if (A.lds_part >= 0) {
    double* pl = dyn + A.lds_part;
    const int n = A.nb * A.pstride;
    for (int i = tid; i < n; i += NT) pl[i] = ld_ag(partG + i);
    __syncthreads();
    partS = pl;
  }
  // FeasibilityCount prefix (MPPIUtils.jl:175): m = rollouts actually run
  if (tid == 0) {
    int tot = 0;
    for (int i = 0; i < A.nb; i++) tot += (int)partS[(size_t)i * A.pstride + 2];
    int m = K, bstar = A.nb, fcount = tot;
    if (tot > P.FC) {
      int cum = 0;
      for (int i = 0; i < A.nb; i++) {
        const int f = (int)partS[(size_t)i * A.pstride + 2];
        if (cum + f > P.FC) { bstar = i; break; }
        cum += f;
      }
      for (int r = 0; r < RPB; r++) {
        const int kr = bstar * RPB + r;
        cum += ld_ag(A.feas_all + (size_t)s * K + kr);
        if (cum == P.FC + 1) { m = kr + 1; break; }
      }
      fcount = P.FC + 1;
    }
    sh_m = m;
    sh_bstar = (m == K) ? A.nb : bstar;
    sh_fc = fcount;
  }
  __syncthreads();
  const int m = sh_m, nfull = sh_bstar;  // blocks [0, nfull) complete; [nfull*RPB, m) partial
  // partial boundary block, recomputed from the stored costs and regenerated controls
  double rho_p = __builtin_inf(), eta_p = 0.0;
  const int p0 = nfull * RPB;
  const bool has_p = p0 < m;
  if (has_p) {
    const int kr = p0 + pair;
    const bool in = kr < m;
    const double cr = in ? ld_ag(A.cost_all + (size_t)s * K + kr) : __builtin_inf();
    rho_p = block_reduce_min(cr, sh_red);
    const double er = in ? mpj_exp(P.nil * (cr - rho_p)) : 0.0;
    if (side == 0) sh_e[pair] = er;
    eta_p = block_reduce_sum(side == 0 ? er : 0.0, sh_red);
  }
  __syncthreads();
  // global ρ
  double rho = rho_p;
  for (int i = tid; i < nfull; i += NT) rho = nanmin(rho, partS[(size_t)i * A.pstride]);
  rho = block_reduce_min(rho, sh_red);
  for (int i = tid; i < nfull; i += NT) scale[i] = mpj_exp(P.nil * (partS[(size_t)i * A.pstride] - rho));
  __syncthreads();
  const double scale_p = has_p ? mpj_exp(P.nil * (rho_p - rho)) : 0.0;
  // η and MPPICtrl = Σ_b scale_b Σ_i e_i u_i  /  η      (fixed order over blocks)
  if (tid == 0) {
    double eta = 0.0;
    for (int i = 0; i < nfull; i++) eta = eta + partS[(size_t)i * A.pstride + 1] * scale[i];
    if (has_p) eta = eta + eta_p * scale_p;
    sh_eta = eta;
  }
  __syncthreads();
  const double inv_eta = 1.0 / sh_eta;
  const double* noiseS = A.noise ? A.noise + (size_t)K * H2 * s : nullptr;
  for (int t = tid; t < H2; t += NT) {
    double acc = 0.0;
#pragma unroll 8
    for (int i = 0; i < nfull; i++) acc = acc + partS[(size_t)i * A.pstride + 4 + t] * scale[i];
    if (has_p) {
      double ap = 0.0;
      for (int r = 0; r < m - p0; r++) {
        const int kr = p0 + r, h = t >> 1;
        double u[2];
        double z[2];
        if (INL) {
          philox_normal2(P, (unsigned)s, (unsigned)kr, (unsigned)h, z);
        } else {
          const double2 zz = reinterpret_cast<const double2*>(noiseS)[(size_t)h * K + kr];
          z[0] = zz.x;
          z[1] = zz.y;
        }
        sample_ctrl(P, z, unom + 2 * h, u);
        ap = ap + sh_e[r] * u[t & 1];
      }
      acc = acc + ap * scale_p;
    }
    Ush[t] = acc * inv_eta;
  }
  __syncthreads();
  MP_STAMP(4);
  for (int t = tid; t < H2; t += NT) A.U_out[(size_t)s * H2 + t] = Ush[t];
  if (tid == 0) {
    A.rc_out[s] = m + 1;
    A.fc_out[s] = sh_fc;
    A.tickets[s] = 0u;  // every block of this scene has arrived
    if (rho != rho) atomicOr(A.flags, 1);
  }
  if (A.fin) {
    // deferred final rollout (final_rollout_kernel on the side stream): snapshot its inputs
    const FinRec R(H, P.n_obs, P.gnx * P.gny);
    double* rec = A.fin + (size_t)s * A.fin_stride;
    for (int t = tid; t < H2; t += NT) {
      rec[R.u + t] = Ush[t];
      rec[R.unom + t] = unom[t];
    }
    if (tid < 7) rec[R.x0 + tid] = X0[tid];
    if (tid == 0) rec[R.ran] = 1.0;
    if (tid < 2) rec[R.goal + tid] = goal[tid];
    for (int i = tid; i < 3 * P.n_obs; i += NT) rec[R.obs + i] = obs[i];
    if (grid) {
      unsigned char* rg = reinterpret_cast<unsigned char*>(rec + R.grid);
      for (int i = tid; i < P.gnx * P.gny; i += NT) rg[i] = grid[i];
    }
    MP_STAMP(5);
    return;
  }
  // final TrajectoryRollout(MPPICtrl) on wave 0 only (its 32 pairs run it redundantly, all write
  // the same values): the other waves leave, so the serial tail owns its SIMD instead of
  // sharing it with an identical copy
  if (tid >= 64) return;
  __builtin_amdgcn_s_setprio(3);  // the serial tail first on its SIMD
  {
    auto ctrl = [&](int j, double* u) { u[0] = Ush[2 * j]; u[1] = Ush[2 * j + 1]; };
    auto store = [&](int, const double*) {};
    const TrajOut traj{A.traj_out + (size_t)s * (H + 1) * 7, 7, 1};  // every pair writes the same values
    int f2;
    const double c2 = rollout_pair(P, X0, goal, obs, grid, unom, tid & 1, ctrl, store, traj, &f2, atab);
    if (tid == 0) {
      A.cost_out[s] = c2;
      A.feas_out[s] = f2;
      if (c2 != c2) atomicOr(A.flags, 1);
    }
  }
  MP_STAMP(5);
}

// Deferred final TrajectoryRollout(MPPICtrl) (MPPIUtils.jl:192-198), one wave per scene on the
// context's side stream, from the FinRec snapshot the plan kernel's last block wrote: the
// same rollout_pair as the in-kernel tail (bit-identical outputs), while the next call's
// rollouts already occupy the rest of the GPU.
__global__ __launch_bounds__(64) void final_rollout_kernel(MppiDev P, const double* fin, int fin_stride,
                                                           int grid_lds, double* traj_out, double* cost_out,
                                                           int* feas_out, int* flags) {
  extern __shared__ double fsh[];
  __shared__ double atab[20];
  const int s = blockIdx.x, tid = threadIdx.x, side = tid & 1, H = P.H;
  const FinRec R(H, P.n_obs, P.gnx * P.gny);
  const double* rec = fin + (size_t)s * fin_stride;
  if (rec[R.ran] == 0.0) return;  // closed loop: the plan kernel of this call skipped the scene
  const int nw = grid_lds ? R.stride : R.grid;  // the grid stays in the record when it does not fit
  for (int i = tid; i < nw; i += 64) fsh[i] = rec[i];
  if (tid == 0) mpj_atan_tab_init(atab);
  __syncthreads();
  // issue priority 0 (lowest): the serial chain fills the issue bubbles of the next call's
  // rollout waves on its SIMD instead of delaying them (the plan kernel ends with its slowest
  // SIMD); measured: prio 0 -> 354 us plan kernel, prio 3 -> 379 us (cfg2, 8 scenes)
  const double* U = fsh + R.u;
  auto ctrl = [&](int j, double* u) { u[0] = U[2 * j]; u[1] = U[2 * j + 1]; };
  auto store = [&](int, const double*) {};
  const unsigned char* grid =
      P.gnx > 0 ? reinterpret_cast<const unsigned char*>((grid_lds ? fsh : rec) + R.grid) : nullptr;
  const TrajOut traj{traj_out + (size_t)s * (H + 1) * 7, 7, 1};
  int f2;
  const double c2 = rollout_pair(P, fsh + R.x0, fsh + R.goal, P.n_obs > 0 ? fsh + R.obs : nullptr, grid,
                                 fsh + R.unom, side, ctrl, store, traj, &f2, atab);
  if (tid == 0) {
    cost_out[s] = c2;
    feas_out[s] = f2;
    if (c2 != c2) atomicOr(flags, 1);
  }
}

// ------------------------------------------------------------- mp_rollout
__global__ __launch_bounds__(NT) void rollout_kernel(MppiDev P, int K, const double* X0, const double* goal,
                                                     const double* ctrl, long long cs, const double* unom,
                                                     const double* obs, const unsigned char* grid, double* traj,
                                                     double* cost, unsigned char* feas, int nb) {
  const int H = P.H;
  const int s = blockIdx.x / nb, b = blockIdx.x % nb;
  const int tid = threadIdx.x, pair = tid >> 1, side = tid & 1;
  __shared__ double atab[20];
  if (tid == 0) mpj_atan_tab_init(atab);
  __syncthreads();
  const int k = b * RPB + pair;
  const bool active = k < K;
  const int kk = active ? k : K - 1;
  const double* cu = ctrl + ((size_t)s * K + kk) * (cs ? (size_t)cs * H : 2);
  auto cf = [&](int j, double* u) {
    const double* q = cu + (size_t)j * cs;
    u[0] = q[0];
    u[1] = q[1];
  };
  auto store = [&](int, const double*) {};
  const TrajOut tr{(traj && active) ? traj + ((size_t)s * K + k) * (H + 1) * 7 : nullptr, 7, 1};
  int f;
  const double c = rollout_pair(P, X0 + 7 * s, goal + 2 * s, obs ? obs + (size_t)3 * P.n_obs * s : nullptr,
                                grid ? grid + (size_t)P.gnx * P.gny * s : nullptr,
                                unom ? unom + (size_t)2 * H * s : nullptr, side, cf, store, tr, &f, atab);
  if (active && side == 0) {
    cost[(size_t)s * K + k] = c;
    feas[(size_t)s * K + k] = (unsigned char)f;
  }
}

// first minimum per scene with Julia isless semantics (DWAUtils.jl:152 `minimum`)
__global__ __launch_bounds__(NT) void argmin_kernel(int K, const double* cost, int* out) {
  __shared__ double sv[NT];
  __shared__ int si[NT];
  const int s = blockIdx.x;
  double bv = 0.0;
  int bi = -1;
  for (int i = threadIdx.x; i < K; i += NT) {
    const double v = cost[(size_t)s * K + i];
    if (bi < 0 || mpj_isless(v, bv)) { bv = v; bi = i; }
  }
  sv[threadIdx.x] = bv;
  si[threadIdx.x] = bi;
  __syncthreads();
  if (threadIdx.x == 0) {
    double v = sv[0];
    int ix = si[0];
    for (int t = 1; t < NT; t++) {
      if (si[t] < 0) continue;
      if (ix < 0 || mpj_isless(sv[t], v) || (!mpj_isless(v, sv[t]) && si[t] < ix)) { v = sv[t]; ix = si[t]; }
    }
    out[s] = ix;
  }
}

// ------------------------------------------------------------ plant (Euler)
// MPPI/main.jl:259-261: states .+= VehicleDynamics(states, u)*δt; one lane pair per vehicle
__global__ __launch_bounds__(64) void euler_kernel(int n, double* states, const double* ctrl, double dt,
                                                   int nsteps, double* his) {
  const int tid = blockIdx.x * 64 + threadIdx.x;
  const int v = tid >> 1, side = tid & 1;
  const int vv = v < n ? v : n - 1;
  __shared__ double atab[20];
  if (threadIdx.x == 0) mpj_atan_tab_init(atab);
  __syncthreads();
  double x[7], d[7];
  for (int i = 0; i < 7; i++) x[i] = states[7 * vv + i];
  const double sr = ctrl[2 * vv], ax = ctrl[2 * vv + 1];
  for (int t = 0; t < nsteps; t++) {
    dyn_pair(x, sr, ax, d, side, atab);
    for (int i = 0; i < 7; i++) x[i] = x[i] + d[i] * dt;
    if (his && v < n && side == 0)
      for (int i = 0; i < 7; i++) his[((size_t)v * nsteps + t) * 7 + i] = x[i];
  }
  if (v < n && side == 0)
    for (int i = 0; i < 7; i++) states[7 * v + i] = x[i];
}


// ------------------------------------------------------- closed loop (plant)
// One replan period of the MPPI closed loop (MPPI/main.jl:55-83) for every scene: the plant
// `states .+= VehicleDynamics(states, u)·δt` for time_idx = step0+1 .. step0+nsub with the
// zero-order-held control row hold[i] of this replan's MPPICtrl, one history row per step and
// the goal check after it.  One lane pair per scene (dyn_pair); every lane runs the same trip
// count (no divergent wave ops in the FDLIBM cores), a finished scene's lanes just stop writing.
// rows: [S][max_steps+1][8] = [time_idx·δt, x...]; st[0..S) n_rows, st[S..2S) live,
// st[2S..3S) n_replans.
__global__ __launch_bounds__(64) void loop_plant_kernel(int S, int H, double* states, const double* U,
                                                        const int* hold, int nsub, double dt, const double* goal,
                                                        double r2, int step0, int max_steps, double* rows, int* st,
                                                        int r) {
  const int tid = blockIdx.x * 64 + threadIdx.x;
  const int v = tid >> 1, side = tid & 1;
  const int vv = v < S ? v : S - 1;
  __shared__ double atab[20];
  if (threadIdx.x == 0) mpj_atan_tab_init(atab);
  __syncthreads();
  int* n_rows = st;
  int* live = st + S;
  int* n_replans = st + 2 * S;
  int act = v < S && live[vv];
  const int act0 = act;
  if (act && side == 0) n_replans[vv] = r + 1;
  double x[7], d[7];
#pragma unroll
  for (int i = 0; i < 7; i++) x[i] = states[7 * vv + i];
  const double g0 = goal[2 * vv], g1 = goal[2 * vv + 1];
  double* row = rows + (size_t)vv * (max_steps + 1) * 8;
  if (step0 == 0 && act && side == 0) {
    row[0] = 0.0;
#pragma unroll
    for (int i = 0; i < 7; i++) row[1 + i] = x[i];
  }
  const double* u = U + (size_t)vv * H * 2;
  int last = step0;
  for (int i = 0; i < nsub; i++) {
    const int t = step0 + i + 1;
    if (t > max_steps) break;  // uniform: the run's time_idx range ends (main.jl:55)
    const int h = hold[i];
    dyn_pair(x, u[2 * h], u[2 * h + 1], d, side, atab);
#pragma unroll
    for (int k = 0; k < 7; k++) x[k] = x[k] + d[k] * dt;
    if (act) {
      last = t;
      if (side == 0) {
        double* q = row + (size_t)t * 8;
        q[0] = (double)t * dt;
#pragma unroll
        for (int k = 0; k < 7; k++) q[1 + k] = x[k];
      }
      const double ex = x[0] - g0, ey = x[1] - g1;
      if (ex * ex + ey * ey <= r2) {  // main.jl:77-79: break after this step's row
        if (side == 0) live[vv] = 0;
        act = 0;
      }
    }
  }
  if (act0 && side == 0) {
    n_rows[vv] = last + 1;
    if (act) {  // still running after the period: carry the state into the next replan
#pragma unroll
      for (int k = 0; k < 7; k++) states[7 * vv + k] = x[k];
      if (last >= max_steps) live[vv] = 0;
    }
  }
}

// ------------------------------------------------------ sharded plan (RCCL)
// One scene's results packed for the all-gather of mp_mppi_plan_sharded, in doubles:
// [U_out 2H | traj_out 7(H+1) | cost | feasible | rollout_count | feasible_count]
__host__ __device__ inline int shard_rec(int H) { return 2 * H + 7 * (H + 1) + 4; }

__global__ __launch_bounds__(256) void shard_pack_kernel(int S, int H, const double* U, const double* traj,
                                                         const double* cost, const int* feas, const int* rc,
                                                         const int* fc, double* out) {
  const int D = shard_rec(H), nu = 2 * H, nt = 7 * (H + 1);
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)S * D) return;
  const int s = (int)(i / D), j = (int)(i % D);
  double v;
  if (j < nu) v = U[(size_t)s * nu + j];
  else if (j < nu + nt) v = traj[(size_t)s * nt + (j - nu)];
  else {
    const int q = j - nu - nt;
    v = q == 0 ? cost[s] : q == 1 ? (double)feas[s] : q == 2 ? (double)rc[s] : (double)fc[s];
  }
  out[i] = v;
}

// ----------------------------------------------------------------- host
static void inv2(const double* A, double* Ai) {
  const double a = A[0], b = A[1], c = A[2], d = A[3];
  if (b == 0.0 && c == 0.0) {
    Ai[0] = 1.0 / a; Ai[1] = 0.0; Ai[2] = 0.0; Ai[3] = 1.0 / d;
    return;
  }
  const bool swap = __builtin_fabs(c) > __builtin_fabs(a);
  const double p11 = swap ? c : a, p12 = swap ? d : b, q11 = swap ? a : c, q12 = swap ? b : d;
  const double l = q11 / p11, u22 = q12 - l * p12;
  const double iu11 = 1.0 / p11, iu22 = 1.0 / u22, iu12 = -(p12 * iu11) * iu22;
  const double m11 = iu11 - iu12 * l, m12 = iu12, m21 = -iu22 * l, m22 = iu22;
  if (swap) { Ai[0] = m12; Ai[1] = m11; Ai[2] = m22; Ai[3] = m21; }
  else { Ai[0] = m11; Ai[1] = m12; Ai[2] = m21; Ai[3] = m22; }
}

static int make_dev_params(mp_ctx* ctx, const mp_mppi_params* p, int K, MppiDev* D) {
  MP_CHECK(ctx, p != nullptr, "params is NULL");
  MP_CHECK(ctx, K >= 1, "SamplingNumber K (%d) must be >= 1", K);
  MP_CHECK(ctx, p->H >= 1 && p->H <= 4096, "horizon N (%d) must be in [1, 4096]", p->H);
  MP_CHECK(ctx, p->n_obs >= 0, "n_obs (%d) must be >= 0", p->n_obs);
  MP_CHECK(ctx, p->dt > 0.0, "dt (%g) must be > 0", p->dt);
  MP_CHECK(ctx, p->grid_nx >= 0 && p->grid_ny >= 0, "grid dims must be >= 0");
  MP_CHECK(ctx, p->noise_mode == MP_NOISE_EXTERNAL || p->noise_mode == MP_NOISE_PHILOX, "bad noise_mode %d",
           p->noise_mode);
  MP_CHECK(ctx, p->calls_in_flight >= 0 && p->calls_in_flight <= 64, "calls_in_flight (%d) must be in [0, 64]",
           p->calls_in_flight);
  D->in_flight = p->calls_in_flight > 1 ? p->calls_in_flight : 1;
  D->K = K;
  D->H = p->H;
  D->FC = p->feasibility_count;
  D->n_obs = p->n_obs;
  D->dt = p->dt;
  D->lambda = p->lambda;
  D->nil = (-1.0) / p->lambda;
  const double* S = p->sigma;
  MP_CHECK(ctx, S[0] > 0.0, "Σ must be positive definite");
  const double l11 = __builtin_sqrt(S[0]);
  const double l21 = S[2] / l11;
  const double r22 = S[3] - l21 * l21;
  MP_CHECK(ctx, r22 > 0.0, "Σ must be positive definite");
  D->L[0] = l11; D->L[1] = 0.0; D->L[2] = l21; D->L[3] = __builtin_sqrt(r22);
  inv2(S, D->Si);
  for (int i = 0; i < 7; i++) { D->XL[i] = p->XL[i]; D->XU[i] = p->XU[i]; }
  for (int i = 0; i < 2; i++) { D->CL[i] = p->CL[i]; D->CU[i] = p->CU[i]; }
  D->slack = p->slack_penalty;
  D->obs_pen = p->obs_penalty;
  D->gnx = p->grid_nx;
  D->gny = p->grid_ny;
  D->gx0 = p->grid_x0; D->gy0 = p->grid_y0; D->gdx = p->grid_dx; D->gdy = p->grid_dy;
  D->noise_mode = p->noise_mode;
  D->ctrl_cost = p->ctrl_cost;
  D->seed = p->seed;
  D->offset = p->offset;
  D->scene_base = p->scene_base;
  return MP_OK;
}

// the plan kernel instance for a block size, lanes per rollout and noise source
using PlanFn = void (*)(MppiDev, PlanArgs);
static PlanFn plan_kernel_for(int BT, int LPR, bool inl) {
#define MP_PLAN_CASE(bt, lpr) \
  if (BT == bt && LPR == lpr) return inl ? mppi_plan_kernel<bt, lpr, true> : mppi_plan_kernel<bt, lpr, false>;
  MP_PLAN_CASE(128, 1)
  MP_PLAN_CASE(128, 2)
  MP_PLAN_CASE(256, 1)
  MP_PLAN_CASE(256, 2)
  MP_PLAN_CASE(512, 1)
  MP_PLAN_CASE(512, 2)
#undef MP_PLAN_CASE
  return nullptr;
}

static int plan_launch(mp_ctx* ctx, const MppiDev& D, int S, const double* X0, const double* goal,
                       const double* U_nom, const double* obstacles, const uint8_t* grid, const double* noise,
                       double* U_out, double* traj_out, double* cost_out, int32_t* feasible_out,
                       int32_t* rc_out, int32_t* fc_out, double* coll_traj, double* coll_ctrl,
                       double* coll_cost, uint8_t* coll_feas, int final_stream, const int* live = nullptr) {
  const int K = D.K, H = D.H;
  // 8-wave blocks once the launch fills every CU with one (the dispatcher then places
  // exactly two waves per SIMD; with 4-wave blocks, two per CU, it can stack 3 + 1 and
  // the slowest SIMD sets the end time), else 4-wave blocks for more CUs at small S.
  // One rollout per lane once that gives every SIMD two waves (S*K >= 2 x 256 CUs x 4 SIMDs x
  // 64 lanes).  Measured (cfg2, K=8192, H=50): 16 scenes, LPR 1 (2 waves/SIMD, the tire chains
  // interleaved in a lane, costs evaluated once) 0.536 ms vs LPR 2 (4 waves/SIMD) 0.703 ms;
  // 8 scenes, LPR 1 (1 wave/SIMD) 0.384 ms vs LPR 2 (2 waves/SIMD) 0.375 ms: a lone wave
  // cannot cover the fp64 dependency latency.
  // With n calls in flight on n contexts (calls_in_flight), the other calls' waves fill the SIMDs too, so the
  // rollouts of all of them count: 8 scenes, two calls alternating over two contexts, LPR 1 1.17-1.19e10
  // rollout-steps/s against LPR 2 1.08-1.10e10; three calls 1.31e10 (r06y, bench driver arguments).
  // (test hook) MPGPU_LPR = 1 / 2 forces the layout: the results are the same bits either way
  // (tests/test_gpu_mppi_lane.py), only the launch shape changes
  const char* lpr_s = getenv("MPGPU_LPR");
  const int lpr_env = lpr_s ? atoi(lpr_s) : 0;
  const int LPR = lpr_env == 1 || lpr_env == 2 ? lpr_env : ((size_t)S * K * D.in_flight >= 131072 ? 1 : 2);
  // Single scene (64 blocks): BT 128 (2 waves per CU on 128 CUs) 0.278 ms vs BT 256 (4 waves, one per
  // SIMD, on 64 CUs) 0.242 ms -- a CU's four SIMDs each holding one wave beat half-filled CUs.
  const int BT = LPR == 1 ? ((size_t)S * ((K + 511) / 512) >= 256 ? 512 : 256)
                          : ((size_t)S * ((K + 255) / 256) >= 256 ? 512 : 256);
  const int RPBh = BT / LPR;
  const int nb = (K + RPBh - 1) / RPBh;
  const int pstride = 4 + 2 * H;
  PlanArgs A;
  A.live = live;
  A.X0 = X0; A.goal = goal; A.unom = U_nom; A.obs = D.n_obs > 0 ? obstacles : nullptr;
  A.grid = D.gnx > 0 ? grid : nullptr;
  A.inline_noise = D.noise_mode == MP_NOISE_PHILOX;
  A.noise = nullptr;
  if (!A.inline_noise) {  // caller's z (parity mode): transposed h-major by noise_prep_kernel
    double* zh = (double*)mp_ws(ctx, WS_NOISE, sizeof(double) * (size_t)S * K * H * 2);
    if (!zh) return MP_ERR_NOMEM;
    const long long n = (long long)S * K * H;
    hipLaunchKernelGGL(noise_prep_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream, D, S, noise,
                       zh);
    MP_HIP(ctx, hipGetLastError());
    A.noise = zh;
  }
  A.cost_all = coll_cost ? coll_cost : (double*)mp_ws(ctx, WS_MPPI_COST, sizeof(double) * (size_t)S * K);
  A.feas_all = coll_feas ? coll_feas : (unsigned char*)mp_ws(ctx, WS_MPPI_FEAS, (size_t)S * K);
  A.part = (double*)mp_ws(ctx, WS_MPPI_PART, sizeof(double) * (size_t)S * nb * pstride);
  if (!A.cost_all || !A.feas_all || !A.part) return MP_ERR_NOMEM;
  A.coll_traj = coll_traj;
  int st = mp_ticket_reserve(ctx, S);
  if (st) return st;
  A.tickets = ctx->tickets;
  A.flags = ctx->flags;
  A.U_out = U_out; A.traj_out = traj_out; A.cost_out = cost_out; A.feas_out = feasible_out;
  A.rc_out = rc_out; A.fc_out = fc_out;
  A.nb = nb;
  A.pstride = pstride;
  // dynamic LDS: [phase-2: 2H + nb] [unom: 2H] [obs: 3 n_obs] [grid bytes] [control lists | staged partials]
  int off = 2 * H + nb;
  A.lds_unom = off;
  off += 2 * H;
  A.lds_cq = off;
  off += 2 * H;
  A.lds_obs = off;
  off += 3 * D.n_obs;
  const size_t gbytes = (size_t)D.gnx * D.gny;
  A.lds_grid = -1;
  if (D.gnx > 0 && (size_t)off * 8 + gbytes <= 48 * 1024) {
    A.lds_grid = off;
    off += (int)((gbytes + 7) / 8);
  }
  // Control lists / staged partials in LDS only while two blocks still fit per CU
  // (multi-scene launches need every block co-resident); otherwise the HBM path.
  const int ctrl_words = RPBh * (2 * H + 1), part_words = nb * pstride;
  A.lds_ctrl = A.lds_part = -1;
  const bool many = (size_t)S * nb > 256;  // more blocks than CUs: keep two per CU resident
  const size_t budget = many ? kCoLds : kMaxLds;
  if ((size_t)(off + (ctrl_words > part_words ? ctrl_words : part_words)) * 8 <= budget) {
    A.lds_ctrl = A.lds_part = off;
    off += ctrl_words > part_words ? ctrl_words : part_words;
  } else if ((size_t)(off + part_words) * 8 <= budget) {
    A.lds_part = off;
    off += part_words;
  }
  // control lists in HBM: the TrajectoryCollection output, or the fallback when LDS is too small
  A.ctrl_all = coll_ctrl;
  if (A.lds_ctrl < 0 && !A.ctrl_all) {
    A.ctrl_all = (double*)mp_ws(ctx, WS_IO14, sizeof(double) * (size_t)S * K * 2 * H);
    if (!A.ctrl_all) return MP_ERR_NOMEM;
  }
  const size_t shmem = sizeof(double) * (size_t)off;
  MP_CHECK(ctx, shmem <= kMaxLds, "K/H/obstacles too large for one scene (dynamic LDS %zu B)", shmem);
  if (!ctx->mppi_lds_attr) {
    MP_HIP(ctx, hipSetDevice(ctx->device));  // the attribute applies to the current device
    for (int bt : {128, 256, 512})
      for (int lpr : {1, 2})
        for (bool inl : {false, true})
          MP_HIP(ctx, hipFuncSetAttribute((const void*)plan_kernel_for(bt, lpr, inl),
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)kMaxLds));
    ctx->mppi_lds_attr = true;
  }
  // deferred final rollout: snapshot ring slot of this call, free once the final rollout of
  // the call MP_FIN_RING back (same slot) is done
  A.fin = nullptr;
  A.fin_stride = 0;
  int par = 0;
  if (final_stream) {
    int st2 = mp_side_init(ctx);
    if (st2) return st2;
    par = ctx->fin_par;
    ctx->fin_par = (par + 1) % MP_FIN_RING;
    const FinRec R(H, D.n_obs, D.gnx * D.gny);
    A.fin_stride = R.stride;
    // every slot of the ring sized at once: a slot first used by a later call would allocate (hipMalloc, which
    // can wait for the device) in the middle of a run of calls -- with calls alternating over two contexts, the
    // bench's first timed calls did
    for (int q = 0; q < MP_FIN_RING; q++)
      if (!mp_ws(ctx, WS_FIN0 + q, sizeof(double) * (size_t)S * R.stride)) return MP_ERR_NOMEM;
    A.fin = (double*)mp_ws(ctx, WS_FIN0 + par, sizeof(double) * (size_t)S * R.stride);
    // The host (not the context stream) waits for the final rollout MP_FIN_RING calls back to
    // have read this slot (long done): a cross-stream wait packet would stall the context
    // stream between kernels, and a wait on the previous call's final rollout (which runs
    // beside the next plan kernel) would hold the host back until the GPU idles.
    MP_HIP(ctx, hipEventSynchronize(ctx->ev_fin[par]));
  }
  A.stamps = nullptr;
  static const bool stamps_on = getenv("MPGPU_STAMPS") != nullptr;
  if (stamps_on) {
    A.stamps = (unsigned long long*)mp_ws(ctx, WS_HA2, sizeof(unsigned long long) * 32 * S * nb);
    MP_HIP(ctx, hipMemsetAsync(A.stamps, 0, sizeof(unsigned long long) * 32 * S * nb, ctx->stream));
  }
  // timing events ride on the dispatch packet (hipExtLaunchKernel), and the stop event doubles
  // as the side stream's plan-done dependency: no marker packets between consecutive plans
  hipEvent_t t_start, t_stop;
  mp_time_pair(ctx, &t_start, &t_stop);
  const dim3 grd(S * nb);
  {
    MppiDev Dl = D;
    void* args[] = {(void*)&Dl, (void*)&A};
    MP_HIP(ctx, hipExtLaunchKernel((const void*)plan_kernel_for(BT, LPR, A.inline_noise != 0), grd, dim3(BT), args,
                                   shmem, ctx->stream, t_start, t_stop, 0));
  }
  MP_HIP(ctx, hipGetLastError());
  if (final_stream) {
    const FinRec R(H, D.n_obs, D.gnx * D.gny);
    const int grid_lds = (size_t)R.stride * 8 <= 64 * 1024;
    const size_t fsh = sizeof(double) * (size_t)(grid_lds ? R.stride : R.grid);
    MP_CHECK(ctx, fsh <= kMaxLds, "final rollout snapshot too large for LDS (%zu B)", fsh);
    if (!ctx->fin_lds_attr) {
      MP_HIP(ctx, hipSetDevice(ctx->device));
      MP_HIP(ctx, hipFuncSetAttribute((const void*)final_rollout_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)kMaxLds));
      ctx->fin_lds_attr = true;
    }
    hipEvent_t plan_done = t_stop;
    if (!plan_done) {
      plan_done = ctx->ev_plan[par];
      MP_HIP(ctx, hipEventRecord(plan_done, ctx->stream));
    }
    MP_HIP(ctx, hipStreamWaitEvent(ctx->side, plan_done, 0));
    hipLaunchKernelGGL(final_rollout_kernel, dim3(S), dim3(64), fsh, ctx->side, D, A.fin, A.fin_stride, grid_lds,
                       traj_out, cost_out, feasible_out, ctx->flags);
    MP_HIP(ctx, hipGetLastError());
    MP_HIP(ctx, hipEventRecord(ctx->ev_fin[par], ctx->side));
  }
  if (stamps_on) {
    std::vector<unsigned long long> h(32 * S * nb);
    MP_HIP(ctx, hipMemcpyAsync(h.data(), A.stamps, h.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
    MP_HIP(ctx, hipStreamSynchronize(ctx->stream));
    unsigned long long t0 = ~0ull, end = 0;
    double d01 = 0, d12 = 0, d23 = 0;
    int last = -1;
    for (int b = 0; b < S * nb; b++) {
      const unsigned long long* q = &h[32 * b];
      t0 = q[0] < t0 ? q[0] : t0;
      d01 += (q[1] - q[0]) / 100.0; d12 += (q[2] - q[1]) / 100.0; d23 += (q[3] - q[2]) / 100.0;
      if (q[5]) last = b;
      end = q[5] > end ? q[5] : end;
      end = q[3] > end ? q[3] : end;
    }
    fprintf(stderr, "[stamps us] blocks=%d mean rollout %.2f partial %.2f ticket %.2f", S * nb, d01 / (S * nb),
            d12 / (S * nb), d23 / (S * nb));
    {  // spread: block start times and phase-1 end times (percentiles)
      std::vector<double> st, en;
      for (int b = 0; b < S * nb; b++) {
        st.push_back((h[32 * b] - t0) / 100.0);
        en.push_back((h[32 * b + 1] - t0) / 100.0);
      }
      std::sort(st.begin(), st.end());
      std::sort(en.begin(), en.end());
      const int n = S * nb;
      fprintf(stderr, " | start p0/50/90/100 %.1f %.1f %.1f %.1f | p1-end p0/50/90/100 %.1f %.1f %.1f %.1f", st[0],
              st[n / 2], st[n * 9 / 10], st[n - 1], en[0], en[n / 2], en[n * 9 / 10], en[n - 1]);
      // per-wave ends and SIMD placement
      std::vector<double> we;
      int hist[9] = {0};  // max waves on one SIMD within a block
      for (int b = 0; b < n; b++) {
        int cnt[4] = {0, 0, 0, 0}, mx = 0;
        for (int w = 0; w < 8; w++) {
          const unsigned long long tw = h[32 * b + 8 + w];
          if (!tw) continue;
          we.push_back((tw - t0) / 100.0);
          const int simd = (int)((h[32 * b + 20 + w] >> 4) & 3);
          mx = std::max(mx, ++cnt[simd]);
        }
        hist[mx]++;
      }
      std::sort(we.begin(), we.end());
      const int m = (int)we.size();
      fprintf(stderr, " | wave-end p0/50/90/100 %.1f %.1f %.1f %.1f | blocks by max waves/SIMD 1:%d 2:%d 3:%d 4:%d",
              we[0], we[m / 2], we[m * 9 / 10], we[m - 1], hist[1], hist[2], hist[3], hist[4]);
    }
    {  // per-XCC wave-end mean / max and block count
      double sum[16] = {0}, mx[16] = {0};
      int cnt[16] = {0}, nbk[16] = {0};
      for (int b = 0; b < S * nb; b++) {
        const int x = (int)(h[32 * b + 30] & 15);
        nbk[x]++;
        for (int w = 0; w < 8; w++) {
          const unsigned long long tw = h[32 * b + 8 + w];
          if (!tw) continue;
          const double v = (tw - t0) / 100.0;
          sum[x] += v; cnt[x]++; mx[x] = std::max(mx[x], v);
        }
      }
      fprintf(stderr, " | xcc(blocks mean/max):");
      for (int x = 0; x < 16; x++)
        if (cnt[x]) fprintf(stderr, " %d(%d %.1f/%.1f)", x, nbk[x], sum[x] / cnt[x], mx[x]);
    }
    if (last >= 0) {
      const unsigned long long* q = &h[32 * last];
      fprintf(stderr, " | last block: start+%.2f combine %.2f final-rollout %.2f | total %.2f", (q[0] - t0) / 100.0,
              (q[4] - q[3]) / 100.0, (q[5] - q[4]) / 100.0, (end - t0) / 100.0);
    }
    fprintf(stderr, "\n");
  }
  return MP_OK;
}

}  // namespace

extern "C" {

int mp_mppi_plan_dev(mp_ctx* ctx, const mp_mppi_params* p, int32_t S, const double* X0, const double* goal,
                     const double* U_nom, const double* obstacles, const uint8_t* grid, const double* noise,
                     double* U_out, double* traj_out, double* cost_out, int32_t* feasible_out,
                     int32_t* rollout_count_out, int32_t* feasible_count_out, double* coll_traj,
                     double* coll_ctrl, double* coll_cost, uint8_t* coll_feas) {
  if (!ctx) return MP_ERR_INVALID;
  MppiDev D;
  int st = make_dev_params(ctx, p, p ? p->K : 0, &D);
  if (st) return st;
  MP_CHECK(ctx, S >= 1, "S (%d) must be >= 1", S);
  MP_CHECK(ctx, X0 && goal && U_nom && U_out && traj_out && cost_out && feasible_out && rollout_count_out &&
               feasible_count_out, "required pointer is NULL");
  MP_CHECK(ctx, p->noise_mode != MP_NOISE_EXTERNAL || noise, "noise is NULL in MP_NOISE_EXTERNAL mode");
  MP_CHECK(ctx, p->n_obs == 0 || obstacles, "obstacles NULL with n_obs > 0");
  MP_CHECK(ctx, p->grid_nx == 0 || grid, "grid NULL with grid_nx > 0");
  MP_CHECK(ctx, p->final_stream == 0 || p->final_stream == 1, "final_stream (%d) must be 0 or 1", p->final_stream);
  return plan_launch(ctx, D, S, X0, goal, U_nom, obstacles, grid, noise, U_out, traj_out, cost_out, feasible_out,
                     rollout_count_out, feasible_count_out, coll_traj, coll_ctrl, coll_cost, coll_feas,
                     p->final_stream);
}

int mp_mppi_plan(mp_ctx* ctx, const mp_mppi_params* p, int32_t S, const double* X0, const double* goal,
                 const double* U_nom, const double* obstacles, const uint8_t* grid, const double* noise,
                 double* U_out, double* traj_out, double* cost_out, int32_t* feasible_out,
                 int32_t* rollout_count_out, int32_t* feasible_count_out, double* coll_traj, double* coll_ctrl,
                 double* coll_cost, uint8_t* coll_feas) {
  if (!ctx) return MP_ERR_INVALID;
  MppiDev D;
  int st = make_dev_params(ctx, p, p ? p->K : 0, &D);
  if (st) return st;
  MP_CHECK(ctx, S >= 1, "S (%d) must be >= 1", S);
  MP_CHECK(ctx, X0 && goal && U_nom && U_out && traj_out && cost_out && feasible_out && rollout_count_out &&
               feasible_count_out, "required pointer is NULL");
  MP_CHECK(ctx, p->noise_mode != MP_NOISE_EXTERNAL || noise, "noise is NULL in MP_NOISE_EXTERNAL mode");
  MP_CHECK(ctx, p->n_obs == 0 || obstacles, "obstacles NULL with n_obs > 0");
  MP_CHECK(ctx, p->grid_nx == 0 || grid, "grid NULL with grid_nx > 0");
  MP_HIP(ctx, hipSetDevice(ctx->device));
  const size_t K = p->K, H = p->H;
  st = MP_OK;
  const double* dX0 = mp_upload(ctx, WS_IO0, X0, 7 * (size_t)S, &st);
  const double* dgoal = mp_upload(ctx, WS_IO1, goal, 2 * (size_t)S, &st);
  const double* dun = mp_upload(ctx, WS_IO2, U_nom, 2 * H * S, &st);
  const double* dobs = mp_upload(ctx, WS_IO3, p->n_obs ? obstacles : nullptr, 3 * (size_t)p->n_obs * S, &st);
  const uint8_t* dgrid = mp_upload(ctx, WS_IO4, p->grid_nx ? grid : nullptr, (size_t)p->grid_nx * p->grid_ny * S, &st);
  const double* dnoise = mp_upload(ctx, WS_IO5, p->noise_mode == MP_NOISE_EXTERNAL ? noise : nullptr, K * H * 2 * S, &st);
  double* dU = mp_alloc_out(ctx, WS_IO6, U_out, 2 * H * S, &st);
  double* dtraj = mp_alloc_out(ctx, WS_IO7, traj_out, (H + 1) * 7 * S, &st);
  double* dcost = mp_alloc_out(ctx, WS_IO8, cost_out, (size_t)S, &st);
  int32_t* dfe = mp_alloc_out(ctx, WS_IO9, feasible_out, (size_t)S, &st);
  int32_t* drc = mp_alloc_out(ctx, WS_IO10, rollout_count_out, (size_t)S, &st);
  int32_t* dfc = mp_alloc_out(ctx, WS_IO11, feasible_count_out, (size_t)S, &st);
  double* dct = mp_alloc_out(ctx, WS_IO12, coll_traj, K * (H + 1) * 7 * S, &st);
  double* dcc = mp_alloc_out(ctx, WS_IO13, coll_ctrl, K * H * 2 * S, &st);
  double* dco = mp_alloc_out(ctx, WS_IO15, coll_cost, K * S, &st);
  uint8_t* dcf = mp_alloc_out(ctx, WS_IO16, coll_feas, K * S, &st);
  if (st) return st;
  MP_HIP(ctx, hipMemsetAsync(ctx->flags, 0, sizeof(int), ctx->stream));
  MP_CHECK(ctx, p->final_stream == 0 || p->final_stream == 1, "final_stream (%d) must be 0 or 1", p->final_stream);
  st = plan_launch(ctx, D, S, dX0, dgoal, dun, dobs, dgrid, dnoise, dU, dtraj, dcost, dfe, drc, dfc, dct, dcc,
                   dco, dcf, p->final_stream);
  if (st) return st;
  if (p->final_stream && (st = mp_ctx_join(ctx))) return st;  // downloads below follow the side stream
  int flag = 0;
  if ((st = mp_download(ctx, U_out, dU, 2 * H * S))) return st;
  if ((st = mp_download(ctx, traj_out, dtraj, (H + 1) * 7 * S))) return st;
  if ((st = mp_download(ctx, cost_out, dcost, (size_t)S))) return st;
  if ((st = mp_download(ctx, feasible_out, dfe, (size_t)S))) return st;
  if ((st = mp_download(ctx, rollout_count_out, drc, (size_t)S))) return st;
  if ((st = mp_download(ctx, feasible_count_out, dfc, (size_t)S))) return st;
  if ((st = mp_download(ctx, coll_traj, dct, K * (H + 1) * 7 * S))) return st;
  if ((st = mp_download(ctx, coll_ctrl, dcc, K * H * 2 * S))) return st;
  if ((st = mp_download(ctx, coll_cost, dco, K * S))) return st;
  if ((st = mp_download(ctx, coll_feas, dcf, K * S))) return st;
  if ((st = mp_download(ctx, &flag, ctx->flags, 1))) return st;
  MP_HIP(ctx, hipStreamSynchronize(ctx->stream));
  if (flag & 1) return mp_fail(ctx, MP_ERR_NUMERIC, "NaN rollout cost (Julia would have produced NaN weights)");
  return MP_OK;
}

int mp_mppi_closed_loop(mp_ctx* ctx, const mp_mppi_params* p, const mp_mppi_loop_params* lp, int32_t S,
                        const double* X0, const double* goal, const double* U_nom0, const double* obstacles,
                        const uint8_t* grid, const int32_t* hold_idx, const double* noise, double* his,
                        int32_t* n_rows, int32_t* n_replans, double* U_log, double* traj_log, double* cost_log,
                        int32_t* feas_log, int32_t* rc_log) {
  if (!ctx) return MP_ERR_INVALID;
  MppiDev D;
  int st = make_dev_params(ctx, p, p ? p->K : 0, &D);
  if (st) return st;
  MP_CHECK(ctx, lp != nullptr, "loop params is NULL");
  MP_CHECK(ctx, S >= 1, "S (%d) must be >= 1", S);
  MP_CHECK(ctx, lp->update_steps >= 1, "update_steps (%d) must be >= 1", lp->update_steps);
  MP_CHECK(ctx, lp->max_steps >= 0, "max_steps (%d) must be >= 0", lp->max_steps);
  MP_CHECK(ctx, lp->plant_dt > 0.0, "plant_dt (%g) must be > 0", lp->plant_dt);
  MP_CHECK(ctx, X0 && goal && U_nom0 && hold_idx && his && n_rows && n_replans, "required pointer is NULL");
  MP_CHECK(ctx, p->noise_mode != MP_NOISE_EXTERNAL || noise, "noise is NULL in MP_NOISE_EXTERNAL mode");
  MP_CHECK(ctx, p->n_obs == 0 || obstacles, "obstacles NULL with n_obs > 0");
  MP_CHECK(ctx, p->grid_nx == 0 || grid, "grid NULL with grid_nx > 0");
  for (int i = 0; i < lp->update_steps; i++)
    MP_CHECK(ctx, hold_idx[i] >= 0 && hold_idx[i] < p->H, "hold_idx[%d] = %d outside [0, H=%d)", i, hold_idx[i],
             p->H);
  MP_HIP(ctx, hipSetDevice(ctx->device));
  const size_t K = p->K, H = p->H, SS = S, nsub = lp->update_steps, M = lp->max_steps;
  const int R = (int)((M + nsub - 1) / nsub);  // replans needed to cover the run
  const size_t RR = R > 0 ? (size_t)R : 1;
  st = MP_OK;
  // device state: the plant states (= the next plan's X0), logs replan-major [R][S]...
  double* dstate = (double*)mp_upload(ctx, WS_IO0, X0, 7 * SS, &st);
  const double* dgoal = mp_upload(ctx, WS_IO1, goal, 2 * SS, &st);
  const double* dU0 = mp_upload(ctx, WS_IO2, U_nom0, 2 * H * SS, &st);
  const double* dobs = mp_upload(ctx, WS_IO3, p->n_obs ? obstacles : nullptr, 3 * (size_t)p->n_obs * SS, &st);
  const uint8_t* dgrid = mp_upload(ctx, WS_IO4, p->grid_nx ? grid : nullptr, (size_t)p->grid_nx * p->grid_ny * SS, &st);
  const double* dnoise =
      mp_upload(ctx, WS_IO5, p->noise_mode == MP_NOISE_EXTERNAL ? noise : nullptr, RR * SS * K * H * 2, &st);
  const int32_t* dhold = mp_upload(ctx, WS_IO15, hold_idx, nsub, &st);
  double* dU = (double*)mp_ws(ctx, WS_IO6, sizeof(double) * RR * SS * H * 2);
  const size_t traj_n = (traj_log ? RR : 1) * SS * (H + 1) * 7;  // without a log: one scratch set
  double* dtraj = (double*)mp_ws(ctx, WS_IO7, sizeof(double) * traj_n);
  double* dcost = (double*)mp_ws(ctx, WS_IO8, sizeof(double) * RR * SS);
  int32_t* dfeas = (int32_t*)mp_ws(ctx, WS_IO9, sizeof(int32_t) * RR * SS);
  int32_t* drc = (int32_t*)mp_ws(ctx, WS_IO10, sizeof(int32_t) * RR * SS);
  int32_t* dfc = (int32_t*)mp_ws(ctx, WS_IO11, sizeof(int32_t) * RR * SS);
  double* drows = (double*)mp_ws(ctx, WS_IO12, sizeof(double) * SS * (M + 1) * 8);
  int32_t* dst = (int32_t*)mp_ws(ctx, WS_IO13, sizeof(int32_t) * 3 * SS);  // n_rows | live | n_replans
  int32_t* pin = (int32_t*)mp_pinned(ctx, sizeof(int32_t) * 2 * SS);
  if (st || !dU || !dtraj || !dcost || !dfeas || !drc || !dfc || !drows || !dst) return st ? st : MP_ERR_NOMEM;
  MP_CHECK(ctx, pin != nullptr, "pinned host buffer allocation failed");
  MP_HIP(ctx, hipMemsetAsync(drows, 0, sizeof(double) * SS * (M + 1) * 8, ctx->stream));
  {  // n_rows = 1, live = 1, n_replans = 0
    std::vector<int32_t> init(3 * SS, 0);
    for (size_t i = 0; i < SS; i++) init[i] = 1, init[SS + i] = M > 0 ? 1 : 0;
    MP_HIP(ctx, hipMemcpyAsync(dst, init.data(), init.size() * 4, hipMemcpyHostToDevice, ctx->stream));
    if (M == 0) {  // no plant step: the history is the start row only
      std::vector<double> r0(SS * 8);
      for (size_t s = 0; s < SS; s++) {
        r0[8 * s] = 0.0;
        for (int i = 0; i < 7; i++) r0[8 * s + 1 + i] = X0[7 * s + i];
      }
      MP_HIP(ctx, hipMemcpy2DAsync(drows, (M + 1) * 8 * sizeof(double), r0.data(), 8 * sizeof(double),
                                   8 * sizeof(double), SS, hipMemcpyHostToDevice, ctx->stream));
    }
    MP_HIP(ctx, hipStreamSynchronize(ctx->stream));  // `init` leaves scope
  }
  MP_HIP(ctx, hipMemsetAsync(ctx->flags, 0, sizeof(int), ctx->stream));
  int32_t* live = dst + SS;
  const int poll = lp->poll_every > 0 ? lp->poll_every : 8;
  const double r2 = lp->goal_radius * lp->goal_radius;
  int pending = -1;  // pinned half holding the last poll's live flags (its copy is in flight)
  hipEvent_t ev_poll[2];
  MP_HIP(ctx, hipEventCreateWithFlags(&ev_poll[0], hipEventDisableTiming));
  MP_HIP(ctx, hipEventCreateWithFlags(&ev_poll[1], hipEventDisableTiming));
  int rc = MP_OK;
  for (int r = 0; r < R; r++) {
    MppiDev Dr = D;
    Dr.offset = p->offset + (unsigned long long)r;  // a fresh Philox counter word per replan
    const double* un = r == 0 ? dU0 : dU + (size_t)(r - 1) * SS * H * 2;  // NominalControls = r.Control
    double* tr = dtraj + (traj_log ? (size_t)r * SS * (H + 1) * 7 : 0);
    rc = plan_launch(ctx, Dr, S, dstate, dgoal, un, dobs, dgrid, dnoise ? dnoise + (size_t)r * SS * K * H * 2 : nullptr,
                     dU + (size_t)r * SS * H * 2, tr, dcost + (size_t)r * SS, dfeas + (size_t)r * SS,
                     drc + (size_t)r * SS, dfc + (size_t)r * SS, nullptr, nullptr, nullptr, nullptr, 1, live);
    if (rc) break;
    hipLaunchKernelGGL(loop_plant_kernel, dim3((unsigned)((2 * SS + 63) / 64)), dim3(64), 0, ctx->stream, S, (int)H,
                       dstate, (const double*)(dU + (size_t)r * SS * H * 2), dhold, (int)nsub, lp->plant_dt, dgoal, r2,
                       (int)(r * nsub), (int)M, drows, dst, r);
    if (hipGetLastError() != hipSuccess) { rc = mp_fail(ctx, MP_ERR_HIP, "loop_plant_kernel launch failed"); break; }
    if ((r + 1) % poll == 0 && r + 1 < R) {
      // the previous poll's flags (one period behind, so the GPU stays fed while the host looks)
      bool done = false;
      if (pending >= 0) {
        if (hipEventSynchronize(ev_poll[pending]) != hipSuccess) { rc = mp_fail(ctx, MP_ERR_HIP, "poll failed"); break; }
        done = true;
        for (size_t s = 0; s < SS; s++) done = done && pin[pending * SS + s] == 0;
      }
      if (done) break;
      const int h = pending < 0 ? 0 : 1 - pending;
      if (hipMemcpyAsync(pin + h * SS, live, sizeof(int32_t) * SS, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
          hipEventRecord(ev_poll[h], ctx->stream) != hipSuccess) {
        rc = mp_fail(ctx, MP_ERR_HIP, "poll copy failed");
        break;
      }
      pending = h;
    }
  }
  if (!rc) rc = mp_ctx_join(ctx);  // the logged final rollouts come from the side stream
  mp_sync_all(ctx);
  hipEventDestroy(ev_poll[0]);
  hipEventDestroy(ev_poll[1]);
  if (rc) return rc;
  // results: [S]-major host layouts
  std::vector<int32_t> hst(3 * SS);
  int flag = 0;
  MP_HIP(ctx, hipMemcpy(hst.data(), dst, hst.size() * 4, hipMemcpyDeviceToHost));
  MP_HIP(ctx, hipMemcpy(his, drows, sizeof(double) * SS * (M + 1) * 8, hipMemcpyDeviceToHost));
  MP_HIP(ctx, hipMemcpy(&flag, ctx->flags, sizeof(int), hipMemcpyDeviceToHost));
  for (size_t s = 0; s < SS; s++) {
    n_rows[s] = hst[s];
    n_replans[s] = hst[2 * SS + s];
  }
  auto gather = [&](auto* host, const auto* dev, size_t per) -> int {  // [R][S][per] -> [S][R][per]
    if (!host || R == 0) return MP_OK;
    using T = std::remove_cv_t<std::remove_pointer_t<decltype(dev)>>;
    std::vector<T> tmp((size_t)R * SS * per);
    MP_HIP(ctx, hipMemcpy(tmp.data(), dev, tmp.size() * sizeof(T), hipMemcpyDeviceToHost));
    for (size_t s = 0; s < SS; s++)
      for (int r = 0; r < R; r++)
        for (size_t i = 0; i < per; i++) host[((size_t)s * R + r) * per + i] = tmp[((size_t)r * SS + s) * per + i];
    return MP_OK;
  };
  if ((st = gather(U_log, dU, H * 2))) return st;
  if ((st = gather(traj_log, dtraj, (H + 1) * 7))) return st;
  if ((st = gather(cost_log, dcost, 1))) return st;
  if ((st = gather(feas_log, dfeas, 1))) return st;
  if ((st = gather(rc_log, drc, 1))) return st;
  if (flag & 1) return mp_fail(ctx, MP_ERR_NUMERIC, "NaN rollout cost in the closed loop");
  return MP_OK;
}

int mp_mppi_plan_sharded(mp_ctx** ctxs, int32_t n, const mp_mppi_params* p, int32_t S, const double* X0,
                         const double* goal, const double* U_nom, const double* obstacles, const uint8_t* grid,
                         const double* noise, double* U_out, double* traj_out, double* cost_out,
                         int32_t* feasible_out, int32_t* rollout_count_out, int32_t* feasible_count_out) {
  if (!ctxs || n < 1 || !ctxs[0]) return MP_ERR_INVALID;
  mp_ctx* c0 = ctxs[0];
  int st = mp_comm_check(ctxs, n);
  if (st) return st;
  MppiDev D;
  if ((st = make_dev_params(c0, p, p ? p->K : 0, &D))) return st;
  MP_CHECK(c0, S >= 1, "S (%d) must be >= 1", S);
  MP_CHECK(c0, X0 && goal && U_nom && U_out && traj_out && cost_out && feasible_out && rollout_count_out &&
               feasible_count_out, "required pointer is NULL");
  MP_CHECK(c0, p->noise_mode != MP_NOISE_EXTERNAL || noise, "noise is NULL in MP_NOISE_EXTERNAL mode");
  MP_CHECK(c0, p->n_obs == 0 || obstacles, "obstacles NULL with n_obs > 0");
  MP_CHECK(c0, p->grid_nx == 0 || grid, "grid NULL with grid_nx > 0");
  MP_CHECK(c0, p->final_stream == 0 || p->final_stream == 1, "final_stream (%d) must be 0 or 1", p->final_stream);
  const size_t K = p->K, H = p->H, Dr = shard_rec((int)H), gb = (size_t)p->grid_nx * p->grid_ny;
  const int base = S / n, rem = S % n, smax = base + (rem > 0);
  auto lo = [&](int r) { return r * base + (r < rem ? r : rem); };
  std::vector<void*> send(n), recv(n);
  // the caller's current device is restored on every return; an error after some ranks have
  // enqueued work drains those ranks first, so nothing of this call is left running
  int dev0 = 0;
  hipGetDevice(&dev0);
  int enq = 0;  // ranks [0, enq) have work enqueued
  auto done = [&](int status) {
    for (int r = 0; r < enq; r++) {
      hipSetDevice(ctxs[r]->device);
      mp_sync_all(ctxs[r]);
    }
    hipSetDevice(dev0);
    return status;
  };
#define MP_SH(call)                                                                       \
  do {                                                                                    \
    hipError_t e_ = (call);                                                               \
    if (e_ != hipSuccess)                                                                 \
      return done(mp_fail(c0, MP_ERR_HIP, "%s: %s", #call, hipGetErrorString(e_)));       \
  } while (0)
  // every rank plans its block [a, b) of scenes (Philox counter word scene_base + a: the same noise as
  // one mp_mppi_plan over all S) and packs its results; all launches are enqueued before any wait
  for (int r = 0; r < n; r++) {
    mp_ctx* c = ctxs[r];
    MP_SH(hipSetDevice(c->device));
    const int a = lo(r), cnt = lo(r + 1) - a;
    const size_t sa = a, sc = cnt;
    send[r] = mp_ws(c, WS_SHARD_SEND, sizeof(double) * (size_t)smax * Dr);
    recv[r] = mp_ws(c, WS_SHARD_RECV, sizeof(double) * (size_t)n * smax * Dr);
    if (!send[r] || !recv[r]) return done(mp_fail(c0, MP_ERR_NOMEM, "rank %d: %s", r, c->err.c_str()));
    // every rank's NaN flag is cleared, also on a rank without scenes: the flags of all ranks are
    // read back below, and a flag left from an earlier call must not report a NaN of this one
    enq = r + 1;
    MP_SH(hipMemsetAsync(c->flags, 0, sizeof(int), c->stream));
    if (cnt == 0) continue;  // more ranks than scenes: this rank only takes part in the gather
    st = MP_OK;
    const double* dX0 = mp_upload(c, WS_IO0, X0 + 7 * sa, 7 * sc, &st);
    const double* dgoal = mp_upload(c, WS_IO1, goal + 2 * sa, 2 * sc, &st);
    const double* dun = mp_upload(c, WS_IO2, U_nom + 2 * H * sa, 2 * H * sc, &st);
    const double* dobs = mp_upload(c, WS_IO3, p->n_obs ? obstacles + 3 * (size_t)p->n_obs * sa : nullptr,
                                   3 * (size_t)p->n_obs * sc, &st);
    const uint8_t* dgrid = mp_upload(c, WS_IO4, gb ? grid + gb * sa : nullptr, gb * sc, &st);
    const double* dnoise = mp_upload(c, WS_IO5, p->noise_mode == MP_NOISE_EXTERNAL ? noise + K * H * 2 * sa : nullptr,
                                     K * H * 2 * sc, &st);
    double* dU = (double*)mp_ws(c, WS_IO6, sizeof(double) * 2 * H * sc);
    double* dtraj = (double*)mp_ws(c, WS_IO7, sizeof(double) * (H + 1) * 7 * sc);
    double* dcost = (double*)mp_ws(c, WS_IO8, sizeof(double) * sc);
    int32_t* dfe = (int32_t*)mp_ws(c, WS_IO9, sizeof(int32_t) * sc);
    int32_t* drc = (int32_t*)mp_ws(c, WS_IO10, sizeof(int32_t) * sc);
    int32_t* dfc = (int32_t*)mp_ws(c, WS_IO11, sizeof(int32_t) * sc);
    if (st || !dU || !dtraj || !dcost || !dfe || !drc || !dfc)
      return done(mp_fail(c0, st ? st : MP_ERR_NOMEM, "rank %d: %s", r, c->err.c_str()));
    MppiDev Dr_ = D;
    Dr_.scene_base = p->scene_base + a;
    if ((st = plan_launch(c, Dr_, cnt, dX0, dgoal, dun, dobs, dgrid, dnoise, dU, dtraj, dcost, dfe, drc, dfc, nullptr,
                          nullptr, nullptr, nullptr, p->final_stream)))
      return done(mp_fail(c0, st, "rank %d: %s", r, c->err.c_str()));
    if (p->final_stream && (st = mp_ctx_join(c))) return done(mp_fail(c0, st, "rank %d: %s", r, c->err.c_str()));
    const long long tot = (long long)cnt * (long long)Dr;
    hipLaunchKernelGGL(shard_pack_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, c->stream, cnt, (int)H,
                       dU, dtraj, dcost, dfe, drc, dfc, (double*)send[r]);
    MP_SH(hipGetLastError());
  }
  // the exchange step: every GPU ends with every scene's results (RCCL all-gather over xGMI)
  if ((st = mp_comm_allgather(ctxs, n, send.data(), recv.data(), sizeof(double) * (size_t)smax * Dr)))
    return done(st);
  std::vector<double> all((size_t)n * smax * Dr);
  MP_SH(hipSetDevice(c0->device));
  MP_SH(hipMemcpyAsync(all.data(), recv[0], all.size() * sizeof(double), hipMemcpyDeviceToHost, c0->stream));
  int nan = 0;
  for (int r = 0; r < n; r++) {
    int f = 0;
    MP_SH(hipSetDevice(ctxs[r]->device));
    MP_SH(hipMemcpyAsync(&f, ctxs[r]->flags, sizeof(int), hipMemcpyDeviceToHost, ctxs[r]->stream));
    MP_SH(hipStreamSynchronize(ctxs[r]->stream));
    nan |= f & 1;
  }
#undef MP_SH
  hipSetDevice(dev0);
  for (int r = 0; r < n; r++)
    for (int s = lo(r), j = 0; s < lo(r + 1); s++, j++) {
      const double* q = all.data() + ((size_t)r * smax + j) * Dr;
      for (size_t t = 0; t < 2 * H; t++) U_out[(size_t)s * 2 * H + t] = q[t];
      for (size_t t = 0; t < 7 * (H + 1); t++) traj_out[(size_t)s * 7 * (H + 1) + t] = q[2 * H + t];
      const double* e = q + 2 * H + 7 * (H + 1);
      cost_out[s] = e[0];
      feasible_out[s] = (int32_t)e[1];
      rollout_count_out[s] = (int32_t)e[2];
      feasible_count_out[s] = (int32_t)e[3];
    }
  if (nan) return mp_fail(c0, MP_ERR_NUMERIC, "NaN rollout cost (Julia would have produced NaN weights)");
  return MP_OK;
}

int mp_rollout(mp_ctx* ctx, const mp_mppi_params* p, int32_t S, int32_t K, const double* X0, const double* goal,
               const double* ctrl, int64_t ctrl_stride_h, const double* U_nom, const double* obstacles,
               const uint8_t* grid, double* traj, double* cost, uint8_t* feas, int32_t* argmin) {
  if (!ctx) return MP_ERR_INVALID;
  MppiDev D;
  int st = make_dev_params(ctx, p, K, &D);
  if (st) return st;
  MP_CHECK(ctx, S >= 1, "S (%d) must be >= 1", S);
  MP_CHECK(ctx, X0 && goal && ctrl && cost && feas, "required pointer is NULL");
  MP_CHECK(ctx, ctrl_stride_h == 0 || ctrl_stride_h == 2, "ctrl_stride_h must be 0 or 2");
  MP_CHECK(ctx, !p->ctrl_cost || U_nom, "U_nom NULL with ctrl_cost");
  MP_CHECK(ctx, p->n_obs == 0 || obstacles, "obstacles NULL with n_obs > 0");
  MP_CHECK(ctx, p->grid_nx == 0 || grid, "grid NULL with grid_nx > 0");
  MP_HIP(ctx, hipSetDevice(ctx->device));
  const size_t H = p->H, KK = K;
  const size_t nctrl = ctrl_stride_h ? KK * H * 2 * S : KK * 2 * S;
  st = MP_OK;
  const double* dX0 = mp_upload(ctx, WS_IO0, X0, 7 * (size_t)S, &st);
  const double* dgoal = mp_upload(ctx, WS_IO1, goal, 2 * (size_t)S, &st);
  const double* dun = mp_upload(ctx, WS_IO2, p->ctrl_cost ? U_nom : nullptr, 2 * H * S, &st);
  const double* dobs = mp_upload(ctx, WS_IO3, p->n_obs ? obstacles : nullptr, 3 * (size_t)p->n_obs * S, &st);
  const uint8_t* dgrid = mp_upload(ctx, WS_IO4, p->grid_nx ? grid : nullptr, (size_t)p->grid_nx * p->grid_ny * S, &st);
  const double* dctrl = mp_upload(ctx, WS_IO5, ctrl, nctrl, &st);
  double* dtraj = mp_alloc_out(ctx, WS_IO6, traj, KK * (H + 1) * 7 * S, &st);
  double* dcost = mp_alloc_out(ctx, WS_IO7, cost, KK * S, &st);
  uint8_t* dfeas = mp_alloc_out(ctx, WS_IO8, feas, KK * S, &st);
  int32_t* dam = mp_alloc_out(ctx, WS_IO9, argmin, (size_t)S, &st);
  if (st) return st;
  const int nb = (K + RPB - 1) / RPB;
  hipLaunchKernelGGL(rollout_kernel, dim3(S * nb), dim3(NT), 0, ctx->stream, D, K, dX0, dgoal, dctrl,
                     (long long)ctrl_stride_h, dun, dobs, dgrid, dtraj, dcost, dfeas, nb);
  MP_HIP(ctx, hipGetLastError());
  if (dam) {
    hipLaunchKernelGGL(argmin_kernel, dim3(S), dim3(NT), 0, ctx->stream, K, dcost, dam);
    MP_HIP(ctx, hipGetLastError());
  }
  if ((st = mp_download(ctx, traj, dtraj, KK * (H + 1) * 7 * S))) return st;
  if ((st = mp_download(ctx, cost, dcost, KK * S))) return st;
  if ((st = mp_download(ctx, feas, dfeas, KK * S))) return st;
  if ((st = mp_download(ctx, argmin, dam, (size_t)S))) return st;
  MP_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return MP_OK;
}

int mp_vehicle_euler(mp_ctx* ctx, int32_t n, double* states, const double* ctrl, double dt, int32_t nsteps,
                     double* his) {
  if (!ctx) return MP_ERR_INVALID;
  MP_CHECK(ctx, n >= 1 && nsteps >= 0 && states && ctrl, "bad arguments to mp_vehicle_euler");
  MP_HIP(ctx, hipSetDevice(ctx->device));
  int st = MP_OK;
  double* ds = (double*)mp_upload(ctx, WS_IO0, states, 7 * (size_t)n, &st);
  const double* dc = mp_upload(ctx, WS_IO1, ctrl, 2 * (size_t)n, &st);
  double* dh = mp_alloc_out(ctx, WS_IO2, his, (size_t)n * nsteps * 7, &st);
  if (st) return st;
  const int blocks = (2 * n + 63) / 64;
  hipLaunchKernelGGL(euler_kernel, dim3(blocks), dim3(64), 0, ctx->stream, n, ds, dc, dt, nsteps, dh);
  MP_HIP(ctx, hipGetLastError());
  if ((st = mp_download(ctx, states, (const double*)ds, 7 * (size_t)n))) return st;
  if ((st = mp_download(ctx, his, (const double*)dh, (size_t)n * nsteps * 7))) return st;
  MP_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return MP_OK;
}

}  // extern "C"
