// Standalone Hybrid A* driver for kernel debugging and phase timing (s_memtime stamps of the RS_connected
// block, the expansion blocks and one mid-search bookkeeping launch).  Build:
//   bash tools/build_variant.sh dbg "-DHA_DEBUG"
//   hipcc --offload-arch=gfx950 -O2 -std=c++17 -o tools/ha_dbg tools/ha_dbg.cpp -Lmotionplanning_amd/lib \
//         -lmpgpu_dbg -Wl,-rpath,'$ORIGIN/../motionplanning_amd/lib'
// (the stamps themselves wait for outstanding loads, so they perturb what they time: use them for
// shares, not absolute latencies)
#include <cmath>
#include <cstdio>
#include <cstring>
#include <thread>
#include <unistd.h>

#include <hip/hip_runtime.h>

#include "../include/mpgpu.h"
extern "C" int mp_ha_debug_buf(int*);

int main() {
  mp_ctx* ctx = nullptr;
  if (mp_ctx_create(0, &ctx)) { printf("ctx: %s\n", mp_last_error(nullptr)); return 1; }
  mp_ha_params p;
  memset(&p, 0, sizeof p);
  p.vehicle_len = 3; p.vehicle_wid = 2; p.minR = 3 / std::tan(M_PI / 6); p.expand_time = 2.5;
  p.res[0] = 0.5; p.res[1] = 0.5; p.res[2] = M_PI / 12;
  double sb[6] = {-5, 10, 0, 10, -M_PI, M_PI};
  memcpy(p.stbound, sb, sizeof sb);
  p.n_walls = 3; p.n_prim = 62; p.n_col = 250; p.max_pops = 5000;
  double node[3] = {7, 0, M_PI / 2}, goal[3] = {0, 0.5, M_PI / 2};
  double walls[15] = {0, -1, 0, 5.5 / 2 + 1, 1, -5.5 / 2, 2.7432 / 2, 0, 1, 2.7432 / 2, 5.5 / 2, 2.7432 / 2, 0, 1, 2.7432 / 2};
  unsigned char ok = 0;
  static double path[501 * 3];
  int len = 0;
  int* buf = nullptr;
  hipHostMalloc((void**)&buf, 1 << 20, hipHostMallocMapped);
  memset(buf, 0, 1 << 20);
  printf("dbg buf %d\n", mp_ha_debug_buf(buf));
  printf("launch\n");
  fflush(stdout);
  int st = -99;
  std::thread th([&] { st = mp_ha_rs_connect(ctx, &p, 1, node, goal, walls, &ok, path, &len); });
  for (int t = 0; t < 20 && st == -99; t++) usleep(250000);
  printf("block0 phases:");
  for (int i = 0; i < 64; i++) printf(" %d", ((volatile int*)buf)[i]);
  printf("\nst=%d\n", st);
  fflush(stdout);
  if (st == -99) _exit(3);
  th.join();
  {
    const unsigned long long* t = reinterpret_cast<const unsigned long long*>(buf + 64 * 64);
    printf("RS block stamps (cycles from [0]):");
    for (int i = 1; i < 16; i++) printf(" [%d]%lld", i, t[i] ? (long long)(t[i] - t[0]) : -1LL);
    printf("\n");
  }
  printf("st %d ok %d len %d end %g %g %g\n", st, ok, len, path[3 * (len - 1)], path[3 * (len - 1) + 1], path[3 * (len - 1) + 2]);
  {  // expand of the same node: block 1 (neighbours 0..15) phase times
    double sc[62 * 3], pc[62 * 250 * 3];
    double steer[31], gear[2] = {1, -1};
    for (int i = 0; i < 31; i++) {
      const double t = i / 30.0, a = -1 / p.minR, b = 1 / p.minR;
      steer[i] = (1 - t) * a + t * b;
    }
    printf("prims %d\n", mp_ha_neighbor_origin(ctx, &p, 31, steer, 2, gear, sc, pc));
    memset(buf, 0, 1 << 20);
    double nb[62 * 3], hh[62];
    int64_t idx[62];
    uint8_t fr[62];
    printf("expand %d\n", mp_ha_expand(ctx, &p, 1, node, goal, walls, nb, idx, fr, hh));
    const unsigned long long* t = reinterpret_cast<const unsigned long long*>(buf + 64 * 64);
    for (int blk = 1; blk <= 4; blk++) {
      printf("expand block %d stamps:", blk);
      for (int i = 1; i < 16; i++) printf(" [%d]%lld", i, t[blk * 16 + i] ? (long long)(t[blk * 16 + i] - t[blk * 16]) : -1LL);
      printf("\n");
    }
  }
  {  // a short plan of the same scene: phase stamps of the last bookkeeping launch (scene 0)
    memset(buf, 0, 1 << 20);
    p.max_pops = 40;
    const double start[3] = {7, 0, M_PI / 2};
    int32_t found, pops, nn, ns, rl;
    static int64_t seq[40];
    static double st[40 * 3], rs[501 * 3];
    printf("plan %d\n", mp_ha_plan(ctx, &p, 1, start, goal, walls, &found, &pops, &nn, seq, &ns, st, &rl, rs));
    const unsigned long long* t = reinterpret_cast<const unsigned long long*>(buf + 64 * 64) + 4096 * 16;
    printf("book stamps (cycles from [0]):");
    for (int i = 1; i < 16; i++) printf(" [%d]%lld", i, t[i] ? (long long)(t[i] - t[0]) : -1LL);
    printf("\npops %d\n", pops);
    // the same after 600 pops (an open list of ~2,000 entries, as late in configs[3]'s longest searches)
    memset(buf, 0, 1 << 20);
    p.max_pops = 600;
    static int64_t seq6[600];
    static double st6[600 * 3];
    printf("plan %d\n", mp_ha_plan(ctx, &p, 1, start, goal, walls, &found, &pops, &nn, seq6, &ns, st6, &rl, rs));
    printf("book stamps at pop %d, %d nodes (cycles from [0]):", pops, nn);
    for (int i = 1; i < 16; i++) printf(" [%d]%lld", i, t[i] ? (long long)(t[i] - t[0]) : -1LL);
    printf("\n");
  }
  mp_ctx_destroy(ctx);
  return 0;
}
