// Reduced reproducer for the rocprofv3 exit crash seen after a cooperative launch (round 5, r05z2:
// rocprofv3 --kernel-trace around a process that ran ha_persist_kernel through hipLaunchCooperativeKernel
// exited 139 in its exit handlers; the same kernel by an ordinary launch exited 0).  One trivial kernel,
// one cooperative (or, with argv[1] = "plain", ordinary) launch of 256 one-wave blocks, synchronise,
// release everything explicitly, return 0:
//   rocprofv3 --kernel-trace --stats -d DIR -o run --output-format csv -- ./coop_exit [plain]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>

__global__ void k_touch(int* out) {
  if (threadIdx.x == 0) out[blockIdx.x] = (int)blockIdx.x;
}

int main(int argc, char** argv) {
  const bool plain = argc > 1 && !strcmp(argv[1], "plain");
  int coop = 0;
  if (hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, 0) != hipSuccess) return 2;
  int* d = nullptr;
  if (hipMalloc(&d, 256 * sizeof(int)) != hipSuccess) return 3;
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 4;
  void* args[] = {&d};
  const hipError_t e = plain || !coop
                           ? hipLaunchKernel((const void*)k_touch, dim3(256), dim3(64), args, 0, s)
                           : hipLaunchCooperativeKernel((const void*)k_touch, dim3(256), dim3(64), args, 0, s);
  if (e != hipSuccess) { printf("launch: %s\n", hipGetErrorString(e)); return 5; }
  if (hipStreamSynchronize(s) != hipSuccess) return 6;
  int h[256];
  if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 7;
  int bad = 0;
  for (int i = 0; i < 256; i++) bad += h[i] != i;
  hipStreamDestroy(s);
  hipFree(d);
  printf("%s launch (coop supported %d): %d wrong\n", plain ? "plain" : "cooperative", coop, bad);
  return bad ? 8 : 0;
}
