// Launch-overhead probe (lab only): per-kernel cost of graph-replayed launches (empty / one wide
// grid) vs a grid barrier inside one launch (bounded spin, so a non-resident grid cannot hang).
// hipcc --offload-arch=gfx950 -O3 launch_probe.hip -o launch_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void k_empty(int* p) {
  if (p && threadIdx.x == 1023 && blockIdx.x == 100000) p[0] = 1;
}

__global__ void k_touch(double* p, int n) {  // each thread writes one double (a tiny level)
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = p[i] * 0.5 + 1.0;
}

__global__ void k_gridbar(unsigned* cnt, int nbar, int* err, double* p, int n) {
  const unsigned nwg = gridDim.x;
  for (int k = 0; k < nbar; ++k) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = p[i] * 0.5 + 1.0;
    __syncthreads();
    if (threadIdx.x == 0) {
      __threadfence();
      atomicAdd(cnt, 1u);
      const unsigned target = (unsigned)(k + 1) * nwg;
      long long spins = 0;
      while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        if (++spins > 20000000) { *err = 1; break; }
        __builtin_amdgcn_s_sleep(1);
      }
      __threadfence();
    }
    __syncthreads();
  }
}

int main() {
  int* err;
  unsigned* cnt;
  double* p;
  hipMalloc(&err, 4);
  hipMalloc(&cnt, 4);
  hipMalloc(&p, 8 << 20);
  hipMemset(err, 0, 4);
  hipMemset(p, 0, 8 << 20);
  hipStream_t s;
  hipStreamCreate(&s);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int NK = 100;
  auto graph_time = [&](auto body) {
    hipGraph_t g;
    hipGraphExec_t ge;
    hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
    for (int i = 0; i < NK; ++i) body();
    hipStreamEndCapture(s, &g);
    hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    for (int r = 0; r < 3; ++r) hipGraphLaunch(ge, s);
    hipEventRecord(e0, s);
    for (int r = 0; r < 10; ++r) hipGraphLaunch(ge, s);
    hipEventRecord(e1, s);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    hipGraphExecDestroy(ge);
    hipGraphDestroy(g);
    return ms * 1e3f / (10 * NK);
  };
  printf("empty 1 WG x 64          : %.2f us per kernel (graph)\n", graph_time([&] { k_empty<<<1, 64, 0, s>>>(nullptr); }));
  printf("empty 1 WG x 1024        : %.2f us\n", graph_time([&] { k_empty<<<1, 1024, 0, s>>>(nullptr); }));
  printf("empty 256 WG x 1024      : %.2f us\n", graph_time([&] { k_empty<<<256, 1024, 0, s>>>(nullptr); }));
  printf("empty 512 WG x 256       : %.2f us\n", graph_time([&] { k_empty<<<512, 256, 0, s>>>(nullptr); }));
  printf("empty 2048 WG x 256      : %.2f us\n", graph_time([&] { k_empty<<<2048, 256, 0, s>>>(nullptr); }));
  printf("touch 1 MB, 512 WG x 256 : %.2f us\n", graph_time([&] { k_touch<<<512, 256, 0, s>>>(p, 131072); }));
  printf("touch 8 MB, 4096 WGx256  : %.2f us\n", graph_time([&] { k_touch<<<4096, 256, 0, s>>>(p, 1048576); }));
  for (int wg : {64, 256}) {
    for (int th : {256, 1024}) {
      hipMemset(cnt, 0, 4);
      const int NB = 200;
      hipEventRecord(e0, s);
      k_gridbar<<<wg, th, 0, s>>>(cnt, NB, err, p, wg * th);
      hipEventRecord(e1, s);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      int he;
      hipMemcpy(&he, err, 4, hipMemcpyDeviceToHost);
      printf("grid barrier %3d WG x %4d: %.2f us per barrier (err=%d)\n", wg, th, ms * 1e3f / NB, he);
    }
  }
  return 0;
}
