// Latency probe (lab only): dependent-chain cycles of fp64 FMA / DPP / LDS and s_barrier cost on
// gfx950, one workgroup, s_memtime stamps.  hipcc --offload-arch=gfx950 -O3 lat_probe.hip -o lat_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

__device__ __forceinline__ long long stamp() {
  long long t;
  asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t));
  return t;
}

template <int CH>
__global__ void k_fma(double* out, long long* t, double a, double b) {
  double x[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) x[c] = threadIdx.x + c;
  __syncthreads();
#pragma unroll
  for (int c = 0; c < CH; ++c) asm volatile("" : "+v"(x[c]));
  long long t0 = stamp();
#pragma unroll
  for (int c = 0; c < CH; ++c) asm volatile("" : "+v"(x[c]) : "s"(t0));
#pragma unroll
  for (int i = 0; i < 64; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) x[c] = __fma_rn(x[c], a, b);
#pragma unroll
  for (int c = 0; c < CH; ++c) asm volatile("" : "+v"(x[c]));
  long long t1 = stamp();
  double s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s += x[c];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) t[0] = t1 - t0;
}

__global__ void k_dpp(double* out, long long* t) {
  double x = threadIdx.x;
  long long t0 = stamp();
  asm volatile("" : "+v"(x) : "s"(t0));
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    const long long v = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(v >> 32), 0x138, 0xF, 0xF, true);
    x = __longlong_as_double(((long long)hi << 32) | (unsigned)lo) + 1.0;
  }
  asm volatile("" : "+v"(x));
  long long t1 = stamp();
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) t[0] = t1 - t0;
}

__global__ void k_lds(double* out, long long* t) {
  __shared__ double sh[1024];
  sh[threadIdx.x] = 0;
  __syncthreads();
  int idx = threadIdx.x & 63;
  long long t0 = stamp();
#pragma unroll 1
  for (int i = 0; i < 64; ++i) idx = (int)sh[idx] + (threadIdx.x & 63);
  long long t1 = stamp();
  out[threadIdx.x] = idx;
  if (threadIdx.x == 0) t[0] = t1 - t0;
}

__global__ void k_bar(double* out, long long* t) {
  long long t0 = stamp();
#pragma unroll 1
  for (int i = 0; i < 64; ++i) __syncthreads();
  long long t1 = stamp();
  if (threadIdx.x == 0) t[0] = t1 - t0;
}

int main() {
  double* out;
  long long* t;
  hipMalloc(&out, 1024 * 8);
  hipMalloc(&t, 8);
  long long h;
  auto run = [&](const char* name, auto launch, int ops) {
    for (int r = 0; r < 3; ++r) launch();
    hipMemcpy(&h, t, 8, hipMemcpyDeviceToHost);
    printf("%-28s %8lld cycles  (%.1f per op)\n", name, h, (double)h / ops);
  };
  run("fma_f64 1 chain x64", [&] { k_fma<1><<<1, 64>>>(out, t, 1.0000001, 1e-9); }, 64);
  run("fma_f64 2 chains x64", [&] { k_fma<2><<<1, 64>>>(out, t, 1.0000001, 1e-9); }, 64);
  run("fma_f64 4 chains x64", [&] { k_fma<4><<<1, 64>>>(out, t, 1.0000001, 1e-9); }, 64);
  run("fma_f64 8 chains x64", [&] { k_fma<8><<<1, 64>>>(out, t, 1.0000001, 1e-9); }, 64);
  run("fma_f64 4 chains, 16 waves", [&] { k_fma<4><<<1, 1024>>>(out, t, 1.0000001, 1e-9); }, 64);
  run("dpp f64 shift+add x64", [&] { k_dpp<<<1, 64>>>(out, t); }, 64);
  run("ds_read chain x64 (1 wave)", [&] { k_lds<<<1, 64>>>(out, t); }, 64);
  run("ds_read chain x64 (16 waves)", [&] { k_lds<<<1, 1024>>>(out, t); }, 64);
  run("s_barrier x64 (16 waves)", [&] { k_bar<<<1, 1024>>>(out, t); }, 64);
  run("s_barrier x64 (4 waves)", [&] { k_bar<<<1, 256>>>(out, t); }, 64);
  hipDeviceSynchronize();
  return 0;
}
