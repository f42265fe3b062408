// Lab: does the size of a copy kernel's argument block set its duration?  A 2-D rectangle copy of R x C doubles
// with (a) a 1.5 KB table of rectangles in the kernel arguments, (b) one rectangle (48 B), (c) the table in device
// memory (pointer argument); HIP-event time per launch over many back-to-back launches, and an empty kernel.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

struct Rect { long long dst, src, dld, sld, rows, cols; };
struct Table { Rect r[32]; };

__global__ __launch_bounds__(256) void k_table(const Table t) {
  const Rect q = t.r[blockIdx.y];
  double* d = (double*)q.dst; const double* s = (const double*)q.src;
  const int cols = (int)q.cols, n = (int)(q.rows * q.cols);
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const int r = i / cols, c = i - r * cols;
    d[r * q.dld + c] = s[r * q.sld + c];
  }
}
__global__ __launch_bounds__(256) void k_one(const Rect q) {
  double* d = (double*)q.dst; const double* s = (const double*)q.src;
  const int cols = (int)q.cols, n = (int)(q.rows * q.cols);
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const int r = i / cols, c = i - r * cols;
    d[r * q.dld + c] = s[r * q.sld + c];
  }
}
__global__ __launch_bounds__(256) void k_dev(const Rect* __restrict__ t) {
  const Rect q = t[blockIdx.y];
  double* d = (double*)q.dst; const double* s = (const double*)q.src;
  const int cols = (int)q.cols, n = (int)(q.rows * q.cols);
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const int r = i / cols, c = i - r * cols;
    d[r * q.dld + c] = s[r * q.sld + c];
  }
}
__global__ void k_empty(int) {}

template <typename F>
static float time_us(F f, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  for (int i = 0; i < 20; ++i) f();
  hipEventRecord(a);
  for (int i = 0; i < reps; ++i) f();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0; hipEventElapsedTime(&ms, a, b);
  return ms * 1e3f / reps;
}

int main() {
  const int R = 128, C = 256, ld = 4224;
  double *src, *dst; Rect* dt;
  hipMalloc(&src, (size_t)R * ld * 8 * 2); hipMalloc(&dst, (size_t)R * ld * 8 * 2); hipMalloc(&dt, sizeof(Table));
  hipMemset(src, 0, (size_t)R * ld * 8 * 2);
  Rect q{(long long)dst, (long long)src, ld, C, R, C};
  Table t{}; t.r[0] = q;
  hipMemcpy(dt, &t, sizeof(Table), hipMemcpyHostToDevice);
  for (int g : {32, 128, 256}) {
    dim3 grid(g, 1);
    printf("grid %4d: table-in-args %6.2f us, one-rect %6.2f us, table-in-memory %6.2f us\n", g,
           time_us([&] { k_table<<<grid, 256>>>(t); }, 2000), time_us([&] { k_one<<<grid, 256>>>(q); }, 2000),
           time_us([&] { k_dev<<<grid, 256>>>(dt); }, 2000));
  }
  printf("empty kernel: %6.2f us\n", time_us([&] { k_empty<<<1, 64>>>(0); }, 2000));
  return 0;
}
