// fea_common.h — shared device helpers for the FEANet HIP kernels (gfx950 / CDNA4).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "feanet_hip.h"

namespace fea {

constexpr int kWave = 64;

// ---------------------------------------------------------------------------
// Cross-lane moves on the full 64-lane wave (DPP wave_shr:1 / wave_shl:1, gfx9 family).
// shr1: lane i receives lane i-1's value; lane 0 keeps `old`.
// shl1: lane i receives lane i+1's value; lane 63 keeps `old`.
// Requires every lane of the wave to be active (callers keep control flow wave-uniform).
// ---------------------------------------------------------------------------
constexpr int kDppWaveShl1 = 0x130;
constexpr int kDppWaveShr1 = 0x138;

template <int CTRL>
__device__ __forceinline__ int dpp_i32(int old, int src) {
  return __builtin_amdgcn_update_dpp(old, src, CTRL, 0xF, 0xF, false);
}

template <int CTRL>
__device__ __forceinline__ float dpp(float v, float old) {
  return __int_as_float(dpp_i32<CTRL>(__float_as_int(old), __float_as_int(v)));
}

template <int CTRL>
__device__ __forceinline__ double dpp(double v, double old) {
  const long long x = __double_as_longlong(v), o = __double_as_longlong(old);
  const int lo = dpp_i32<CTRL>((int)o, (int)x);
  const int hi = dpp_i32<CTRL>((int)(o >> 32), (int)(x >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

template <int CTRL>
__device__ __forceinline__ int dpp(int v, int old) {
  return dpp_i32<CTRL>(old, v);
}

template <typename T>
__device__ __forceinline__ T shr1(T v, T old) { return dpp<kDppWaveShr1>(v, old); }
template <typename T>
__device__ __forceinline__ T shl1(T v, T old) { return dpp<kDppWaveShl1>(v, old); }

// Same shifts with 0 shifted in at the wave edge by the DPP bound control (no `old` operand to
// materialise: one instruction per 32-bit half instead of a zeroing move plus the DPP move).
template <int CTRL>
__device__ __forceinline__ int dppz_i32(int src) {
  return __builtin_amdgcn_update_dpp(0, src, CTRL, 0xF, 0xF, true);
}
template <int CTRL>
__device__ __forceinline__ double dppz(double v) {
  const long long x = __double_as_longlong(v);
  const int lo = dppz_i32<CTRL>((int)x), hi = dppz_i32<CTRL>((int)(x >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
template <int CTRL>
__device__ __forceinline__ float dppz(float v) { return __int_as_float(dppz_i32<CTRL>(__float_as_int(v))); }
template <int CTRL>
__device__ __forceinline__ int dppz(int v) { return dppz_i32<CTRL>(v); }
template <typename T>
__device__ __forceinline__ T shr1z(T v) { return dppz<kDppWaveShr1>(v); }
template <typename T>
__device__ __forceinline__ T shl1z(T v) { return dppz<kDppWaveShl1>(v); }

// Pin a value as computed on every lane: stops the compiler from sinking its (branch-free)
// computation under the lane mask of a later select/store, so independent row chains stay in one
// basic block where they can be interleaved.
template <typename T>
__device__ __forceinline__ T keep(T x) {
  asm volatile("" : "+v"(x));
  return x;
}

// ---------------------------------------------------------------------------
// XCD-aware block remap (bijective for any grid size): the dispatcher deals blocks
// round-robin over the 8 XCDs, so blocks b, b+8, ... share an L2.  Remapping gives each
// XCD a CONTIGUOUS range of logical tiles, so vertically/horizontally adjacent tiles
// (which share halo rows/lines) are served by one L2.  Placement changes speed only.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int xcd_remap(int bid, int nblk) {
  const int xcd = bid & 7;
  const int q = nblk >> 3, r = nblk & 7;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }

// Deterministic wave-level sum (fixed butterfly order).
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// Fixed-order reduction of `n` partials per sample -> sqrt.  One 256-thread block per sample.
// (internal linkage: each translation unit launches its own copy)
static __global__ __launch_bounds__(256) void k_norm_final(const double* __restrict__ part, long long n,
                                                           double* __restrict__ out) {
  __shared__ double sh[256];
  const double* p = part + blockIdx.x * n;
  double s = 0.0;
  for (long long i = threadIdx.x; i < n; i += 256) s += p[i];
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) sh[threadIdx.x] += sh[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[blockIdx.x] = sqrt(sh[0]);
}

}  // namespace fea

#define FEA_LAUNCH_CHECK()                   \
  do {                                       \
    hipError_t _e = hipGetLastError();       \
    return _e == hipSuccess ? 0 : (int)_e;   \
  } while (0)
