// stream_probe.hip — lab kernels (not part of the product library): what limits a 2-read + 1-write
// stream over fields far larger than the Infinity Cache (8193^2 fp64: ~540 MB per field)?
//
// Every variant moves exactly the same bytes: `units` 1 KiB pieces of u and f read, of out written
// (one 16-byte load per lane per piece), out = u + c*f, nontemporal stores as the product kernels use
// at this size.  Only the ORDER in which a wave visits its pieces differs:
//   MODE 0 "linear": wave w takes `rb` consecutive pieces of the flat buffers (a copy kernel);
//   MODE 1 "strip" : the product kernels' order — wave (row task t, strip s) walks rows
//                    t*rb .. t*rb+rb-1 of a 128-column strip, consecutive pieces one row pitch
//                    (`ld` doubles) apart;
//   MODE 2 "tile"  : pieces laid out strip-major (all rows of strip 0, then strip 1 ...), so the
//                    strip-march of MODE 1 reads consecutive addresses (a column-strip-blocked layout).
// Launch: 4 waves per 256-thread workgroup, consecutive waves take consecutive tasks; `remap` applies
// the product's XCD remap to the workgroup index.
#include <hip/hip_runtime.h>

#include "fea_common.h"

using namespace fea;

namespace {
typedef double d2 __attribute__((ext_vector_type(2)));

template <int MODE>
__device__ __forceinline__ long long piece(long long task, int k, int rb, int nstrips, int ld, int rows) {
  if constexpr (MODE == 0) {
    return (task * rb + k) * 128;
  } else if constexpr (MODE == 1) {
    const long long t = task / nstrips, s = task - t * nstrips;
    return (t * rb + k) * (long long)ld + s * 128;
  } else {
    const long long t = task / nstrips, s = task - t * nstrips;
    return (s * rows + t * rb + k) * 128;
  }
}

template <int MODE>
__global__ __launch_bounds__(256) void probe(const double* __restrict__ u, const double* __restrict__ f,
                                             double* __restrict__ out, long long ntask, int rb, int nstrips, int ld,
                                             int rows, int remap) {
  const int bid = remap ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const long long task = (long long)bid * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  if (task >= ntask) return;
  const int lane = threadIdx.x & 63;
  const long long o0 = piece<MODE>(task, 0, rb, nstrips, ld, rows) + 2 * lane;
  d2 un = *reinterpret_cast<const d2*>(u + o0);
  d2 fn = *reinterpret_cast<const d2*>(f + o0);
  for (int k = 0; k < rb; ++k) {
    const long long o = piece<MODE>(task, k, rb, nstrips, ld, rows) + 2 * lane;
    const d2 uc = un, fc = fn;
    if (k + 1 < rb) {
      const long long o1 = piece<MODE>(task, k + 1, rb, nstrips, ld, rows) + 2 * lane;
      un = *reinterpret_cast<const d2*>(u + o1);
      fn = *reinterpret_cast<const d2*>(f + o1);
    }
    const d2 r = uc + 0.6666 * fc;
    __builtin_nontemporal_store(r, reinterpret_cast<d2*>(out + o));
  }
}
}  // namespace

// rows x (nstrips * 128) doubles per field, row pitch ld (MODE 1) — rows % rb == 0.
extern "C" int lab_stream_probe(int mode, const double* u, const double* f, double* out, int rows, int nstrips,
                                int ld, int rb, int remap, hipStream_t st) {
  if (rb < 1 || rows % rb || ld < nstrips * 128) return -1;
  const long long ntask = (long long)(rows / rb) * nstrips;
  const dim3 grid((unsigned)((ntask + 3) / 4));
  switch (mode) {
    case 0: hipLaunchKernelGGL(probe<0>, grid, dim3(256), 0, st, u, f, out, ntask, rb, nstrips, ld, rows, remap); break;
    case 1: hipLaunchKernelGGL(probe<1>, grid, dim3(256), 0, st, u, f, out, ntask, rb, nstrips, ld, rows, remap); break;
    case 2: hipLaunchKernelGGL(probe<2>, grid, dim3(256), 0, st, u, f, out, ntask, rb, nstrips, ld, rows, remap); break;
    default: return -1;
  }
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------------
// flow<NR, NW, DEPTH, NTL, NTS>: the streaming ceiling.  NR input streams read, NW output streams
// written (out_j = sum of inputs + j), linear 1 KiB pieces, `rb` consecutive pieces per wave, DEPTH
// pieces of every input in flight per wave (a register ring), nontemporal loads / stores by flag.
// ---------------------------------------------------------------------------------------------------
namespace {
template <int NR, int NW, int DEPTH, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void flow(const double* __restrict__ in0, const double* __restrict__ in1,
                                            double* __restrict__ out0, double* __restrict__ out1, long long ntask,
                                            int rb) {
  const long long task = (long long)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  if (task >= ntask) return;
  const int lane = threadIdx.x & 63;
  const long long base = task * rb * 128 + 2 * lane;
  const double* ins[2] = {in0, in1};
  double* outs[2] = {out0, out1};
  d2 ring[DEPTH][NR > 0 ? NR : 1];
  auto ld = [&](int k, int j) -> d2 {
    const d2* p = reinterpret_cast<const d2*>(ins[j] + base + (long long)k * 128);
    if constexpr (NTL) return __builtin_nontemporal_load(p);
    else return *p;
  };
#pragma unroll
  for (int i = 0; i < DEPTH; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) ring[i][j] = (i < rb) ? ld(i, j) : d2{0.0, 0.0};
  d2 acc = {0.0, 0.0};
  for (int k = 0; k < rb; k += DEPTH) {
#pragma unroll
    for (int i = 0; i < DEPTH; ++i) {
      d2 v = {1.0, 2.0};
#pragma unroll
      for (int j = 0; j < NR; ++j) {
        v += ring[i][j];
        if (k + i + DEPTH < rb) ring[i][j] = ld(k + i + DEPTH, j);
      }
      if (k + i < rb) {
#pragma unroll
        for (int j = 0; j < NW; ++j) {
          d2* p = reinterpret_cast<d2*>(outs[j] + base + (long long)(k + i) * 128);
          const d2 w = v + (double)j;
          if constexpr (NTS) __builtin_nontemporal_store(w, p);
          else *p = w;
        }
      }
      acc += v;
    }
  }
  if constexpr (NW == 0) {
    if (acc[0] == 123.456) out0[base] = acc[1];  // keeps the reads alive
  }
}

template <int NR, int NW, int DEPTH, bool NTL, bool NTS>
int flow_launch(const double* a, const double* b, double* c, double* d, long long pieces, int rb, hipStream_t st) {
  const long long ntask = pieces / rb;
  hipLaunchKernelGGL((flow<NR, NW, DEPTH, NTL, NTS>), dim3((unsigned)((ntask + 3) / 4)), dim3(256), 0, st, a, b, c, d,
                     ntask, rb);
  return (int)hipGetLastError();
}
}  // namespace

// variant = NR*10000 + NW*1000 + DEPTH*100 + NTL*10 + NTS
extern "C" int lab_flow(int variant, const double* a, const double* b, double* c, double* d, long long pieces, int rb,
                        hipStream_t st) {
  if (rb < 1 || pieces % rb) return -1;
  switch (variant) {
#define F_(nr, nw, dp, ntl, nts) \
  case nr * 10000 + nw * 1000 + dp * 100 + ntl * 10 + nts: return flow_launch<nr, nw, dp, ntl, nts>(a, b, c, d, pieces, rb, st);
    F_(1, 0, 1, 0, 0) F_(1, 0, 2, 0, 0) F_(1, 0, 4, 0, 0) F_(1, 0, 8, 0, 0) F_(1, 0, 4, 1, 0)
    F_(2, 0, 2, 0, 0) F_(2, 0, 4, 0, 0)
    F_(0, 1, 1, 0, 0) F_(0, 1, 1, 0, 1)
    F_(1, 1, 1, 0, 1) F_(1, 1, 2, 0, 1) F_(1, 1, 4, 0, 1) F_(1, 1, 8, 0, 1) F_(1, 1, 2, 0, 0) F_(1, 1, 4, 1, 1)
    F_(2, 1, 1, 0, 1) F_(2, 1, 2, 0, 1) F_(2, 1, 4, 0, 1) F_(2, 1, 8, 0, 1) F_(2, 1, 2, 0, 0) F_(2, 1, 4, 0, 0)
    F_(2, 1, 4, 1, 1) F_(2, 1, 2, 1, 1)
#undef F_
    default: return -1;
  }
}
