// sweep_lab.hip — variants of the fine-level Poisson fp64 Jacobi sweep for A/B timing
// (not part of the product library).  Same framed layout and arithmetic as fea_mg_sweep_f64.
//   NV : 16-byte vectors per lane per row (sub-strips of 128 columns; strip = 128*NV columns)
//   PF : rows of u in flight ahead of the row being computed (f: PF-1 ahead, min 1)
//   NT : nontemporal stores of u'
#include <hip/hip_runtime.h>
#include "fea_common.h"

using namespace fea;

namespace {
constexpr int A = 16, OFF = 15;

__device__ __forceinline__ double rdlane(double v, int l) {
  const long long x = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)x, l);
  const int hi = __builtin_amdgcn_readlane((int)(x >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

typedef double d2 __attribute__((ext_vector_type(2)));

template <int NV>
struct Raw {
  d2 x[NV];
  d2 h;
};
template <int NV>
struct Win {
  double a[NV][4];
};

template <int NV>
__device__ __forceinline__ Raw<NV> raw(const double* rp, int lane) {
  Raw<NV> r;
#pragma unroll
  for (int j = 0; j < NV; ++j) r.x[j] = *reinterpret_cast<const d2*>(rp + j * 128 + 2 * lane);
  r.h = d2{0.0, 0.0};
  if (lane == 0 || lane == 63) r.h = *reinterpret_cast<const d2*>(rp + (lane == 0 ? -2 : NV * 128));
  return r;
}

template <int NV>
__device__ __forceinline__ Win<NV> fin(const Raw<NV>& r) {
  Win<NV> w;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    w.a[j][1] = r.x[j][0];
    w.a[j][2] = r.x[j][1];
    const double lo = (j == 0) ? r.h[1] : rdlane(r.x[j - 1][1], 63);
    const double ro = (j == NV - 1) ? r.h[0] : rdlane(r.x[j + 1][0], 0);
    w.a[j][0] = shr1(r.x[j][1], lo);
    w.a[j][3] = shl1(r.x[j][0], ro);
  }
  return w;
}

template <int NV, int PF, bool NT>
__global__ __launch_bounds__(256) void lab_sweep(const double* __restrict__ u, const double* __restrict__ f,
                                                 double* __restrict__ out, const double* __restrict__ ktab,
                                                 const double* __restrict__ omd, int N, int ld, int rb, int nstrips,
                                                 int ntr) {
  const int nsg = (nstrips + 3) / 4;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int t = bid / nsg;
  const int s = (bid - t * nsg) * 4 + (threadIdx.x >> 6);
  if (s >= nstrips || t >= ntr) return;
  const int lane = threadIdx.x & 63;
  const int c0 = 1 + s * 128 * NV;
  const int r0 = 1 + t * rb;
  const int r1 = min(r0 + rb, N - 1);
  double ks[9];
#pragma unroll
  for (int d = 0; d < 9; ++d) ks[d] = ktab[d];
  const double om = omd[0];
  const long long poff = OFF + c0;
  const double* ub = u + poff;
  const double* fb = f + poff;
  double* ob = out + poff;
  auto rowo = [&](int r) -> long long { return (long long)(min(r, N) + 1) * ld; };
  constexpr int FP = PF > 1 ? PF - 1 : 1;  // f rows ahead
  Win<NV> w0 = fin(raw<NV>(ub + rowo(r0 - 1), lane));
  Win<NV> w1 = fin(raw<NV>(ub + rowo(r0), lane));
  Raw<NV> ring[PF];
#pragma unroll
  for (int i = 0; i < PF; ++i) ring[i] = raw<NV>(ub + rowo(r0 + 1 + i), lane);
  d2 fr[FP][NV];
#pragma unroll
  for (int i = 0; i < FP; ++i)
#pragma unroll
    for (int j = 0; j < NV; ++j) fr[i][j] = *reinterpret_cast<const d2*>(fb + rowo(r0 + i) + j * 128 + 2 * lane);
  for (int r = r0; r < r1; ++r) {
    const Raw<NV> nn = raw<NV>(ub + rowo(r + 1 + PF), lane);
    d2 fn[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) fn[j] = *reinterpret_cast<const d2*>(fb + rowo(r + FP) + j * 128 + 2 * lane);
    const Win<NV> w2 = fin(ring[0]);
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      d2 o;
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        double acc = ks[0] * w0.a[j][k];
        acc += ks[1] * w0.a[j][k + 1];
        acc += ks[2] * w0.a[j][k + 2];
        acc += ks[3] * w1.a[j][k];
        acc += ks[4] * w1.a[j][k + 1];
        acc += ks[5] * w1.a[j][k + 2];
        acc += ks[6] * w2.a[j][k];
        acc += ks[7] * w2.a[j][k + 1];
        acc += ks[8] * w2.a[j][k + 2];
        o[k] = om * (fr[0][j][k] - acc) + w1.a[j][k + 1];
      }
      const int cl = c0 + j * 128 + 2 * lane;
      double* p = ob + rowo(r) + j * 128 + 2 * lane;
      if (cl + 1 <= N - 2) {
        if constexpr (NT)
          __builtin_nontemporal_store(o, reinterpret_cast<d2*>(p));
        else
          *reinterpret_cast<d2*>(p) = o;
      } else if (cl <= N - 2) {
        p[0] = o[0];
      }
    }
    w0 = w1;
    w1 = w2;
#pragma unroll
    for (int i = 0; i < PF - 1; ++i) ring[i] = ring[i + 1];
    ring[PF - 1] = nn;
#pragma unroll
    for (int i = 0; i < FP - 1; ++i)
#pragma unroll
      for (int j = 0; j < NV; ++j) fr[i][j] = fr[i + 1][j];
#pragma unroll
    for (int j = 0; j < NV; ++j) fr[FP - 1][j] = fn[j];
  }
}

template <int NV, int PF, bool NT>
int launch(const double* u, const double* f, double* out, const double* ktab, const double* omd, int N, int ld,
           int rb, hipStream_t st) {
  const int nstrips = (N - 2 + 128 * NV - 1) / (128 * NV);
  const int ntr = (N - 2 + rb - 1) / rb;
  const int grid = ntr * ((nstrips + 3) / 4);
  hipLaunchKernelGGL((lab_sweep<NV, PF, NT>), dim3(grid), dim3(256), 0, st, u, f, out, ktab, omd, N, ld, rb, nstrips,
                     ntr);
  return (int)hipGetLastError();
}
}  // namespace

extern "C" int lab_sweep_f64(int variant, const double* u, const double* f, double* out, const double* ktab,
                             const double* omd, int N, int ld, int rb, hipStream_t st) {
  // variant = NV*100 + PF*10 + NT
  switch (variant) {
#define V_(nv, pf, nt) \
  case nv * 100 + pf * 10 + nt: return launch<nv, pf, nt>(u, f, out, ktab, omd, N, ld, rb, st);
    V_(1, 1, 0) V_(1, 1, 1) V_(1, 2, 0) V_(1, 2, 1) V_(1, 3, 0) V_(1, 3, 1)
    V_(2, 1, 0) V_(2, 1, 1) V_(2, 2, 0) V_(2, 2, 1)
    V_(4, 1, 0) V_(4, 1, 1)
#undef V_
    default: return -1;
  }
}
