// sr_lab.hip — overlapped-strip variant of the fused sweep+residual+restriction (fp64 Poisson) for
// A/B timing against fea_mg_sweep_restrict_f64 (not part of the product library).
// A wave loads 128 columns starting 2 left of its first owned column and owns the middle 122: the
// u' / residual values its edge lanes get wrong are never stored, so no edge-lane recompute.
#include <hip/hip_runtime.h>
#include "fea_common.h"

using namespace fea;

namespace {
constexpr int OFF = 15;   // frame offset (fp64)
constexpr int S = 122;    // owned fine columns per strip
typedef double d2 __attribute__((ext_vector_type(2)));

struct Win {  // a[0] = col-1, a[1], a[2] own, a[3] = col+2
  double a[4];
};

__device__ __forceinline__ Win mk(const d2 x) {
  Win w;
  w.a[1] = x[0];
  w.a[2] = x[1];
  w.a[0] = shr1(x[1], 0.0);
  w.a[3] = shl1(x[0], 0.0);
  return w;
}
__device__ __forceinline__ Win mk2(double x0, double x1) {
  Win w;
  w.a[1] = x0;
  w.a[2] = x1;
  w.a[0] = shr1(x1, 0.0);
  w.a[3] = shl1(x0, 0.0);
  return w;
}

__device__ __forceinline__ double kap(const Win& a, const Win& b, const Win& c, int k, const double (&ks)[9]) {
  double acc = ks[0] * a.a[k];
  acc += ks[1] * a.a[k + 1];
  acc += ks[2] * a.a[k + 2];
  acc += ks[3] * b.a[k];
  acc += ks[4] * b.a[k + 1];
  acc += ks[5] * b.a[k + 2];
  acc += ks[6] * c.a[k];
  acc += ks[7] * c.a[k + 1];
  acc += ks[8] * c.a[k + 2];
  return acc;
}

template <bool NT, int R>
__global__ __launch_bounds__(256) void sr_ovl(const double* __restrict__ u, const double* __restrict__ f,
                                              double* __restrict__ uo, double* __restrict__ fc,
                                              const double* __restrict__ ktab, const double* __restrict__ omd,
                                              const double* __restrict__ rtab, double w0, int H, int W, int ld,
                                              int ldc, int rb, int nstrips, int ntr) {
  const int nsg = (nstrips + 3) / 4;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int t = bid / nsg;
  const int s = (bid - t * nsg) * 4 + (threadIdx.x >> 6);
  if (s >= nstrips || t >= ntr) return;
  const int lane = threadIdx.x & 63;
  const int Hc = (H + 1) / 2, Wc = (W + 1) / 2;
  const int c0 = 1 + s * S;       // first owned fine column
  const int cs = c0 - 2;          // first loaded column (16-byte aligned)
  const int cl = cs + 2 * lane;   // lane's first column
  const int I0 = 1 + t * (rb / 2);
  const int I1 = min(I0 + rb / 2, Hc - 1);
  double ks[9], rs[9];
#pragma unroll
  for (int d = 0; d < 9; ++d) {
    ks[d] = ktab[d];
    rs[d] = rtab[d];
  }
  const double om = omd[0];
  const bool cin0 = cl >= 1 && cl <= W - 2, cin1 = cl + 1 >= 1 && cl + 1 <= W - 2;
  const bool own = lane >= 1 && lane <= 61;                 // owned columns cl, cl+1 (strip middle)
  const bool st0 = own && cl <= W - 2, st1 = own && cl + 1 <= W - 2;
  const int J = (cl + 1) / 2;                               // coarse column of (cl, cl+1, cl+2)
  const bool cst = own && J <= Wc - 2;
  const double* ub = u + OFF + cs;
  const double* fb = f + OFF + cs;
  double* ob = uo + OFF + cs;
  double* cb = fc + OFF + J;
  auto rowo = [&](int r) -> long long { return (long long)(min(max(r, -1), H) + 1) * ld; };
  auto ld2 = [&](const double* b, int y) -> d2 { return *reinterpret_cast<const d2*>(b + rowo(y) + 2 * lane); };
  // u'(y) own values from u rows y-1..y+1 (windows) and f(y)
  auto sweep = [&](const Win& a, const Win& b, const Win& c, const d2 fy, int y, double& o0, double& o1) {
    const bool rin = y >= 1 && y <= H - 2;
    const double v0 = om * (fy[0] - kap(a, b, c, 0, ks)) + b.a[1];
    const double v1 = om * (fy[1] - kap(a, b, c, 1, ks)) + b.a[2];
    o0 = (rin && cin0) ? v0 : b.a[1];
    o1 = (rin && cin1) ? v1 : b.a[2];
  };
  auto store_u = [&](int y, double o0, double o1) {
    const bool ownr = y >= 2 * I0 - 1 && (y < 2 * I1 - 1 || I1 == Hc - 1) && y <= H - 2;
    if (ownr) {
      double* p = ob + rowo(y) + 2 * lane;
      if (st0 && st1) {
        d2 v = {o0, o1};
        if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<d2*>(p));
        else *reinterpret_cast<d2*>(p) = v;
      } else if (st0) {
        p[0] = o0;
      }
    }
  };
  // residual row -> restriction contribution (row weight ky) for the lane's coarse column
  auto rrow = [&](const Win& a, const Win& b, const Win& c, const d2 fy, int ky) -> double {
    const double r0 = fy[0] - kap(a, b, c, 0, ks);
    const double r1 = fy[1] - kap(a, b, c, 1, ks);
    const double r2 = shl1(r0, 0.0);  // column cl+2 from the next lane
    double tt = rs[ky * 3 + 0] * r0;
    tt += rs[ky * 3 + 1] * r1;
    tt += rs[ky * 3 + 2] * r2;
    return tt;
  };
  const int ya = 2 * I0 - 1;  // first residual row
  // ring of raw rows ahead of use: ru[i] = u row (next + i), rf[i] = f row (next + i - 1)
  Win X0 = mk(ld2(ub, ya - 2)), X1 = mk(ld2(ub, ya - 1)), X2 = mk(ld2(ub, ya)), X3 = mk(ld2(ub, ya + 1));
  d2 F1 = ld2(fb, ya - 1), F2 = ld2(fb, ya), F3 = ld2(fb, ya + 1);
  d2 ru[R], rf[R];
#pragma unroll
  for (int i = 0; i < R; ++i) {
    ru[i] = ld2(ub, ya + 2 + i);
    rf[i] = ld2(fb, ya + 2 + i);
  }
  double p0, p1, q0, q1, s0, s1;
  Win X4 = mk(ru[0]);
  d2 F4 = rf[0];
  sweep(X0, X1, X2, F1, ya - 1, p0, p1);  // u'(ya-1)
  sweep(X1, X2, X3, F2, ya, q0, q1);      // u'(ya)
  store_u(ya, q0, q1);
  sweep(X2, X3, X4, F3, ya + 1, s0, s1);  // u'(ya+1)
  store_u(ya + 1, s0, s1);
  Win Up = mk2(p0, p1), Uc = mk2(q0, q1), Un = mk2(s0, s1);
  double acc = rrow(Up, Uc, Un, F2, 0);   // residual row ya -> coarse I0 with ky = 0
  // rotate: ring[0] (row ya+2) consumed as X4 / F4
  auto shift = [&](int next_row) {
#pragma unroll
    for (int i = 0; i + 1 < R; ++i) {
      ru[i] = ru[i + 1];
      rf[i] = rf[i + 1];
    }
    ru[R - 1] = ld2(ub, next_row);
    rf[R - 1] = ld2(fb, next_row);
  };
  shift(ya + 2 + R);
  // state for coarse row I: u' rows 2I-1 (Uc), 2I (Un); u rows 2I (X3), 2I+1 (X4); f rows 2I (F3),
  // 2I+1 (F4); ring rows 2I+2 ...
  for (int I = I0; I < I1; ++I) {
    const Win X5 = mk(ru[0]);             // u row 2I+2
    const d2 F5 = rf[0];
    shift(2 * I + 2 + R);
    double a0, a1;
    sweep(X3, X4, X5, F4, 2 * I + 1, a0, a1);  // u'(2I+1)
    store_u(2 * I + 1, a0, a1);
    const Win U1 = mk2(a0, a1);
    acc += rrow(Uc, Un, U1, F3, 1);       // residual row 2I
    const Win X6 = mk(ru[0]);             // u row 2I+3
    const d2 F6 = rf[0];
    shift(2 * I + 3 + R);
    double b0, b1;
    sweep(X4, X5, X6, F5, 2 * I + 2, b0, b1);  // u'(2I+2)
    store_u(2 * I + 2, b0, b1);
    const Win U2 = mk2(b0, b1);
    const double rr = rrow(Un, U1, U2, F4, 2);  // residual row 2I+1: ky = 2 for I
    const double o = w0 * (acc + rr);
    if (cst) cb[(long long)(I + 1) * ldc] = o;
    acc = rrow(Un, U1, U2, F4, 0);        // ... and ky = 0 for I+1
    Uc = U1;
    Un = U2;
    X3 = X5;
    X4 = X6;
    F3 = F5;
    F4 = F6;
  }
}

template <int R>
int launch(bool nt, const double* u, const double* f, double* uo, double* fc, const double* ktab, const double* omd,
           const double* rtab, double w0, int H, int W, int ld, int ldc, int rb, hipStream_t st) {
  const int nstrips = (W - 2 + S - 1) / S;
  const int Hc = (H + 1) / 2;
  const int ntr = (Hc - 2 + rb / 2 - 1) / (rb / 2);
  const int grid = ntr * ((nstrips + 3) / 4);
  if (nt)
    hipLaunchKernelGGL((sr_ovl<true, R>), dim3(grid), dim3(256), 0, st, u, f, uo, fc, ktab, omd, rtab, w0, H, W, ld,
                       ldc, rb, nstrips, ntr);
  else
    hipLaunchKernelGGL((sr_ovl<false, R>), dim3(grid), dim3(256), 0, st, u, f, uo, fc, ktab, omd, rtab, w0, H, W,
                       ld, ldc, rb, nstrips, ntr);
  return (int)hipGetLastError();
}
}  // namespace

extern "C" int lab_sr_f64(int var, const double* u, const double* f, double* uo, double* fc, const double* ktab,
                          const double* omd, const double* rtab, double w0, int H, int W, int ld, int ldc, int rb,
                          hipStream_t st) {
  const bool nt = var % 10;
  switch (var / 10) {
    case 1: return launch<1>(nt, u, f, uo, fc, ktab, omd, rtab, w0, H, W, ld, ldc, rb, st);
    case 2: return launch<2>(nt, u, f, uo, fc, ktab, omd, rtab, w0, H, W, ld, ldc, rb, st);
    case 4: return launch<4>(nt, u, f, uo, fc, ktab, omd, rtab, w0, H, W, ld, ldc, rb, st);
    case 6: return launch<6>(nt, u, f, uo, fc, ktab, omd, rtab, w0, H, W, ld, ldc, rb, st);
    default: return -1;
  }
}
