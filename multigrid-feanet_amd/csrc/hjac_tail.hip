// hjac_tail.hip — the coarse end of the learned-smoother V-cycle in ONE launch.
//
// MultiGrid.Step with mode='hjac' (M-FEANet-mg_test.ipynb:27346-27372, Relax = HJacIterator.HRelax :147-155)
// runs, below the finest levels, a V-cycle whose every relaxation is one HRelax sweep
//     j = J(u, f);  d_0 = j - u;  d_l = (W_l * d_(l-1)) . g;  u' = j + d_nl
// and whose coarse levels start from a zero guess.  Streamed level by level (feanet_amd.schedule.hjac_schedule)
// that is four launches per level and direction, each a few microseconds of latency on levels of <= 65^2 nodes
// (8-11 us per fea_mg_hsweep launch there, profiles/r03z_configs/trace_hjac4097.txt).  Here one 1024-thread
// workgroup per sample keeps every level of the coarse end (f and u of each level, two scratch fields of the top
// level's size, pattern maps and tables) resident in LDS and runs the whole sub-cycle — zero-guess pre-sweeps,
// residual + restriction, the coarsest sweeps, prolongation + correction, post-sweeps — with workgroup barriers
// between the phases.  It reads f_t once from HBM and writes u_t once, in the framed layout.
//
// Every node value is the same expression, in the same order, as the per-level kernels the streamed schedule
// runs (fea_mg_hsweep, fea_mg_residual_restrict with a stored iterate, fea_mg_prolong_add; -ffp-contract=on),
// so the result is bitwise theirs (tests/test_gpu_hnet.py).  An HRelax sweep is nl + 1 phases:
//   P0:        A = j, B = d_0 (interior; 0 elsewhere)
//   layer 0:   nl == 1: u = A + conv_0(B);  else u = A, A = conv_0(B)
//   layer l:   last: u = u + conv_l(.);     else the other scratch field = conv_l(.)
#include "fea_common.h"

namespace fea {

constexpr int kHTailThreads = 1024;
constexpr int kHTailMaxLevels = 8;
constexpr int kHTailMaxN = 65;
constexpr int kHTailLdsBytes = 160 * 1024 - 1024;
constexpr int kHTailTS = 10;  // table stride (9 weights + omega/d)
constexpr int kHTailMaxLayers = 3;

template <typename T>
struct HTailArgs {
  const T* f_t;
  T* u_t;
  const uint8_t* pid;  // compact concatenated per-level maps (NULL: single pattern)
  const T* ktab;
  const T* omd;
  const T* rtab;
  const T* ptab;
  const T* hw;
  T w0, w1;
  int Ht, Wt, nlev, ld_t;
  long long bs_t;
  int ntab, nl, nu1, nu2;
  int zmask;  // 0 (staged weight loads)
};

__host__ __device__ inline int htail_n(int n0, int k) { return ((n0 - 1) >> k) + 1; }

__host__ __device__ inline long long htail_elems(int Ht, int Wt, int nlev) {
  long long s = 0;
  for (int k = 0; k < nlev; ++k) s += (long long)htail_n(Ht, k) * htail_n(Wt, k);
  return s;
}

// f and u of every level, two scratch fields of the top level, the tables, the pattern maps
template <typename T>
__host__ __device__ inline long long htail_lds_bytes(int Ht, int Wt, int nlev, bool multi) {
  const long long e = htail_elems(Ht, Wt, nlev);
  long long b = (2 * e + 2LL * Ht * Wt) * (long long)sizeof(T);
  b += (3LL * FEA_MAX_PATTERNS * kHTailTS + kHTailMaxLayers * 9) * sizeof(T);
  if (multi) b += (e + 15) / 16 * 16;
  return b;
}

template <typename T, bool MULTI>
struct HTail {
  const HTailArgs<T>& a;
  const T* ktb;  // ntab x 10 (weights, omega/d)
  const T* rtb;
  const T* ptb;
  const T* hk;   // nl x 9
  T ks[9], rs[9], ps[9], om0;
  int tid;
  mutable int z;  // 0; "changed" by an empty asm at every pass (stage()): the weights are re-read per pass

  template <typename U>
  __device__ __forceinline__ static U kload(const U* p, int i) {  // scalar read-only load (constant space)
    return ((const __attribute__((address_space(4))) U*)p)[i];
  }
  // fp64 single-pattern: each pass re-reads its weights (after the barrier, hoisted to the pass's start) instead
  // of keeping all 28 in SGPRs the compiler parks in VGPR lanes
  static constexpr bool kStage = !MULTI && sizeof(T) == 8;
  __device__ __forceinline__ void stage() const {
    if constexpr (kStage) asm volatile("" : "+s"(z));
  }

  __device__ __forceinline__ T kw(const uint8_t* pk, int i, int d) const {
    if constexpr (MULTI) return ktb[pk[i] * kHTailTS + d];
    else if constexpr (kStage) return kload(a.ktab, z + d);
    return ks[d];
  }
  __device__ __forceinline__ T omk(const uint8_t* pk, int i) const {
    if constexpr (MULTI) return ktb[pk[i] * kHTailTS + 9];
    else if constexpr (kStage) return kload(a.omd, z);
    return om0;
  }
  __device__ __forceinline__ T rw(const uint8_t* pk, int i, int d) const {
    if constexpr (MULTI) return rtb[pk[i] * kHTailTS + d];
    else if constexpr (kStage) return kload(a.rtab, z + d);
    return rs[d];
  }
  __device__ __forceinline__ T pw(const uint8_t* pk, int i, int d) const {
    if constexpr (MULTI) return ptb[pk[i] * kHTailTS + d];
    else if constexpr (kStage) return kload(a.ptab, z + d);
    return ps[d];
  }
  // (K x)(i) at an interior node of a W-wide level (taps in row-major order, the weight by the tap node's pattern)
  __device__ __forceinline__ T kx(const T* x, const uint8_t* pk, int i, int W) const {
    const int n = i - W, s = i + W;
    T acc = kw(pk, n - 1, 0) * x[n - 1];
    acc += kw(pk, n, 1) * x[n];
    acc += kw(pk, n + 1, 2) * x[n + 1];
    acc += kw(pk, i - 1, 3) * x[i - 1];
    acc += kw(pk, i, 4) * x[i];
    acc += kw(pk, i + 1, 5) * x[i + 1];
    acc += kw(pk, s - 1, 6) * x[s - 1];
    acc += kw(pk, s, 7) * x[s];
    acc += kw(pk, s + 1, 8) * x[s + 1];
    return acc;
  }
  // HNet layer l (cross-correlation, zero padding) at an interior node
  __device__ __forceinline__ T conv(const T* d, int l, int i, int W) const {
    const T* h = hk + l * 9;  // (LDS)
    const int n = i - W, s = i + W;
    T acc = h[0] * d[n - 1];
    acc += h[1] * d[n];
    acc += h[2] * d[n + 1];
    acc += h[3] * d[i - 1];
    acc += h[4] * d[i];
    acc += h[5] * d[i + 1];
    acc += h[6] * d[s - 1];
    acc += h[7] * d[s];
    acc += h[8] * d[s + 1];
    return acc;
  }
  // i / W for the tail's node indices (i < 65 * 65, W <= 65): (i + 0.5) / W lies at least 0.5 / W from an
  // integer, far beyond the float rounding of the product, so the truncation is the exact quotient (an integer
  // division is ~25 VALU per node and pass here)
  __device__ __forceinline__ static int divw(int i, int W) {
    return (int)(((float)i + 0.5f) * __frcp_rn((float)W));
  }
  __device__ __forceinline__ static bool inner(int i, int H, int W) {
    const int y = divw(i, W), c = i - y * W;
    return y >= 1 && y <= H - 2 && c >= 1 && c <= W - 2;
  }

  // one HRelax sweep of u in place (A, B: scratch fields of >= H*W)
  __device__ void hrelax(int H, int W, const T* f, T* u, const uint8_t* pk, T* A, T* B) const {
    const int n = H * W;
    stage();
    for (int i = tid; i < n; i += kHTailThreads) {
      T j = T(0), d = T(0);
      if (inner(i, H, W)) {
        const T acc = kx(u, pk, i, W);
        j = omk(pk, i) * (f[i] - acc) + u[i];
        d = j - u[i];
      }
      A[i] = j;
      B[i] = d;
    }
    __syncthreads();
    const int nl = a.nl;
    if (nl == 0) {
      for (int i = tid; i < n; i += kHTailThreads)
        if (inner(i, H, W)) u[i] = A[i];
      __syncthreads();
      return;
    }
    for (int l = 0; l < nl; ++l) {
      const T* src = (l & 1) ? A : B;
      T* dst = (l & 1) ? B : A;
      const bool last = l == nl - 1;
      for (int i = tid; i < n; i += kHTailThreads) {
        const bool in = inner(i, H, W);
        const T c = in ? conv(src, l, i, W) : T(0);
        if (l == 0) {
          if (last) {
            if (in) u[i] = A[i] + c;
          } else {
            if (in) u[i] = A[i];
            A[i] = c;  // d_1 (the same thread read A[i] above)
          }
        } else if (last) {
          if (in) u[i] = u[i] + c;
        } else {
          dst[i] = c;
        }
      }
      __syncthreads();
    }
  }

  // f_c = w0 R (f - K u) on the coarse interior (fea_mg_residual_restrict with a stored iterate)
  __device__ void restrict_(int H, int W, const T* f, const T* u, const uint8_t* pk, T* fc) const {
    const int Hc = (H + 1) / 2, Wc = (W + 1) / 2;
    const int n = (Hc - 2) * (Wc - 2);
    stage();
    for (int t = tid; t < n; t += kHTailThreads) {
      const int I = divw(t, Wc - 2) + 1, J = t - (I - 1) * (Wc - 2) + 1;
      T r[9];
#pragma unroll
      for (int dy = 0; dy < 3; ++dy)
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
          const int i = (2 * I - 1 + dy) * W + 2 * J - 1 + dx;
          r[dy * 3 + dx] = f[i] - kx(u, pk, i, W);
        }
      const int i0 = (2 * I - 1) * W + 2 * J - 1;
      T acc = rw(pk, i0, 0) * r[0];
      acc += rw(pk, i0 + 1, 1) * r[1];
      acc += rw(pk, i0 + 2, 2) * r[2];
      acc += rw(pk, i0 + W, 3) * r[3];
      acc += rw(pk, i0 + W + 1, 4) * r[4];
      acc += rw(pk, i0 + W + 2, 5) * r[5];
      acc += rw(pk, i0 + 2 * W, 6) * r[6];
      acc += rw(pk, i0 + 2 * W + 1, 7) * r[7];
      acc += rw(pk, i0 + 2 * W + 2, 8) * r[8];
      fc[I * Wc + J] = a.w0 * acc;
    }
    __syncthreads();
  }

  // coarse row a's contribution at fine column x with row tap ky (crow_term of framed_ops.hip)
  __device__ __forceinline__ T crow(const T* e, const uint8_t* pc, int Wc, int ar, int ky, int x) const {
    if (!(x & 1)) {  // even fine column: one coarse node, kx = 1
      const int i = ar * Wc + x / 2;
      return pw(pc, i, ky * 3 + 1) * e[i];
    }
    const int i = ar * Wc + (x - 1) / 2;  // odd: coarse nodes (x-1)/2 (kx = 2) and (x+1)/2 (kx = 0)
    T t = pw(pc, i, ky * 3 + 2) * e[i];
    t += pw(pc, i + 1, ky * 3 + 0) * e[i + 1];
    return t;
  }
  // u += w1 P e on the fine interior (fea_mg_prolong_add)
  __device__ void prolong_add(int H, int W, T* u, const T* e, const uint8_t* pc) const {
    const int Wc = (W + 1) / 2;
    const T w1 = a.w1;
    stage();
    for (int i = tid; i < H * W; i += kHTailThreads) {
      if (!inner(i, H, W)) continue;
      const int y = divw(i, W), x = i - y * W;
      if (!(y & 1)) {
        u[i] += w1 * crow(e, pc, Wc, y / 2, 1, x);
      } else {
        const T t = crow(e, pc, Wc, (y - 1) / 2, 2, x) + crow(e, pc, Wc, (y + 1) / 2, 0, x);
        u[i] += w1 * t;
      }
    }
    __syncthreads();
  }
};

template <typename T, bool MULTI>
__global__ __launch_bounds__(kHTailThreads) void k_hjac_tail(HTailArgs<T> a) {
  __shared__ __attribute__((aligned(16))) char smem[kHTailLdsBytes];
  const int tid = threadIdx.x;
  const int Ht = a.Ht, Wt = a.Wt, nlev = a.nlev;
  const long long e = htail_elems(Ht, Wt, nlev);
  T* fs = reinterpret_cast<T*>(smem);  // f of every level
  T* us = fs + e;                      // u of every level
  T* A = us + e;                       // scratch (top level's size)
  T* Bf = A + Ht * Wt;
  T* tabs = Bf + Ht * Wt;
  T* ktb = tabs;
  T* rtb = ktb + FEA_MAX_PATTERNS * kHTailTS;
  T* ptb = rtb + FEA_MAX_PATTERNS * kHTailTS;
  T* hk = ptb + FEA_MAX_PATTERNS * kHTailTS;
  uint8_t* pl = reinterpret_cast<uint8_t*>(hk + kHTailMaxLayers * 9);
  const T* fg = a.f_t + (long long)blockIdx.x * a.bs_t + (128 / (int)sizeof(T) - 1);

  // zero every level's f and u (boundaries stay zero), load the tables, maps and f_t
  for (long long i = tid; i < 2 * e; i += kHTailThreads) fs[i] = T(0);
  for (int i = tid; i < a.ntab * kHTailTS; i += kHTailThreads) {
    const int p = i / kHTailTS, d = i - p * kHTailTS;
    ktb[i] = d == 9 ? a.omd[p] : a.ktab[p * 9 + d];
    rtb[i] = d == 9 ? T(0) : a.rtab[p * 9 + d];
    ptb[i] = d == 9 ? T(0) : a.ptab[p * 9 + d];
  }
  for (int i = tid; i < a.nl * 9; i += kHTailThreads) hk[i] = a.hw[i];
  if constexpr (MULTI)
    for (long long i = tid; i < e; i += kHTailThreads) pl[i] = a.pid[i];
  __syncthreads();
  for (int i = tid; i < Ht * Wt; i += kHTailThreads) {
    const int r = i / Wt, c = i - r * Wt;
    fs[i] = fg[(long long)(r + 1) * a.ld_t + c];
  }
  HTail<T, MULTI> t{a, ktb, rtb, ptb, hk, {}, {}, {}, T(0), tid, a.zmask};
  if constexpr (!MULTI) {
#pragma unroll
    for (int d = 0; d < 9; ++d) {
      t.ks[d] = a.ktab[d];
      t.rs[d] = a.rtab[d];
      t.ps[d] = a.ptab[d];
    }
    t.om0 = a.omd[0];
  }
  __syncthreads();

  // down: nu1 zero-guess pre-sweeps, residual + restriction
  long long o = 0;
  for (int k = 0; k < nlev - 1; ++k) {
    const int H = htail_n(Ht, k), W = htail_n(Wt, k);
    for (int s = 0; s < a.nu1; ++s) t.hrelax(H, W, fs + o, us + o, pl + o, A, Bf);
    t.restrict_(H, W, fs + o, us + o, pl + o, fs + o + H * W);
    o += H * W;
  }
  {  // coarsest: nu1 + nu2 sweeps from zero
    const int H = htail_n(Ht, nlev - 1), W = htail_n(Wt, nlev - 1);
    for (int s = 0; s < a.nu1 + a.nu2; ++s) t.hrelax(H, W, fs + o, us + o, pl + o, A, Bf);
  }
  // up: prolongation + correction, nu2 post-sweeps
  for (int k = nlev - 2; k >= 0; --k) {
    const int H = htail_n(Ht, k), W = htail_n(Wt, k);
    const long long oc = o;
    o -= H * W;
    t.prolong_add(H, W, us + o, us + oc, pl + oc);
    for (int s = 0; s < a.nu2; ++s) t.hrelax(H, W, fs + o, us + o, pl + o, A, Bf);
  }
  T* dst = a.u_t + (long long)blockIdx.x * a.bs_t + (128 / (int)sizeof(T) - 1);
  for (int i = tid; i < Ht * Wt; i += kHTailThreads) {
    const int r = i / Wt, c = i - r * Wt;
    if (r > 0 && r < Ht - 1 && c > 0 && c < Wt - 1) dst[(long long)(r + 1) * a.ld_t + c] = us[i];
  }
}

// ---------------------------------------------------------------------------------------------------------------
// V(1,1) fast path (k_hjac_tail_fast): ONE workgroup barrier per level and direction.  A wave owns a block of rows
// and streams them through register windows exactly as the level kernels do (hnet_ops.hip hsweep_task, with one
// column per lane: lane c = column c, levels are <= 65 wide, column 64 a boundary column read as 0): every HRelax
// stage one row behind the previous one, neighbour columns by DPP, the halo rows of its block recomputed instead of
// exchanged.  Per level going down, one pass: the zero-guess sweep, its residual and the restriction (hsweep MODE 2,
// ZERO), the pre-smoothed iterate's owned rows kept in LDS; at the coarsest level two sweeps; going up, one pass:
// prolongation + correction + sweep (hsweep MODE 1) into a scratch field (the top level straight to HBM).  Same
// per-node expressions, in the same order, as those kernels: bitwise the general path and the streamed schedule
// (tests/test_gpu_hnet.py::test_hjac_tail_bitwise).  The general path below takes ~50 barrier phases at 33^2 x 5 levels.
// ---------------------------------------------------------------------------------------------------------------
template <typename T>
struct HW1 {  // a row at the lane's column: a[0] = left neighbour, a[1] = own, a[2] = right neighbour
  T a[3];
};
template <typename T>
__device__ __forceinline__ HW1<T> hw1(T x) {
  HW1<T> w;
  w.a[1] = x;
  w.a[0] = shr1z(x);
  w.a[2] = shl1z(x);
  return w;
}
__device__ __forceinline__ HW1<int> hp1(int p) {  // pattern table-row offsets (pattern * kHTailTS)
  HW1<int> w;
  w.a[1] = p * kHTailTS;
  w.a[0] = shr1z(p) * kHTailTS;
  w.a[2] = shl1z(p) * kHTailTS;
  return w;
}

template <typename T, bool MULTI, int NL>
struct HTailFast {
  const HTailArgs<T>& a;
  const T* ktb;  // LDS tables (MULTI)
  const T* rtb;
  const T* ptb;
  int lane;

  template <typename U>
  __device__ __forceinline__ static U cl(const U* p, int i) {  // scalar read-only load
    return ((const __attribute__((address_space(4))) U*)p)[i];
  }
  // (K x) at the lane's column from a 3-row window (hsweep_task's tap order), weights by the tap node's pattern
  __device__ __forceinline__ T kx(const HW1<T>& x0, const HW1<T>& x1, const HW1<T>& x2, const HW1<int>& p0,
                                  const HW1<int>& p1, const HW1<int>& p2, const T (&ks)[9]) const {
    T acc;
    if constexpr (!MULTI) {
      acc = ks[0] * x0.a[0];
      acc += ks[1] * x0.a[1];
      acc += ks[2] * x0.a[2];
      acc += ks[3] * x1.a[0];
      acc += ks[4] * x1.a[1];
      acc += ks[5] * x1.a[2];
      acc += ks[6] * x2.a[0];
      acc += ks[7] * x2.a[1];
      acc += ks[8] * x2.a[2];
    } else {
      acc = ktb[p0.a[0] + 0] * x0.a[0];
      acc += ktb[p0.a[1] + 1] * x0.a[1];
      acc += ktb[p0.a[2] + 2] * x0.a[2];
      acc += ktb[p1.a[0] + 3] * x1.a[0];
      acc += ktb[p1.a[1] + 4] * x1.a[1];
      acc += ktb[p1.a[2] + 5] * x1.a[2];
      acc += ktb[p2.a[0] + 6] * x2.a[0];
      acc += ktb[p2.a[1] + 7] * x2.a[1];
      acc += ktb[p2.a[2] + 8] * x2.a[2];
    }
    return acc;
  }

  // One pass over level (H x W, pitch W) for the out rows [ra, rb] (MODE 0: a sweep; MODE 1: prolongation +
  // correction + sweep; MODE 2: zero-guess sweep + residual + restriction of the coarse rows [I0, I1)).
  //   u: the iterate (nullptr: zero guess); e / pkc: level k+1's correction and map (MODE 1); f, pk: level k's;
  //   dst: out rows [o0, o1) at interior columns (MODE 0/1: the result; MODE 2: the pre-smoothed iterate);
  //   fc: level k+1's right-hand side (MODE 2).  dst_g / ldg: the top level's result goes to HBM instead.
  template <int MODE>
  __device__ void pass(int H, int W, const T* u, const T* f, const uint8_t* pk, const T* e, const uint8_t* pkc,
                       T* dst, int o0, int o1, T* dst_g, long long ldg, T* fc, int I0, int I1, int ra, int rb) const {
    constexpr int HALO = NL + 1;
    const int Wc = (W + 1) / 2, Hc = (H + 1) / 2;
    const bool cin = lane >= 1 && lane <= W - 2;
    const int lc = min(lane, W - 1);
    auto ldrow = [&](const T* x, int y) -> T {  // row y of a level field at the lane's column (0 off the level)
      const T v = x[min(max(y, 0), H - 1) * W + lc];
      return (y >= 0 && y < H && lane < W) ? v : T(0);
    };
    auto ldpat = [&](int y) -> int {
      if constexpr (MULTI) {
        const int p = pk[min(max(y, 0), H - 1) * W + lc];
        return (y >= 0 && y < H && lane < W) ? p : 0;
      }
      return 0;
    };
    T ks[9], hk[NL > 0 ? NL : 1][9], t2[9];
    T om = 0;
    // weights: scalar loads re-issued stage by stage (hsweep_task's staged weights): z is 0 at run time, and an
    // empty asm "changes" it before each stage, so the loads stay where they are used
    int z = 0;
    auto stage = [&]() __attribute__((always_inline)) {
      if constexpr (sizeof(T) == 8) asm volatile("" : "+s"(z));
    };
    auto stage_ks = [&]() __attribute__((always_inline)) {
      stage();
      if constexpr (!MULTI) {
#pragma unroll
        for (int d = 0; d < 9; ++d) ks[d] = cl(a.ktab, z + d);
        om = cl(a.omd, z);
      }
    };
    auto stage_t2 = [&]() __attribute__((always_inline)) {
      stage();
      if constexpr (!MULTI && MODE != 0) {
#pragma unroll
        for (int d = 0; d < 9; ++d) t2[d] = cl(MODE == 1 ? a.ptab : a.rtab, z + d);
      }
    };
    auto stage_hk = [&](int l) __attribute__((always_inline)) {
      stage();
#pragma unroll
      for (int d = 0; d < 9; ++d) hk[l][d] = cl(a.hw, z + l * 9 + d);
    };
    // MODE 1: the corrected iterate x(y) = u(y) + w1 P(e) on the interior (hsweep_task MODE 1 / prolong_add)
    const int jl = lane >> 1;
    auto ecol = [&](int I, int J) -> T {  // e(I, J) on level k+1's interior, else 0 (the framed zeros; the scratch
      //                                       fields are reused at other pitches, so their boundary is not read)
      const T v = e[min(max(I, 0), Hc - 1) * Wc + min(J, Wc - 1)];
      return (I >= 1 && I <= Hc - 2 && J >= 1 && J <= Wc - 2) ? v : T(0);
    };
    auto epat = [&](int I, int J) -> int {
      if constexpr (MULTI) {
        const int p = pkc[min(max(I, 0), Hc - 1) * Wc + min(J, Wc - 1)];
        return (I >= 0 && I < Hc && J < Wc) ? p * kHTailTS : 0;
      }
      return 0;
    };
    auto cterm = [&](int I, int ky) -> T {  // coarse row I's contribution at the lane's column (crow_term)
      if (lane & 1) {  // odd fine column c: coarse nodes (c-1)/2 (kx = 2) and (c+1)/2 (kx = 0)
        T t = (MULTI ? ptb[epat(I, jl) + ky * 3 + 2] : t2[ky * 3 + 2]) * ecol(I, jl);
        t += (MULTI ? ptb[epat(I, jl + 1) + ky * 3 + 0] : t2[ky * 3 + 0]) * ecol(I, jl + 1);
        return t;
      }
      return (MULTI ? ptb[epat(I, jl) + ky * 3 + 1] : t2[ky * 3 + 1]) * ecol(I, jl);  // even: node c/2, kx = 1
    };

    HW1<T> U0{}, U1{}, U2{};
    HW1<int> P0{}, P1{}, P2{};
    HW1<T> D[NL > 0 ? NL : 1][3] = {};
    T J[NL + 1];
#pragma unroll
    for (int i = 0; i <= NL; ++i) J[i] = T(0);
    HW1<T> O0{}, O1{}, O2{};
    HW1<int> Q0{}, Q1{}, Q2{};
    T Ra[3] = {}, Rb[3] = {};
    HW1<int> PRa{}, PRb{};
    // steps y = ra - HALO .. rb + HALO: u(y) enters, j / d_0 of row y-1, d_l of row y-1-l, out of row y-1-NL (and
    // MODE 2 the residual of row y-2-NL)
    const int ys = ra - HALO, ye = rb + HALO;
    for (int y = ys; y <= ye; ++y) {
      z = __builtin_amdgcn_readfirstlane(y & a.zmask);
      T uy = (u != nullptr) ? ldrow(u, y) : T(0);
      const int py = ldpat(y);
      if constexpr (MODE == 1) {
        stage_t2();
        const bool yin = y >= 1 && y <= H - 2;
        T xk;
        if (!(y & 1)) {
          xk = uy + a.w1 * cterm(y >> 1, 1);
        } else {
          const T tt = cterm((y - 1) >> 1, 2) + cterm((y + 1) >> 1, 0);
          xk = uy + a.w1 * tt;
        }
        uy = (yin && cin) ? xk : uy;
      }
      U0 = U1;
      U1 = U2;
      U2 = hw1<T>(uy);
      if constexpr (MULTI) {
        P0 = P1;
        P1 = P2;
        P2 = hp1(py);
      }
      // j and d_0 of row y-1
      stage_ks();
      const int yj = y - 1;
      const bool rin = yj >= 1 && yj <= H - 2;
      const T fy1 = ldrow(f, yj);
      const T acc = kx(U0, U1, U2, P0, P1, P2, ks);
      const T omk = MULTI ? ktb[P1.a[1] + 9] : om;
      const T jv = omk * (fy1 - acc) + U1.a[1];
      const T d0 = (rin && cin) ? jv - U1.a[1] : T(0);
#pragma unroll
      for (int i = NL; i > 0; --i) J[i] = J[i - 1];
      J[0] = jv;
      if constexpr (NL > 0) {
        D[0][0] = D[0][1];
        D[0][1] = D[0][2];
        D[0][2] = hw1<T>(d0);
      }
      const int yo = y - 1 - NL;
      T o = NL == 0 ? J[0] : T(0);
#pragma unroll
      for (int l = 1; l <= NL; ++l) {
        stage_hk(l - 1);
        const int yl = y - 1 - l;
        const bool lin = yl >= 1 && yl <= H - 2;
        const HW1<T>& A = D[l - 1][0];
        const HW1<T>& Bw = D[l - 1][1];
        const HW1<T>& C = D[l - 1][2];
        T c = hk[l - 1][0] * A.a[0];
        c += hk[l - 1][1] * A.a[1];
        c += hk[l - 1][2] * A.a[2];
        c += hk[l - 1][3] * Bw.a[0];
        c += hk[l - 1][4] * Bw.a[1];
        c += hk[l - 1][5] * Bw.a[2];
        c += hk[l - 1][6] * C.a[0];
        c += hk[l - 1][7] * C.a[1];
        c += hk[l - 1][8] * C.a[2];
        const T dl = (lin && cin) ? c : T(0);
        if (l < NL) {
          D[l][0] = D[l][1];
          D[l][1] = D[l][2];
          D[l][2] = hw1<T>(dl);
        } else {
          o = J[NL] + dl;
        }
      }
      const bool oin = yo >= 1 && yo <= H - 2;
      if (yo >= o0 && yo < o1 && cin) {  // (wave-uniform row test)
        if (dst_g) dst_g[(long long)(yo + 1) * ldg + lane] = o;
        else dst[yo * W + lane] = o;
      }
      if constexpr (MODE == 2) {
        // the out row as the buffer holds it (the zero guess off the interior), the residual of row yo - 1, and the
        // restriction of the coarse row it closes (hsweep_task MODE 2)
        const T ob = (oin && cin) ? o : T(0);
        O0 = O1;
        O1 = O2;
        O2 = hw1<T>(ob);
        if constexpr (MULTI) {
          Q0 = Q1;
          Q1 = Q2;
          Q2 = hp1(ldpat(yo));
        }
        const int yr = yo - 1;
        stage_ks();
        if (yr >= ra + 1) {
          const T r = ldrow(f, yr) - kx(O0, O1, O2, Q0, Q1, Q2, ks);
          T rw[3];
          rw[1] = r;
          rw[0] = shr1z(r);
          rw[2] = shl1z(r);
          stage_t2();
          if (!(yr & 1)) {  // row 2I
#pragma unroll
            for (int k = 0; k < 3; ++k) Rb[k] = rw[k];
            PRb = Q1;
          } else {
            if (yr > ra + 1) {  // row 2I+1 closes coarse row I = (yr - 1) / 2 (taps at columns c-1, c, c+1)
              const int I = (yr - 1) / 2;
              T acc2;
              if constexpr (!MULTI) {
                acc2 = t2[0] * Ra[0];
                acc2 += t2[1] * Ra[1];
                acc2 += t2[2] * Ra[2];
                acc2 += t2[3] * Rb[0];
                acc2 += t2[4] * Rb[1];
                acc2 += t2[5] * Rb[2];
                acc2 += t2[6] * rw[0];
                acc2 += t2[7] * rw[1];
                acc2 += t2[8] * rw[2];
              } else {
                acc2 = rtb[PRa.a[0] + 0] * Ra[0];
                acc2 += rtb[PRa.a[1] + 1] * Ra[1];
                acc2 += rtb[PRa.a[2] + 2] * Ra[2];
                acc2 += rtb[PRb.a[0] + 3] * Rb[0];
                acc2 += rtb[PRb.a[1] + 4] * Rb[1];
                acc2 += rtb[PRb.a[2] + 5] * Rb[2];
                acc2 += rtb[Q1.a[0] + 6] * rw[0];
                acc2 += rtb[Q1.a[1] + 7] * rw[1];
                acc2 += rtb[Q1.a[2] + 8] * rw[2];
              }
              const int Jc = lane >> 1;
              if (I >= I0 && I < I1 && !(lane & 1) && Jc >= 1 && Jc <= Wc - 2) fc[I * Wc + Jc] = a.w0 * acc2;
            }
#pragma unroll
            for (int k = 0; k < 3; ++k) Ra[k] = rw[k];
            PRa = Q1;
          }
        }
      }
    }
  }
};

// rows [1, n+1) split over the waves: [r0, r1) of wave wv (r1 <= r0 when it has none)
__device__ __forceinline__ void htail_split(int n, int wv, int& r0, int& r1) {
  constexpr int NW = kHTailThreads / 64;
  const int per = (n + NW - 1) / NW;
  r0 = 1 + wv * per;
  r1 = min(n + 1, r0 + per);
}

template <typename T, bool MULTI, int NL>
__global__ __launch_bounds__(kHTailThreads) void k_hjac_tail_fast(HTailArgs<T> a) {
  __shared__ __attribute__((aligned(16))) char smem[kHTailLdsBytes];
  const int tid = threadIdx.x;
  const int Ht = a.Ht, Wt = a.Wt, nlev = a.nlev;
  const long long e = htail_elems(Ht, Wt, nlev);
  T* fs = reinterpret_cast<T*>(smem);  // f of every level
  T* us = fs + e;                      // the pre-smoothed iterate of every level above the coarsest
  T* S[2] = {us + e, us + e + Ht * Wt};  // up-pass results, alternating by level
  T* tabs = S[1] + Ht * Wt;
  T* ktb = tabs;
  T* rtb = ktb + FEA_MAX_PATTERNS * kHTailTS;
  T* ptb = rtb + FEA_MAX_PATTERNS * kHTailTS;
  uint8_t* pl = reinterpret_cast<uint8_t*>(ptb + FEA_MAX_PATTERNS * kHTailTS + kHTailMaxLayers * 9);
  const T* fg = a.f_t + (long long)blockIdx.x * a.bs_t + (128 / (int)sizeof(T) - 1);
  // zero the f and scratch regions (boundaries and unwritten rows read as 0), tables, maps, f_t
  for (long long i = tid; i < 2 * e + 2LL * Ht * Wt; i += kHTailThreads) fs[i] = T(0);
  if constexpr (MULTI) {
    for (int i = tid; i < a.ntab * kHTailTS; i += kHTailThreads) {
      const int p = i / kHTailTS, d = i - p * kHTailTS;
      ktb[i] = d == 9 ? a.omd[p] : a.ktab[p * 9 + d];
      rtb[i] = d == 9 ? T(0) : a.rtab[p * 9 + d];
      ptb[i] = d == 9 ? T(0) : a.ptab[p * 9 + d];
    }
    for (long long i = tid; i < e; i += kHTailThreads) pl[i] = a.pid[i];
  }
  __syncthreads();
  for (int i = tid; i < Ht * Wt; i += kHTailThreads) {
    const int r = i / Wt, c = i - r * Wt;
    fs[i] = fg[(long long)(r + 1) * a.ld_t + c];
  }
  __syncthreads();
  const int wv = tid >> 6, lane = tid & 63;
  HTailFast<T, MULTI, NL> t{a, ktb, rtb, ptb, lane};
  // down: per level one pass (zero-guess sweep, residual, restriction)
  long long o = 0;
  for (int k = 0; k < nlev - 1; ++k) {
    const int H = htail_n(Ht, k), W = htail_n(Wt, k), Hc = (H + 1) / 2;
    int I0, I1;
    htail_split(Hc - 2, wv, I0, I1);
    if (I0 < I1) {  // owned fine rows 2I0-1 .. 2I1-2 (and H-2 with the last coarse row)
      const int r1 = I1 == Hc - 1 ? H - 1 : 2 * I1 - 1;
      t.template pass<2>(H, W, nullptr, fs + o, pl + o, nullptr, nullptr, us + o, 2 * I0 - 1, r1, nullptr, 0,
                         fs + o + H * W, I0, I1, 2 * I0 - 2, 2 * I1);
    }
    o += H * W;
    __syncthreads();
  }
  T* ug = a.u_t + (long long)blockIdx.x * a.bs_t + (128 / (int)sizeof(T) - 1);
  // coarsest: two sweeps from zero (the first into the other scratch field)
  {
    const int k = nlev - 1, H = htail_n(Ht, k), W = htail_n(Wt, k);
    int y0, y1;
    htail_split(H - 2, wv, y0, y1);
    T* mid = S[(k + 1) & 1];
    if (y0 < y1)
      t.template pass<0>(H, W, nullptr, fs + o, pl + o, nullptr, nullptr, mid, y0, y1, nullptr, 0, nullptr, 0, 0,
                         y0, y1 - 1);
    __syncthreads();
    if (y0 < y1)  // (nlev == 1: the coarsest is the top level, its result goes to HBM)
      t.template pass<0>(H, W, mid, fs + o, pl + o, nullptr, nullptr, S[k & 1], y0, y1, k == 0 ? ug : nullptr,
                         a.ld_t, nullptr, 0, 0, y0, y1 - 1);
    __syncthreads();
  }
  // up: per level one pass (prolongation + correction + sweep); the top level writes u_t in HBM
  for (int k = nlev - 2; k >= 0; --k) {
    const int H = htail_n(Ht, k), W = htail_n(Wt, k);
    const long long oc = o;
    o -= H * W;
    int y0, y1;
    htail_split(H - 2, wv, y0, y1);
    if (y0 < y1)
      t.template pass<1>(H, W, us + o, fs + o, pl + o, S[(k + 1) & 1], pl + oc, S[k & 1], y0, y1,
                         k == 0 ? ug : nullptr, a.ld_t, nullptr, 0, 0, y0, y1 - 1);
    if (k > 0) __syncthreads();
  }
}

}  // namespace fea

using namespace fea;

extern "C" size_t fea_mg_hjac_tail_lds_bytes(int Ht, int Wt, int nlev, int elem_size, int multi) {
  if (Ht < 3 || Wt < 3 || nlev < 1 || nlev > kHTailMaxLevels) return 0;
  return elem_size == 8 ? (size_t)htail_lds_bytes<double>(Ht, Wt, nlev, multi != 0)
                        : (size_t)htail_lds_bytes<float>(Ht, Wt, nlev, multi != 0);
}

#ifndef FEA_HTAIL_FAST
#define FEA_HTAIL_FAST 1
#endif
constexpr bool kHTailFast = FEA_HTAIL_FAST != 0;

template <typename T, bool MULTI>
static void htail_fast_nl(int nl, int B, hipStream_t s, const HTailArgs<T>& a) {
  switch (nl) {
    case 0: k_hjac_tail_fast<T, MULTI, 0><<<B, kHTailThreads, 0, s>>>(a); break;
    case 1: k_hjac_tail_fast<T, MULTI, 1><<<B, kHTailThreads, 0, s>>>(a); break;
    case 2: k_hjac_tail_fast<T, MULTI, 2><<<B, kHTailThreads, 0, s>>>(a); break;
    default: k_hjac_tail_fast<T, MULTI, 3><<<B, kHTailThreads, 0, s>>>(a); break;
  }
}

// (n - 1) divisible by 2^(nlev-1), every level >= 3 nodes
static inline bool htail_dim_ok(int n, int nlev) {
  if (n < 3 || n > kHTailMaxN) return false;
  for (int k = 1; k < nlev; ++k) {
    if ((n - 1) & 1) return false;
    n = (n + 1) / 2;
    if (n < 3) return false;
  }
  return true;
}

#define FEA_HTAIL_API(SUF, T)                                                                                  \
  extern "C" int fea_mg_hjac_tail_##SUF(const T* f_t, T* u_t, int Ht, int Wt, int nlev, int ld_t, long long bs_t, \
                                        const uint8_t* pid_levels, const T* ktab, const T* omd, int ntab,      \
                                        const T* rtab, const T* ptab, const T* hw, int nlayers, T w0, T w1,     \
                                        int nu1, int nu2, int B, void* stream) {                               \
    if (!f_t || !u_t || !ktab || !omd || !rtab || !ptab || (!hw && nlayers > 0) || B <= 0 || B > 65535)        \
      return FEA_EINVAL;                                                                                       \
    if (nlev < 1 || nlev > kHTailMaxLevels || nlayers < 0 || nlayers > kHTailMaxLayers || nu1 < 0 || nu2 < 0)   \
      return FEA_EINVAL;                                                                                       \
    if (!htail_dim_ok(Ht, nlev) || !htail_dim_ok(Wt, nlev) || ld_t < Wt + 128 / (int)sizeof(T) ||             \
        bs_t < (long long)(Ht + 2) * ld_t)                                                                     \
      return FEA_EINVAL;                                                                                       \
    const bool multi = ntab > 1;                                                                               \
    if (ntab < 1 || ntab > FEA_MAX_PATTERNS || (multi && !pid_levels)) return FEA_EINVAL;                      \
    if (htail_lds_bytes<T>(Ht, Wt, nlev, multi) > kHTailLdsBytes) return FEA_EINVAL;                          \
    HTailArgs<T> a{f_t, u_t, pid_levels, ktab, omd, rtab, ptab, hw, w0, w1, Ht, Wt, nlev, ld_t, bs_t, ntab,     \
                   nlayers, nu1, nu2};                                                                         \
    hipStream_t s_ = (hipStream_t)stream;                                                                      \
    if (nu1 == 1 && nu2 == 1 && kHTailFast) {  /* V(1,1): the row-wave path */                                 \
      if (multi) htail_fast_nl<T, true>(nlayers, B, s_, a);                                                      \
      else htail_fast_nl<T, false>(nlayers, B, s_, a);                                                           \
    } else if (multi) k_hjac_tail<T, true><<<B, kHTailThreads, 0, s_>>>(a);                                    \
    else k_hjac_tail<T, false><<<B, kHTailThreads, 0, s_>>>(a);                                                \
    FEA_LAUNCH_CHECK();                                                                                        \
  }

FEA_HTAIL_API(f32, float)
FEA_HTAIL_API(f64, double)
