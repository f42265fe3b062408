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

}  // namespace fea

using namespace fea;

extern "C" size_t fea_mg_hjac_tail_lds_bytes(int Ht, int Wt, int nlev, int elem_size, int multi) {
  if (Ht < 3 || Wt < 3 || nlev < 1 || nlev > kHTailMaxLevels) return 0;
  return elem_size == 8 ? (size_t)htail_lds_bytes<double>(Ht, Wt, nlev, multi != 0)
                        : (size_t)htail_lds_bytes<float>(Ht, Wt, nlev, multi != 0);
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
    if (multi) k_hjac_tail<T, true><<<B, kHTailThreads, 0, s_>>>(a);                                           \
    else k_hjac_tail<T, false><<<B, kHTailThreads, 0, s_>>>(a);                                                \
    FEA_LAUNCH_CHECK();                                                                                        \
  }

FEA_HTAIL_API(f32, float)
FEA_HTAIL_API(f64, double)
