// coarse_tail.hip — the coarse end of the V-cycle (levels with H, W <= 65) in ONE launch.
//
// Below ~129^2 nodes a level's kernels are pure launch/latency cost (each level is a few
// microseconds of work spread thin over the chip, twice per V-cycle).  Here one 1024-thread
// workgroup per right-hand side keeps every coarse level (v ping-pong + f, pattern ids, tables)
// resident in LDS (<= ~147 KB of the 160 KB per CU at N_t = 65 in fp64) and runs the whole
// coarse sub-cycle — pre-smoothing, residual, restriction, coarsest sweeps, prolongation +
// correction, post-smoothing — with workgroup barriers between the phases.  It reads f_t once
// from HBM and writes v_t once, in the framed layout the level kernels use.
//
// Semantics = the coarse part of feanet_amd.schedule.vcycle_schedule (every coarse level starts
// from a zero guess with zero Dirichlet data, FEANet/multigrid.py:171-172; coarsest level gets
// nu1 + nu2 sweeps; q2 = MM_Interface_error.ipynb's grids[0] pre-smoothing, i.e. none here).
#include "fea_common.h"

namespace fea {

constexpr int kTailThreads = 1024;
constexpr int kTailMaxLevels = 8;
constexpr int kTailMaxN = 65;  // per dimension
constexpr int kTailLdsBytes = 160 * 1024 - 1024;
constexpr int kTS = 10;  // table stride (9 weights + omega/d)

#ifdef FEA_TAIL_TRACE  // lab builds only (tools/lab/tail_lab.py): a timestamp after every barrier
__device__ long long g_tail_trace[256];
#define FEA_TAIL_SYNC()                                                            \
  do {                                                                             \
    __syncthreads();                                                               \
    if (threadIdx.x == 0 && blockIdx.x == 0 && nph < 256) g_tail_trace[nph] = clock64(); \
    ++nph;                                                                         \
  } while (0)
#else
#define FEA_TAIL_SYNC() __syncthreads()
#endif

template <typename T>
struct TailArgs {
  const T* f_t;
  T* v_t;
  const uint8_t* pid;  // compact concatenated per-level maps (NULL: single pattern)
  const T* ktab;
  const T* omd;
  const T* rtab;
  const T* ptab;
  T w0, w1;
  int Ht, Wt, nlev, ld_t;
  long long bs_t;
  int ntab, nu1, nu2, q2;
};

__host__ __device__ inline long long tail_elems(int Ht, int Wt, int nlev) {
  long long s = 0;
  for (int k = 0, H = Ht, W = Wt; k < nlev; ++k, H = (H + 1) / 2, W = (W + 1) / 2) s += (long long)H * W;
  return s;
}

template <typename T>
__host__ __device__ inline long long tail_lds_bytes(int Ht, int Wt, int nlev, bool multi) {
  const long long e = tail_elems(Ht, Wt, nlev);
  long long b = 3 * e * (long long)sizeof(T);
  if (multi) b += (e + 15) / 16 * 16;
  b += 3LL * FEA_MAX_PATTERNS * kTS * sizeof(T);
  return b;
}

__device__ __forceinline__ int tail_n(int n0, int k) { return ((n0 - 1) >> k) + 1; }
__device__ __forceinline__ int tail_off(int Ht, int Wt, int k) {  // element offset of level k in a region
  int o = 0;
  for (int j = 0; j < k; ++j) o += tail_n(Ht, j) * tail_n(Wt, j);
  return o;
}


// ---------------------------------------------------------------------------------------------
// Fused V(1,1) coarse sub-cycle: one workgroup barrier per level and direction.  Wave w of the 16
// owns a contiguous block of rows of each level, lane c is column c (levels are <= 65 wide; column
// 64 is a boundary column, read as 0), horizontal neighbours come from DPP row shifts, vertical ones
// from a sliding window of rows in registers — so a level's 9-point stencil costs ~1 LDS read per
// node instead of 9.  Per level:
//   down:   v = omd f (stored: the pre-smoothed iterate), r = f - K v on the rows the wave's coarse
//           rows need (v recomputed there, it is pointwise), f_c = w0 R r       -> barrier
//   coarsest: v1 = omd f, v2 = v1 + omd (f - K v1)                               -> barrier
//   up:     x = v + w1 P e (rows the wave's sweep reads), v' = x + omd (f - K x) -> barrier
//           (level 0: v' goes straight to HBM)
// Every node value is the same expression, in the same order, as the general path (bitwise).
// ---------------------------------------------------------------------------------------------
template <typename T, bool MULTI>
__device__ __forceinline__ void tail_fast(const TailArgs<T>& a, T* va, T* vb, T* fs, const T* ktb, const T* rtb,
                                          const T* ptb, const uint8_t* pl, int wv, int lane
#ifdef FEA_TAIL_TRACE
                                          , int& nph
#endif
) {
  constexpr int kWaves = kTailThreads / 64;
  const int nlev = a.nlev, Ht = a.Ht, Wt = a.Wt;
  // single-pattern tables in registers (uniform)
  T kr[9], rr[9], pr[9], om0 = T(0);
  if constexpr (!MULTI) {
#pragma unroll
    for (int d = 0; d < 9; ++d) {
      kr[d] = ktb[d];
      rr[d] = rtb[d];
      pr[d] = ptb[d];
    }
    om0 = ktb[9];
  }
  unsigned cur = 0;  // bit k set: level k's current iterate is in vb
  auto curp = [&](int k, int o) -> T* { return ((cur >> k) & 1u) ? vb + o : va + o; };
  auto othp = [&](int k, int o) -> T* { return ((cur >> k) & 1u) ? va + o : vb + o; };
  auto inside = [&](int H, int N, int r) { return r >= 1 && r <= H - 2 && lane >= 1 && lane <= N - 2; };
  auto pat = [&](const uint8_t* pk, int H, int N, int r) -> int {
    if constexpr (MULTI) return (r >= 0 && r < H && lane < N) ? (int)pk[r * N + lane] : 0;
    return 0;
  };
  auto omega = [&](int p) -> T {
    if constexpr (MULTI) return ktb[p * kTS + 9];
    return om0;
  };
  // K x at a row from rows (xm, x0, xp) and their pattern ids: DPP for the column neighbours.
  // Must be called wave-uniformly.
  auto Krow = [&](T xm, T x0, T xp, int qm, int q0, int qp) -> T {
    const T xs[3] = {xm, x0, xp};
    const int qs[3] = {qm, q0, qp};
    T acc = 0;
#pragma unroll
    for (int dr = 0; dr < 3; ++dr) {
      const T l = shr1(xs[dr], T(0)), r = shl1(xs[dr], T(0));
      if constexpr (MULTI) {
        const int ql = shr1(qs[dr], 0), qr = shl1(qs[dr], 0);
        acc += ktb[ql * kTS + dr * 3 + 0] * l;
        acc += ktb[qs[dr] * kTS + dr * 3 + 1] * xs[dr];
        acc += ktb[qr * kTS + dr * 3 + 2] * r;
      } else {
        acc += kr[dr * 3 + 0] * l;
        acc += kr[dr * 3 + 1] * xs[dr];
        acc += kr[dr * 3 + 2] * r;
      }
    }
    return acc;
  };
  auto block = [&](int n, int& b0, int& b1) {  // this wave's share of rows 1..n (contiguous)
    const int per = (n + kWaves - 1) / kWaves;
    b0 = 1 + wv * per;
    b1 = min(n + 1, b0 + per);
  };

  // ------------------------------------------------------------------ down
  int o = 0;
  for (int k = 0; k + 1 < nlev; ++k) {
    const int H = tail_n(Ht, k), N = tail_n(Wt, k), Hc = (H + 1) / 2, Nc = (N + 1) / 2;
    const int on = o + H * N;
    const T* f = fs + o;
    const uint8_t* pk = pl + o;
    T* v = curp(k, o);
    T* fc = fs + on;
    int y0, y1;
    block(H - 2, y0, y1);
    for (int y = y0; y < y1; ++y)
      if (inside(H, N, y)) v[y * N + lane] = omega(pat(pk, H, N, y)) * f[y * N + lane];
    int I0, I1;
    block(Hc - 2, I0, I1);
    if (I0 < I1) {
      // pre-smoothed iterate v = omd f on row y (0 off the interior), recomputed in registers
      auto vrow = [&](int y) -> T {
        return inside(H, N, y) ? omega(pat(pk, H, N, y)) * f[y * N + lane] : T(0);
      };
      auto rrow = [&](T vm, T v0, T vp, int qm, int q0, int qp, int y) -> T {
        const T kv = Krow(vm, v0, vp, qm, q0, qp);
        return inside(H, N, y) ? f[y * N + lane] - kv : T(0);
      };
      int y = 2 * I0 - 1;  // first residual row
      T vm = vrow(y - 1), v0 = vrow(y), vp = vrow(y + 1);
      int qm = pat(pk, H, N, y - 1), q0 = pat(pk, H, N, y), qp = pat(pk, H, N, y + 1);
      T ra = rrow(vm, v0, vp, qm, q0, qp, y);
      int pa = q0;
      for (int I = I0; I < I1; ++I) {
        // rows 2I and 2I+1 of the residual
        vm = v0; v0 = vp; vp = vrow(2 * I + 1);
        qm = q0; q0 = qp; qp = pat(pk, H, N, 2 * I + 1);
        const T rb = rrow(vm, v0, vp, qm, q0, qp, 2 * I);
        const int pb = q0;
        vm = v0; v0 = vp; vp = vrow(2 * I + 2);
        qm = q0; q0 = qp; qp = pat(pk, H, N, 2 * I + 2);
        const T rc = rrow(vm, v0, vp, qm, q0, qp, 2 * I + 1);
        const int pc = q0;
        const T rs[3] = {ra, rb, rc};
        const int ps[3] = {pa, pb, pc};
        T acc = 0;
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          const T l = shr1(rs[ky], T(0)), r = shl1(rs[ky], T(0));
          if constexpr (MULTI) {
            const int pl_ = shr1(ps[ky], 0), pr_ = shl1(ps[ky], 0);
            acc += rtb[pl_ * kTS + ky * 3 + 0] * l;
            acc += rtb[ps[ky] * kTS + ky * 3 + 1] * rs[ky];
            acc += rtb[pr_ * kTS + ky * 3 + 2] * r;
          } else {
            acc += rr[ky * 3 + 0] * l;
            acc += rr[ky * 3 + 1] * rs[ky];
            acc += rr[ky * 3 + 2] * r;
          }
        }
        const int J = lane >> 1;
        if (!(lane & 1) && J >= 1 && J <= Nc - 2) fc[I * Nc + J] = a.w0 * acc;
        ra = rc;
        pa = pc;
      }
    }
    o = on;
    FEA_TAIL_SYNC();
  }
  // ------------------------------------------------------------------ coarsest: 2 sweeps
  T* const vt = a.v_t + (long long)blockIdx.x * a.bs_t + (128 / (int)sizeof(T) - 1);
  {
    const int k = nlev - 1, H = tail_n(Ht, k), N = tail_n(Wt, k);
    const T* f = fs + o;
    const uint8_t* pk = pl + o;
    auto vrow = [&](int y) -> T { return inside(H, N, y) ? omega(pat(pk, H, N, y)) * f[y * N + lane] : T(0); };
    T* out = othp(k, o);
    int y0, y1;
    block(H - 2, y0, y1);
    if (y0 < y1) {
      T vm = vrow(y0 - 1), v0 = vrow(y0);
      int qm = pat(pk, H, N, y0 - 1), q0 = pat(pk, H, N, y0);
      for (int y = y0; y < y1; ++y) {
        const T vp = vrow(y + 1);
        const int qp = pat(pk, H, N, y + 1);
        const T kv = Krow(vm, v0, vp, qm, q0, qp);
        if (inside(H, N, y)) {
          const T w = omega(q0) * (f[y * N + lane] - kv) + v0;
          if (k == 0) vt[(long long)(y + 1) * a.ld_t + lane] = w;
          else out[y * N + lane] = w;
        }
        vm = v0; v0 = vp;
        qm = q0; q0 = qp;
      }
    }
    cur ^= 1u << k;
    if (k > 0) FEA_TAIL_SYNC();
  }
  // ------------------------------------------------------------------ up
  for (int k = nlev - 2; k >= 0; --k) {
    const int H = tail_n(Ht, k), N = tail_n(Wt, k), Hc = (H + 1) / 2, Nc = (N + 1) / 2;
    const int oc = o;
    o -= H * N;
    const T* f = fs + o;
    const uint8_t* pk = pl + o;
    const uint8_t* pkc = pl + oc;
    T* v = curp(k, o);
    const T* e = curp(k + 1, oc);
    T* out = othp(k, o);
    int y0, y1;
    block(H - 2, y0, y1);
    // (a) v += w1 P e on this wave's rows, in place (the general path's prolong_add, same order)
    for (int y = y0; y < y1; ++y) {
      if (!inside(H, N, y)) continue;
      T acc = 0;
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const int cy = y + 1 - ky;
        if (cy & 1) continue;
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const int cx = lane + 1 - kx;
          if (cx & 1) continue;
          const int I = cy >> 1, J = cx >> 1;
          const bool ein = I >= 1 && I <= Hc - 2 && J >= 1 && J <= Nc - 2;
          const int j = I * Nc + J;
          const T ev = ein ? e[j] : T(0);
          if constexpr (MULTI) acc += ptb[(int)pkc[j] * kTS + ky * 3 + kx] * ev;
          else acc += pr[ky * 3 + kx] * ev;
        }
      }
      v[y * N + lane] += a.w1 * acc;
    }
    FEA_TAIL_SYNC();
    // (b) one sweep from the corrected iterate (rows from LDS, columns by DPP)
    auto xrow = [&](int y) -> T { return inside(H, N, y) ? v[y * N + lane] : T(0); };
    if (y0 < y1) {
      T xm = xrow(y0 - 1), x0 = xrow(y0);
      int qm = pat(pk, H, N, y0 - 1), q0 = pat(pk, H, N, y0);
      for (int y = y0; y < y1; ++y) {
        const T xp = xrow(y + 1);
        const int qp = pat(pk, H, N, y + 1);
        const T kx_ = Krow(xm, x0, xp, qm, q0, qp);
        if (inside(H, N, y)) {
          const T w = omega(q0) * (f[y * N + lane] - kx_) + x0;
          if (k == 0) vt[(long long)(y + 1) * a.ld_t + lane] = w;
          else out[y * N + lane] = w;
        }
        xm = x0; x0 = xp;
        qm = q0; q0 = qp;
      }
    }
    cur ^= 1u << k;
    if (k > 0) FEA_TAIL_SYNC();
  }
}

template <typename T, bool MULTI>
__global__ __launch_bounds__(kTailThreads) void k_mg_coarse_tail(TailArgs<T> a) {
  __shared__ __attribute__((aligned(16))) char smem[kTailLdsBytes];
  const int tid = threadIdx.x;
  const int nlev = a.nlev, Ht = a.Ht, Wt = a.Wt;
#ifdef FEA_TAIL_TRACE
  int nph = 0;
  if (tid == 0 && blockIdx.x == 0) g_tail_trace[255] = clock64();
#endif
  const int tot = tail_off(Ht, Wt, nlev);
  T* va = reinterpret_cast<T*>(smem);
  T* vb = va + tot;
  T* fs = vb + tot;
  T* ktb = fs + tot;  // [16][10]: stencil + omega/d
  T* rtb = ktb + FEA_MAX_PATTERNS * kTS;
  T* ptb = rtb + FEA_MAX_PATTERNS * kTS;
  uint8_t* pl = reinterpret_cast<uint8_t*>(ptb + FEA_MAX_PATTERNS * kTS);

  // V(1,1) (the default MultiGrid.Step / iterate schedule) runs the fused row-wave path below; it
  // masks every read outside a level's interior, so only the general path needs zeroed buffers
  const bool fast = a.nu1 == 1 && a.nu2 == 1 && !a.q2;
  if (!fast) {
    for (int i = tid; i < 3 * tot; i += kTailThreads) va[i] = T(0);
    FEA_TAIL_SYNC();  // the zero fill must land before f_t is staged into the same region
  }
  const int nt = MULTI ? a.ntab : 1;
  for (int i = tid; i < nt * kTS; i += kTailThreads) {
    const int p = i / kTS, d = i - p * kTS;
    ktb[i] = d == 9 ? a.omd[p] : a.ktab[p * 9 + d];
    rtb[i] = d == 9 ? T(0) : a.rtab[p * 9 + d];
    ptb[i] = d == 9 ? T(0) : a.ptab[p * 9 + d];
  }
  if constexpr (MULTI)
    for (int i = tid; i < tot; i += kTailThreads) pl[i] = a.pid[i];
  const int wv = tid >> 6, lane = tid & 63;  // wave = row group, lane = column (Wt <= 65)
  constexpr int kWaves = kTailThreads / 64;
  {
    const T* src = a.f_t + (long long)blockIdx.x * a.bs_t + (128 / (int)sizeof(T) - 1);
    constexpr int kRows = (kTailMaxN + kWaves - 1) / kWaves;  // rows per wave, all loads in flight at once
    T buf[kRows], b64[kRows];
#pragma unroll
    for (int i = 0; i < kRows; ++i) {
      const int r = wv + i * kWaves;
      const T* row = src + (long long)(r + 1) * a.ld_t;
      buf[i] = (r < Ht && lane < Wt) ? row[lane] : T(0);
      b64[i] = (r < Ht && lane == 0 && Wt == 65) ? row[64] : T(0);
    }
#pragma unroll
    for (int i = 0; i < kRows; ++i) {
      const int r = wv + i * kWaves;
      if (r < Ht && lane < Wt) fs[r * Wt + lane] = buf[i];
      if (r < Ht && lane == 0 && Wt == 65) fs[r * Wt + 64] = b64[i];
    }
  }
  FEA_TAIL_SYNC();
  if (fast) {
    tail_fast<T, MULTI>(a, va, vb, fs, ktb, rtb, ptb, pl, wv, lane
#ifdef FEA_TAIL_TRACE
                        , nph
#endif
    );
    return;
  }

  // pattern offset (into a stride-10 table) of node j of a level whose map starts at pk
  auto P = [&](const uint8_t* pk, int j) -> int { return MULTI ? pk[j] * kTS : 0; };
  auto Ku = [&](int N, const uint8_t* pk, const T* u, int r, int c) -> T {  // N = row pitch (W)
    const int i0 = (r - 1) * N + c - 1;
    T acc = 0;
#pragma unroll
    for (int dr = 0; dr < 3; ++dr)
#pragma unroll
      for (int dc = 0; dc < 3; ++dc) {
        const int j = i0 + dr * N + dc;
        acc += ktb[P(pk, j) + dr * 3 + dc] * u[j];
      }
    return acc;
  };
  // threads as a 32 x 32 grid over the interior nodes (no per-node integer division)
  const int tx = tid & 31, ty = tid >> 5;
  auto sweep = [&](int H, int N, const uint8_t* pk, const T* f, const T* src, T* dst, bool zero) {
    for (int r = 1 + ty; r <= H - 2; r += 32)
      for (int c = 1 + tx; c <= N - 2; c += 32) {
        const int i = r * N + c;
        const T om = ktb[P(pk, i) + 9];
        dst[i] = zero ? om * f[i] : om * (f[i] - Ku(N, pk, src, r, c)) + src[i];
      }
    FEA_TAIL_SYNC();
  };
  auto residual = [&](int H, int N, const uint8_t* pk, const T* f, const T* src, T* dst) {
    for (int r = 1 + ty; r <= H - 2; r += 32)
      for (int c = 1 + tx; c <= N - 2; c += 32) dst[r * N + c] = f[r * N + c] - Ku(N, pk, src, r, c);
    FEA_TAIL_SYNC();
  };
  auto restrict_ = [&](int H, int N, const uint8_t* pk, const T* res, T* fc) {  // fine residual -> coarse f
    const int Nc = (N + 1) / 2, Hc = (H + 1) / 2;
    for (int I = 1 + ty; I <= Hc - 2; I += 32)
      for (int J = 1 + tx; J <= Nc - 2; J += 32) {
      T acc = 0;
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const int j = (2 * I - 1 + ky) * N + (2 * J - 1 + kx);
          acc += rtb[P(pk, j) + ky * 3 + kx] * res[j];
        }
      fc[I * Nc + J] = a.w0 * acc;
    }
    FEA_TAIL_SYNC();
  };
  auto prolong_add = [&](int H, int N, const uint8_t* pkc, T* v, const T* e) {  // v += w1 P e, interior
    const int Nc = (N + 1) / 2;
    for (int y = 1 + ty; y <= H - 2; y += 32)
      for (int x = 1 + tx; x <= N - 2; x += 32) {
      T acc = 0;
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const int cy = y + 1 - ky;
        if (cy & 1) continue;
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const int cx = x + 1 - kx;
          if (cx & 1) continue;
          const int j = (cy >> 1) * Nc + (cx >> 1);
          acc += ptb[P(pkc, j) + ky * 3 + kx] * e[j];
        }
      }
      v[y * N + x] += a.w1 * acc;
    }
    FEA_TAIL_SYNC();
  };

  // level k's regions start at element offset o (running sums, no per-phase recomputation)
  unsigned cur = 0;  // bit k set: level k's current iterate is in vb
  auto curp = [&](int k, int o) -> T* { return ((cur >> k) & 1u) ? vb + o : va + o; };
  auto othp = [&](int k, int o) -> T* { return ((cur >> k) & 1u) ? va + o : vb + o; };
  auto flip = [&](int k) { cur ^= (1u << k); };

  const bool presmooth = a.nu1 > 0 && !a.q2;
  int o = 0;
  for (int k = 0; k + 1 < nlev; ++k) {
    const int H = tail_n(Ht, k), N = tail_n(Wt, k);
    const int on = o + H * N;
    if (presmooth) {
      sweep(H, N, pl + o, fs + o, nullptr, curp(k, o), true);
      for (int s = 1; s < a.nu1; ++s) {
        sweep(H, N, pl + o, fs + o, curp(k, o), othp(k, o), false);
        flip(k);
      }
    }
    residual(H, N, pl + o, fs + o, curp(k, o), othp(k, o));
    restrict_(H, N, pl + o, othp(k, o), fs + on);
    o = on;
  }
  {
    const int k = nlev - 1, H = tail_n(Ht, k), N = tail_n(Wt, k);
    const int ncs = a.q2 ? a.nu2 : a.nu1 + a.nu2;
    if (ncs > 0) {
      sweep(H, N, pl + o, fs + o, nullptr, curp(k, o), true);
      for (int s = 1; s < ncs; ++s) {
        sweep(H, N, pl + o, fs + o, curp(k, o), othp(k, o), false);
        flip(k);
      }
    }
  }
  for (int k = nlev - 2; k >= 0; --k) {
    const int H = tail_n(Ht, k), N = tail_n(Wt, k);
    const int oc = o;  // level k + 1
    o -= H * N;
    prolong_add(H, N, pl + oc, curp(k, o), curp(k + 1, oc));
    for (int s = 0; s < a.nu2; ++s) {
      sweep(H, N, pl + o, fs + o, curp(k, o), othp(k, o), false);
      flip(k);
    }
  }
  {
    const T* v = curp(0, 0);
    T* dst = a.v_t + (long long)blockIdx.x * a.bs_t + (128 / (int)sizeof(T) - 1);
    for (int i = tid; i < Ht * Wt; i += kTailThreads) {
      const int r = i / Wt, c = i - r * Wt;
      if (r > 0 && r < Ht - 1 && c > 0 && c < Wt - 1) dst[(long long)(r + 1) * a.ld_t + c] = v[i];
    }
  }
}

}  // namespace fea

using namespace fea;

extern "C" size_t fea_mg_coarse_tail_lds_bytes(int Ht, int Wt, int nlev, int elem_size, int multi) {
  if (Ht < 3 || Wt < 3 || nlev < 1 || nlev > kTailMaxLevels) return 0;
  return elem_size == 8 ? (size_t)tail_lds_bytes<double>(Ht, Wt, nlev, multi != 0)
                        : (size_t)tail_lds_bytes<float>(Ht, Wt, nlev, multi != 0);
}

// (n - 1) divisible by 2^(nlev-1) and every level >= 3 nodes
static inline bool tail_dim_ok(int n, int nlev) {
  if (n < 3 || n > kTailMaxN) return false;
  for (int k = 1; k < nlev; ++k) {
    if ((n - 1) & 1) return false;
    n = (n + 1) / 2;
    if (n < 3) return false;
  }
  return true;
}

#define FEA_TAIL_API(SUF, T)                                                                                  \
  extern "C" int fea_mg_coarse_tail_##SUF(const T* f_t, T* v_t, int Ht, int Wt, int nlev, int ld_t,          \
                                          long long bs_t,                                                      \
                                          const uint8_t* pid_levels, const T* ktab, const T* omd, int ntab,    \
                                          const T* rtab, const T* ptab, T w0, T w1, int nu1, int nu2, int q2,  \
                                          int B, void* stream) {                                               \
    if (!f_t || !v_t || !ktab || !omd || !rtab || !ptab || B <= 0 || nlev < 1 || nlev > kTailMaxLevels)       \
      return FEA_EINVAL;                                                                                      \
    if (!tail_dim_ok(Ht, nlev) || !tail_dim_ok(Wt, nlev) || nu1 < 0 || nu2 < 0) return FEA_EINVAL;           \
    const bool multi = ntab > 1;                                                                              \
    if (ntab < 1 || ntab > FEA_MAX_PATTERNS || (multi && !pid_levels)) return FEA_EINVAL;                     \
    if (tail_lds_bytes<T>(Ht, Wt, nlev, multi) > kTailLdsBytes) return FEA_EINVAL;                           \
    TailArgs<T> a{f_t, v_t, pid_levels, ktab, omd, rtab, ptab, w0, w1, Ht, Wt, nlev, ld_t, bs_t, ntab, nu1, nu2,  \
                  q2};                                                                                        \
    if (multi) k_mg_coarse_tail<T, true><<<B, kTailThreads, 0, (hipStream_t)stream>>>(a);                     \
    else k_mg_coarse_tail<T, false><<<B, kTailThreads, 0, (hipStream_t)stream>>>(a);                          \
    FEA_LAUNCH_CHECK();                                                                                       \
  }

FEA_TAIL_API(f32, float)
FEA_TAIL_API(f64, double)

#ifdef FEA_TAIL_TRACE
extern "C" int fea_tail_trace_read(long long* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_tail_trace), sizeof(long long) * 256, 0, hipMemcpyDeviceToHost);
}
#endif
