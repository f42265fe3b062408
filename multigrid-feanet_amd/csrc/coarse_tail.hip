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

#include <utility>

namespace fea {

// threads per tail workgroup (one per sample; waves split each level's rows).  FEA_TAIL_THREADS: lab builds
#ifndef FEA_TAIL_THREADS
#define FEA_TAIL_THREADS 1024
#endif
constexpr int kTailThreads = FEA_TAIL_THREADS;
static_assert(kTailThreads % 64 == 0 && kTailThreads >= 256 && kTailThreads <= 1024, "tail: 4..16 waves");
constexpr int kTailMaxLevels = 8;
constexpr int kTailMaxN = 65;  // per dimension
constexpr int kTailLdsBytes = 160 * 1024 - 1024;
constexpr int kTS = 10;  // table stride (9 weights + omega/d)
#ifndef FEA_KSYM  // two-material K from the centre's table row (see framed_ops.hip kapply)
#define FEA_KSYM 1
#endif

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
// Fused V(1,1) coarse sub-cycle, laid out for latency: ONE workgroup barrier per level and
// direction, and inside a phase every LDS load of a wave is issued up front (clamped addresses,
// results masked by selects instead of branches) so the row chains run back to back instead of
// waiting on one load at a time.  Wave w of the 16 owns a contiguous block of rows of each level,
// lane c is column c (levels are <= 65 wide; column 64 is a boundary column, read as 0),
// horizontal neighbours come from DPP row shifts, each row shifted once.  Per level:
//   down:     v = omd f on the rows the wave's coarse rows need (pointwise, never stored),
//             r = f - K v, f_c = w0 R r  (level 0 reads f_t straight from HBM)       -> barrier
//   coarsest: v1 = omd f, v2 = v1 + omd (f - K v1)                                   -> barrier
//   up:       x = omd f + w1 P e on the rows the wave's sweep reads (the zero-guess pre-smoothed
//             iterate recomputed, as the streaming kernels do), v' = x + omd (f - K x) -> barrier
//             (level 0: v' goes straight to HBM)
// Every node value is the same expression, in the same order, as the general path (bitwise):
// acc chains start from 0 and add the taps in (row, column) order; x = fma(w1, P e, omd f).
// ---------------------------------------------------------------------------------------------
constexpr int kTailDownRows = (31 + kTailThreads / 64 - 1) / (kTailThreads / 64);  // coarse rows per wave going down:
//                                                                                   Hc - 2 <= 31 (2 over 16 waves)
constexpr int kTailUpRows = (63 + kTailThreads / 64 - 1) / (kTailThreads / 64);  // fine rows per wave going up / at the
//                                                                                 coarsest level: H - 2 <= 63 (4)
// FEA_TAIL_LATE_SYNC: the two-material 65^2 tail takes its staging barrier inside the first phase (down_rows SYNC)
#ifndef FEA_TAIL_LATE_SYNC
#define FEA_TAIL_LATE_SYNC 1
#endif
constexpr bool kTailLateSync = FEA_TAIL_LATE_SYNC != 0;

// HT != 0: the grid is HT x HT with NLEV levels, known at compile time (every BASELINE configuration
// ends in the 65^2 .. 3^2 tail), so level sizes, offsets and rows per wave fold into immediates.
template <typename T, bool MULTI, int HT = 0, bool EXT = false>
struct TailFast {
  const TailArgs<T>& a;
  T* es;               // per-level corrections (up-sweep outputs), level regions like fs
  T* fs;               // per-level right-hand sides
  const T* ktb;        // LDS tables (MULTI)
  const T* rtb;
  const T* ptb;
  const uint8_t* pl;   // LDS pattern maps (MULTI)
  const T* fg;         // row 0 of this sample's f_t (framed, HBM)
  T* vg;               // row 0 of this sample's v_t
  int ld, wv, lane;
  T kr[9], rr[9], pr[9], om0;

  __device__ __forceinline__ int Hk(int k) const { return HT ? ((HT - 1) >> k) + 1 : tail_n(a.Ht, k); }
  __device__ __forceinline__ int Nk(int k) const { return HT ? ((HT - 1) >> k) + 1 : tail_n(a.Wt, k); }

  // p: byte offset of a pattern's table row (pat(): pattern * kTS * sizeof(T)), so a table read is one
  // ds_read at p with the tap as its immediate offset
  __device__ __forceinline__ T tb(const T* t, int p, int d) const {
    return *reinterpret_cast<const T*>(reinterpret_cast<const char*>(t) + p + d * (int)sizeof(T));
  }
  __device__ __forceinline__ T omega(int p) const {
    if constexpr (MULTI) return tb(ktb, p, 9);
    return om0;
  }
  __device__ __forceinline__ T kw(int p, int d) const {
    if constexpr (MULTI) return tb(ktb, p, d);
    return kr[d];
  }
  __device__ __forceinline__ T rw(int p, int d) const {
    if constexpr (MULTI) return tb(rtb, p, d);
    return rr[d];
  }
  __device__ __forceinline__ T pw(int p, int d) const {
    if constexpr (MULTI) return tb(ptb, p, d);
    return pr[d];
  }
  __device__ __forceinline__ bool inside(int H, int N, int y) const {
    return y >= 1 && y <= H - 2 && lane >= 1 && lane <= N - 2;
  }
  // table-row byte offset of node (y, lane)'s pattern (0 off the level), loaded unconditionally
  __device__ __forceinline__ int pat(const uint8_t* pk, int H, int N, int y) const {
    if constexpr (MULTI) {
      const int p = pk[min(max(y, 0), H - 1) * N + min(lane, N - 1)];
      return (y >= 0 && y < H && lane < N) ? p * (kTS * (int)sizeof(T)) : 0;
    }
    return 0;
  }
  // (K x) on row j of a register window: rows j-1..j+1 with their DPP-shifted copies
  template <int R>
  __device__ __forceinline__ T Kx(int j, const T (&xl)[R], const T (&x)[R], const T (&xr)[R], const int (&ql)[R],
                                  const int (&q)[R], const int (&qr)[R]) const {
    T acc = 0;
    if constexpr (MULTI && FEA_KSYM) {  // the centre's table row, mirrored taps (framed_ops.hip kapply): same bits
#pragma unroll
      for (int dr = 0; dr < 3; ++dr) {
        acc += kw(q[j], 8 - dr * 3) * xl[j - 1 + dr];
        acc += kw(q[j], 7 - dr * 3) * x[j - 1 + dr];
        acc += kw(q[j], 6 - dr * 3) * xr[j - 1 + dr];
      }
      return acc;
    }
#pragma unroll
    for (int dr = 0; dr < 3; ++dr) {
      acc += kw(ql[j - 1 + dr], dr * 3 + 0) * xl[j - 1 + dr];
      acc += kw(q[j - 1 + dr], dr * 3 + 1) * x[j - 1 + dr];
      acc += kw(qr[j - 1 + dr], dr * 3 + 2) * xr[j - 1 + dr];
    }
    return acc;
  }
  template <int R>
  __device__ __forceinline__ void shift(const T (&x)[R], T (&xl)[R], T (&xr)[R]) const {
#pragma unroll
    for (int j = 0; j < R; ++j) {
      xl[j] = shr1z(x[j]);
      xr[j] = shl1z(x[j]);
    }
  }
  template <int R>
  __device__ __forceinline__ void shift(const int (&q)[R], int (&ql)[R], int (&qr)[R]) const {
#pragma unroll
    for (int j = 0; j < R; ++j) {
      if constexpr (MULTI) {
        ql[j] = shr1z(q[j]);
        qr[j] = shl1z(q[j]);
      } else {
        ql[j] = qr[j] = 0;
      }
    }
  }

  // level k (offset o) -> f_{k+1}; PER coarse rows per wave.  GLOBAL: f_k is f_t in HBM (level 0);
  // the wave then also writes the rows it loaded into LDS for the up phase (overlapping rows of
  // neighbouring waves are written twice with the same value), which replaces a separate staging pass.
  // SYNC (the first phase of a two-material FIX65 tail): the workgroup barrier that makes the staged tables and
  // pattern maps visible is taken here, after this phase's f_t rows were requested from HBM, so the two memory
  // round trips overlap instead of following each other (every wave has rows in that phase: 31 coarse rows over
  // 16 waves).
  template <bool GLOBAL, int PER, bool SYNC = false>
  __device__ __forceinline__ void down_rows(int k, int o, int I0, int I1) const {
    constexpr int R = 2 * PER + 3;
    const int H = Hk(k), N = Nk(k), Hc = (H + 1) / 2, Nc = (N + 1) / 2;
    T* f = fs + o;
    const uint8_t* pk = pl + o;
    T* fc = fs + o + H * N;
    const int yb = 2 * I0 - 2;  // rows yb .. yb + R - 1 (residual rows yb + 1 .. yb + R - 2)
    T fr[R], v[R], vl[R], vr[R], r[R], rl[R], rrt[R];
    int q[R], ql[R], qr[R];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int y = min(yb + j, H - 1);
      if constexpr (GLOBAL) fr[j] = fg[(long long)y * ld + lane];
      else fr[j] = f[y * N + lane];
    }
    if constexpr (SYNC) __syncthreads();
#pragma unroll
    for (int j = 0; j < R; ++j) q[j] = pat(pk, H, N, yb + j);
    if constexpr (GLOBAL) {
#pragma unroll
      for (int j = 0; j < R; ++j)
        if (yb + j < H && lane < N) f[(yb + j) * N + lane] = fr[j];
    }
#pragma unroll
    for (int j = 0; j < R; ++j) v[j] = inside(H, N, yb + j) ? omega(q[j]) * fr[j] : T(0);
    shift(v, vl, vr);
    shift(q, ql, qr);
    r[0] = r[R - 1] = T(0);
#pragma unroll
    for (int j = 1; j < R - 1; ++j) {
      const T kv = keep(Kx(j, vl, v, vr, ql, q, qr));
      r[j] = inside(H, N, yb + j) ? fr[j] - kv : T(0);
    }
    shift(r, rl, rrt);
    const int J = lane >> 1;
    const bool st = !(lane & 1) && J >= 1 && J <= Nc - 2;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      if (I0 + i >= I1) break;
      T acc = 0;
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const int j = 2 * i + 1 + ky;
        acc += rw(ql[j], ky * 3 + 0) * rl[j];
        acc += rw(q[j], ky * 3 + 1) * r[j];
        acc += rw(qr[j], ky * 3 + 2) * rrt[j];
      }
      acc = keep(acc);
      if (st) fc[(I0 + i) * Nc + J] = a.w0 * acc;
    }
  }
  template <bool GLOBAL>
  __device__ __forceinline__ void down(int k, int o) const {
    constexpr int kWaves = kTailThreads / 64;
    const int Hc = (Hk(k) + 1) / 2;
    const int per = (Hc - 2 + kWaves - 1) / kWaves;  // <= kTailDownRows
    const int I0 = 1 + wv * per, I1 = min(Hc - 1, I0 + per);
    if constexpr (GLOBAL && MULTI && HT == 65 && kTailLateSync) {  // 31 coarse rows: every wave has two
      down_rows<true, kTailDownRows, true>(k, o, I0, I1);
      return;
    }
    if (I0 >= I1) return;  // wave-uniform
    if (per == 1) down_rows<GLOBAL, 1>(k, o, I0, I1);
    else down_rows<GLOBAL, kTailDownRows>(k, o, I0, I1);
  }

  // coarsest level k: v1 = omd f, v2 = v1 + omd (f - K v1); PER rows per wave
  template <int PER>
  __device__ __forceinline__ void coarsest_rows(int k, int o, int y0, int y1) const {
    constexpr int R = PER + 2;
    const int H = Hk(k), N = Nk(k);
    const T* f = fs + o;
    const uint8_t* pk = pl + o;
    const int yb = y0 - 1;
    T fr[R], v[R], vl[R], vr[R];
    int q[R], ql[R], qr[R];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      fr[j] = f[min(yb + j, H - 1) * N + lane];
      q[j] = pat(pk, H, N, yb + j);
    }
#pragma unroll
    for (int j = 0; j < R; ++j) v[j] = inside(H, N, yb + j) ? omega(q[j]) * fr[j] : T(0);
    shift(v, vl, vr);
    shift(q, ql, qr);
#pragma unroll
    for (int j = 1; j < R - 1; ++j) {
      const int y = yb + j;
      if (y >= y1) break;
      const T kv = Kx(j, vl, v, vr, ql, q, qr);
      const T w = keep(omega(q[j]) * (fr[j] - kv) + v[j]);
      if (inside(H, N, y)) {
        if (k == 0 && !EXT) vg[(long long)y * ld + lane] = w;
        else es[o + y * N + lane] = w;
      }
    }
  }

  // level k (offset o) from the correction of level k + 1 (offset oc): x = omd f + w1 P e, one sweep.
  // PAR = parity of the wave's first window row, so every coarse-row index is a compile-time constant;
  // PER rows per wave.
  template <int PAR, int PER>
  __device__ __forceinline__ void up_rows(int k, int o, int oc, int y0, int y1) const {
    constexpr int R = PER + 2;                // x rows y0-1 .. y0+R-2
    constexpr int C = (PAR + R) / 2 + 1;      // coarse rows Ib .. Ib+C-1 that they touch
    const int H = Hk(k), N = Nk(k), Hc = (H + 1) / 2, Nc = (N + 1) / 2;
    const T* f = fs + o;
    const T* e = es + oc;
    const uint8_t* pk = pl + o;
    const uint8_t* pkc = pl + oc;
    const int yb = y0 - 1, Ib = yb >> 1;  // yb = 2 Ib + PAR
    const int Ja = (lane + 1) >> 1, Jb = (lane - 1) >> 1;  // even lane: Ja only (kx = 1); odd: Ja (kx = 0), Jb (kx = 2)
    const bool odd = lane & 1;
    T fr[R], ea[C], eb[C];
    int q[R], pa[C], pb[C];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      fr[j] = f[min(yb + j, H - 1) * N + lane];
      q[j] = pat(pk, H, N, yb + j);
    }
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const int I = Ib + c, Ic = min(I, Hc - 1);
      const bool iin = I >= 1 && I <= Hc - 2;
      const int jA = min(Ja, Nc - 1), jB = max(Jb, 0);
      const T va = e[Ic * Nc + jA], vb = e[Ic * Nc + jB];
      ea[c] = (iin && Ja >= 1 && Ja <= Nc - 2) ? va : T(0);
      eb[c] = (iin && Jb >= 1 && Jb <= Nc - 2) ? vb : T(0);
      if constexpr (MULTI) {
        pa[c] = pkc[Ic * Nc + jA] * (kTS * (int)sizeof(T));
        pb[c] = pkc[Ic * Nc + jB] * (kTS * (int)sizeof(T));
      } else {
        pa[c] = pb[c] = 0;
      }
    }
    T x[R], xl[R], xr[R];
    int ql[R], qr[R];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      T acc = 0;
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        if ((PAR + j + 1 - ky) & 1) continue;  // coarse row (y + 1 - ky) / 2 exists only for even y + 1 - ky
        const int c = (PAR + j + 1 - ky) >> 1;
        const T cfa = odd ? pw(pa[c], ky * 3 + 0) : pw(pa[c], ky * 3 + 1);
        const T t = acc + cfa * ea[c];
        const T t2 = t + pw(pb[c], ky * 3 + 2) * eb[c];
        acc = odd ? t2 : t;
      }
      const T v0 = omega(q[j]) * fr[j];
      const T xv = keep(v0 + a.w1 * acc);
      x[j] = inside(H, N, yb + j) ? xv : T(0);
    }
    shift(x, xl, xr);
    shift(q, ql, qr);
#pragma unroll
    for (int j = 1; j < R - 1; ++j) {
      const int y = yb + j;
      if (y >= y1) break;
      const T kx = Kx(j, xl, x, xr, ql, q, qr);
      const T w = keep(omega(q[j]) * (fr[j] - kx) + x[j]);
      if (inside(H, N, y)) {
        if (k == 0 && !EXT) vg[(long long)y * ld + lane] = w;
        else es[o + y * N + lane] = w;
      }
    }
  }

  // rows 1 .. H-2 of level k over the 16 waves: dispatch on the rows per wave (<= kTailUpRows)
  template <int PAR>
  __device__ __forceinline__ void up_par(int k, int o, int oc, int per, int y0, int y1) const {
    switch (per) {
      case 1: up_rows<PAR, 1>(k, o, oc, y0, y1); break;
      case 2: up_rows<PAR, 2>(k, o, oc, y0, y1); break;
      case 3: up_rows<PAR, 3>(k, o, oc, y0, y1); break;
      default: up_rows<PAR, kTailUpRows>(k, o, oc, y0, y1); break;
    }
  }
  __device__ __forceinline__ void up(int k, int o, int oc) const {
    constexpr int kWaves = kTailThreads / 64;
    const int H = Hk(k);
    const int per = (H - 2 + kWaves - 1) / kWaves;
    const int y0 = 1 + wv * per, y1 = min(H - 1, y0 + per);
    if (y0 >= y1) return;
    if ((y0 - 1) & 1) up_par<1>(k, o, oc, per, y0, y1);
    else up_par<0>(k, o, oc, per, y0, y1);
  }
  __device__ __forceinline__ void coarsest(int k, int o) const {
    constexpr int kWaves = kTailThreads / 64;
    const int H = Hk(k);
    const int per = (H - 2 + kWaves - 1) / kWaves;
    const int y0 = 1 + wv * per, y1 = min(H - 1, y0 + per);
    if (y0 >= y1) return;
    switch (per) {
      case 1: coarsest_rows<1>(k, o, y0, y1); break;
      case 2: coarsest_rows<2>(k, o, y0, y1); break;
      case 3: coarsest_rows<3>(k, o, y0, y1); break;
      default: coarsest_rows<kTailUpRows>(k, o, y0, y1); break;
    }
  }
};

template <typename T, bool MULTI, int HT = 0, int NLEV = 0, bool EXT = false>
__device__ __forceinline__ void tail_fast(const TailArgs<T>& a, T* es, T* fs, const T* ktb, const T* rtb,
                                          const T* ptb, const uint8_t* pl, int wv, int lane
#ifdef FEA_TAIL_TRACE
                                          , int& nph
#endif
) {
  const int nlev = NLEV ? NLEV : a.nlev;
  const long long s0 = (long long)blockIdx.x * a.bs_t + (128 / (int)sizeof(T) - 1) + a.ld_t;
  TailFast<T, MULTI, HT, EXT> t{a, es, fs, ktb, rtb, ptb, pl, a.f_t + s0, a.v_t + s0, a.ld_t, wv, lane};
  if constexpr (!MULTI) {  // single-pattern tables in registers (uniform loads)
#pragma unroll
    for (int d = 0; d < 9; ++d) {
      t.kr[d] = a.ktab[d];
      t.rr[d] = a.rtab[d];
      t.pr[d] = a.ptab[d];
    }
    t.om0 = a.omd[0];
  }
  // ------------------------------------------------------------------ down
  // (NLEV != 0: the level loops unroll, so k, the level sizes and offsets are constants in every phase)
  int o = 0;
  auto down = [&](int k) {
    if (k == 0 && !EXT) t.template down<true>(k, o);  // (EXT: level 0's f is already in LDS)
    else t.template down<false>(k, o);
    o += t.Hk(k) * t.Nk(k);
    FEA_TAIL_SYNC();
  };
  auto up = [&](int k) {
    const int oc = o;
    o -= t.Hk(k) * t.Nk(k);
    t.up(k, o, oc);
    if (k > 0) FEA_TAIL_SYNC();
  };
  if constexpr (NLEV != 0) {
#pragma unroll
    for (int k = 0; k + 1 < NLEV; ++k) down(k);
  } else {
    for (int k = 0; k + 1 < nlev; ++k) down(k);
  }
  // ------------------------------------------------------------------ coarsest: 2 sweeps
  t.coarsest(nlev - 1, o);
  if (nlev > 1) FEA_TAIL_SYNC();
  // ------------------------------------------------------------------ up
  if constexpr (NLEV != 0) {
#pragma unroll
    for (int k = NLEV - 2; k >= 0; --k) up(k);
  } else {
    for (int k = nlev - 2; k >= 0; --k) up(k);
  }
}

// FIX65: the V(1,1) 65^2 / 6-level tail of every BASELINE configuration only — a kernel of its own, so the
// register allocation is that path's alone (sharing one kernel with the general paths spilled 16 VGPRs of
// the fp64 single-pattern variant to scratch, reloaded inside the phases).
// FAST: any V(1,1) tail (the fused row-wave path) as a kernel without the general path, for the same reason
// (sharing one kernel spilled 68 B per lane of the fp64 single-pattern variant: C2's 65 -> 33 tail took 11.2 us).
template <typename T, bool MULTI, bool FIX65 = false, bool FAST = false>
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
  const bool fast = FIX65 || FAST || (a.nu1 == 1 && a.nu2 == 1 && !a.q2);
  if (!fast) {
    for (int i = tid; i < 3 * tot; i += kTailThreads) va[i] = T(0);
    FEA_TAIL_SYNC();  // the zero fill must land before f_t is staged into the same region
  }
  if (MULTI || !fast) {  // (the single-pattern fast path keeps its tables in registers)
    const int nt = MULTI ? a.ntab : 1;
    for (int i = tid; i < nt * kTS; i += kTailThreads) {
      const int p = i / kTS, d = i - p * kTS;
      ktb[i] = d == 9 ? a.omd[p] : a.ktab[p * 9 + d];
      rtb[i] = d == 9 ? T(0) : a.rtab[p * 9 + d];
      ptb[i] = d == 9 ? T(0) : a.ptab[p * 9 + d];
    }
  }
  if constexpr (MULTI)
    for (int i = tid; i < tot; i += kTailThreads) pl[i] = a.pid[i];
  const int wv = tid >> 6, lane = tid & 63;  // wave = row group, lane = column (Wt <= 65)
  constexpr int kWaves = kTailThreads / 64;
  if (!fast || (!FIX65 && nlev == 1)) {
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
  if constexpr (FIX65) {
    // the first down phase reads f_t from HBM itself and stages it for the up phase; single pattern:
    // the tables come from uniform loads, so nothing has to land before it
    if (MULTI && !kTailLateSync) FEA_TAIL_SYNC();  // (else the first phase takes it after its HBM loads)
    tail_fast<T, MULTI, 65, 6>(a, va, fs, ktb, rtb, ptb, pl, wv, lane
#ifdef FEA_TAIL_TRACE
                               , nph
#endif
    );
    return;
  } else if (fast) {
    if (MULTI || nlev == 1) FEA_TAIL_SYNC();
    tail_fast<T, MULTI>(a, va, fs, ktb, rtb, ptb, pl, wv, lane
#ifdef FEA_TAIL_TRACE
                        , nph
#endif
    );
    return;
  }
  FEA_TAIL_SYNC();

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
  // threads as a 32 x (threads / 32) grid over the interior nodes (no per-node integer division)
  constexpr int kTy = kTailThreads / 32;
  const int tx = tid & 31, ty = tid >> 5;
  auto sweep = [&](int H, int N, const uint8_t* pk, const T* f, const T* src, T* dst, bool zero) {
    for (int r = 1 + ty; r <= H - 2; r += kTy)
      for (int c = 1 + tx; c <= N - 2; c += 32) {
        const int i = r * N + c;
        const T om = ktb[P(pk, i) + 9];
        dst[i] = zero ? om * f[i] : om * (f[i] - Ku(N, pk, src, r, c)) + src[i];
      }
    FEA_TAIL_SYNC();
  };
  auto residual = [&](int H, int N, const uint8_t* pk, const T* f, const T* src, T* dst) {
    for (int r = 1 + ty; r <= H - 2; r += kTy)
      for (int c = 1 + tx; c <= N - 2; c += 32) dst[r * N + c] = f[r * N + c] - Ku(N, pk, src, r, c);
    FEA_TAIL_SYNC();
  };
  auto restrict_ = [&](int H, int N, const uint8_t* pk, const T* res, T* fc) {  // fine residual -> coarse f
    const int Nc = (N + 1) / 2, Hc = (H + 1) / 2;
    for (int I = 1 + ty; I <= Hc - 2; I += kTy)
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
    for (int y = 1 + ty; y <= H - 2; y += kTy)
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

// ---------------------------------------------------------------------------------------------
// The tail extended by ONE streamed level on top (fea_mg_coarse_tail_ext).  Level X (2 Ht - 1 rows x
// 2 Wt - 1 columns, framed in HBM) goes down and up inside the tail's launch: its zero-guess restriction
// (k_mg_zero_restrict: v = omd f, f_t = w0 R(f - K v)) writes level t's right-hand side straight into the
// tail's LDS before the sub-cycle, and its recomputed-iterate prolongation + sweep (k_mg_prolong_zu_ovl:
// x = omd f + w1 P e_t, v_X = omd (f - K x) + x) reads level t's correction from LDS after it — two launches
// of the 129^2 level (~5 us each, a boundary plus a row chain on a few waves) and the HBM round trips of f_t
// and v_t disappear.  Every node value is the same expression, in the same order, as in those streaming kernels
// (bitwise: tests/test_gpu_mg.py::test_coarse_tail_ext_bitwise).  Lane L holds level X's columns 2L+1, 2L+2 (one
// aligned 16-B fp64 / 8-B fp32 vector per row; its outer neighbours by DPP); the 16 waves split the rows.
// Single pattern, V(1,1) (the streaming kernels' zero-guess forms).
// ---------------------------------------------------------------------------------------------
template <typename T>
struct ExtArgs {
  const T* f;  // level X right-hand side (framed)
  T* v;        // level X iterate out (framed; interior written)
  int H, W, ld;
  long long bs;
};

template <typename T>
struct ExtV {  // a row at the lane's columns and their neighbours: a[0..3] = columns 2L .. 2L+3
  T a[4];
};
template <typename T>
__device__ __forceinline__ ExtV<T> ext_win(T x0, T x1) {  // (own_row of framed_ops.hip)
  ExtV<T> w;
  w.a[1] = x0;
  w.a[2] = x1;
  w.a[0] = shr1z(x1);
  w.a[3] = shl1z(x0);
  return w;
}
// (K x) at the lane's column k (0: 2L+1, 1: 2L+2): kapply's taps and order (framed_ops.hip)
template <typename T>
__device__ __forceinline__ T ext_k(const ExtV<T>& w0, const ExtV<T>& w1, const ExtV<T>& w2, int k,
                                   const T (&ks)[9]) {
  T acc = ks[0] * w0.a[k];
  acc += ks[1] * w0.a[k + 1];
  acc += ks[2] * w0.a[k + 2];
  acc += ks[3] * w1.a[k];
  acc += ks[4] * w1.a[k + 1];
  acc += ks[5] * w1.a[k + 2];
  acc += ks[6] * w2.a[k];
  acc += ks[7] * w2.a[k + 1];
  acc += ks[8] * w2.a[k + 2];
  return acc;
}
// crow_term (framed_ops.hip) at the lane's column k from a coarse row's values at columns L (ea) and L+1 (eb)
template <typename T>
__device__ __forceinline__ T ext_ct(T ea, T eb, int ky, int k, const T (&ps)[9]) {
  if (k == 1) return ps[ky * 3 + 1] * eb;  // even fine column 2L+2: coarse node L+1, kx = 1
  T t = ps[ky * 3 + 2] * ea;              // odd fine column 2L+1: coarse nodes L (kx = 2) and L+1 (kx = 0)
  t += ps[ky * 3 + 0] * eb;
  return t;
}
template <typename Fn, int... J>
__device__ __forceinline__ void ext_unroll(Fn&& fn, std::integer_sequence<int, J...>) {  // fn(1) .. fn(PER)
  (fn(std::integral_constant<int, J + 1>{}), ...);
}
template <typename T>
__device__ __forceinline__ void ext_load(const T* p, T& x0, T& x1) {
  typedef T v2 __attribute__((ext_vector_type(2)));
  const v2 v = *reinterpret_cast<const v2*>(p);
  x0 = v[0];
  x1 = v[1];
}

// level X -> fs0 (level t's right-hand side, Ht x Wt, pitch Wt, interior written): coarse rows [I0, I1) per wave.
// The rows stream through a 3-row window (all loads issued first); every second residual row closes a coarse row.
template <typename T>
__device__ __forceinline__ void ext_down(const TailArgs<T>& a, const ExtArgs<T>& x, T* fs0, int Ht, int Wt, int wv,
                                         int lane) {
  constexpr int PER = (63 + kTailThreads / 64 - 1) / (kTailThreads / 64), R = 2 * PER + 3;  // Ht - 2 <= 63 coarse rows
  constexpr int NW = kTailThreads / 64;
  const int per = (Ht - 2 + NW - 1) / NW;
  const int I0 = 1 + wv * per, I1 = min(Ht - 1, I0 + per);
  if (I0 >= I1) return;  // wave-uniform
  const int H = x.H, W = x.W;
  const int yb = 2 * I0 - 2;  // fine rows yb .. yb + R - 1
  const int c0 = 2 * lane + 1;
  // lanes past the grid load the last interior pair (masked; their values only feed masked neighbours)
  const T* fb = x.f + (long long)blockIdx.x * x.bs + (128 / (int)sizeof(T) - 1) + min(c0, W - 2);
  T f0[R], f1[R];
#pragma unroll
  for (int j = 0; j < R; ++j) ext_load(fb + (long long)(min(yb + j, H - 1) + 1) * x.ld, f0[j], f1[j]);
  T ks[9], rs[9];
#pragma unroll
  for (int d = 0; d < 9; ++d) {
    ks[d] = a.ktab[d];
    rs[d] = a.rtab[d];
  }
  const T om = a.omd[0], w0 = a.w0;
  const bool cin0 = c0 <= W - 2, cin1 = c0 + 1 <= W - 2;
  auto vrow = [&](int j) {
    const int y = yb + j;
    const bool rin = y >= 1 && y <= H - 2;
    return ext_win<T>((rin && cin0) ? om * f0[j] : T(0), (rin && cin1) ? om * f1[j] : T(0));
  };
  ExtV<T> va = vrow(0), vb = vrow(1);
  T ra[3], rb[3];  // the last two residual rows at columns 2L+1, 2L+2, 2L+3 (odd row 2I-1, then even row 2I)
  const int J = lane + 1;  // coarse column of fine column 2L+2
#pragma unroll
  for (int j = 1; j < R - 1; ++j) {
    const ExtV<T> vc = vrow(j + 1);
    T r[3];
    r[0] = f0[j] - ext_k<T>(va, vb, vc, 0, ks);
    r[1] = f1[j] - ext_k<T>(va, vb, vc, 1, ks);
    r[2] = shl1z(r[0]);
    va = vb;
    vb = vc;
    if (j >= 3 && (j & 1)) {  // rows j-2, j-1, j = 2I-1, 2I, 2I+1 with I = I0 + (j-3)/2
      const int I = I0 + (j - 3) / 2;
      if (I >= I1) break;  // wave-uniform
      T acc = rs[0] * ra[0];
      acc += rs[1] * ra[1];
      acc += rs[2] * ra[2];
      acc += rs[3] * rb[0];
      acc += rs[4] * rb[1];
      acc += rs[5] * rb[2];
      acc += rs[6] * r[0];
      acc += rs[7] * r[1];
      acc += rs[8] * r[2];
      if (J <= Wt - 2) fs0[I * Wt + J] = w0 * acc;
    }
    if (j & 1) {
#pragma unroll
      for (int k = 0; k < 3; ++k) ra[k] = r[k];
    } else {
#pragma unroll
      for (int k = 0; k < 3; ++k) rb[k] = r[k];
    }
  }
}

// es0 (level t's correction, Ht x Wt, pitch Wt, interior valid) -> level X's iterate on fine rows [y0, y1) per wave
template <typename T>
__device__ __forceinline__ void ext_up(const TailArgs<T>& a, const ExtArgs<T>& x, const T* es0, int Ht, int Wt, int wv,
                                       int lane) {
  constexpr int PER = 2 * ((127 + kTailThreads / 32 - 1) / (kTailThreads / 32)), R = PER + 2;  // x rows y0-1 .. y0+PER
  constexpr int NW = kTailThreads / 64;
  const int H = x.H, W = x.W;
  const int per = 2 * ((H - 2 + 2 * NW - 1) / (2 * NW));  // even: y0 - 1 is even on every wave
  const int y0 = 1 + wv * per, y1 = min(H - 1, y0 + per);
  if (y0 >= y1) return;  // wave-uniform
  const int c0 = 2 * lane + 1;
  const long long boff = (long long)blockIdx.x * x.bs + (128 / (int)sizeof(T) - 1);
  const T* fb = x.f + boff + min(c0, W - 2);
  T f0[R], f1[R];
#pragma unroll
  for (int j = 0; j < R; ++j) ext_load(fb + (long long)(min(y0 - 1 + j, H - 1) + 1) * x.ld, f0[j], f1[j]);
  const int cb = (y0 - 1) >> 1;
  // coarse row cb + m at columns L (ea) and L+1 (eb), read from LDS where used (0 off the interior, as the
  // framed zeros)
  const bool ja = lane >= 1 && lane <= Wt - 2, jb = lane + 1 <= Wt - 2;
  const int la = min(lane, Wt - 1), lb = min(lane + 1, Wt - 1);
  auto ea = [&](int m) {
    const int I = cb + m;
    const T v = es0[min(I, Ht - 1) * Wt + la];
    return (I >= 1 && I <= Ht - 2 && ja) ? v : T(0);
  };
  auto eb = [&](int m) {
    const int I = cb + m;
    const T v = es0[min(I, Ht - 1) * Wt + lb];
    return (I >= 1 && I <= Ht - 2 && jb) ? v : T(0);
  };
  T ks[9], ps[9];
#pragma unroll
  for (int d = 0; d < 9; ++d) {
    ks[d] = a.ktab[d];
    ps[d] = a.ptab[d];
  }
  const T om = a.omd[0], w1 = a.w1;
  const bool cin0 = c0 <= W - 2, cin1 = c0 + 1 <= W - 2;
  auto xrow = [&](auto jc) {  // x of row y0 - 1 + j (its parity is j's)
    constexpr int j = decltype(jc)::value;
    const int y = y0 - 1 + j;
    const bool rin = y >= 1 && y <= H - 2;
    T xv[2];
    xv[0] = (rin && cin0) ? om * f0[j] : T(0);
    xv[1] = (rin && cin1) ? om * f1[j] : T(0);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      if constexpr ((j & 1) == 0) {
        xv[k] += w1 * ext_ct<T>(ea(j / 2), eb(j / 2), 1, k, ps);
      } else {
        const T t = ext_ct<T>(ea(j / 2), eb(j / 2), 2, k, ps) + ext_ct<T>(ea(j / 2 + 1), eb(j / 2 + 1), 0, k, ps);
        xv[k] += w1 * t;
      }
    }
    return ext_win<T>(xv[0], xv[1]);
  };
  T* vb_ = x.v + boff + c0;
  ExtV<T> A = xrow(std::integral_constant<int, 0>{}), B = xrow(std::integral_constant<int, 1>{});
  auto emit = [&](auto jc) {  // row y0 - 1 + j from the windows j-1 (A), j (B), j+1 (C)
    constexpr int j = decltype(jc)::value;
    const ExtV<T> Cw = xrow(std::integral_constant<int, j + 1>{});
    const int y = y0 - 1 + j;
    if (y < y1) {  // wave-uniform
      T o[2];
      o[0] = om * (f0[j] - ext_k<T>(A, B, Cw, 0, ks)) + B.a[1];
      o[1] = om * (f1[j] - ext_k<T>(A, B, Cw, 1, ks)) + B.a[2];
      T* p = vb_ + (long long)(y + 1) * x.ld;
      if (cin1) {
        typedef T v2 __attribute__((ext_vector_type(2)));
        v2 v;
        v[0] = o[0];
        v[1] = o[1];
        *reinterpret_cast<v2*>(p) = v;
      } else if (cin0) {
        p[0] = o[0];
      }
    }
    A = B;
    B = Cw;
  };
  ext_unroll(emit, std::make_integer_sequence<int, PER>{});
}

template <typename T, bool FIX65>
__global__ __launch_bounds__(kTailThreads) void k_mg_coarse_tail_ext(TailArgs<T> a, ExtArgs<T> x) {
  __shared__ __attribute__((aligned(16))) char smem[kTailLdsBytes];
  const int tid = threadIdx.x;
  const int Ht = FIX65 ? 65 : a.Ht, Wt = FIX65 ? 65 : a.Wt;
  const int tot = tail_off(Ht, Wt, FIX65 ? 6 : a.nlev);
  T* es = reinterpret_cast<T*>(smem);  // the fast path's two regions: corrections, right-hand sides
  T* fs = es + tot;
  const int wv = tid >> 6, lane = tid & 63;
  ext_down<T>(a, x, fs, Ht, Wt, wv, lane);
  __syncthreads();
#ifdef FEA_TAIL_TRACE
  int nph = 0;
#define FEA_EXT_NPH , nph
#else
#define FEA_EXT_NPH
#endif
  if constexpr (FIX65) tail_fast<T, false, 65, 6, true>(a, es, fs, nullptr, nullptr, nullptr, nullptr, wv, lane FEA_EXT_NPH);
  else tail_fast<T, false, 0, 0, true>(a, es, fs, nullptr, nullptr, nullptr, nullptr, wv, lane FEA_EXT_NPH);
#undef FEA_EXT_NPH
  __syncthreads();
  ext_up<T>(a, x, es, Ht, Wt, wv, lane);
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
    const bool fix65 = Ht == 65 && Wt == 65 && nlev == 6 && nu1 == 1 && nu2 == 1 && !q2;                     \
    hipStream_t s_ = (hipStream_t)stream;                                                                     \
    const bool v11 = nu1 == 1 && nu2 == 1 && !q2;                                                             \
    if (multi && fix65) k_mg_coarse_tail<T, true, true><<<B, kTailThreads, 0, s_>>>(a);                       \
    else if (multi && v11) k_mg_coarse_tail<T, true, false, true><<<B, kTailThreads, 0, s_>>>(a);             \
    else if (multi) k_mg_coarse_tail<T, true><<<B, kTailThreads, 0, s_>>>(a);                                  \
    else if (fix65) k_mg_coarse_tail<T, false, true><<<B, kTailThreads, 0, s_>>>(a);                          \
    else if (v11) k_mg_coarse_tail<T, false, false, true><<<B, kTailThreads, 0, s_>>>(a);                     \
    else k_mg_coarse_tail<T, false><<<B, kTailThreads, 0, s_>>>(a);                                            \
    FEA_LAUNCH_CHECK();                                                                                       \
  }

FEA_TAIL_API(f32, float)
FEA_TAIL_API(f64, double)

#define FEA_TAIL_EXT_API(SUF, T)                                                                              \
  extern "C" int fea_mg_coarse_tail_ext_##SUF(const T* f_x, T* v_x, int Hx, int Wx, int ld_x, long long bs_x,  \
                                              int nlev, const T* ktab, const T* omd, int ntab, const T* rtab,   \
                                              const T* ptab, T w0, T w1, int B, void* stream) {                \
    if (!f_x || !v_x || !ktab || !omd || !rtab || !ptab || B <= 0 || nlev < 1 || nlev > kTailMaxLevels)       \
      return FEA_EINVAL;                                                                                      \
    if (ntab != 1 || Hx < 5 || Wx < 5 || !(Hx & 1) || !(Wx & 1)) return FEA_EINVAL;                            \
    const int Ht = (Hx + 1) / 2, Wt = (Wx + 1) / 2;                                                           \
    if (!tail_dim_ok(Ht, nlev) || !tail_dim_ok(Wt, nlev)) return FEA_EINVAL;                                  \
    if (ld_x < Wx + 128 / (int)sizeof(T) || bs_x < (long long)(Hx + 2) * ld_x) return FEA_EINVAL;              \
    if (tail_lds_bytes<T>(Ht, Wt, nlev, false) > kTailLdsBytes) return FEA_EINVAL;                            \
    TailArgs<T> a{f_x, v_x, nullptr, ktab, omd, rtab, ptab, w0, w1, Ht, Wt, nlev, ld_x, bs_x, 1, 1, 1, 0};       \
    ExtArgs<T> x{f_x, v_x, Hx, Wx, ld_x, bs_x};                                                               \
    hipStream_t s_ = (hipStream_t)stream;                                                                     \
    if (Ht == 65 && Wt == 65 && nlev == 6) k_mg_coarse_tail_ext<T, true><<<B, kTailThreads, 0, s_>>>(a, x);     \
    else k_mg_coarse_tail_ext<T, false><<<B, kTailThreads, 0, s_>>>(a, x);                                    \
    FEA_LAUNCH_CHECK();                                                                                       \
  }

FEA_TAIL_EXT_API(f32, float)
FEA_TAIL_EXT_API(f64, double)

#ifdef FEA_TAIL_TRACE
extern "C" int fea_tail_trace_read(long long* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_tail_trace), sizeof(long long) * 256, 0, hipMemcpyDeviceToHost);
}
#endif
