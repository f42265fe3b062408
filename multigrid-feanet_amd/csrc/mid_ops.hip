// mid_ops.hip — several consecutive coarse levels of the V-cycle in ONE launch.
//
// Between the bandwidth-bound fine levels and the LDS-resident coarse tail sit levels of 129^2 ..
// 1025^2 nodes whose per-level kernels are latency-bound (~5 us each for ~1 MB of data, twice per
// V-cycle).  Their V(1,1) work is a pure function of data that is already on the device:
//
//   down (zero-guess pre-sweep, FEANet/multigrid.py:171-172 then :168-170, per level l = a..a+k-1):
//       v_l = omd f_l (interior, 0 on the boundary);   f_{l+1} = w0 R(f_l - K v_l)
//   up (prolongation + correction + post-sweep, :177-181, per level l = a+k-1 .. a):
//       x_l = v_l + w1 P(u_{l+1});                     u_l = x_l + omd (f_l - K x_l)   (interior)
//
// so k levels fuse into one launch of independent TILES with recomputed halos (no grid-wide
// synchronisation):
//   k_mg_mid_down: a workgroup owns a T x T tile of f_{a+k}; it stages the f_a region the tile
//     depends on (2^k T + 3 (2^k - 1) per side) in LDS and restricts it level by level in LDS
//     (residual rows in a scratch region, restriction into the next level's region), writing the
//     rows/columns of f_{a+1} .. f_{a+k} it owns to HBM (the up pass and the coarse tail read them).
//   k_mg_mid_up: a workgroup owns a T x T tile of u_a; it stages u_{a+k} and f_a .. f_{a+k-1} on the
//     regions the tile depends on (x_l needs u_{l+1} on a region ~half its size plus a 1-node halo)
//     and runs prolongation + correction + sweep level by level in LDS; only u_a goes to HBM (the
//     intermediate iterates have no other reader).
//
// Every node value is computed with the same expression, in the same order, as the per-level
// kernels (k_mg_resid_restrict zero-guess mode, k_mg_prolong ZU mode; fp-contract=on), so the
// result is bitwise that of the per-level launches.  Two-material problems (per-pattern tables,
// uint8 pattern maps per level) are supported; the regions are read in the framed layout of
// fea_mg_layout at every level.
#include "fea_common.h"

namespace fea {

constexpr int kMidThreads = 1024;
constexpr int kMidMaxK = 4;
constexpr int kMidLdsBytes = 160 * 1024 - 2048;
constexpr int kMS = 10;  // table stride: 9 weights + omega/d

#ifdef FEA_MID_TRACE  // lab builds only (tools/lab/mid_trace.py): s_memrealtime per workgroup and phase
__device__ long long g_mid_trace[4096];
#define FEA_MID_MARK(slot) \
  if (threadIdx.x == 0) g_mid_trace[slot] = (long long)__builtin_amdgcn_s_memrealtime()
#define FEA_MID_SYNC(ph)                                                                   \
  do {                                                                                     \
    __syncthreads();                                                                       \
    if (blockIdx.x == 0 && threadIdx.x == 0) g_mid_trace[2048 + (ph)] = (long long)__builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define FEA_MID_WAVE_MARK(slot)                                                              \
  if (blockIdx.x == 0 && (threadIdx.x & 63) == 0)                                            \
  g_mid_trace[3072 + (slot) * 16 + (threadIdx.x >> 6)] = (long long)__builtin_amdgcn_s_memrealtime()
#else
#define FEA_MID_MARK(slot)
#define FEA_MID_SYNC(ph) __syncthreads()
#define FEA_MID_WAVE_MARK(slot)
#endif

template <typename T>
struct MidArgs {
  const T* f[kMidMaxK + 1];  // down: f_a (in), f_{a+1..a+k} (out, via fo); up: f_a .. f_{a+k-1}
  T* fo[kMidMaxK + 1];
  const uint8_t* pid[kMidMaxK + 1];  // per-level pattern maps (MULTI), framed, one per mesh
  int H[kMidMaxK + 1], W[kMidMaxK + 1], ld[kMidMaxK + 1];
  long long bs[kMidMaxK + 1];
  const T* e;  // up: u_{a+k}
  T* out;      // up: u_a
  const T* ktab;
  const T* omd;
  const T* xtab;  // down: R kernels, up: P kernels
  T w;            // down: w0, up: w1
  int k, ntab, nx;
  int TR, TC, ntr, ntc;  // tile size and tiles per dimension (at level a+k down, level a up)
  // down, gathered top level (a domain-decomposed run's agglomerated coarse problem): f_a is read from the
  // all-gather's buffer gsrc ([Pr * Pc][B][gcr][gcc]: rank blocks of gcr x gcc interior nodes, rank order) and
  // each tile places the nodes it owns into the framed f_a (fo[0]) for the later launches — the placement copy
  // folded into the launch that reads the blocks first
  const T* gsrc;
  int gB, gPc, gcr, gcc;
};

// One region of a level: rows [r0, r0+nr), columns [c0, c0+nc), row-major in LDS.
struct Reg {
  int r0, c0, nr, nc;
};

__device__ __forceinline__ bool interior(int H, int W, int y, int c) {
  return y >= 1 && y <= H - 2 && c >= 1 && c <= W - 2;
}

// Coefficient tables (9 weights + omega/d per pattern, and the transfer kernels) go through LDS for
// every problem: threads issue their table element's load together with the region loads (one
// memory round trip for the whole preamble; scalar loads of the tables would be waited for before
// the region loads could be addressed) and store it after; the single-pattern kernels then read
// their weights from LDS into registers (broadcast reads).
template <typename T>
struct TabLoad {
  T k, x;
};
template <typename T>
__device__ __forceinline__ TabLoad<T> tables_issue(const T* ktab, const T* omd, const T* xtab, int ntab, int nx) {
  const int i = threadIdx.x, ix = (int)threadIdx.x - 512;
  const int ik = min(i, ntab * kMS - 1), jx = min(max(ix, 0), nx * kMS - 1);
  const int pk = ik / kMS, dk = ik - pk * kMS, px = jx / kMS, dx = jx - px * kMS;
  TabLoad<T> t;
  t.k = dk == 9 ? omd[pk] : ktab[pk * 9 + dk];
  t.x = dx == 9 ? T(0) : xtab[px * 9 + (dx == 9 ? 0 : dx)];
  return t;
}
template <typename T>
__device__ __forceinline__ void tables_commit(const TabLoad<T>& t, T* ktb, T* xtb, int ntab, int nx) {
  const int i = threadIdx.x, ix = (int)threadIdx.x - 512;
  if (i < ntab * kMS) ktb[i] = t.k;
  if (ix >= 0 && ix < nx * kMS) xtb[ix] = t.x;
}

// Staging: every load of a launch's input regions is issued before the first LDS store, so the
// whole stage costs one memory round trip (a plain copy loop waits for each load in turn).  Wave w
// takes region rows w, w+16, ... (regions are <= 64 columns: lane = column).
constexpr int kStageRows = 5;  // rows per wave per region in one batch (regions <= 80 rows)
template <typename E>
struct StageJob {
  const E* src;  // framed level (sample base), element (r, c) at src[(r+1)*ld + off + c]
  E* dst;
  Reg g;
  int H, W, ld, off;
};
template <typename E, int N>
__device__ __forceinline__ void stage_batch(const StageJob<E> (&jobs)[N]) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  constexpr int NW = kMidThreads / 64;
  for (int base = 0;; base += kStageRows * NW) {
    E v[N][kStageRows];
    bool more = false;
    // unconditional loads from clamped (always valid) addresses; the masks are applied at the
    // stores, after every load is in flight (a conditional load would be waited for at its branch)
#pragma unroll
    for (int q = 0; q < N; ++q) {
      const StageJob<E>& J = jobs[q];
      const int c = min(max(J.g.c0 + lane, 0), J.W - 1);
#pragma unroll
      for (int i = 0; i < kStageRows; ++i) {
        const int yy = base + wv + i * NW;  // wave-uniform: rows past the region are not loaded
        const int y = min(max(J.g.r0 + yy, 0), J.H - 1);
        v[q][i] = E(0);
        if (yy < J.g.nr) v[q][i] = J.src[(long long)(y + 1) * J.ld + J.off + c];
      }
      more |= base + kStageRows * NW < J.g.nr;
    }
#pragma unroll
    for (int q = 0; q < N; ++q) {
      const StageJob<E>& J = jobs[q];
      const int c = J.g.c0 + lane;
      const bool cok = c >= 0 && c < J.W;
#pragma unroll
      for (int i = 0; i < kStageRows; ++i) {
        const int yy = base + wv + i * NW, y = J.g.r0 + yy;
        if (yy < J.g.nr && lane < J.g.nc) J.dst[yy * J.g.nc + lane] = (cok && y >= 0 && y < J.H) ? v[q][i] : E(0);
      }
    }
    if (!more) break;
  }
}

// LDS bytes of one down / up launch with a full T x T tile (host: tile choice; device: carving)
__host__ __device__ inline void mid_down_regions(int k, int TR, int TC, Reg* g) {
  g[k] = Reg{0, 0, TR, TC};
  for (int j = k - 1; j >= 0; --j) g[j] = Reg{0, 0, 2 * g[j + 1].nr + 3, 2 * g[j + 1].nc + 3};
}
__host__ __device__ inline long long mid_down_lds(int k, int TR, int TC, int esz, bool multi) {
  Reg g[kMidMaxK + 1];
  mid_down_regions(k, TR, TC, g);
  long long e = 0, pb = 0, rmax = 0;
  for (int j = 0; j <= k; ++j) {
    e += (long long)g[j].nr * g[j].nc;
    if (multi && j < k) pb += ((long long)g[j].nr * g[j].nc + 15) / 16 * 16;
    if (j < k) rmax = rmax > (long long)(g[j].nr - 2) * g[j].nc ? rmax : (long long)(g[j].nr - 2) * g[j].nc;
  }
  if (g[0].nc > 64) return 1LL << 40;  // row-wave kernels: a region row fits one wave
  return (e + rmax) * esz + pb + 2LL * FEA_MAX_PATTERNS * kMS * esz + 64;
}
// up: the u region of level j+1 covering the x region [r0-1, r0+nr] of level j (same for columns)
__host__ __device__ inline Reg mid_coarse_of(const Reg& u) {
  const int r0 = (u.r0 - 1) >> 1, r1 = (u.r0 + u.nr + 1) >> 1;  // inclusive
  const int c0 = (u.c0 - 1) >> 1, c1 = (u.c0 + u.nc + 1) >> 1;
  return Reg{r0, c0, r1 - r0 + 1, c1 - c0 + 1};
}
__host__ __device__ inline long long mid_up_lds(int k, int TR, int TC, int esz, bool multi) {
  // region sizes below the tile level depend on the tile's alignment: take the worst over every
  // residue of the tile index that reaches level k (rows and columns alike)
  long long worst = 0;
  for (int t = 0; t < (2 << k); ++t) {
    Reg u = Reg{1 + t * TR, 1 + t * TC, TR, TC};
    if (TC + 2 > 64) return 1LL << 40;  // row-wave kernels: a region row fits one wave
    long long e = 0, pb = 0, xmax = 0;
    for (int j = 0; j < k; ++j) {
      const long long xn = (long long)(u.nr + 2) * (u.nc + 2);
      e += xn;  // f on the x region
      if (multi) pb += (xn + 15) / 16 * 16;
      xmax = xmax > xn ? xmax : xn;
      u = mid_coarse_of(u);
      e += (long long)u.nr * u.nc;  // u_{j+1}
    }
    if (multi) pb += ((long long)u.nr * u.nc + 15) / 16 * 16;
    const long long b = (e + xmax) * esz + pb + 2LL * FEA_MAX_PATTERNS * kMS * esz + 64;
    worst = worst > b ? worst : b;
  }
  return worst;
}

// ---------------------------------------------------------------------------------------------
// down: f_a -> f_{a+1} .. f_{a+k}
// ---------------------------------------------------------------------------------------------
template <typename T, bool MULTI, int K, bool GATH = false>
__global__ __launch_bounds__(kMidThreads) void k_mg_mid_down(MidArgs<T> a) {
  __shared__ __attribute__((aligned(16))) char smem[kMidLdsBytes];
  FEA_MID_MARK(2 * blockIdx.x);
  constexpr int OFF = 128 / (int)sizeof(T) - 1;
  constexpr int k = K;  // compile-time: every per-level array below stays in registers
  const int tiles = a.ntr * a.ntc;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int b = bid / tiles, t = bid - b * tiles, ti = t / a.ntc, tj = t - ti * a.ntc;
  // regions: level k = the tile of f_{a+k}; level j = the f_j rows/columns that tile depends on
  Reg g[kMidMaxK + 1];
  // owned rows/columns per level [os, oe): the tile at level k; a finer level owns the fine nodes
  // 2I-1 .. 2I'-1 of its coarse range (through the last boundary-adjacent row for the last tile)
  int os_r[kMidMaxK + 1], os_c[kMidMaxK + 1], oe_r[kMidMaxK + 1], oe_c[kMidMaxK + 1];
  {
    const int r0 = 1 + ti * a.TR, c0 = 1 + tj * a.TC;
    g[k] = Reg{r0, c0, min(r0 + a.TR, a.H[k] - 1) - r0, min(c0 + a.TC, a.W[k] - 1) - c0};
    os_r[k] = g[k].r0;
    os_c[k] = g[k].c0;
    oe_r[k] = g[k].r0 + g[k].nr;
    oe_c[k] = g[k].c0 + g[k].nc;
#pragma unroll
    for (int j = k - 1; j >= 0; --j) {
      g[j] = Reg{2 * g[j + 1].r0 - 2, 2 * g[j + 1].c0 - 2, 2 * g[j + 1].nr + 3, 2 * g[j + 1].nc + 3};
      os_r[j] = 2 * os_r[j + 1] - 1;
      os_c[j] = 2 * os_c[j + 1] - 1;
      oe_r[j] = oe_r[j + 1] == a.H[j + 1] - 1 ? a.H[j] - 1 : 2 * oe_r[j + 1] - 1;
      oe_c[j] = oe_c[j + 1] == a.W[j + 1] - 1 ? a.W[j] - 1 : 2 * oe_c[j + 1] - 1;
    }
  }
  // LDS carve: F[0..k], R scratch, tables, pattern regions
  T* F[kMidMaxK + 1];
  T* p = reinterpret_cast<T*>(smem);
  long long rmax = 0;
#pragma unroll
  for (int j = 0; j <= k; ++j) {
    F[j] = p;
    p += g[j].nr * g[j].nc;
    if (j < k) rmax = max(rmax, (long long)(g[j].nr - 2) * g[j].nc);
  }
  T* Rs = p;
  p += rmax;
  T* ktb = p;
  T* xtb = ktb + FEA_MAX_PATTERNS * kMS;
  uint8_t* P[kMidMaxK + 1];
  uint8_t* q = reinterpret_cast<uint8_t*>(xtb + FEA_MAX_PATTERNS * kMS);
#pragma unroll
  for (int j = 0; j < k; ++j) {
    P[j] = q;
    if constexpr (MULTI) q += (g[j].nr * g[j].nc + 15) / 16 * 16;
  }
  // single pattern: weights in registers from uniform loads and the top level read straight from
  // HBM by the first phase (no staging pass, nothing to wait for before it); two materials: tables
  // and the pattern maps of every level go through LDS first
  T ks[9], rs[9], om = T(0);
  if constexpr (MULTI) {
    const TabLoad<T> tl = tables_issue<T>(a.ktab, a.omd, a.xtab, a.ntab, a.nx);
    StageJob<uint8_t> jp[k];
#pragma unroll
    for (int j = 0; j < k; ++j) jp[j] = {a.pid[j], P[j], g[j], a.H[j], a.W[j], a.ld[j], OFF};
    stage_batch<uint8_t, k>(jp);
    tables_commit<T>(tl, ktb, xtb, a.ntab, a.nx);
    FEA_MID_SYNC(0);
  } else {
#pragma unroll
    for (int d = 0; d < 9; ++d) {
      ks[d] = a.ktab[d];
      rs[d] = a.xtab[d];
    }
    om = a.omd[0];
  }

  // Per level: wave w owns a contiguous block of coarse-region rows; for each chunk of <= 2 of them it
  // loads the 2 PER + 3 fine-region rows they depend on at once (LDS, or HBM on the top level),
  // forms v = omd f, the residual rows r = f - K v and their restriction in registers (column
  // neighbours by DPP, each row shifted once), so a level costs one barrier and one load round trip.
  // Per-node expressions and their order are those of k_mg_resid_restrict (zero-guess mode).
  constexpr int NW = kMidThreads / 64;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < k; ++j) {
    const Reg G = g[j], C = g[j + 1];
    const int H = a.H[j], W = a.W[j], Hc = a.H[j + 1], Wc = a.W[j + 1];
    const T* f = F[j];
    const uint8_t* pj = P[j];
    // row-wave form (regions are <= 64 columns): lane = column G.c0 + lane
    const int c = G.c0 + lane;
    const bool lv = lane < G.nc;
    const bool cin = lv && c >= 1 && c <= W - 2;
    const T* src = a.f[0] + (long long)b * a.bs[0] + OFF + min(max(c, 0), W - 1);  // top level, row -1
    const int ld0 = a.ld[0];
    // gathered top level: the lane's column inside its rank block (nodes 1 .. W-1 lie in blocks)
    const int gcl = min(max(c, 1), W - 1) - 1;
    const int gbi = GATH ? gcl / a.gcc : 0, gbc = gcl - gbi * a.gcc;
    auto gload = [&](int y) -> T {
      const int yy = min(max(y, 1), H - 1) - 1;
      const int ri = yy / a.gcr, rr = yy - ri * a.gcr;
      const T v = a.gsrc[(((long long)(ri * a.gPc + gbi) * a.gB + b) * a.gcr + rr) * a.gcc + gbc];
      return (y >= 1 && y <= H - 1 && c >= 1 && c <= W - 1) ? v : T(0);
    };
    T* const place = a.fo[0] + (long long)b * a.bs[0] + OFF + c;
    T* fc = F[j + 1];
    T* go = a.fo[j + 1] + (long long)b * a.bs[j + 1];
    const int ldc = a.ld[j + 1];
    const int JJ = (lane - 2) >> 1;  // even lane 2 + 2 JJ holds fine column 2J
    const int J = C.c0 + JJ;
    const bool outl = !(lane & 1) && lane >= 2 && JJ < C.nc;
    const bool jin = J >= 1 && J <= Wc - 2, jown = J >= os_c[j + 1] && J < oe_c[j + 1];
    auto rows = [&](auto per_c, auto glob_c, int II0, int II1) {
      constexpr int PER = decltype(per_c)::value;
      constexpr bool GLOB = decltype(glob_c)::value;
      constexpr int R = 2 * PER + 3;  // fine-region rows 2 II0 .. 2 II0 + R - 1
      T fr[R], v[R], vl[R], vh[R], r[R], rl[R], rh[R];
      int pr[R], pl[R], ph[R];
#pragma unroll
      for (int d = 0; d < R; ++d) {
        const int rr = 2 * II0 + d, y = G.r0 + rr;
        if constexpr (GLOB && GATH) fr[d] = gload(y);
        else if constexpr (GLOB) fr[d] = src[(long long)(min(max(y, 0), H - 1) + 1) * ld0];
        else fr[d] = f[min(rr, G.nr - 1) * G.nc + lane];
        pr[d] = 0;
        if constexpr (MULTI) {
          const int pv = pj[min(rr, G.nr - 1) * G.nc + min(lane, G.nc - 1)];
          pr[d] = lv ? pv : 0;
        }
      }
#pragma unroll
      for (int d = 0; d < R; ++d) {
        const int y = G.r0 + 2 * II0 + d;
        const bool in = cin && y >= 1 && y <= H - 2;
        T om_ = om;
        if constexpr (MULTI) om_ = ktb[pr[d] * kMS + 9];
        v[d] = in ? om_ * fr[d] : T(0);
        vl[d] = shr1z(v[d]);
        vh[d] = shl1z(v[d]);
        pl[d] = ph[d] = 0;
        if constexpr (MULTI) {
          pl[d] = shr1z(pr[d]);
          ph[d] = shl1z(pr[d]);
        }
      }
      if constexpr (GLOB && GATH) {
        {  // placement of the tile's own interior nodes of the gathered top level
          const bool oc = lv && c >= os_c[0] && c < oe_c[0] && c >= 1 && c <= W - 2;
#pragma unroll
          for (int d = 0; d < R; ++d) {
            const int y = G.r0 + 2 * II0 + d;
            if (oc && y >= os_r[0] && y < oe_r[0] && y >= 1 && y <= H - 2) place[(long long)(y + 1) * ld0] = fr[d];
          }
        }
      }
      r[0] = r[R - 1] = T(0);
#pragma unroll
      for (int d = 1; d < R - 1; ++d) {
        // (1) residual row: kapply order, rows d-1, d, d+1, columns left to right
        T acc;
        if constexpr (!MULTI) {
          acc = ks[0] * vl[d - 1];
          acc += ks[1] * v[d - 1];
          acc += ks[2] * vh[d - 1];
          acc += ks[3] * vl[d];
          acc += ks[4] * v[d];
          acc += ks[5] * vh[d];
          acc += ks[6] * vl[d + 1];
          acc += ks[7] * v[d + 1];
          acc += ks[8] * vh[d + 1];
        } else {
          acc = ktb[pl[d - 1] * kMS + 0] * vl[d - 1];
          acc += ktb[pr[d - 1] * kMS + 1] * v[d - 1];
          acc += ktb[ph[d - 1] * kMS + 2] * vh[d - 1];
          acc += ktb[pl[d] * kMS + 3] * vl[d];
          acc += ktb[pr[d] * kMS + 4] * v[d];
          acc += ktb[ph[d] * kMS + 5] * vh[d];
          acc += ktb[pl[d + 1] * kMS + 6] * vl[d + 1];
          acc += ktb[pr[d + 1] * kMS + 7] * v[d + 1];
          acc += ktb[ph[d + 1] * kMS + 8] * vh[d + 1];
        }
        acc = keep(acc);
        const int y = G.r0 + 2 * II0 + d;
        const bool in = cin && y >= 1 && y <= H - 2;
        r[d] = in ? fr[d] - acc : T(0);
        rl[d] = shr1z(r[d]);
        rh[d] = shl1z(r[d]);
      }
      // (2) restriction of coarse rows II0 + i: residual rows 2i+1 .. 2i+3 of the window
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        if (II0 + i >= II1) break;
        T acc = T(0);
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          const int d = 2 * i + 1 + ky;
          if constexpr (!MULTI) {
            if (ky == 0) acc = rs[0] * rl[d];
            else acc += rs[ky * 3 + 0] * rl[d];
            acc += rs[ky * 3 + 1] * r[d];
            acc += rs[ky * 3 + 2] * rh[d];
          } else {
            if (ky == 0) acc = xtb[pl[d] * kMS + 0] * rl[d];
            else acc += xtb[pl[d] * kMS + ky * 3 + 0] * rl[d];
            acc += xtb[pr[d] * kMS + ky * 3 + 1] * r[d];
            acc += xtb[ph[d] * kMS + ky * 3 + 2] * rh[d];
          }
        }
        acc = keep(acc);
        const int II = II0 + i, I = C.r0 + II;
        if (outl) {
          T o = T(0);
          if (I >= 1 && I <= Hc - 2 && jin) {
            o = a.w * acc;
            if (I >= os_r[j + 1] && I < oe_r[j + 1] && jown) go[(long long)(I + 1) * ldc + OFF + J] = o;
          }
          fc[II * C.nc + JJ] = o;
        }
      }
    };
    const int per = (C.nr + NW - 1) / NW;
    const int II0 = wv * per, II1 = min(C.nr, II0 + per);
    for (int s0 = II0; s0 < II1; s0 += 2) {  // wave-uniform chunks of <= 2 coarse rows
      const int s1 = min(s0 + 2, II1);
      if (s1 - s0 == 2) {
        if (j == 0) rows(std::integral_constant<int, 2>{}, std::true_type{}, s0, s1);
        else rows(std::integral_constant<int, 2>{}, std::false_type{}, s0, s1);
      } else {
        if (j == 0) rows(std::integral_constant<int, 1>{}, std::true_type{}, s0, s1);
        else rows(std::integral_constant<int, 1>{}, std::false_type{}, s0, s1);
      }
    }
    if (j + 1 < k) FEA_MID_SYNC(1 + j);
  }
  FEA_MID_MARK(2 * blockIdx.x + 1);
}

// ---------------------------------------------------------------------------------------------
// up: u_{a+k}, f_a .. f_{a+k-1} -> u_a
// ---------------------------------------------------------------------------------------------
// The up pass's per-level geometry (regions and LDS carve offsets), kept in LDS: every level reloads its
// own after the barrier in front of it, so none of it is live across the levels (held in registers through
// the unrolled level loop it pushed the two-material kernels past 128 VGPRs: scratch spills reloaded at
// every barrier).
struct MidUpGeo {
  Reg u[kMidMaxK + 1];
  int fx[kMidMaxK], uo[kMidMaxK + 1], po[kMidMaxK + 1], ko;
};

template <typename T, bool MULTI, int K>
__global__ __launch_bounds__(kMidThreads) void k_mg_mid_up(MidArgs<T> a) {
  __shared__ __attribute__((aligned(16))) char smem[kMidLdsBytes];
  __shared__ MidUpGeo geo;
  FEA_MID_MARK(2 * blockIdx.x);
  constexpr int OFF = 128 / (int)sizeof(T) - 1;
  constexpr int k = K;
  const int tiles = a.ntr * a.ntc;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int b = bid / tiles, t = bid - b * tiles, ti = t / a.ntc, tj = t - ti * a.ntc;
  // u regions: level 0 = the tile of u_a; level j+1 = the coarse nodes x_j's prolongation reads
  Reg u[kMidMaxK + 1];
  {
    const int r0 = 1 + ti * a.TR, c0 = 1 + tj * a.TC;
    u[0] = Reg{r0, c0, min(r0 + a.TR, a.H[0] - 1) - r0, min(c0 + a.TC, a.W[0] - 1) - c0};
#pragma unroll
    for (int j = 0; j < k; ++j) u[j + 1] = mid_coarse_of(u[j]);
  }
  auto xreg = [&](int j) { return Reg{u[j].r0 - 1, u[j].c0 - 1, u[j].nr + 2, u[j].nc + 2}; };
  // LDS carve: Fx[j] (f on x region j), U[j+1], X scratch, tables, patterns
  T* Fx[kMidMaxK];
  T* U[kMidMaxK + 1];
  T* p = reinterpret_cast<T*>(smem);
  int xmax = 0;
#pragma unroll
  for (int j = 0; j < k; ++j) {
    const Reg x = xreg(j);
    Fx[j] = p;
    p += x.nr * x.nc;
    xmax = max(xmax, x.nr * x.nc);
    U[j + 1] = p;
    p += u[j + 1].nr * u[j + 1].nc;
  }
  T* X = p;
  p += xmax;
  T* ktb0 = p;
  T* xtb0 = ktb0 + FEA_MAX_PATTERNS * kMS;
  uint8_t* P[kMidMaxK + 1];
  uint8_t* q = reinterpret_cast<uint8_t*>(xtb0 + FEA_MAX_PATTERNS * kMS);
#pragma unroll
  for (int j = 0; j <= k; ++j) {
    P[j] = q;
    if constexpr (MULTI) {
      const Reg x = j < k ? xreg(j) : u[k];
      q += (x.nr * x.nc + 15) / 16 * 16;
    }
  }
  const TabLoad<T> tl = tables_issue<T>(a.ktab, a.omd, a.xtab, a.ntab, a.nx);
  // stage everything up front (one round of memory latency for the whole launch)
  {
    StageJob<T> jf[k + 1];
#pragma unroll
    for (int j = 0; j < k; ++j) jf[j] = {a.f[j] + (long long)b * a.bs[j], Fx[j], xreg(j), a.H[j], a.W[j], a.ld[j], OFF};
    jf[k] = {a.e + (long long)b * a.bs[k], U[k], u[k], a.H[k], a.W[k], a.ld[k], OFF};
    if constexpr (MULTI) {
      StageJob<uint8_t> jp[k + 1];
#pragma unroll
      for (int j = 0; j <= k; ++j) jp[j] = {a.pid[j], P[j], j < k ? xreg(j) : u[k], a.H[j], a.W[j], a.ld[j], OFF};
      stage_batch<uint8_t, k + 1>(jp);
    }
    FEA_MID_WAVE_MARK(0);
    stage_batch<T, k + 1>(jf);
    FEA_MID_WAVE_MARK(1);
  }
  tables_commit<T>(tl, ktb0, xtb0, a.ntab, a.nx);
  if (MULTI && threadIdx.x == 0) {
#pragma unroll
    for (int j = 0; j <= k; ++j) {
      geo.u[j] = u[j];
      if (j < k) geo.fx[j] = (int)(Fx[j] - reinterpret_cast<T*>(smem));
      if (j > 0) geo.uo[j] = (int)(U[j] - reinterpret_cast<T*>(smem));
      geo.po[j] = (int)(P[j] - reinterpret_cast<uint8_t*>(smem));
    }
    geo.ko = (int)(ktb0 - reinterpret_cast<T*>(smem));
  }
  FEA_MID_SYNC(0);
  T ks[9], ps[9], om = T(0);
  if constexpr (!MULTI) {
#pragma unroll
    for (int d = 0; d < 9; ++d) {
      ks[d] = ktb0[d];
      ps[d] = xtb0[d];
    }
    om = ktb0[9];
  }

  // Per level: wave w owns a contiguous block of u-region rows; for each chunk of <= 4 of them it forms
  // the corrected iterate x = v + w1 P(e) on the chunk's rows plus one halo row on each side (every
  // LDS load of the chunk issued up front), then the sweep u = x + omd (f - K x) — one barrier per
  // level (the halo rows of x are recomputed by both neighbouring waves, bitwise the same values).
  // Per-node expressions and their order are those of k_mg_prolong (ZU mode).
  constexpr int NW = kMidThreads / 64;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int j = k - 1; j >= 0; --j) {
    // this level's geometry, from LDS (see MidUpGeo)
    // (LDS loads are not known to be uniform: readfirstlane puts the values back into scalar registers)
    auto rfl = [](int v) { return __builtin_amdgcn_readfirstlane(v); };
    auto greg = [&](int i) { return Reg{rfl(geo.u[i].r0), rfl(geo.u[i].c0), rfl(geo.u[i].nr), rfl(geo.u[i].nc)}; };
    // (single pattern: few enough registers to keep it all live, which is faster)
    T* const sb = reinterpret_cast<T*>(smem);
    const uint8_t* const sp = reinterpret_cast<const uint8_t*>(smem);
    const Reg U0 = MULTI ? greg(j) : u[j], C = MULTI ? greg(j + 1) : u[j + 1];
    const Reg x = Reg{U0.r0 - 1, U0.c0 - 1, U0.nr + 2, U0.nc + 2};
    const int H = a.H[j], W = a.W[j];
    const T* f = MULTI ? sb + rfl(geo.fx[j]) : Fx[j];
    const T* e = MULTI ? sb + rfl(geo.uo[j + 1]) : U[j + 1];
    const uint8_t* pj = MULTI ? sp + rfl(geo.po[j]) : P[j];
    const uint8_t* pc = MULTI ? sp + rfl(geo.po[j + 1]) : P[j + 1];
    const T* ktb = MULTI ? sb + rfl(geo.ko) : ktb0;
    const T* xtb = ktb + FEA_MAX_PATTERNS * kMS;
    // the coarse pattern map region: x region of level j+1 (j+1 < k) or its u region (j+1 == k)
    const Reg PC = (j + 1 < k) ? Reg{C.r0 - 1, C.c0 - 1, C.nr + 2, C.nc + 2} : C;
    // row-wave form (regions <= 64 columns): lane = column x.c0 + lane
    const int c = x.c0 + lane;
    const bool lv = lane < x.nc;
    const bool cing = lv && c >= 0 && c < W;
    const bool cin = lv && c >= 1 && c <= W - 2;
    // coarse columns of the prolongation: odd c reads (c-1)/2 (kx = 2) and (c+1)/2 (kx = 0), even c
    // reads c/2 (kx = 1) = the right one; both loads are issued (clamped), the parity selects
    const int cL = (c - 1) >> 1, cR = cL + 1;
    const int iL = min(max(cL - C.c0, 0), C.nc - 1), iR = min(max(cR - C.c0, 0), C.nc - 1);
    const int qL = min(max(cL - PC.c0, 0), PC.nc - 1), qR = min(max(cR - PC.c0, 0), PC.nc - 1);
    const bool codd = (c & 1) != 0;
    T* un = j > 0 ? (MULTI ? sb + rfl(geo.uo[j]) : U[j]) : nullptr;
    T* go = j == 0 ? a.out + (long long)b * a.bs[0] : nullptr;
    const bool lo = lane >= 1 && lane <= U0.nc;  // u-region column c = U0.c0 + lane - 1
    auto rows = [&](auto par_c, auto per_c, int yy0, int yy1) {
      constexpr int PAR = decltype(par_c)::value;  // parity of the first x row's grid row
      constexpr int PER = decltype(per_c)::value;
      constexpr int R = PER + 2;                   // x-region rows yy0 .. yy0 + R - 1
      constexpr int NC = (PAR + R) / 2 + 1;        // coarse rows Ib .. Ib + NC - 1 they read
      const int yf = x.r0 + yy0, Ib = yf >> 1;     // yf = 2 Ib + PAR
      T fr[R], eL[NC], eR[NC];
      int pr[R], pL[NC], pR[NC];
#pragma unroll
      for (int d = 0; d < R; ++d) {
        const int i = min(yy0 + d, x.nr - 1) * x.nc + lane;
        fr[d] = f[i];
        pr[d] = 0;
        if constexpr (MULTI) {
          const int pv = pj[min(yy0 + d, x.nr - 1) * x.nc + min(lane, x.nc - 1)];
          pr[d] = lv ? pv : 0;
        }
      }
#pragma unroll
      for (int q = 0; q < NC; ++q) {
        const int ci = min(max(Ib + q - C.r0, 0), C.nr - 1);
        eL[q] = e[ci * C.nc + iL];
        eR[q] = e[ci * C.nc + iR];
        pL[q] = pR[q] = 0;
        if constexpr (MULTI) {
          const int pi = min(max(Ib + q - PC.r0, 0), PC.nr - 1);
          pL[q] = pc[pi * PC.nc + qL];
          pR[q] = pc[pi * PC.nc + qR];
        }
      }
      // (1) x = v + w1 P(e) (k_mg_prolong: correct_even / correct_odd, crow_term)
      auto term = [&](int q, int ky) -> T {
        T wl, wm, wr;
        if constexpr (MULTI) {
          wl = xtb[pL[q] * kMS + ky * 3 + 2];
          wr = xtb[pR[q] * kMS + ky * 3 + 0];
          wm = xtb[pR[q] * kMS + ky * 3 + 1];
        } else {
          wl = ps[ky * 3 + 2];
          wr = ps[ky * 3 + 0];
          wm = ps[ky * 3 + 1];
        }
        T tt;
        if (codd) {
          tt = wl * eL[q];
          tt += wr * eR[q];
        } else {
          tt = wm * eR[q];
        }
        return tt;
      };
      T xv[R], xl[R], xh[R];
      int ql_[R], qh_[R];
#pragma unroll
      for (int d = 0; d < R; ++d) {
        const int y = yf + d;
        T v = T(0);
        if (cin && y >= 1 && y <= H - 2) {
          if constexpr (MULTI) v = ktb[pr[d] * kMS + 9] * fr[d];
          else v = om * fr[d];
        }
        if (((PAR + d) & 1) == 0) {
          v += a.w * term((PAR + d) >> 1, 1);
        } else {
          const T tt = term((PAR + d - 1) >> 1, 2) + term((PAR + d + 1) >> 1, 0);
          v += a.w * tt;
        }
        v = keep(v);
        xv[d] = (cing && y >= 0 && y < H) ? v : T(0);
        xl[d] = shr1z(xv[d]);
        xh[d] = shl1z(xv[d]);
        ql_[d] = qh_[d] = 0;
        if constexpr (MULTI) {
          ql_[d] = shr1z(pr[d]);
          qh_[d] = shl1z(pr[d]);
        }
      }
      // (2) u = x + omd (f - K x) on the u rows (interior), 0 on boundary nodes
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int yy = yy0 + i;
        if (yy >= yy1) break;
        T acc;
        if constexpr (!MULTI) {
          acc = ks[0] * xl[i];
          acc += ks[1] * xv[i];
          acc += ks[2] * xh[i];
          acc += ks[3] * xl[i + 1];
          acc += ks[4] * xv[i + 1];
          acc += ks[5] * xh[i + 1];
          acc += ks[6] * xl[i + 2];
          acc += ks[7] * xv[i + 2];
          acc += ks[8] * xh[i + 2];
        } else {
          acc = ktb[ql_[i] * kMS + 0] * xl[i];
          acc += ktb[pr[i] * kMS + 1] * xv[i];
          acc += ktb[qh_[i] * kMS + 2] * xh[i];
          acc += ktb[ql_[i + 1] * kMS + 3] * xl[i + 1];
          acc += ktb[pr[i + 1] * kMS + 4] * xv[i + 1];
          acc += ktb[qh_[i + 1] * kMS + 5] * xh[i + 1];
          acc += ktb[ql_[i + 2] * kMS + 6] * xl[i + 2];
          acc += ktb[pr[i + 2] * kMS + 7] * xv[i + 2];
          acc += ktb[qh_[i + 2] * kMS + 8] * xh[i + 2];
        }
        const int y = U0.r0 + yy;
        T om_ = om;
        if constexpr (MULTI) om_ = ktb[pr[i + 1] * kMS + 9];
        const T ov = keep(om_ * (fr[i + 1] - acc) + xv[i + 1]);
        if (lo) {
          T o = T(0);
          if (cin && y >= 1 && y <= H - 2) {
            o = ov;
            if (go) go[(long long)(y + 1) * a.ld[0] + OFF + c] = o;
          }
          if (un) un[yy * U0.nc + lane - 1] = o;
        }
      }
    };
    auto chunk = [&](auto per_c, int s0, int s1) {
      if ((x.r0 + s0) & 1) rows(std::integral_constant<int, 1>{}, per_c, s0, s1);
      else rows(std::integral_constant<int, 0>{}, per_c, s0, s1);
    };
    const int per = (U0.nr + NW - 1) / NW;
    const int Y0 = wv * per, Y1 = min(U0.nr, Y0 + per);
    constexpr int CH = MULTI ? 2 : 4;  // (two materials: the pattern windows need the registers)
    for (int s0 = Y0; s0 < Y1; s0 += CH) {  // wave-uniform chunks of <= CH u rows
      const int n = min(CH, Y1 - s0);
      if constexpr (CH == 4) {
        if (n == 4) chunk(std::integral_constant<int, 4>{}, s0, s0 + 4);
        else if (n == 3) chunk(std::integral_constant<int, 3>{}, s0, s0 + 3);
        else if (n == 2) chunk(std::integral_constant<int, 2>{}, s0, s0 + 2);
        else chunk(std::integral_constant<int, 1>{}, s0, s0 + 1);
      } else {
        if (n == 2) chunk(std::integral_constant<int, 2>{}, s0, s0 + 2);
        else chunk(std::integral_constant<int, 1>{}, s0, s0 + 1);
      }
    }
    if (j > 0) FEA_MID_SYNC(1 + (k - 1 - j));
  }
  FEA_MID_MARK(2 * blockIdx.x + 1);
}

}  // namespace fea

using namespace fea;

template <typename T>
static int mid_fill(MidArgs<T>& a, int k, int B, int H, int W, int TR, int TC) {
  if (k < 1 || k > kMidMaxK || B <= 0 || B > 65535 || TR < 1 || TC < 1) return FEA_EINVAL;
  a.k = k;
  for (int j = 0; j <= k; ++j) {
    if (H < 3 || W < 3 || (j < k && (!(H & 1) || !(W & 1)))) return FEA_EINVAL;
    a.H[j] = H;
    a.W[j] = W;
    if (fea_mg_layout(H, W, (int)sizeof(T), &a.ld[j], &a.bs[j]) != 0) return FEA_EINVAL;
    H = (H + 1) / 2;
    W = (W + 1) / 2;
  }
  a.TR = TR;
  a.TC = TC;
  return 0;
}

template <typename T, bool MULTI, typename Kern>
static void mid_launch(Kern k1, Kern k2, Kern k3, Kern k4, int k, dim3 grid, void* stream, const MidArgs<T>& a) {
  Kern kern = k == 1 ? k1 : k == 2 ? k2 : k == 3 ? k3 : k4;
  hipLaunchKernelGGL(kern, grid, dim3(kMidThreads), 0, (hipStream_t)stream, a);
}

#define FEA_MID_API(SUF, T)                                                                                      \
  extern "C" int fea_mg_mid_down_##SUF(const T* const* f, const uint8_t* const* pid, int k, int B, int H, int W, \
                                       const T* ktab, const T* omd, int ntab, const T* rtab, int nrtab, T w0,    \
                                       int TR, int TC, void* stream) {                                          \
    MidArgs<T> a = {};                                                                                           \
    if (!f || !ktab || !omd || !rtab || ntab < 1 || ntab > FEA_MAX_PATTERNS) return FEA_EINVAL;                \
    const bool multi = ntab > 1;                                                                                 \
    if ((multi && (!pid || nrtab != ntab)) || (!multi && nrtab != 1)) return FEA_EINVAL;                        \
    if (mid_fill<T>(a, k, B, H, W, TR, TC)) return FEA_EINVAL;                                                   \
    if (mid_down_lds(k, TR, TC, (int)sizeof(T), multi) > kMidLdsBytes) return FEA_EINVAL;                       \
    for (int j = 0; j <= k; ++j) {                                                                               \
      if (!f[j] || (multi && j < k && !pid[j])) return FEA_EINVAL;                                              \
      a.f[j] = f[j];                                                                                             \
      a.fo[j] = const_cast<T*>(f[j]);                                                                            \
      a.pid[j] = multi && j < k ? pid[j] : nullptr;                                                              \
    }                                                                                                            \
    a.ktab = ktab; a.omd = omd; a.xtab = rtab; a.w = w0; a.ntab = ntab; a.nx = nrtab;                           \
    a.ntr = (a.H[k] - 2 + TR - 1) / TR;                                                                          \
    a.ntc = (a.W[k] - 2 + TC - 1) / TC;                                                                          \
    const dim3 grid(B * a.ntr * a.ntc);                                                                          \
    if (multi) mid_launch<T, true>(k_mg_mid_down<T, true, 1>, k_mg_mid_down<T, true, 2>,                       \
                                   k_mg_mid_down<T, true, 3>, k_mg_mid_down<T, true, 4>, k, grid, stream, a);     \
    else mid_launch<T, false>(k_mg_mid_down<T, false, 1>, k_mg_mid_down<T, false, 2>,                             \
                              k_mg_mid_down<T, false, 3>, k_mg_mid_down<T, false, 4>, k, grid, stream, a);        \
    FEA_LAUNCH_CHECK();                                                                                          \
  }                                                                                                              \
  extern "C" int fea_mg_mid_down_gathered_##SUF(const T* const* f, const uint8_t* const* pid, int k, int B, int H, \
                                                int W, const T* ktab, const T* omd, int ntab, const T* rtab,      \
                                                int nrtab, T w0, int TR, int TC, const T* gsrc, int Pr, int Pc,    \
                                                int gcr, int gcc, void* stream) {                                 \
    MidArgs<T> a = {};                                                                                           \
    if (!f || !ktab || !omd || !rtab || !gsrc || ntab < 1 || ntab > FEA_MAX_PATTERNS) return FEA_EINVAL;       \
    if (Pr < 1 || Pc < 1 || gcr < 1 || gcc < 1 || H - 1 != Pr * gcr || W - 1 != Pc * gcc) return FEA_EINVAL;    \
    const bool multi = ntab > 1;                                                                                 \
    if ((multi && (!pid || nrtab != ntab)) || (!multi && nrtab != 1)) return FEA_EINVAL;                        \
    if (mid_fill<T>(a, k, B, H, W, TR, TC)) return FEA_EINVAL;                                                   \
    if (mid_down_lds(k, TR, TC, (int)sizeof(T), multi) > kMidLdsBytes) return FEA_EINVAL;                       \
    for (int j = 0; j <= k; ++j) {                                                                               \
      if (!f[j] || (multi && j < k && !pid[j])) return FEA_EINVAL;                                              \
      a.f[j] = f[j];                                                                                             \
      a.fo[j] = const_cast<T*>(f[j]);                                                                            \
      a.pid[j] = multi && j < k ? pid[j] : nullptr;                                                              \
    }                                                                                                            \
    a.ktab = ktab; a.omd = omd; a.xtab = rtab; a.w = w0; a.ntab = ntab; a.nx = nrtab;                           \
    a.gsrc = gsrc; a.gB = B; a.gPc = Pc; a.gcr = gcr; a.gcc = gcc;                                               \
    a.ntr = (a.H[k] - 2 + TR - 1) / TR;                                                                          \
    a.ntc = (a.W[k] - 2 + TC - 1) / TC;                                                                          \
    const dim3 grid(B * a.ntr * a.ntc);                                                                          \
    if (multi) mid_launch<T, true>(k_mg_mid_down<T, true, 1, true>, k_mg_mid_down<T, true, 2, true>,           \
                                   k_mg_mid_down<T, true, 3, true>, k_mg_mid_down<T, true, 4, true>, k, grid,     \
                                   stream, a);                                                                    \
    else mid_launch<T, false>(k_mg_mid_down<T, false, 1, true>, k_mg_mid_down<T, false, 2, true>,                 \
                              k_mg_mid_down<T, false, 3, true>, k_mg_mid_down<T, false, 4, true>, k, grid,        \
                              stream, a);                                                                         \
    FEA_LAUNCH_CHECK();                                                                                          \
  }                                                                                                              \
  extern "C" int fea_mg_mid_up_##SUF(const T* const* f, const T* e, T* out, const uint8_t* const* pid, int k,   \
                                     int B, int H, int W, const T* ktab, const T* omd, int ntab, const T* ptab,  \
                                     int nptab, T w1, int TR, int TC, void* stream) {                            \
    MidArgs<T> a = {};                                                                                           \
    if (!f || !e || !out || !ktab || !omd || !ptab || ntab < 1 || ntab > FEA_MAX_PATTERNS) return FEA_EINVAL;  \
    const bool multi = ntab > 1;                                                                                 \
    if ((multi && (!pid || nptab != ntab)) || (!multi && nptab != 1)) return FEA_EINVAL;                        \
    if (mid_fill<T>(a, k, B, H, W, TR, TC)) return FEA_EINVAL;                                                   \
    if (mid_up_lds(k, TR, TC, (int)sizeof(T), multi) > kMidLdsBytes) return FEA_EINVAL;                         \
    for (int j = 0; j <= k; ++j) {                                                                               \
      if ((j < k && (!f[j] || f[j] == out)) || (multi && !pid[j])) return FEA_EINVAL;                           \
      a.f[j] = j < k ? f[j] : nullptr;                                                                           \
      a.pid[j] = multi ? pid[j] : nullptr;                                                                       \
    }                                                                                                            \
    if (e == out) return FEA_EINVAL;                                                                             \
    a.e = e; a.out = out;                                                                                        \
    a.ktab = ktab; a.omd = omd; a.xtab = ptab; a.w = w1; a.ntab = ntab; a.nx = nptab;                           \
    a.ntr = (a.H[0] - 2 + TR - 1) / TR;                                                                          \
    a.ntc = (a.W[0] - 2 + TC - 1) / TC;                                                                          \
    const dim3 grid(B * a.ntr * a.ntc);                                                                          \
    if (multi) mid_launch<T, true>(k_mg_mid_up<T, true, 1>, k_mg_mid_up<T, true, 2>, k_mg_mid_up<T, true, 3>,     \
                                   k_mg_mid_up<T, true, 4>, k, grid, stream, a);                                  \
    else mid_launch<T, false>(k_mg_mid_up<T, false, 1>, k_mg_mid_up<T, false, 2>, k_mg_mid_up<T, false, 3>,      \
                              k_mg_mid_up<T, false, 4>, k, grid, stream, a);                                      \
    FEA_LAUNCH_CHECK();                                                                                          \
  }

FEA_MID_API(f32, float)
FEA_MID_API(f64, double)

#ifdef FEA_MID_TRACE
extern "C" int fea_mid_trace_read(long long* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_mid_trace), sizeof(long long) * 4096, 0, hipMemcpyDeviceToHost);
}
#endif

extern "C" long long fea_mg_mid_lds_bytes(int up, int k, int TR, int TC, int elem_size, int multi) {
  if (k < 1 || k > kMidMaxK || TR < 1 || TC < 1 || (elem_size != 4 && elem_size != 8)) return -1;
  const long long b = up ? mid_up_lds(k, TR, TC, elem_size, multi != 0) : mid_down_lds(k, TR, TC, elem_size, multi != 0);
  return b <= kMidLdsBytes ? b : -1;
}
