// hmid_ops.hip — two consecutive coarse levels of the learned-smoother (HJac) V-cycle in ONE launch each way.
//
// MultiGrid.Step with mode='hjac' (M-FEANet-mg_test.ipynb:27346-27372, Relax = HJacIterator.HRelax :147-155) runs,
// with the fused schedule (feanet_amd.schedule.hjac_schedule(fuse=True)), per coarse level l and V(1,1):
//   down: out_l = HRelax(0, f_l) stored; f_(l+1) = w0 R(f_l - K out_l)      (fea_mg_hsweep_restrict, zero guess)
//   up:   x = out_l + w1 P(e_(l+1)); u_l = HRelax(x, f_l)                    (fea_mg_prolong_hsweep)
// with HRelax(u, f): j = J(u, f); d_0 = j - u; d_k = (W_k * d_(k-1)) . g; result j + d_nl (interior).
// Between the fine levels and the LDS-resident HJac tail (hjac_tail.hip) sit levels of 129^2 .. 513^2 nodes whose
// streaming launches are bound by the per-wave chain of rows, ~10-14 us each (profiles/r05_configs/
// trace_hjac4097.txt) whatever their size.  Here two levels run per launch as independent TILES with recomputed
// halos (no grid-wide synchronisation), every stage an LDS pass of the whole workgroup:
//   k_hmid_down: a workgroup owns a T x T tile of f_(a+2); it stages the f_a region that tile depends on and runs
//     both levels' sweep, residual and restriction in LDS, writing the nodes of u_a, f_(a+1), u_(a+1), f_(a+2) it
//     owns (the up leg and the tail read them).
//   k_hmid_up: a workgroup owns a T x T tile of the new u_a; it stages u_a, f_a, u_(a+1), f_(a+1) and e = u_(a+2)
//     on the regions the tile depends on, runs level a+1's prolongation + correction + sweep into LDS and then
//     level a's; only u_a goes to HBM (the new u_(a+1) has no other reader).
// Every node value is the same expression, in the same order, as in the streaming kernels (hnet_ops.hip MODE 2 /
// MODE 1; -ffp-contract=on), so the results are bitwise theirs (tests/test_gpu_hnet.py).
#include "fea_common.h"

namespace fea {

constexpr int kHMThreads = 1024;
constexpr int kHMLdsBytes = 160 * 1024 - 2048;
constexpr int kHMS = 10;          // table stride: 9 weights + omega/d
constexpr int kHMMaxLayers = 3;

#ifdef FEA_HMID_TRACE  // lab builds only (tools/lab/hmid_trace.py): s_memrealtime per workgroup and phase
__device__ long long g_hm_trace[4096];
#define FEA_HM_MARK(slot) \
  if (threadIdx.x == 0) g_hm_trace[slot] = (long long)__builtin_amdgcn_s_memrealtime()
#define FEA_HM_SYNC(ph)                                                                                         \
  do {                                                                                                          \
    __syncthreads();                                                                                            \
    if (blockIdx.x == 0 && threadIdx.x == 0) g_hm_trace[2048 + (ph)] = (long long)__builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define FEA_HM_MARK(slot)
#define FEA_HM_SYNC(ph) __syncthreads()
#endif

// A region of a level: rows [r0, r0+nr), columns [c0, c0+nc), row-major in LDS.
struct HMReg {
  int r0, c0, nr, nc;
};

// the fine nodes the restriction of coarse region c depends on: residual rows 2 r0 - 1 .. 2 (r0 + nr - 1) + 1,
// the swept iterate one node further, its stage chain (nl layers) nl more
__host__ __device__ inline HMReg hm_down_parent(const HMReg& c, int nl) {
  const int h = 2 + nl;
  return HMReg{2 * c.r0 - h, 2 * c.c0 - h, 2 * c.nr - 1 + 2 * h, 2 * c.nc - 1 + 2 * h};
}
__host__ __device__ inline HMReg hm_grow(const HMReg& g, int h) {
  return HMReg{g.r0 - h, g.c0 - h, g.nr + 2 * h, g.nc + 2 * h};
}
// the coarse nodes the prolongation onto the fine region x reads (rows floor(y/2) and floor(y/2) + 1)
__host__ __device__ inline HMReg hm_coarse_of(const HMReg& x) {
  const int r0 = x.r0 >> 1, r1 = ((x.r0 + x.nr - 1) >> 1) + 1;
  const int c0 = x.c0 >> 1, c1 = ((x.c0 + x.nc - 1) >> 1) + 1;
  return HMReg{r0, c0, r1 - r0 + 1, c1 - c0 + 1};
}
__host__ __device__ inline long long hm_n(const HMReg& g) { return (long long)g.nr * g.nc; }
__host__ __device__ inline long long hm_al16(long long b) { return (b + 15) / 16 * 16; }

__host__ __device__ inline long long hm_tables_bytes(int esz) {
  return hm_al16((2LL * FEA_MAX_PATTERNS * kHMS + kHMMaxLayers * 9) * esz);
}
// down: F_a, three scratch fields of level a's region, F_(a+1); pattern maps of both levels
__host__ __device__ inline long long hm_down_lds(int TT, int nl, int esz, bool multi) {
  const HMReg g2{1, 1, TT, TT};
  const HMReg g1 = hm_down_parent(g2, nl), g0 = hm_down_parent(g1, nl);
  long long b = hm_al16((4 * hm_n(g0) + hm_n(g1)) * esz) + hm_tables_bytes(esz);
  if (multi) b += hm_al16(hm_n(g0)) + hm_al16(hm_n(g1));
  return b;
}
struct HMUpGeo {
  HMReg t, xa, c1, x1, c2;
};
__host__ __device__ inline HMUpGeo hm_up_geo(int r0, int c0, int nr, int nc, int nl) {
  HMUpGeo q;
  q.t = HMReg{r0, c0, nr, nc};
  q.xa = hm_grow(q.t, nl + 1);
  q.c1 = hm_coarse_of(q.xa);
  q.x1 = hm_grow(q.c1, nl + 1);
  q.c2 = hm_coarse_of(q.x1);
  return q;
}
// up: u and f of level a's and level a+1's regions, three scratch fields (the larger region), the new u_(a+1) and
// e = u_(a+2) on the coarse regions; pattern maps of the three levels.  Region sizes below the tile depend on the
// tile's alignment: the worst over the residues of its origin mod 4.
__host__ __device__ inline long long hm_up_lds(int TT, int nl, int esz, bool multi) {
  long long worst = 0;
  for (int t = 0; t < 4; ++t) {
    const HMUpGeo q = hm_up_geo(1 + t * TT, 1 + t * TT, TT, TT, nl);
    const long long sa = hm_n(q.xa), s1 = hm_n(q.x1), sm = sa > s1 ? sa : s1;
    long long b = hm_al16((2 * sa + 2 * s1 + 3 * sm + hm_n(q.c1) + hm_n(q.c2)) * esz) + hm_tables_bytes(esz);
    if (multi) b += hm_al16(sa) + hm_al16(s1) + hm_al16(hm_n(q.c2));
    worst = worst > b ? worst : b;
  }
  return worst;
}

template <typename T>
struct HMArgs {
  const T* f[3];    // level a, a+1, a+2 (down: f_a in; up: f_a, f_(a+1))
  T* fo[3];         // down: f_(a+1), f_(a+2) out
  const T* u[2];    // up: the stored iterates u_a, u_(a+1)
  T* uo[2];         // down: u_a, u_(a+1) out
  const T* e;       // up: u_(a+2)
  T* out;           // up: the new u_a
  const uint8_t* pid[3];
  int H[3], W[3], ld[3];
  long long bs[3];
  const T* ktab;
  const T* omd;
  const T* xtab;    // down: R kernels, up: P kernels
  const T* hw;
  T w;              // down: w0, up: w1
  int ntab, nx, nl, TT, ntr, ntc;
};

__device__ __forceinline__ bool hm_inner(int y, int x, int H, int W) {
  return y >= 1 && y <= H - 2 && x >= 1 && x <= W - 2;
}
// i / w for the region's node indices (i < 2^13, w <= 128): (i + 0.5) / w lies at least 0.5 / w from an integer,
// far beyond the float rounding of the product, so the truncation is the exact quotient
__device__ __forceinline__ int hm_divw(int i, int w) { return (int)(((float)i + 0.5f) * __frcp_rn((float)w)); }

// every node of g shrunk by s on each side: fn(LDS index, grid row, grid column)
template <typename Fn>
__device__ __forceinline__ void hm_for(const HMReg& g, int s, Fn&& fn) {
  const int w = g.nc - 2 * s, n = w * (g.nr - 2 * s);
  for (int i = threadIdx.x; i < n; i += kHMThreads) {
    const int yy = hm_divw(i, w), xx = i - yy * w;
    const int y = yy + s, x = xx + s;
    fn(y * g.nc + x, g.r0 + y, g.c0 + x);
  }
}

// Staging: every load of a job list is issued (from clamped, always valid addresses) before the first LDS store,
// so a stage costs one memory round trip; nodes outside the grid are stored as 0.
template <typename E>
struct HMStage {
  const E* src;  // framed level of the sample: node (r, c) at src[(r + 1) * ld + c] (the frame offset folded in)
  E* dst;
  HMReg g;
  int H, W, ld;
};
template <typename E, int N>
__device__ __forceinline__ void hm_stage(const HMStage<E> (&J)[N]) {
  constexpr int M = 4;
  const int tid = threadIdx.x;
  for (int base = 0;; base += M * kHMThreads) {
    E v[N][M];
    bool more = false;
#pragma unroll
    for (int q = 0; q < N; ++q) {
      const int n = J[q].g.nr * J[q].g.nc;
#pragma unroll
      for (int m = 0; m < M; ++m) {
        const int i = min(base + m * kHMThreads + tid, n - 1);
        const int y = hm_divw(i, J[q].g.nc), x = i - y * J[q].g.nc;
        const int r = min(max(J[q].g.r0 + y, 0), J[q].H - 1), c = min(max(J[q].g.c0 + x, 0), J[q].W - 1);
        v[q][m] = J[q].src[(long long)(r + 1) * J[q].ld + c];
      }
      more |= base + M * kHMThreads < n;
    }
#pragma unroll
    for (int q = 0; q < N; ++q) {
      const int n = J[q].g.nr * J[q].g.nc;
#pragma unroll
      for (int m = 0; m < M; ++m) {
        const int i = base + m * kHMThreads + tid;
        if (i < n) {
          const int y = hm_divw(i, J[q].g.nc), x = i - y * J[q].g.nc;
          const int r = J[q].g.r0 + y, c = J[q].g.c0 + x;
          J[q].dst[i] = (r >= 0 && r < J[q].H && c >= 0 && c < J[q].W) ? v[q][m] : E(0);
        }
      }
    }
    if (!more) break;
  }
}

// weights: two materials from the LDS tables (by the tap node's pattern), one material from registers
template <typename T, bool MULTI>
struct HMW {
  const T* ktb;  // ntab x 10 (9 weights + omega/d)
  const T* xtb;  // R or P kernels, ntab x 10
  const T* hk;   // nl x 9 (LDS)
  T ks[9], xs[9], om;
  __device__ __forceinline__ T kw(const uint8_t* p, int i, int d) const {
    if constexpr (MULTI) return ktb[p[i] * kHMS + d];
    else return ks[d];
  }
  __device__ __forceinline__ T omk(const uint8_t* p, int i) const {
    if constexpr (MULTI) return ktb[p[i] * kHMS + 9];
    else return om;
  }
  __device__ __forceinline__ T xw(const uint8_t* p, int i, int d) const {
    if constexpr (MULTI) return xtb[p[i] * kHMS + d];
    else return xs[d];
  }
  // (K x)(i): taps in row-major order (rows i-w, i, i+w; columns left to right), the weight by the tap's pattern
  __device__ __forceinline__ T kx(const T* x, const uint8_t* p, int i, int w) const {
    const int n = i - w, s = i + w;
    T acc = kw(p, n - 1, 0) * x[n - 1];
    acc += kw(p, n, 1) * x[n];
    acc += kw(p, n + 1, 2) * x[n + 1];
    acc += kw(p, i - 1, 3) * x[i - 1];
    acc += kw(p, i, 4) * x[i];
    acc += kw(p, i + 1, 5) * x[i + 1];
    acc += kw(p, s - 1, 6) * x[s - 1];
    acc += kw(p, s, 7) * x[s];
    acc += kw(p, s + 1, 8) * x[s + 1];
    return acc;
  }
  // HNet layer l (cross-correlation, zero padding outside the interior: the fields hold 0 there)
  __device__ __forceinline__ T conv(const T* d, int l, int i, int w) const {
    const T* h = hk + l * 9;
    const int n = i - w, s = i + w;
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
};

template <typename T, bool MULTI>
__device__ __forceinline__ HMW<T, MULTI> hm_tables(const HMArgs<T>& a, T* ktb, T* xtb, T* hk) {
  const int tid = threadIdx.x;
  HMW<T, MULTI> w{ktb, xtb, hk, {}, {}, T(0)};
  if constexpr (MULTI) {
    for (int i = tid; i < a.ntab * kHMS; i += kHMThreads) {
      const int p = i / kHMS, d = i - p * kHMS;
      ktb[i] = d == 9 ? a.omd[p] : a.ktab[p * 9 + d];
      xtb[i] = d == 9 ? T(0) : a.xtab[p * 9 + d];
    }
  } else {
#pragma unroll
    for (int d = 0; d < 9; ++d) {
      w.ks[d] = a.ktab[d];
      w.xs[d] = a.xtab[d];
    }
    w.om = a.omd[0];
  }
  if (tid < a.nl * 9) hk[tid] = a.hw[tid];
  return w;
}

// ---------------------------------------------------------------------------------------------------------------
// down: f_a -> u_a, f_(a+1), u_(a+1), f_(a+2)
// ---------------------------------------------------------------------------------------------------------------
template <typename T, bool MULTI>
__global__ __launch_bounds__(kHMThreads) void k_hmid_down(HMArgs<T> a) {
  __shared__ __attribute__((aligned(16))) char smem[kHMLdsBytes];
  FEA_HM_MARK(2 * blockIdx.x);
  [[maybe_unused]] int ph = 0;
  constexpr int OFF = 128 / (int)sizeof(T) - 1;
  const int nl = a.nl;
  const int tiles = a.ntr * a.ntc;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int b = bid / tiles, t = bid - b * tiles, ti = t / a.ntc, tj = t - ti * a.ntc;
  // regions: level 2 = the tile of f_(a+2); level j = the nodes of level j the next level's region depends on.
  // Owned nodes per level [os, oe): the tile at level 2; a finer level owns the fine nodes 2I-1 .. 2I'-1 of its
  // coarse range (through the last interior row for the last tile)
  HMReg g[3];
  int os_r[3], os_c[3], oe_r[3], oe_c[3];
  {
    const int r0 = 1 + ti * a.TT, c0 = 1 + tj * a.TT;
    g[2] = HMReg{r0, c0, min(r0 + a.TT, a.H[2] - 1) - r0, min(c0 + a.TT, a.W[2] - 1) - c0};
    os_r[2] = g[2].r0;
    os_c[2] = g[2].c0;
    oe_r[2] = g[2].r0 + g[2].nr;
    oe_c[2] = g[2].c0 + g[2].nc;
#pragma unroll
    for (int j = 1; j >= 0; --j) {
      g[j] = hm_down_parent(g[j + 1], nl);
      os_r[j] = 2 * os_r[j + 1] - 1;
      os_c[j] = 2 * os_c[j + 1] - 1;
      oe_r[j] = oe_r[j + 1] == a.H[j + 1] - 1 ? a.H[j] - 1 : 2 * oe_r[j + 1] - 1;
      oe_c[j] = oe_c[j + 1] == a.W[j + 1] - 1 ? a.W[j] - 1 : 2 * oe_c[j + 1] - 1;
    }
  }
  // LDS carve: F0, JD, A, B (level a's region), F1, tables, pattern maps
  const int S0 = g[0].nr * g[0].nc, S1 = g[1].nr * g[1].nc;
  T* F0 = reinterpret_cast<T*>(smem);
  T* JD = F0 + S0;
  T* A = JD + S0;
  T* Bf = A + S0;
  T* F1 = Bf + S0;
  T* ktb = reinterpret_cast<T*>(smem + hm_al16((4LL * S0 + S1) * sizeof(T)));
  T* xtb = ktb + FEA_MAX_PATTERNS * kHMS;
  T* hk = xtb + FEA_MAX_PATTERNS * kHMS;
  uint8_t* P0 = reinterpret_cast<uint8_t*>(ktb) + hm_tables_bytes(sizeof(T));
  uint8_t* P1 = P0 + hm_al16(S0);
  {
    HMStage<T> jf[1] = {{a.f[0] + (long long)b * a.bs[0] + OFF, F0, g[0], a.H[0], a.W[0], a.ld[0]}};
    if constexpr (MULTI) {
      HMStage<uint8_t> jp[2] = {{a.pid[0] + OFF, P0, g[0], a.H[0], a.W[0], a.ld[0]},
                                {a.pid[1] + OFF, P1, g[1], a.H[1], a.W[1], a.ld[1]}};
      hm_stage<uint8_t, 2>(jp);
    }
    hm_stage<T, 1>(jf);
  }
  const HMW<T, MULTI> wt = hm_tables<T, MULTI>(a, ktb, xtb, hk);
  FEA_HM_SYNC(++ph);

#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const HMReg G = g[j], C = g[j + 1];
    const int H = a.H[j], W = a.W[j], Hc = a.H[j + 1], Wc = a.W[j + 1], w = G.nc;
    const T* F = j == 0 ? F0 : F1;
    const uint8_t* P = j == 0 ? P0 : P1;
    // j = J(0, f) = omd (f - K 0) + 0 and d_0 = j - 0 on the interior, 0 elsewhere: K 0 is +0 exactly (the
    // stencil's centre weight is positive), so j = omd f + 0 (the fused multiply-add of the streaming kernel)
    hm_for(G, 0, [&](int i, int y, int x) { JD[i] = hm_inner(y, x, H, W) ? wt.omk(P, i) * F[i] + T(0) : T(0); });
    FEA_HM_SYNC(++ph);
    // d_l = (W_(l-1) * d_(l-1)) . g (d_1 in A, d_2 in B, d_3 in A); the last layer forms the iterate j + d_nl on
    // the interior, 0 elsewhere (the zero guess's boundary values)
    const T* out = JD;
    for (int l = 1; l <= nl; ++l) {
      const T* src = l == 1 ? JD : ((l & 1) ? Bf : A);
      T* dst = (l & 1) ? A : Bf;
      const bool last = l == nl;
      hm_for(G, l, [&](int i, int y, int x) {
        const bool in = hm_inner(y, x, H, W);
        const T c = in ? wt.conv(src, l - 1, i, w) : T(0);
        dst[i] = last ? (in ? JD[i] + c : T(0)) : c;
      });
      out = dst;
      FEA_HM_SYNC(++ph);
    }
    // the level's iterate: the nodes this tile owns
    {
      T* uo = a.uo[j] + (long long)b * a.bs[j] + OFF;
      const int ld = a.ld[j];
      hm_for(G, nl, [&](int i, int y, int x) {
        if (hm_inner(y, x, H, W) && y >= os_r[j] && y < oe_r[j] && x >= os_c[j] && x < oe_c[j])
          uo[(long long)(y + 1) * ld + x] = out[i];
      });
    }
    // residual + restriction of every coarse node of C (k_mg_resid_restrict's expressions): the next level's f in
    // LDS (j = 0) and the owned nodes in HBM
    {
      T* fo = a.fo[j + 1] + (long long)b * a.bs[j + 1] + OFF;
      const int ldc = a.ld[j + 1];
      hm_for(C, 0, [&](int ic, int I, int J) {
        const bool inc = hm_inner(I, J, Hc, Wc);
        T fc = T(0);
        if (inc) {
          const int i0 = (2 * I - 1 - G.r0) * w + (2 * J - 1 - G.c0);  // fine node (2I-1, 2J-1)
          T r[9];
#pragma unroll
          for (int dy = 0; dy < 3; ++dy)
#pragma unroll
            for (int dx = 0; dx < 3; ++dx) {
              const int n = i0 + dy * w + dx;
              r[dy * 3 + dx] = F[n] - wt.kx(out, P, n, w);
            }
          T acc = wt.xw(P, i0, 0) * r[0];
          acc += wt.xw(P, i0 + 1, 1) * r[1];
          acc += wt.xw(P, i0 + 2, 2) * r[2];
          acc += wt.xw(P, i0 + w, 3) * r[3];
          acc += wt.xw(P, i0 + w + 1, 4) * r[4];
          acc += wt.xw(P, i0 + w + 2, 5) * r[5];
          acc += wt.xw(P, i0 + 2 * w, 6) * r[6];
          acc += wt.xw(P, i0 + 2 * w + 1, 7) * r[7];
          acc += wt.xw(P, i0 + 2 * w + 2, 8) * r[8];
          fc = a.w * acc;
          if (I >= os_r[j + 1] && I < oe_r[j + 1] && J >= os_c[j + 1] && J < oe_c[j + 1])
            fo[(long long)(I + 1) * ldc + J] = fc;
        }
        if (j == 0) F1[ic] = fc;
      });
    }
    if (j == 0) FEA_HM_SYNC(++ph);
  }
  FEA_HM_MARK(2 * blockIdx.x + 1);
}

// ---------------------------------------------------------------------------------------------------------------
// up: u_a, f_a, u_(a+1), f_(a+1), e = u_(a+2) -> the new u_a
// ---------------------------------------------------------------------------------------------------------------
template <typename T, bool MULTI>
__global__ __launch_bounds__(kHMThreads) void k_hmid_up(HMArgs<T> a) {
  __shared__ __attribute__((aligned(16))) char smem[kHMLdsBytes];
  FEA_HM_MARK(2 * blockIdx.x);
  [[maybe_unused]] int ph = 0;
  constexpr int OFF = 128 / (int)sizeof(T) - 1;
  const int nl = a.nl;
  const int tiles = a.ntr * a.ntc;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int b = bid / tiles, t = bid - b * tiles, ti = t / a.ntc, tj = t - ti * a.ntc;
  // regions: the tile of u_a, level a's iterate region (tile + nl + 1: the sweep's stencil and stage chain), the
  // coarse nodes its prolongation reads (where the new u_(a+1) is needed), level a+1's iterate region around
  // them, and the nodes of e its prolongation reads
  const int r0 = 1 + ti * a.TT, c0 = 1 + tj * a.TT;
  const HMUpGeo q = hm_up_geo(r0, c0, min(r0 + a.TT, a.H[0] - 1) - r0, min(c0 + a.TT, a.W[0] - 1) - c0, nl);
  const int Sa = (int)hm_n(q.xa), S1 = (int)hm_n(q.x1), Sm = max(Sa, S1);
  const int Sc1 = (int)hm_n(q.c1), Sc2 = (int)hm_n(q.c2);
  T* Ua = reinterpret_cast<T*>(smem);
  T* Fa = Ua + Sa;
  T* U1 = Fa + Sa;
  T* F1 = U1 + S1;
  T* JJ = F1 + S1;
  T* A = JJ + Sm;
  T* Bf = A + Sm;
  T* E1 = Bf + Sm;
  T* E2 = E1 + Sc1;
  T* ktb = reinterpret_cast<T*>(smem + hm_al16((2LL * Sa + 2LL * S1 + 3LL * Sm + Sc1 + Sc2) * sizeof(T)));
  T* xtb = ktb + FEA_MAX_PATTERNS * kHMS;
  T* hk = xtb + FEA_MAX_PATTERNS * kHMS;
  uint8_t* Pa = reinterpret_cast<uint8_t*>(ktb) + hm_tables_bytes(sizeof(T));
  uint8_t* P1 = Pa + hm_al16(Sa);
  uint8_t* P2 = P1 + hm_al16(S1);
  {
    HMStage<T> jf[5] = {{a.u[0] + (long long)b * a.bs[0] + OFF, Ua, q.xa, a.H[0], a.W[0], a.ld[0]},
                        {a.f[0] + (long long)b * a.bs[0] + OFF, Fa, q.xa, a.H[0], a.W[0], a.ld[0]},
                        {a.u[1] + (long long)b * a.bs[1] + OFF, U1, q.x1, a.H[1], a.W[1], a.ld[1]},
                        {a.f[1] + (long long)b * a.bs[1] + OFF, F1, q.x1, a.H[1], a.W[1], a.ld[1]},
                        {a.e + (long long)b * a.bs[2] + OFF, E2, q.c2, a.H[2], a.W[2], a.ld[2]}};
    if constexpr (MULTI) {
      HMStage<uint8_t> jp[3] = {{a.pid[0] + OFF, Pa, q.xa, a.H[0], a.W[0], a.ld[0]},
                                {a.pid[1] + OFF, P1, q.x1, a.H[1], a.W[1], a.ld[1]},
                                {a.pid[2] + OFF, P2, q.c2, a.H[2], a.W[2], a.ld[2]}};
      hm_stage<uint8_t, 3>(jp);
    }
    hm_stage<T, 5>(jf);
  }
  const HMW<T, MULTI> wt = hm_tables<T, MULTI>(a, ktb, xtb, hk);
  FEA_HM_SYNC(++ph);

  const T w1 = a.w;
#pragma unroll
  for (int j = 1; j >= 0; --j) {
    const HMReg G = j == 1 ? q.x1 : q.xa;    // the level's iterate region
    const HMReg GE = j == 1 ? q.c2 : q.c1;   // the coarse values its prolongation reads
    const HMReg GP = j == 1 ? q.c2 : q.x1;   // the region of the coarse pattern map that holds them
    const int H = a.H[j], W = a.W[j], w = G.nc;
    T* U = j == 1 ? U1 : Ua;
    const T* F = j == 1 ? F1 : Fa;
    const uint8_t* P = j == 1 ? P1 : Pa;
    const T* E = j == 1 ? E2 : E1;
    const uint8_t* PE = j == 1 ? P2 : P1;
    // coarse row ar's contribution at fine column x with row tap ky (crow_term of framed_ops.hip)
    auto crow = [&](int ar, int ky, int x) -> T {
      const int ie = (ar - GE.r0) * GE.nc - GE.c0, ip = (ar - GP.r0) * GP.nc - GP.c0;
      if (!(x & 1)) {  // even fine column: one coarse node, kx = 1
        const int c = x >> 1;
        return wt.xw(PE, ip + c, ky * 3 + 1) * E[ie + c];
      }
      const int c = x >> 1;  // odd: coarse nodes (x-1)/2 (kx = 2) and (x+1)/2 (kx = 0)
      T tt = wt.xw(PE, ip + c, ky * 3 + 2) * E[ie + c];
      tt += wt.xw(PE, ip + c + 1, ky * 3 + 0) * E[ie + c + 1];
      return tt;
    };
    // x = u + w1 P(e) on the interior (correct_even / correct_odd of k_mg_prolong), in place
    hm_for(G, 0, [&](int i, int y, int x) {
      if (hm_inner(y, x, H, W)) {
        if (!(y & 1)) {
          U[i] = U[i] + w1 * crow(y >> 1, 1, x);
        } else {
          const T tt = crow(y >> 1, 2, x) + crow((y >> 1) + 1, 0, x);
          U[i] = U[i] + w1 * tt;
        }
      }
    });
    FEA_HM_SYNC(++ph);
    // the level's result: into E1 (level a+1, on its coarse region; 0 off the interior, as the buffer holds there)
    // or HBM (level a, the tile)
    T* uo = a.out + (long long)b * a.bs[0] + OFF;
    const int ld0 = a.ld[0];
    auto emit = [&](int y, int x, T o) {
      if (j == 1) E1[(y - q.c1.r0) * q.c1.nc + (x - q.c1.c0)] = o;
      else if (hm_inner(y, x, H, W)) uo[(long long)(y + 1) * ld0 + x] = o;
    };
    // j = omd (f - K x) + x; d_0 = j - x (interior)
    hm_for(G, 1, [&](int i, int y, int x) {
      const T acc = wt.kx(U, P, i, w);
      const T jv = wt.omk(P, i) * (F[i] - acc) + U[i];
      const bool in = hm_inner(y, x, H, W);
      if (nl == 0) {
        emit(y, x, in ? jv : T(0));
      } else {
        JJ[i] = jv;
        A[i] = in ? jv - U[i] : T(0);
      }
    });
    FEA_HM_SYNC(++ph);
    // d_l (d_0 in A, d_1 in B, d_2 in A); the last layer: j + d_nl
    for (int l = 1; l <= nl; ++l) {
      const T* src = (l & 1) ? A : Bf;
      T* dst = (l & 1) ? Bf : A;
      const bool last = l == nl;
      hm_for(G, 1 + l, [&](int i, int y, int x) {
        const bool in = hm_inner(y, x, H, W);
        const T c = in ? wt.conv(src, l - 1, i, w) : T(0);
        if (!last) dst[i] = c;
        else emit(y, x, in ? JJ[i] + c : T(0));
      });
      FEA_HM_SYNC(++ph);
    }
  }
  FEA_HM_MARK(2 * blockIdx.x + 1);
}

}  // namespace fea

using namespace fea;

template <typename T>
static int hm_fill(HMArgs<T>& a, int B, int H, int W, int nl, int TT) {
  if (B <= 0 || B > 65535 || TT < 1 || nl < 0 || nl > kHMMaxLayers) return FEA_EINVAL;
  for (int j = 0; j < 3; ++j) {
    if (H < 3 || W < 3 || (j < 2 && (!(H & 1) || !(W & 1)))) return FEA_EINVAL;
    a.H[j] = H;
    a.W[j] = W;
    if (fea_mg_layout(H, W, (int)sizeof(T), &a.ld[j], &a.bs[j]) != 0) return FEA_EINVAL;
    H = (H + 1) / 2;
    W = (W + 1) / 2;
  }
  a.nl = nl;
  a.TT = TT;
  return 0;
}

#define FEA_HMID_API(SUF, T)                                                                                       \
  extern "C" int fea_mg_hmid_down_##SUF(const T* const* f, T* const* u, const uint8_t* const* pid, int B, int H,   \
                                        int W, const T* ktab, const T* omd, int ntab, const T* hw, int nlayers,    \
                                        const T* rtab, int nrtab, T w0, int TT, void* stream) {                    \
    HMArgs<T> a = {};                                                                                              \
    if (!f || !u || !ktab || !omd || !rtab || (!hw && nlayers > 0) || ntab < 1 || ntab > FEA_MAX_PATTERNS)        \
      return FEA_EINVAL;                                                                                           \
    const bool multi = ntab > 1;                                                                                   \
    if ((multi && (!pid || nrtab != ntab)) || (!multi && nrtab != 1)) return FEA_EINVAL;                          \
    if (hm_fill<T>(a, B, H, W, nlayers, TT)) return FEA_EINVAL;                                                    \
    if (hm_down_lds(TT, nlayers, (int)sizeof(T), multi) > kHMLdsBytes) return FEA_EINVAL;                          \
    for (int j = 0; j < 3; ++j) {                                                                                  \
      if (!f[j] || (j < 2 && (!u[j] || u[j] == f[j])) || (multi && j < 2 && !pid[j])) return FEA_EINVAL;         \
      a.f[j] = f[j];                                                                                               \
      a.fo[j] = const_cast<T*>(f[j]);                                                                              \
      a.pid[j] = multi && j < 2 ? pid[j] : nullptr;                                                                \
    }                                                                                                              \
    a.uo[0] = u[0];                                                                                                \
    a.uo[1] = u[1];                                                                                                \
    a.ktab = ktab; a.omd = omd; a.xtab = rtab; a.hw = hw; a.w = w0; a.ntab = ntab; a.nx = nrtab;                  \
    a.ntr = (a.H[2] - 2 + TT - 1) / TT;                                                                            \
    a.ntc = (a.W[2] - 2 + TT - 1) / TT;                                                                            \
    const dim3 grid(B * a.ntr * a.ntc);                                                                            \
    hipStream_t s_ = (hipStream_t)stream;                                                                          \
    if (multi) k_hmid_down<T, true><<<grid, kHMThreads, 0, s_>>>(a);                                               \
    else k_hmid_down<T, false><<<grid, kHMThreads, 0, s_>>>(a);                                                    \
    FEA_LAUNCH_CHECK();                                                                                            \
  }                                                                                                                \
  extern "C" int fea_mg_hmid_up_##SUF(const T* const* f, const T* const* u, const T* e, T* out,                    \
                                      const uint8_t* const* pid, int B, int H, int W, const T* ktab, const T* omd, \
                                      int ntab, const T* hw, int nlayers, const T* ptab, int nptab, T w1, int TT,  \
                                      void* stream) {                                                              \
    HMArgs<T> a = {};                                                                                              \
    if (!f || !u || !e || !out || !ktab || !omd || !ptab || (!hw && nlayers > 0) || ntab < 1 ||                    \
        ntab > FEA_MAX_PATTERNS)                                                                                   \
      return FEA_EINVAL;                                                                                           \
    const bool multi = ntab > 1;                                                                                   \
    if ((multi && (!pid || nptab != ntab)) || (!multi && nptab != 1)) return FEA_EINVAL;                          \
    if (hm_fill<T>(a, B, H, W, nlayers, TT)) return FEA_EINVAL;                                                    \
    if (hm_up_lds(TT, nlayers, (int)sizeof(T), multi) > kHMLdsBytes) return FEA_EINVAL;                            \
    for (int j = 0; j < 3; ++j)                                                                                    \
      if (multi && !pid[j]) return FEA_EINVAL;                                                                     \
    for (int j = 0; j < 2; ++j) {                                                                                  \
      if (!f[j] || !u[j] || (j == 0 && (out == f[j] || out == u[j]))) return FEA_EINVAL;                           \
      a.f[j] = f[j];                                                                                               \
      a.u[j] = u[j];                                                                                               \
    }                                                                                                              \
    if (out == e) return FEA_EINVAL;                                                                               \
    for (int j = 0; j < 3; ++j) a.pid[j] = multi ? pid[j] : nullptr;                                               \
    a.e = e; a.out = out;                                                                                          \
    a.ktab = ktab; a.omd = omd; a.xtab = ptab; a.hw = hw; a.w = w1; a.ntab = ntab; a.nx = nptab;                  \
    a.ntr = (a.H[0] - 2 + TT - 1) / TT;                                                                            \
    a.ntc = (a.W[0] - 2 + TT - 1) / TT;                                                                            \
    const dim3 grid(B * a.ntr * a.ntc);                                                                            \
    hipStream_t s_ = (hipStream_t)stream;                                                                          \
    if (multi) k_hmid_up<T, true><<<grid, kHMThreads, 0, s_>>>(a);                                                 \
    else k_hmid_up<T, false><<<grid, kHMThreads, 0, s_>>>(a);                                                      \
    FEA_LAUNCH_CHECK();                                                                                            \
  }

FEA_HMID_API(f32, float)
FEA_HMID_API(f64, double)

#ifdef FEA_HMID_TRACE
extern "C" int fea_hmid_trace_read(long long* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_hm_trace), sizeof(long long) * 4096, 0, hipMemcpyDeviceToHost);
}
#endif

extern "C" long long fea_mg_hmid_lds_bytes(int up, int TT, int nlayers, int elem_size, int multi) {
  if (TT < 1 || nlayers < 0 || nlayers > kHMMaxLayers || (elem_size != 4 && elem_size != 8)) return -1;
  const long long b = up ? hm_up_lds(TT, nlayers, elem_size, multi != 0) : hm_down_lds(TT, nlayers, elem_size, multi != 0);
  return b <= kHMLdsBytes ? b : -1;
}
