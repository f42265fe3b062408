// hnet_ops.hip — one sweep of the learned smoother of M-FEANet-mg_test.ipynb (HJacIterator.HRelax,
// :147-155, HNet.forward :104-106) fused into one pass over a framed level:
//
//   j   = J(u, f)                         (weighted Jacobi, jacobi.py:39-47)
//   d_0 = j - u                           (zero on the boundary: u holds the Dirichlet values)
//   d_k = (W_k * d_{k-1}) . g             k = 1..nl, 3x3 cross-correlation, zero padding, g = interior
//   out = j + d_nl                        (interior; the boundary keeps u)
//
// SURVEY §8f row 1 ("fuse Jacobi with three masked 3x3 convs").  Round 2 staged an LDS tile of 16 rows plus
// a 4-node halo per workgroup (0.12 of the HBM peak at 4097^2 fp64, 15-24 us per launch on small levels: one
// workgroup per tile, every stage an LDS pass with a barrier); the streaming form below replaced it: register
// windows, DPP neighbours, every stage of a node in the same wave.  Work per node: 9 (K u) + 9 nl FMAs; HBM
// traffic ~ read u, read f, write out (+ the tasks' halo rows, served by the L2).  The arithmetic per node is
// the same expression at every node (fp-contract=on), so results do not depend on the geometry.
#include "fea_common.h"

#include <type_traits>
#include <utility>

namespace fea {

constexpr int kHMaxLayers = 3;    // HNet(nb_layers=3) (M-FEANet-mg_test.ipynb:222)
// input rows in flight per wave (1 or 2 steps ahead).  Same-lease A/B on MI355X: profiles/r04_hjac
#ifndef FEA_HSWEEP_PF
#define FEA_HSWEEP_PF 2
#endif
constexpr int kHPrefetch = FEA_HSWEEP_PF;
static_assert(kHPrefetch == 1 || kHPrefetch == 2, "hsweep prefetch of 1 or 2 rows");
// rows in flight of the sweep + restriction kernel with the 6-step loop body (the fine level's, 227 -> 231 VGPRs, two
// waves per SIMD either way): 3 -> 4097^2 fp64 111.4 -> 106.0 us (same lease, profiles/r05_hjac/prefetch3_ab.txt).
// The prolongation variant stays at 2 (3 spills it at its three-wave register cap).
#ifndef FEA_HSWEEP_PF6
#define FEA_HSWEEP_PF6 3
#endif
constexpr int kHTS = 10;          // LDS table stride (9 weights + omega/d)
// Weights: the stencil / HNet / transfer weights (up to 46 doubles: more than the SGPR file holds beside the
// kernel's addresses) are re-read with scalar loads at every row step, stage by stage, each stage's loads held
// behind an empty asm that "changes" their offset — hoisted out of the loop, or loaded all at the step's start,
// the compiler parks them (and with them the loop's other scalars) in VGPR lanes and pays a v_readlane per 32-bit
// half at every use (~95 VALU per step of the fp64 sweep+restriction, as many as its FMAs).

// steps per loop body: 6 (the 3-row windows' period x the 2-slot ring: the window rotations become register
// renamings) for the sweep+restriction of a stored iterate, 2 elsewhere (the longer body costs those kernels their
// third wave per SIMD: 4097^2 fp64 sweep+restriction 133.4 -> 116.8 us at 6, prolongation+sweep 103.5 -> 114.2 us;
// same-lease A/B, profiles/r04_hjac).  FEA_HS_UNROLL overrides both (lab builds).
// the fp64 single-pattern prolongation+sweep: 6 steps per body held to 168 VGPRs (three waves per SIMD)
template <typename T, bool MULTI, int MODE, bool RAW>
constexpr bool hs_mode1_wide() {
  return MODE == 1 && sizeof(T) == 8 && !MULTI && !RAW;
}
template <typename T, bool MULTI, int MODE, bool ZERO, bool RAW>
constexpr int hs_unroll_steps() {
#ifdef FEA_HS_UNROLL
  return FEA_HS_UNROLL;
#else
  return (MODE == 2 && !ZERO) || hs_mode1_wide<T, MULTI, MODE, RAW>() ? 6 : 2;
#endif
}

template <int N, typename Fn, int... I>
__device__ __forceinline__ void hs_unroll_(Fn&& fn, std::integer_sequence<int, I...>) {
  (fn(std::integral_constant<int, I>{}), ...);
}
template <int N, typename Fn>
__device__ __forceinline__ void hs_unroll(Fn&& fn) {
  hs_unroll_<N>(fn, std::make_integer_sequence<int, N>{});
}

// a read-only load through the constant address space: scalar (s_load) for a uniform address
template <typename T>
__device__ __forceinline__ T cload(const T* p, int i) {
  return ((const __attribute__((address_space(4))) T*)p)[i];
}

// ---------------------------------------------------------------------------------------------------------
// Streaming form (the one the API launches): a wave owns a strip of S columns and marches down its rows with
// register windows, all stages of the sweep skewed by one row each — u(y) loaded at step y; j and d_0 of row
// y-1; d_1 of row y-2; ...; d_NL and out of row y-1-NL.  Neighbour columns come from the adjacent lane by DPP;
// each stage's values are wrong on the outermost loaded column of the wave (no neighbour there), so a wave
// loads HLN halo lanes on each side (NL+1 columns) and its middle lanes own the strip: no halo loads, no LDS
// staging, no barriers.  Rows: the task recomputes NL+1 input rows above and below its own (the L2 serves
// the second read).  Same per-node expressions in the same order as the tile form above, so the results are
// bitwise those of the round-2 tile form (and independent of the strip and task geometry).
// ---------------------------------------------------------------------------------------------------------
template <typename T>
struct HVec;
template <>
struct HVec<double> { typedef double type __attribute__((ext_vector_type(2))); static constexpr int V = 2; };
template <>
struct HVec<float> { typedef float type __attribute__((ext_vector_type(4))); static constexpr int V = 4; };

template <typename T, int V>
struct HWin {  // a row's values on the lane's columns with the left and right neighbour columns
  T a[V + 2];
};

template <typename T, int V>
__device__ __forceinline__ HWin<T, V> hwin(const T (&x)[V]) {
  HWin<T, V> w;
#pragma unroll
  for (int k = 0; k < V; ++k) w.a[k + 1] = x[k];
  w.a[0] = shr1z(x[V - 1]);
  w.a[V + 1] = shl1z(x[0]);
  return w;
}

template <typename T, int V>
__device__ __forceinline__ void hload(const T* p, T (&x)[V]) {
  const typename HVec<T>::type v = *reinterpret_cast<const typename HVec<T>::type*>(p);
#pragma unroll
  for (int k = 0; k < V; ++k) x[k] = v[k];
}

template <typename T, int V>
__device__ __forceinline__ void hstore(T* p, const T (&x)[V], const bool (&m)[V]) {  // interior columns only
  bool all = true;
#pragma unroll
  for (int k = 0; k < V; ++k) all = all && m[k];
  if (all) {
    typename HVec<T>::type v;
#pragma unroll
    for (int k = 0; k < V; ++k) v[k] = x[k];
    *reinterpret_cast<typename HVec<T>::type*>(p) = v;
  } else {
#pragma unroll
    for (int k = 0; k < V; ++k)
      if (m[k]) p[k] = x[k];
  }
}

template <int V>
__device__ __forceinline__ void hpload(const uint8_t* p, int (&o)[V]) {
  if constexpr (V == 2) {
    const unsigned v = *reinterpret_cast<const unsigned short*>(p);
    o[0] = v & 0xff;
    o[1] = v >> 8;
  } else {
    const unsigned v = *reinterpret_cast<const unsigned*>(p);
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = (v >> (8 * k)) & 0xff;
  }
}

template <int V>
__device__ __forceinline__ HWin<int, V> hpwin(const int (&x)[V]) {  // pattern offsets (pattern * kHTS)
  HWin<int, V> w;
#pragma unroll
  for (int k = 0; k < V; ++k) w.a[k + 1] = x[k] * kHTS;
  w.a[0] = shr1z(x[V - 1]) * kHTS;
  w.a[V + 1] = shl1z(x[0]) * kHTS;
  return w;
}

template <typename T>
struct HSArgs {
  const T* u;
  const T* u_raw;
  const T* f;
  T* out;
  const uint8_t* pid;
  const T* ktab;
  const T* omd;
  const T* hw;
  int ntab;
  int H, W, ld;
  long long bs;
  int nstrips, ntr, rb;
  int zmask;  // 0 (the weight loads' offset the compiler cannot fold)
  // MODE 1 (prolongation + correction first): the sweep's iterate is x = u + w1 P(ec)
  const T* ec;
  const uint8_t* pidc;
  const T* ptab;
  T w1;
  // MODE 2 (residual + restriction after): fc = w0 R(f - K out)
  T* fc;
  const T* rtab;
  T w0;
  int Hc, Wc, ldc;
  long long bsc;
};

// MODE 0: the sweep alone (fea_mg_hsweep).
// MODE 1: prolongation + correction + sweep (fea_mg_prolong_hsweep): the loaded row u(y) becomes
//   x(y) = u(y) + w1 P(ec) on the interior (k_mg_prolong<SWEEP = false>'s expressions: correct_even / correct_odd)
//   as it enters the window, so the corrected iterate is never stored.
// MODE 2: sweep + residual + restriction (fea_mg_hsweep_restrict): out rows enter a 3-row window (boundary nodes
//   hold the iterate's values there, as in the buffer the separate kernels would read), the residual f - K out of
//   the middle row is formed one row later and three residual rows close a coarse row (k_mg_resid_restrict's
//   expressions); the wave loads two more halo columns per side and a task owns rb/2 coarse rows.
// geometry of a wave's task (shared by the kernel's interior test and the task body)
template <typename T, int NL, int MODE>
struct HSGeo {
  static constexpr int V = HVec<T>::V;
  static constexpr int HALO = NL + 1;  // columns / rows the stage chain reaches on each side
  // MODE 1: the corrected iterate is wrong on the leftmost loaded column too (its left coarse node comes from a
  // lane the wave does not have); MODE 2: the residual and the restriction reach one column each further
  static constexpr int HALOC = HALO + (MODE == 2 ? 2 : MODE == 1 ? 1 : 0);
  static constexpr int HLN = (HALOC + V - 1) / V;  // halo lanes per side
  static constexpr int S = (64 - 2 * HLN) * V;     // owned columns per strip
};

// out rows owned [r0, r1) and computed [rc0, rc1) of row task t (MODE 2: coarse rows [I0, I1))
template <int MODE>
__device__ __forceinline__ void hs_rows(int t, int rb, int H, int Hc, int& r0, int& r1, int& rc0, int& rc1, int& I0,
                                        int& I1) {
  I0 = I1 = 0;
  if constexpr (MODE == 2) {
    I0 = 1 + t * (rb / 2);
    I1 = min(I0 + rb / 2, Hc - 1);
    r0 = 2 * I0 - 1;
    r1 = I1 == Hc - 1 ? H - 1 : 2 * I1 - 1;
    rc0 = 2 * I0 - 2;
    rc1 = 2 * I1 + 1;
  } else {
    r0 = 1 + t * rb;
    r1 = min(r0 + rb, H - 1);
    rc0 = r0;
    rc1 = r1;
  }
}

// FEA_HS_INNER (lab): a wave whose task lies inside the grid with its whole reach (every row it streams, every column
// its lanes load, every coarse row it reads) runs the EDGE = false body: no boundary / edge selects (j - u, the masked
// HNet stages, the prolonged correction, the out row's stand-in values), no row or lane clamps, no partial stores,
// no loads of the iterate's boundary values.  Same per-node expressions: bitwise the general body (GPU hnet tests
// pass with it).  Measured slower, so off: the interior body has 19 % fewer VALU per step (800 vs 990 per 6-step
// loop of the fp64 sweep + restriction, same 231 VGPRs) yet the 4097^2 MG-HJac cycle ran 411 instead of 396 us
// (fea_mg_hsweep_restrict 123 vs 111 us, same lease, three alternations; profiles/r06_ab/hjac_inner_rejected.txt):
// the kernel then carries both bodies (7186 instead of 4290 instructions) and waves of both kinds share each CU's
// instruction cache.
#ifndef FEA_HS_INNER
#define FEA_HS_INNER 0
#endif

// One (row task, strip) of the streaming sweep (see k_mg_hsweep_strip).
template <typename T, bool MULTI, bool ZERO, bool RAW, int NL, int MODE, bool EDGE>
__device__ __forceinline__ void hsweep_task(const HSArgs<T>& g, int b, int t, int s, const T* tab, const T* tb2) {
  static_assert(MODE != 1 || !ZERO, "the prolongation variant corrects a stored iterate");
  using G = HSGeo<T, NL, MODE>;
  constexpr int V = HVec<T>::V;
  constexpr int Q = V / 2;
  constexpr int HALO = G::HALO;
  constexpr int HLN = G::HLN;
  constexpr int S = G::S;
  constexpr int OFF = 128 / (int)sizeof(T) - 1;
  const int lane = lane_id();
  const int H = g.H, W = g.W, ld = g.ld;
  const int cs = 1 + s * S - HLN * V;  // first loaded column
  const int cl = cs + V * lane;
  const int ll = EDGE ? min(lane, (W - 1 - cs) / V) : lane;  // lanes past the last column re-read a valid line
  const bool own = lane >= HLN && lane < 64 - HLN;
  int r0, r1, rc0, rc1, I0, I1;
  hs_rows<MODE>(t, g.rb, H, g.Hc, r0, r1, rc0, rc1, I0, I1);
  bool cin[V], cgr[V];
#pragma unroll
  for (int k = 0; k < V; ++k) {
    cin[k] = !EDGE || (cl + k >= 1 && cl + k <= W - 2);
    cgr[k] = !EDGE || (cl + k >= 0 && cl + k <= W - 1);
  }
  T ks[9], om = 0, hk[NL > 0 ? NL : 1][9], t2[9];
  if constexpr (!MULTI) {
#pragma unroll
    for (int d = 0; d < 9; ++d) {
      ks[d] = g.ktab[d];
      if constexpr (MODE != 0) t2[d] = (MODE == 1 ? g.ptab : g.rtab)[d];
    }
    om = g.omd[0];
  }
#pragma unroll
  for (int l = 0; l < NL; ++l)
#pragma unroll
    for (int d = 0; d < 9; ++d) hk[l][d] = g.hw[l * 9 + d];
  const long long boff = (long long)b * g.bs + OFF + cs;
  const T* __restrict__ ub = ZERO ? nullptr : g.u + boff;
  const T* __restrict__ rb_ = RAW ? g.u_raw + boff : nullptr;
  const T* __restrict__ fb = g.f + boff;
  T* __restrict__ ob = g.out + boff;
  const uint8_t* __restrict__ pb = MULTI ? g.pid + OFF + cs : nullptr;
  auto rowo = [&](int r) -> long long {
    if constexpr (EDGE) r = min(max(r, -1), H);
    return (long long)(r + 1) * ld + V * ll;
  };

  // MODE 1: the lane's coarse values (cl + 1) / 2 + q, q < Q, and the left lane's last one (DPP)
  const int jc = (cs + 1) / 2;
  const int llc = MODE == 1 ? (EDGE ? min(lane, (g.Wc - 1 - jc) / Q) : lane) : 0;
  const T* __restrict__ eb = MODE == 1 ? g.ec + (long long)b * g.bsc + OFF + jc + Q * llc : nullptr;
  const uint8_t* __restrict__ pcb = (MODE == 1 && MULTI) ? g.pidc + OFF + jc + Q * llc : nullptr;
  struct CR {  // coarse row: e[0] = column (cl-1)/2 (left lane), e[1..Q] = own; pattern offsets o[]
    T e[Q + 1];
    int o[Q + 1];
  };
  struct CRaw {
    T x[Q];
    int p[Q];
  };
  auto crow_ld = [&](int a) {
    CRaw r;
    if constexpr (EDGE) a = min(max(a, -1), g.Hc);
    const long long o = (long long)(a + 1) * g.ldc;
    if constexpr (MODE == 1) {
      if constexpr (Q == 1) {
        r.x[0] = eb[o];
      } else {
        typedef T v2 __attribute__((ext_vector_type(2)));  // Q == 2: fp32, 8-byte aligned (jc is odd, OFF odd)
        const v2 v = *reinterpret_cast<const v2*>(eb + o);
#pragma unroll
        for (int q = 0; q < Q; ++q) r.x[q] = v[q];
      }
      if constexpr (MULTI) {
#pragma unroll
        for (int q = 0; q < Q; ++q) r.p[q] = pcb[o + q];
      }
    }
    return r;
  };
  auto crow_fin = [&](const CRaw& r) {
    CR c{};
#pragma unroll
    for (int q = 0; q < Q; ++q) c.e[q + 1] = r.x[q];
    c.e[0] = shr1z(r.x[Q - 1]);
    if constexpr (MULTI) {
#pragma unroll
      for (int q = 0; q < Q; ++q) c.o[q + 1] = r.p[q] * kHTS;
      c.o[0] = shr1z(r.p[Q - 1]) * kHTS;
    }
    return c;
  };
  // crow_term (framed_ops.hip) at own column k: coarse row c's contribution with row tap ky
  auto cterm = [&](const CR& c, int k, int ky) -> T {
    if (k & 1) {  // even fine column (cl odd): one coarse node, kx = 1
      const int i = (k + 1) / 2;
      return (MULTI ? tb2[c.o[i] + ky * 3 + 1] : t2[ky * 3 + 1]) * c.e[i];
    }
    const int i = k / 2;  // odd fine column: coarse nodes i (kx = 2) and i + 1 (kx = 0)
    T tt = (MULTI ? tb2[c.o[i] + ky * 3 + 2] : t2[ky * 3 + 2]) * c.e[i];
    tt += (MULTI ? tb2[c.o[i + 1] + ky * 3 + 0] : t2[ky * 3 + 0]) * c.e[i + 1];
    return tt;
  };

  HWin<T, V> U0{}, U1{}, U2{};           // u rows y-2, y-1, y
  HWin<int, V> P0{}, P1{}, P2{};         // pattern offsets of the same rows
  HWin<T, V> D[NL > 0 ? NL : 1][3] = {}; // d_l windows: d_l of rows (y-1-l)-2 .. (y-1-l)
  T J[NL + 1][V];                        // j of rows y-1 .. y-1-NL
#pragma unroll
  for (int i = 0; i <= NL; ++i)
#pragma unroll
    for (int k = 0; k < V; ++k) J[i][k] = T(0);
  // MODE 2: out windows (rows yo-2 .. yo), their patterns, the residual rows 2I-1 (Ra), 2I (Rb) of a coarse row
  HWin<T, V> O0{}, O1{}, O2{};
  HWin<int, V> Q0{}, Q1{}, Q2{};
  T Ra[V + 1], Rb[V + 1];
  HWin<int, V> PRa{}, PRb{};
#pragma unroll
  for (int k = 0; k <= V; ++k) Ra[k] = Rb[k] = T(0);
  // the first step's row is even (one more fill step on odd starts: nothing it computes is stored), so every
  // unrolled step knows its row parity at compile time
  const int y0 = (rc0 - HALO) & ~1, y1 = rc1 - 1 + HALO;
  // input rows PF steps ahead, in a ring of PF slots indexed by the step's position (compile-time after the
  // unroll below): step y consumes u(y), pid(y), f(y-1) (RAW: u_raw(y-1); MODE 2: f and pid of its residual row
  // y-2-NL, the iterate of its out row y-1-NL) and refills the slot with the rows of step y+PF at once
  constexpr int PF = (MODE == 2 && hs_unroll_steps<T, MULTI, MODE, ZERO, RAW>() == 6) ? FEA_HSWEEP_PF6 : kHPrefetch;
  T ur[PF][V], fr_[PF][V], rw_[PF][V], frr[PF][V], uo[PF][V];
  int pr[PF][V], po[PF][V];
  // MODE 2 needs the iterate's values of an out row only where they stand in for the sweep (boundary nodes)
  auto need_uo = [&](int yy) { return EDGE && (!(yy >= 1 && yy <= H - 2) || !cin[0] || !cin[V - 1]); };
  auto fill = [&](int sl, int y) {
#pragma unroll
    for (int k = 0; k < V; ++k) ur[sl][k] = T(0);
    if constexpr (!ZERO) hload<T, V>(ub + rowo(y), ur[sl]);
    if constexpr (MULTI) hpload<V>(pb + rowo(y), pr[sl]);
    hload<T, V>(fb + rowo(y - 1), fr_[sl]);
    if constexpr (RAW) hload<T, V>(rb_ + rowo(y - 1), rw_[sl]);
    if constexpr (MODE == 2) {
      hload<T, V>(fb + rowo(y - 2 - NL), frr[sl]);
      if constexpr (MULTI) hpload<V>(pb + rowo(y - 1 - NL), po[sl]);
      if constexpr (!ZERO && EDGE) {
#pragma unroll
        for (int k = 0; k < V; ++k) uo[sl][k] = T(0);
        if (need_uo(y - 1 - NL)) hload<T, V>(ub + rowo(y - 1 - NL), uo[sl]);
      }
    }
  };
#pragma unroll
  for (int d = 0; d < PF; ++d) fill(d, y0 + d);
  // MODE 1: coarse rows floor(y/2) (Clo) and floor(y/2) + 1 (Chi) of the row entering the window; nC = the next
  CR Clo{}, Chi{};
  CRaw nC{};
  if constexpr (MODE == 1) {
    const int a0 = y0 >> 1;  // floor (y0 may be negative: rows outside the grid get no correction)
    Clo = crow_fin(crow_ld(a0));
    Chi = crow_fin(crow_ld(a0 + 1));
    nC = crow_ld(a0 + 2);
  }
  auto step = [&](int y, auto pos_c) __attribute__((always_inline)) {
    constexpr int SL = decltype(pos_c)::value % PF;
    constexpr bool ODD = decltype(pos_c)::value & 1;  // y odd (y0 is even)
    int z = __builtin_amdgcn_readfirstlane(y & g.zmask);  // 0 at run time, unknown to the compiler: the weight loads stay in the step
    // stage barrier: z is "changed" by an empty asm, so the weight loads after it cannot be hoisted above it —
    // each stage's weights are loaded just before the stage and die after it (one stage's worth of SGPRs live).
    // fp64 only: 4097^2 MG-HJac 486 -> 456 us (prolongation+sweep 101.6 -> 96.7 us, level 1 38.3 -> 30.5 us);
    // the fp32 129^2 cycle ran 1 % slower with them (profiles/r04_hjac/staged_weights_ab.txt)
    auto stage_ks = [&]() __attribute__((always_inline)) {
      if constexpr (sizeof(T) == 8) asm volatile("" : "+s"(z));  // (fp32: measured without the barriers)
      if constexpr (!MULTI) {
#pragma unroll
        for (int d = 0; d < 9; ++d) ks[d] = cload(g.ktab, z + d);
        om = cload(g.omd, z);
      }
    };
    auto stage_t2 = [&]() __attribute__((always_inline)) {
      if constexpr (sizeof(T) == 8) asm volatile("" : "+s"(z));  // (fp32: measured without the barriers)
      if constexpr (!MULTI && MODE != 0) {
#pragma unroll
        for (int d = 0; d < 9; ++d) t2[d] = cload(MODE == 1 ? g.ptab : g.rtab, z + d);
      }
    };
    auto stage_hk = [&](int l) __attribute__((always_inline)) {
      if constexpr (sizeof(T) == 8) asm volatile("" : "+s"(z));  // (fp32: measured without the barriers)
#pragma unroll
      for (int d = 0; d < 9; ++d) hk[l][d] = cload(g.hw, z + l * 9 + d);
    };
    // this step's rows (their loads were issued two steps ago), then the slot's refill for step y+2
    T uy[V], fy1[V], raw[V], fres[V], uout[V];
    int py[V], pout[V];
#pragma unroll
    for (int k = 0; k < V; ++k) {
      uy[k] = ur[SL][k];
      fy1[k] = fr_[SL][k];
      py[k] = MULTI ? pr[SL][k] : 0;
      raw[k] = RAW ? rw_[SL][k] : T(0);
      fres[k] = MODE == 2 ? frr[SL][k] : T(0);
      uout[k] = (MODE == 2 && !ZERO && EDGE) ? uo[SL][k] : T(0);
      pout[k] = (MODE == 2 && MULTI) ? po[SL][k] : 0;
    }
    fill(SL, y + PF);  // (rows past the task's last are clamped into the frame: loaded, never used)
    if constexpr (MODE == 1) {
      stage_t2();
      // x(y) = u(y) + w1 P(ec) on the interior (correct_even / correct_odd of k_mg_prolong)
      const bool yin = !EDGE || (y >= 1 && y <= H - 2);
#pragma unroll
      for (int k = 0; k < V; ++k) {  // (branch-free: a select, not a divergent branch per column)
        T xk;
        if constexpr (!ODD) {
          xk = uy[k] + g.w1 * cterm(Clo, k, 1);
        } else {
          const T tt = cterm(Clo, k, 2) + cterm(Chi, k, 0);
          xk = uy[k] + g.w1 * tt;
        }
        uy[k] = (yin && cin[k]) ? xk : uy[k];
      }
      if constexpr (ODD) {  // the next row (even) starts the next coarse row pair
        Clo = Chi;
        Chi = crow_fin(nC);
        nC = crow_ld((y >> 1) + 3);
      }
    }
    U0 = U1;
    U1 = U2;
    U2 = hwin<T, V>(uy);
    if constexpr (MULTI) {
      P0 = P1;
      P1 = P2;
      P2 = hpwin<V>(py);
    }
    // j and d_0 of row y-1
    stage_ks();
    const int yj = y - 1;
    const bool rin = !EDGE || (yj >= 1 && yj <= H - 2), rgr = !EDGE || (yj >= 0 && yj <= H - 1);
    T d0[V], jv[V];
#pragma unroll
    for (int k = 0; k < V; ++k) {
      T acc;
      if constexpr (!MULTI) {
        acc = ks[0] * U0.a[k];
        acc += ks[1] * U0.a[k + 1];
        acc += ks[2] * U0.a[k + 2];
        acc += ks[3] * U1.a[k];
        acc += ks[4] * U1.a[k + 1];
        acc += ks[5] * U1.a[k + 2];
        acc += ks[6] * U2.a[k];
        acc += ks[7] * U2.a[k + 1];
        acc += ks[8] * U2.a[k + 2];
      } else {
        acc = tab[P0.a[k] + 0] * U0.a[k];
        acc += tab[P0.a[k + 1] + 1] * U0.a[k + 1];
        acc += tab[P0.a[k + 2] + 2] * U0.a[k + 2];
        acc += tab[P1.a[k] + 3] * U1.a[k];
        acc += tab[P1.a[k + 1] + 4] * U1.a[k + 1];
        acc += tab[P1.a[k + 2] + 5] * U1.a[k + 2];
        acc += tab[P2.a[k] + 6] * U2.a[k];
        acc += tab[P2.a[k + 1] + 7] * U2.a[k + 1];
        acc += tab[P2.a[k + 2] + 8] * U2.a[k + 2];
      }
      const T omk = MULTI ? tab[P1.a[k + 1] + 9] : om;
      jv[k] = omk * (fy1[k] - acc) + U1.a[k + 1];
      T d = T(0);
      if (rin && cin[k]) {
        d = jv[k] - U1.a[k + 1];
      } else if (RAW && rgr && cgr[k]) {
        d = U1.a[k + 1] - raw[k];
      }
      d0[k] = d;
    }
    // j ring: J[i] = j of row y-1-i
#pragma unroll
    for (int i = NL; i > 0; --i)
#pragma unroll
      for (int k = 0; k < V; ++k) J[i][k] = J[i - 1][k];
#pragma unroll
    for (int k = 0; k < V; ++k) J[0][k] = jv[k];
    if constexpr (NL > 0) {
      D[0][0] = D[0][1];
      D[0][1] = D[0][2];
      D[0][2] = hwin<T, V>(d0);
    }
    // out row yo = y-1-NL: j + d_NL on the interior
    const int yo = y - 1 - NL;
    T o[V];
    if constexpr (NL == 0) {
#pragma unroll
      for (int k = 0; k < V; ++k) o[k] = J[0][k];
    }
    // d_l of row y-1-l from the d_(l-1) window of rows y-1-l-1 .. y-1-l+1
#pragma unroll
    for (int l = 1; l <= NL; ++l) {
      stage_hk(l - 1);
      const int yl = y - 1 - l;
      const bool lin = !EDGE || (yl >= 1 && yl <= H - 2);
      T dl[V];
#pragma unroll
      for (int k = 0; k < V; ++k) {
        const HWin<T, V>& A = D[l - 1][0];
        const HWin<T, V>& Bw = D[l - 1][1];
        const HWin<T, V>& C = D[l - 1][2];
        T acc = hk[l - 1][0] * A.a[k];
        acc += hk[l - 1][1] * A.a[k + 1];
        acc += hk[l - 1][2] * A.a[k + 2];
        acc += hk[l - 1][3] * Bw.a[k];
        acc += hk[l - 1][4] * Bw.a[k + 1];
        acc += hk[l - 1][5] * Bw.a[k + 2];
        acc += hk[l - 1][6] * C.a[k];
        acc += hk[l - 1][7] * C.a[k + 1];
        acc += hk[l - 1][8] * C.a[k + 2];
        dl[k] = (lin && cin[k]) ? acc : T(0);
      }
      if (l < NL) {
        D[l][0] = D[l][1];
        D[l][1] = D[l][2];
        D[l][2] = hwin<T, V>(dl);
      } else {
#pragma unroll
        for (int k = 0; k < V; ++k) o[k] = J[NL][k] + dl[k];
      }
    }
    if (own && yo >= r0 && yo < r1) hstore<T, V>(ob + (long long)(yo + 1) * ld + V * lane, o, cin);
    if constexpr (MODE == 2) {
      // the out row as the buffer would hold it: the iterate's own values off the interior
      const bool oin = !EDGE || (yo >= 1 && yo <= H - 2);
#pragma unroll
      for (int k = 0; k < V; ++k) o[k] = (oin && cin[k]) ? o[k] : uout[k];
      O0 = O1;
      O1 = O2;
      O2 = hwin<T, V>(o);
      if constexpr (MULTI) {
        Q0 = Q1;
        Q1 = Q2;
        Q2 = hpwin<V>(pout);
      }
      // residual row yr = yo - 1 (fea_mg_residual_restrict's resid), then the restriction of its coarse row
      const int yr = yo - 1;
      stage_ks();
      if (yr >= rc0 + 1) {
        T r[V + 1];
        const T(&fr)[V] = fres;
#pragma unroll
        for (int k = 0; k < V; ++k) {
          T acc;
          if constexpr (!MULTI) {
            acc = ks[0] * O0.a[k];
            acc += ks[1] * O0.a[k + 1];
            acc += ks[2] * O0.a[k + 2];
            acc += ks[3] * O1.a[k];
            acc += ks[4] * O1.a[k + 1];
            acc += ks[5] * O1.a[k + 2];
            acc += ks[6] * O2.a[k];
            acc += ks[7] * O2.a[k + 1];
            acc += ks[8] * O2.a[k + 2];
          } else {
            acc = tab[Q0.a[k] + 0] * O0.a[k];
            acc += tab[Q0.a[k + 1] + 1] * O0.a[k + 1];
            acc += tab[Q0.a[k + 2] + 2] * O0.a[k + 2];
            acc += tab[Q1.a[k] + 3] * O1.a[k];
            acc += tab[Q1.a[k + 1] + 4] * O1.a[k + 1];
            acc += tab[Q1.a[k + 2] + 5] * O1.a[k + 2];
            acc += tab[Q2.a[k] + 6] * O2.a[k];
            acc += tab[Q2.a[k + 1] + 7] * O2.a[k + 1];
            acc += tab[Q2.a[k + 2] + 8] * O2.a[k + 2];
          }
          r[k] = fr[k] - acc;
        }
        r[V] = shl1z(r[0]);  // column cl+V from the next lane
        stage_t2();
        if constexpr (((ODD ? 1 : 0) + NL) % 2 == 0) {  // row 2I (yr = y - 2 - NL)
#pragma unroll
          for (int k = 0; k <= V; ++k) Rb[k] = r[k];
          PRb = Q1;
        } else {
          if (yr > rc0 + 1) {  // row 2I+1 closes coarse row I = (yr - 1) / 2
            const int I = (yr - 1) / 2;
            T oc[Q];
#pragma unroll
            for (int q = 0; q < Q; ++q) {
              T acc;
              if constexpr (!MULTI) {
                acc = t2[0] * Ra[2 * q];
                acc += t2[1] * Ra[2 * q + 1];
                acc += t2[2] * Ra[2 * q + 2];
                acc += t2[3] * Rb[2 * q];
                acc += t2[4] * Rb[2 * q + 1];
                acc += t2[5] * Rb[2 * q + 2];
                acc += t2[6] * r[2 * q];
                acc += t2[7] * r[2 * q + 1];
                acc += t2[8] * r[2 * q + 2];
              } else {
                acc = tb2[PRa.a[2 * q + 1] + 0] * Ra[2 * q];
                acc += tb2[PRa.a[2 * q + 2] + 1] * Ra[2 * q + 1];
                acc += tb2[PRa.a[2 * q + 3] + 2] * Ra[2 * q + 2];
                acc += tb2[PRb.a[2 * q + 1] + 3] * Rb[2 * q];
                acc += tb2[PRb.a[2 * q + 2] + 4] * Rb[2 * q + 1];
                acc += tb2[PRb.a[2 * q + 3] + 5] * Rb[2 * q + 2];
                acc += tb2[Q1.a[2 * q + 1] + 6] * r[2 * q];
                acc += tb2[Q1.a[2 * q + 2] + 7] * r[2 * q + 1];
                acc += tb2[Q1.a[2 * q + 3] + 8] * r[2 * q + 2];
              }
              oc[q] = g.w0 * acc;
            }
            const int Jl = (cl + 1) / 2;
            if (own && I >= I0 && I < I1) {
              T* cp = g.fc + (long long)b * g.bsc + OFF + (long long)(I + 1) * g.ldc + Jl;
#pragma unroll
              for (int q = 0; q < Q; ++q)
                if (!EDGE || Jl + q <= g.Wc - 2) cp[q] = oc[q];
            }
          }
#pragma unroll
          for (int k = 0; k <= V; ++k) Ra[k] = r[k];
          PRa = Q1;
        }
      }
    }
  };
  // the loop body holds U steps (hs_unroll_steps), the remainder one by one
  constexpr int U = hs_unroll_steps<T, MULTI, MODE, ZERO, RAW>();
  static_assert(U % PF == 0 && U % 2 == 0, "hsweep unroll: even, a multiple of the prefetch ring");
  int y = y0;
  for (; y + U - 1 <= y1; y += U) hs_unroll<U>([&](auto i) __attribute__((always_inline)) { step(y + decltype(i)::value, i); });
  hs_unroll<U - 1>([&](auto i) __attribute__((always_inline)) {
    if (y + decltype(i)::value <= y1) step(y + decltype(i)::value, i);
  });
}

template <typename T, bool MULTI, bool ZERO, bool RAW, int NL, int MODE>
__global__ __launch_bounds__(256)
__attribute__((amdgpu_waves_per_eu(hs_mode1_wide<T, MULTI, MODE, RAW>() ? 3 : 1))) void k_mg_hsweep_strip(HSArgs<T> g) {
  using G = HSGeo<T, NL, MODE>;
  constexpr int V = HVec<T>::V;
  __shared__ T tab[MULTI ? FEA_MAX_PATTERNS * kHTS : 1];
  __shared__ T tb2[(MULTI && MODE != 0) ? FEA_MAX_PATTERNS * kHTS : 1];  // P (MODE 1) or R (MODE 2) kernels
  if constexpr (MULTI) {
    for (int i = threadIdx.x; i < g.ntab * kHTS; i += 256) {
      const int p = i / kHTS, d = i - p * kHTS;
      tab[i] = d == 9 ? g.omd[p] : g.ktab[p * 9 + d];
      if constexpr (MODE != 0) tb2[i] = d == 9 ? T(0) : (MODE == 1 ? g.ptab : g.rtab)[p * 9 + d];
    }
    __syncthreads();
  }
  // (row task, strip) pairs of one sample in linear order, four per workgroup
  const int per = g.ntr * g.nstrips;
  const int wpb = (per + 3) / 4;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int b = bid / wpb;
  const int w = (bid - b * wpb) * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  if (w >= per) return;
  const int t = w / g.nstrips, s = w - t * g.nstrips;
  if constexpr (FEA_HS_INNER != 0) {
    // interior: the rows streamed (from the first fill step 2 + NL rows above the first computed one, through the
    // prefetch past the last), the loaded columns and (MODE 1) the coarse rows read all lie strictly inside the grid
    int r0, r1, rc0, rc1, I0, I1;
    hs_rows<MODE>(t, g.rb, g.H, g.Hc, r0, r1, rc0, rc1, I0, I1);
    const int cs = 1 + s * G::S - G::HLN * V;
    const int ya = ((rc0 - G::HALO) & ~1) - 3 - NL, yz = rc1 + G::HALO + 4;
    const bool inner = cs >= 1 && cs + 64 * V - 1 <= g.W - 2 && ya >= 1 && yz <= g.H - 2 &&
                       (MODE != 1 || ((ya >> 1) - 1 >= 1 && (yz >> 1) + 4 <= g.Hc - 2));
    if (__builtin_amdgcn_readfirstlane((int)inner)) {  // wave-uniform (scalar branch)
      hsweep_task<T, MULTI, ZERO, RAW, NL, MODE, false>(g, b, t, s, tab, tb2);
      return;
    }
  }
  hsweep_task<T, MULTI, ZERO, RAW, NL, MODE, true>(g, b, t, s, tab, tb2);
}

}  // namespace fea

using namespace fea;

template <typename T, bool MULTI, bool ZERO, bool RAW, int MODE>
static void hs_launch_nl(int nl, dim3 grid, hipStream_t s, const HSArgs<T>& g) {
  switch (nl) {
    case 0: k_mg_hsweep_strip<T, MULTI, ZERO, RAW, 0, MODE><<<grid, 256, 0, s>>>(g); break;
    case 1: k_mg_hsweep_strip<T, MULTI, ZERO, RAW, 1, MODE><<<grid, 256, 0, s>>>(g); break;
    case 2: k_mg_hsweep_strip<T, MULTI, ZERO, RAW, 2, MODE><<<grid, 256, 0, s>>>(g); break;
    default: k_mg_hsweep_strip<T, MULTI, ZERO, RAW, 3, MODE><<<grid, 256, 0, s>>>(g); break;
  }
}

template <typename T, int MODE>
static void hs_dispatch(bool multi, bool zero, bool raw, int nl, dim3 grid, hipStream_t s, const HSArgs<T>& g) {
  if constexpr (MODE == 1) {
    if (raw) {
      if (multi) hs_launch_nl<T, true, false, true, 1>(nl, grid, s, g);
      else hs_launch_nl<T, false, false, true, 1>(nl, grid, s, g);
    } else {
      if (multi) hs_launch_nl<T, true, false, false, 1>(nl, grid, s, g);
      else hs_launch_nl<T, false, false, false, 1>(nl, grid, s, g);
    }
  } else if (zero) {
    if (multi) hs_launch_nl<T, true, true, false, MODE>(nl, grid, s, g);
    else hs_launch_nl<T, false, true, false, MODE>(nl, grid, s, g);
  } else if (raw) {
    if (multi) hs_launch_nl<T, true, false, true, MODE>(nl, grid, s, g);
    else hs_launch_nl<T, false, false, true, MODE>(nl, grid, s, g);
  } else {
    if (multi) hs_launch_nl<T, true, false, false, MODE>(nl, grid, s, g);
    else hs_launch_nl<T, false, false, false, MODE>(nl, grid, s, g);
  }
}

static int hs_num_cus() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cached[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cached[dev] = n;
  }
  return cached[dev];
}

#ifndef FEA_HSWEEP_BALANCED
#define FEA_HSWEEP_BALANCED 1
#endif

// Row tasks: `unit` rows each (MODE 2 counts coarse rows, 2 fine rows per unit), a task streams k*unit + ovh
// rows (the stage chain's halo rows above and below its own).  Balanced (the cycle join's rule, framed_ops.hip
// balanced_rb): the slowest CU runs ceil(workgroups / CUs) tasks back to back, so the cost of a task height is
// that count times the rows a task streams; among the heights that keep >= 2048 waves in flight the cheapest
// wins (4097^2 fp64 sweep+restriction: 504 workgroups of 74 rows, 2 per CU, instead of 576 of 64: a quarter of
// the CUs ran a third task; "2048" is FEA_HS_MINW, now 1536).  Levels too small for 2048 waves at any height take the cheapest height outright:
// there every CU holds at most one or two tasks and the task's chain of rows is the time.  Results are bitwise
// independent of the task height.
// the fewest waves a balanced hsweep launch may have: 1536 (4097^2 MG-HJac 397.4 -> 393.3 us, fine sweep +
// restriction 111 -> 109 us, against 2048; 1024 measured the same as 1536; profiles/r06_ab/hjac_minw.txt)
#ifndef FEA_HS_MINW
#define FEA_HS_MINW 1536
#endif
static int hs_units_per_task(int B, int nstrips, int rows_u, int k, int ovh) {
#if FEA_HSWEEP_BALANCED
  const long long ncu = hs_num_cus();
  long long best_ok = -1, best_any = -1;
  int u_ok = 0, u_any = 1;
  for (int u = 1; u <= rows_u && k * u <= 256; ++u) {
    const long long ntr = (rows_u + u - 1) / u, waves = (long long)B * nstrips * ntr;
    const long long wgs = (long long)B * ((ntr * nstrips + 3) / 4);
    const long long cost = ((wgs + ncu - 1) / ncu) * (k * u + ovh);
    if (waves >= FEA_HS_MINW && (best_ok < 0 || cost < best_ok)) best_ok = cost, u_ok = u;
    if (best_any < 0 || cost < best_any) best_any = cost, u_any = u;
  }
  return best_ok >= 0 ? u_ok : u_any;
#else
  // the largest of 64 / 32 / 16 / 8 rows that still gives >= 2048 waves
  for (int rb = 64; rb > 8; rb /= 2)
    if ((long long)B * nstrips * ((rows_u * k + rb - 1) / rb) >= 2048) return rb / k;
  return 8 / k;
#endif
}

template <typename T, int MODE>
static int hsweep_launch(HSArgs<T> g, int nl, int B, hipStream_t s) {
  constexpr int V = HVec<T>::V;
  const int hln = (nl + 1 + (MODE == 2 ? 2 : MODE == 1 ? 1 : 0) + V - 1) / V;
  const int S = (64 - 2 * hln) * V;
  // (lanes past the grid's last column re-read the last valid line: loads stay within columns < W + V)
  g.nstrips = (g.W - 2 + S - 1) / S;
  const int rows = MODE == 2 ? g.Hc - 2 : g.H - 2;  // MODE 2 tasks count coarse rows (rb / 2 each)
  const int k = MODE == 2 ? 2 : 1;
  const int ovh = 2 * (nl + 1) + (MODE == 2 ? 2 : 0);
  const int u = hs_units_per_task(B, g.nstrips, rows, k, ovh);
  g.rb = k * u;
  g.ntr = (rows + u - 1) / u;
  const dim3 grid((unsigned)(B * ((g.ntr * g.nstrips + 3) / 4)));
  hs_dispatch<T, MODE>(g.ntab > 1, !g.u, g.u_raw != nullptr, nl, grid, s, g);
  FEA_LAUNCH_CHECK();
}

static inline bool hs_layout_ok(int H, int W, int ld, long long bs, int esz) {
  return H >= 3 && W >= 3 && ld >= W + 128 / esz && bs >= (long long)(H + 2) * ld;
}

#define FEA_HNET_API(SUF, T)                                                                                \
  extern "C" int fea_mg_hsweep_##SUF(const T* u, const T* u_raw, const T* f, T* out, const uint8_t* pid,     \
                                     const T* ktab,                                                          \
                                     const T* omd, int ntab, const T* hw, int nlayers, int B, int H, int W,  \
                                     int ld, long long bs, void* stream) {                                   \
    if (!f || !out || !ktab || !omd || (!hw && nlayers > 0) || out == u || B <= 0 || B > 65535) return FEA_EINVAL; \
    if (nlayers < 0 || nlayers > kHMaxLayers || !hs_layout_ok(H, W, ld, bs, sizeof(T))) return FEA_EINVAL;    \
    if (ntab < 1 || ntab > FEA_MAX_PATTERNS || (ntab > 1 && !pid)) return FEA_EINVAL;                         \
    if (u_raw && !u) return FEA_EINVAL;                                                                      \
    HSArgs<T> g{};                                                                                           \
    g.u = u; g.u_raw = u_raw; g.f = f; g.out = out; g.pid = pid; g.ktab = ktab; g.omd = omd; g.hw = hw;       \
    g.ntab = ntab; g.H = H; g.W = W; g.ld = ld; g.bs = bs;                                                    \
    return hsweep_launch<T, 0>(g, nlayers, B, (hipStream_t)stream);                                          \
  }                                                                                                          \
  extern "C" int fea_mg_hsweep_restrict_##SUF(const T* u, const T* u_raw, const T* f, T* out, T* fc,           \
                                              const uint8_t* pid, const T* ktab, const T* omd, int ntab,       \
                                              const T* hw, int nlayers, const T* rtab, int nrtab, T w0, int B,  \
                                              int H, int W, int ld, long long bs, int ldc, long long bsc,       \
                                              void* stream) {                                                  \
    if (!f || !out || !fc || !ktab || !omd || !rtab || (!hw && nlayers > 0) || out == u || B <= 0 ||         \
        B > 65535)                                                                                           \
      return FEA_EINVAL;                                                                                     \
    if (nlayers < 0 || nlayers > kHMaxLayers || !hs_layout_ok(H, W, ld, bs, sizeof(T)) || !(H & 1) || !(W & 1)) \
      return FEA_EINVAL;                                                                                     \
    const int Hc = (H + 1) / 2, Wc = (W + 1) / 2;                                                            \
    if (!hs_layout_ok(Hc, Wc, ldc, bsc, sizeof(T))) return FEA_EINVAL;                                        \
    if (ntab < 1 || ntab > FEA_MAX_PATTERNS || (ntab > 1 && !pid) || (nrtab != ntab && nrtab != 1) ||        \
        (ntab > 1 && nrtab == 1))                                                                            \
      return FEA_EINVAL;                                                                                     \
    if (u_raw && !u) return FEA_EINVAL;                                                                      \
    HSArgs<T> g{};                                                                                           \
    g.u = u; g.u_raw = u_raw; g.f = f; g.out = out; g.pid = pid; g.ktab = ktab; g.omd = omd; g.hw = hw;       \
    g.ntab = ntab; g.H = H; g.W = W; g.ld = ld; g.bs = bs;                                                    \
    g.fc = fc; g.rtab = rtab; g.w0 = w0; g.Hc = Hc; g.Wc = Wc; g.ldc = ldc; g.bsc = bsc;                      \
    return hsweep_launch<T, 2>(g, nlayers, B, (hipStream_t)stream);                                          \
  }                                                                                                          \
  extern "C" int fea_mg_prolong_hsweep_##SUF(const T* u, const T* u_raw, const T* ec, const T* f, T* out,       \
                                             const uint8_t* pid,                                               \
                                             const uint8_t* pidc, const T* ktab, const T* omd, int ntab,        \
                                             const T* hw, int nlayers, const T* ptab, int nptab, T w1, int B,   \
                                             int H, int W, int ld, long long bs, int ldc, long long bsc,        \
                                             void* stream) {                                                   \
    if (!u || !ec || !f || !out || !ktab || !omd || !ptab || (!hw && nlayers > 0) || out == u || B <= 0 ||   \
        B > 65535)                                                                                           \
      return FEA_EINVAL;                                                                                     \
    if (nlayers < 0 || nlayers > kHMaxLayers || !hs_layout_ok(H, W, ld, bs, sizeof(T)) || !(H & 1) || !(W & 1)) \
      return FEA_EINVAL;                                                                                     \
    const int Hc = (H + 1) / 2, Wc = (W + 1) / 2;                                                            \
    if (!hs_layout_ok(Hc, Wc, ldc, bsc, sizeof(T))) return FEA_EINVAL;                                        \
    if (ntab < 1 || ntab > FEA_MAX_PATTERNS || (nptab != ntab && nptab != 1) ||                              \
        (ntab > 1 && (!pid || !pidc || nptab == 1)))                                                          \
      return FEA_EINVAL;                                                                                     \
    HSArgs<T> g{};                                                                                           \
    g.u = u; g.u_raw = u_raw; g.f = f; g.out = out; g.pid = pid; g.ktab = ktab; g.omd = omd; g.hw = hw;       \
    g.ntab = ntab; g.H = H; g.W = W; g.ld = ld; g.bs = bs;                                                    \
    g.ec = ec; g.pidc = pidc; g.ptab = ptab; g.w1 = w1; g.Hc = Hc; g.Wc = Wc; g.ldc = ldc; g.bsc = bsc;       \
    return hsweep_launch<T, 1>(g, nlayers, B, (hipStream_t)stream);                                          \
  }

FEA_HNET_API(f32, float)
FEA_HNET_API(f64, double)
