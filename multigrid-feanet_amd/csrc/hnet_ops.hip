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

namespace fea {

constexpr int kHMaxLayers = 3;    // HNet(nb_layers=3) (M-FEANet-mg_test.ipynb:222)
constexpr int kHTS = 10;          // LDS table stride (9 weights + omega/d)

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
  w.a[0] = shr1(x[V - 1], T(0));
  w.a[V + 1] = shl1(x[0], T(0));
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
  w.a[0] = shr1(x[V - 1], 0) * kHTS;
  w.a[V + 1] = shl1(x[0], 0) * kHTS;
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
};

template <typename T, bool MULTI, bool ZERO, bool RAW, int NL>
__global__ __launch_bounds__(256) void k_mg_hsweep_strip(HSArgs<T> g) {
  constexpr int V = HVec<T>::V;
  constexpr int HALO = NL + 1;                 // columns / rows the stage chain reaches on each side
  constexpr int HLN = (HALO + V - 1) / V;      // halo lanes per side
  constexpr int S = (64 - 2 * HLN) * V;        // owned columns per strip
  constexpr int OFF = 128 / (int)sizeof(T) - 1;
  __shared__ T tab[MULTI ? FEA_MAX_PATTERNS * kHTS : 1];
  if constexpr (MULTI) {
    for (int i = threadIdx.x; i < g.ntab * kHTS; i += 256) {
      const int p = i / kHTS, d = i - p * kHTS;
      tab[i] = d == 9 ? g.omd[p] : g.ktab[p * 9 + d];
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
  const int lane = lane_id();
  const int H = g.H, W = g.W, ld = g.ld;
  const int cs = 1 + s * S - HLN * V;  // first loaded column
  const int cl = cs + V * lane;
  const int ll = min(lane, (W - 1 - cs) / V);  // lanes past the last column re-read a valid line
  const bool own = lane >= HLN && lane < 64 - HLN;
  const int r0 = 1 + t * g.rb, r1 = min(r0 + g.rb, H - 1);
  bool cin[V], cgr[V];
#pragma unroll
  for (int k = 0; k < V; ++k) {
    cin[k] = cl + k >= 1 && cl + k <= W - 2;
    cgr[k] = cl + k >= 0 && cl + k <= W - 1;
  }
  T ks[9], om = 0, hk[NL > 0 ? NL : 1][9];
  if constexpr (!MULTI) {
#pragma unroll
    for (int d = 0; d < 9; ++d) ks[d] = g.ktab[d];
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
  auto rowo = [&](int r) -> long long { return (long long)(min(max(r, -1), H) + 1) * ld + V * ll; };

  HWin<T, V> U0{}, U1{}, U2{};           // u rows y-2, y-1, y
  HWin<int, V> P0{}, P1{}, P2{};         // pattern offsets of the same rows
  HWin<T, V> D[NL > 0 ? NL : 1][3] = {}; // d_l windows: d_l of rows (y-1-l)-2 .. (y-1-l)
  T J[NL + 1][V];                        // j of rows y-1 .. y-1-NL
#pragma unroll
  for (int i = 0; i <= NL; ++i)
#pragma unroll
    for (int k = 0; k < V; ++k) J[i][k] = T(0);
  const int y0 = r0 - HALO, y1 = r1 - 1 + HALO;
  T un[V], fn[V];
  int pn[V];
#pragma unroll
  for (int k = 0; k < V; ++k) { un[k] = T(0); pn[k] = 0; }
  if constexpr (!ZERO) hload<T, V>(ub + rowo(y0), un);
  if constexpr (MULTI) hpload<V>(pb + rowo(y0), pn);
  hload<T, V>(fb + rowo(y0 - 1), fn);
  for (int y = y0; y <= y1; ++y) {
    // rotate the u window in row y (loaded one step ahead); f of row y-1
    T uy[V], fy1[V];
    int py[V];
#pragma unroll
    for (int k = 0; k < V; ++k) { uy[k] = un[k]; fy1[k] = fn[k]; py[k] = pn[k]; }
    if (y + 1 <= y1) {
      if constexpr (!ZERO) hload<T, V>(ub + rowo(y + 1), un);
      if constexpr (MULTI) hpload<V>(pb + rowo(y + 1), pn);
    }
    hload<T, V>(fb + rowo(y), fn);
    U0 = U1;
    U1 = U2;
    U2 = hwin<T, V>(uy);
    if constexpr (MULTI) {
      P0 = P1;
      P1 = P2;
      P2 = hpwin<V>(py);
    }
    // j and d_0 of row y-1
    const int yj = y - 1;
    const bool rin = yj >= 1 && yj <= H - 2, rgr = yj >= 0 && yj <= H - 1;
    T d0[V], jv[V];
    T raw[V];
    if constexpr (RAW) {
      hload<T, V>(rb_ + rowo(yj), raw);
    }
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
    // d_l of row y-1-l from the d_(l-1) window of rows y-1-l-1 .. y-1-l+1
#pragma unroll
    for (int l = 1; l <= NL; ++l) {
      const int yl = y - 1 - l;
      const bool lin = yl >= 1 && yl <= H - 2;
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
        // out of row y-1-NL = j + d_NL on the owned interior nodes
        const int yo = y - 1 - NL;
        if (own && yo >= r0 && yo < r1) {
          T o[V];
#pragma unroll
          for (int k = 0; k < V; ++k) o[k] = J[NL][k] + dl[k];
          hstore<T, V>(ob + (long long)(yo + 1) * ld + V * lane, o, cin);
        }
      }
    }
    if constexpr (NL == 0) {
      const int yo = y - 1;
      if (own && yo >= r0 && yo < r1) hstore<T, V>(ob + (long long)(yo + 1) * ld + V * lane, J[0], cin);
    }
  }
}

}  // namespace fea

using namespace fea;

template <typename T, bool MULTI, bool ZERO, bool RAW>
static void hs_launch_nl(int nl, dim3 grid, hipStream_t s, const HSArgs<T>& g) {
  switch (nl) {
    case 0: k_mg_hsweep_strip<T, MULTI, ZERO, RAW, 0><<<grid, 256, 0, s>>>(g); break;
    case 1: k_mg_hsweep_strip<T, MULTI, ZERO, RAW, 1><<<grid, 256, 0, s>>>(g); break;
    case 2: k_mg_hsweep_strip<T, MULTI, ZERO, RAW, 2><<<grid, 256, 0, s>>>(g); break;
    default: k_mg_hsweep_strip<T, MULTI, ZERO, RAW, 3><<<grid, 256, 0, s>>>(g); break;
  }
}

template <typename T>
static int hsweep_strip_launch(const T* u, const T* u_raw, const T* f, T* out, const uint8_t* pid, const T* ktab,
                               const T* omd, int ntab, const T* hw, int nl, int B, int H, int W, int ld, long long bs,
                               hipStream_t s) {
  constexpr int V = HVec<T>::V;
  const int hln = (nl + 1 + V - 1) / V;
  const int S = (64 - 2 * hln) * V;
  // (lanes past the grid's last column re-read the last valid line: loads stay within columns < W + V)
  HSArgs<T> g{u, u_raw, f, out, pid, ktab, omd, hw, ntab, H, W, ld, bs, 0, 0, 0};
  g.nstrips = (W - 2 + S - 1) / S;
  // rows per task: the largest of 64 / 32 / 16 / 8 that still gives >= 2048 waves (each task recomputes nl + 1
  // rows above and below its own)
  g.rb = 8;
  for (int rb = 64; rb > 8; rb /= 2)
    if ((long long)B * g.nstrips * ((H - 2 + rb - 1) / rb) >= 2048) {
      g.rb = rb;
      break;
    }
  g.ntr = (H - 2 + g.rb - 1) / g.rb;
  const dim3 grid((unsigned)(B * ((g.ntr * g.nstrips + 3) / 4)));
  const bool multi = ntab > 1;
  if (!u) {
    if (multi) hs_launch_nl<T, true, true, false>(nl, grid, s, g);
    else hs_launch_nl<T, false, true, false>(nl, grid, s, g);
  } else if (u_raw) {
    if (multi) hs_launch_nl<T, true, false, true>(nl, grid, s, g);
    else hs_launch_nl<T, false, false, true>(nl, grid, s, g);
  } else {
    if (multi) hs_launch_nl<T, true, false, false>(nl, grid, s, g);
    else hs_launch_nl<T, false, false, false>(nl, grid, s, g);
  }
  FEA_LAUNCH_CHECK();
}

#define FEA_HNET_API(SUF, T)                                                                                \
  extern "C" int fea_mg_hsweep_##SUF(const T* u, const T* u_raw, const T* f, T* out, const uint8_t* pid,     \
                                     const T* ktab,                                                          \
                                     const T* omd, int ntab, const T* hw, int nlayers, int B, int H, int W,  \
                                     int ld, long long bs, void* stream) {                                   \
    if (!f || !out || !ktab || !omd || (!hw && nlayers > 0) || out == u || B <= 0 || B > 65535) return FEA_EINVAL; \
    if (H < 3 || W < 3 || nlayers < 0 || nlayers > kHMaxLayers) return FEA_EINVAL;                           \
    if (ntab < 1 || ntab > FEA_MAX_PATTERNS || (ntab > 1 && !pid)) return FEA_EINVAL;                         \
    if (ld < W + 128 / (int)sizeof(T) || bs < (long long)(H + 2) * ld) return FEA_EINVAL;                     \
    if (u_raw && !u) return FEA_EINVAL;                                                                      \
    return hsweep_strip_launch<T>(u, u_raw, f, out, pid, ktab, omd, ntab, hw, nlayers, B, H, W, ld, bs,         \
                                  (hipStream_t)stream);                                                        \
  }

FEA_HNET_API(f32, float)
FEA_HNET_API(f64, double)
