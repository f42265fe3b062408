// hnet_ops.hip — one sweep of the learned smoother of M-FEANet-mg_test.ipynb (HJacIterator.HRelax,
// :147-155, HNet.forward :104-106) fused into one pass over a framed level:
//
//   j   = J(u, f)                         (weighted Jacobi, jacobi.py:39-47)
//   d_0 = j - u                           (zero on the boundary: u holds the Dirichlet values)
//   d_k = (W_k * d_{k-1}) . g             k = 1..nl, 3x3 cross-correlation, zero padding, g = interior
//   out = j + d_nl                        (interior; the boundary keeps u)
//
// SURVEY §8f row 1 ("fuse Jacobi with three masked 3x3 convs, halo 4 in LDS").  A workgroup owns a
// kHT x TW tile of interior nodes and stages u on the tile plus a halo of nl+1 rows/columns in LDS;
// d_0 is formed on halo nl, each conv layer shrinks the valid halo by one, the last layer lands on
// the tile.  Work per node: 9 (K u) + 9 nl FMAs, all operands from LDS; HBM traffic ~ read u, read f,
// write out (+ halo re-reads served by L2).  The arithmetic per node is the same expression at
// every node (fp-contract=on), so results do not depend on the tiling.
#include "fea_common.h"

namespace fea {

constexpr int kHT = 16;           // tile rows
constexpr int kHThreads = 256;
constexpr int kHMaxLayers = 3;    // HNet(nb_layers=3) (M-FEANet-mg_test.ipynb:222)
constexpr int kHHalo = kHMaxLayers + 1;
constexpr int kHTS = 10;          // LDS table stride (9 weights + omega/d)

template <typename T>
struct HTile {
  static constexpr int TW = 1024 / (int)sizeof(T);  // tile columns: 1 KiB of a row
  static constexpr int RU = kHT + 2 * kHHalo;       // staged u rows / columns
  static constexpr int CU = TW + 2 * kHHalo;
};

template <typename T>
struct HArgs {
  const T* u;
  const T* u_raw;  // optional: the caller's un-reset iterate (d_0 = u - u_raw on boundary nodes)
  const T* f;
  T* out;
  const uint8_t* pid;
  const T* ktab;
  const T* omd;
  const T* hw;
  int ntab, nl;
  int H, W, ld;
  long long bs;
};

template <typename T, bool MULTI, bool ZERO>
__global__ __launch_bounds__(kHThreads) void k_mg_hsweep(HArgs<T> a) {
  using G = HTile<T>;
  constexpr int RU = G::RU, CU = G::CU, TW = G::TW;
  __shared__ T su[RU * CU];                 // u on tile + halo 4 (0 outside the grid)
  __shared__ T sd0[RU * CU];                // d ping-pong (same indexing as su)
  __shared__ T sd1[RU * CU];
  __shared__ uint8_t sp[MULTI ? RU * CU : 1];
  __shared__ T tab[MULTI ? FEA_MAX_PATTERNS * kHTS : kHTS];
  const int tid = threadIdx.x;
  const int H = a.H, W = a.W, ld = a.ld, nl = a.nl;
  const int r0 = 1 + blockIdx.y * kHT, c0 = 1 + blockIdx.x * TW;  // tile origin (grid coordinates)
  const int gy0 = r0 - kHHalo, gx0 = c0 - kHHalo;                   // staged region origin
  const long long boff = (long long)blockIdx.z * a.bs + (128 / (int)sizeof(T) - 1);
  const T* __restrict__ ub = ZERO ? nullptr : a.u + boff;
  const T* __restrict__ fb = a.f + boff;
  T* __restrict__ ob = a.out + boff;
  auto gidx = [&](int r, int c) -> long long { return (long long)(r + 1) * ld + c; };

  const int nt = MULTI ? a.ntab : 1;
  for (int i = tid; i < nt * kHTS; i += kHThreads) {
    const int p = i / kHTS, d = i - p * kHTS;
    tab[i] = d == 9 ? a.omd[p] : a.ktab[p * 9 + d];
  }
  __shared__ T hw[kHMaxLayers * 9];  // conv weights (uniform; LDS so the layer loop can index them)
  for (int i = tid; i < kHMaxLayers * 9; i += kHThreads) hw[i] = i < nl * 9 ? a.hw[i] : T(0);
  for (int i = tid; i < RU * CU; i += kHThreads) {
    const int y = i / CU, x = i - y * CU;
    const int r = gy0 + y, c = gx0 + x;
    const bool in = r >= 0 && r < H && c >= 0 && c < W;
    su[i] = (!ZERO && in) ? ub[gidx(r, c)] : T(0);
    if constexpr (MULTI) sp[i] = in ? a.pid[(128 / (int)sizeof(T) - 1) + gidx(r, c)] : 0;
  }
  __syncthreads();

  auto interior = [&](int y, int x) {
    const int r = gy0 + y, c = gx0 + x;
    return r >= 1 && r <= H - 2 && c >= 1 && c <= W - 2;
  };
  auto jac = [&](int y, int x) -> T {  // j = u + (omega/d)(f - K u) at staged position (y, x)
    const int i = y * CU + x;
    T acc;
    if constexpr (!MULTI) {
      acc = tab[0] * su[i - CU - 1];
      acc += tab[1] * su[i - CU];
      acc += tab[2] * su[i - CU + 1];
      acc += tab[3] * su[i - 1];
      acc += tab[4] * su[i];
      acc += tab[5] * su[i + 1];
      acc += tab[6] * su[i + CU - 1];
      acc += tab[7] * su[i + CU];
      acc += tab[8] * su[i + CU + 1];
    } else {
      acc = tab[sp[i - CU - 1] * kHTS + 0] * su[i - CU - 1];
      acc += tab[sp[i - CU] * kHTS + 1] * su[i - CU];
      acc += tab[sp[i - CU + 1] * kHTS + 2] * su[i - CU + 1];
      acc += tab[sp[i - 1] * kHTS + 3] * su[i - 1];
      acc += tab[sp[i] * kHTS + 4] * su[i];
      acc += tab[sp[i + 1] * kHTS + 5] * su[i + 1];
      acc += tab[sp[i + CU - 1] * kHTS + 6] * su[i + CU - 1];
      acc += tab[sp[i + CU] * kHTS + 7] * su[i + CU];
      acc += tab[sp[i + CU + 1] * kHTS + 8] * su[i + CU + 1];
    }
    const T om = MULTI ? tab[sp[i] * kHTS + 9] : tab[9];
    return om * (fb[gidx(gy0 + y, gx0 + x)] - acc) + su[i];
  };
  auto conv = [&](const T* s, int i, const T* w) -> T {
    T acc = w[0] * s[i - CU - 1];
    acc += w[1] * s[i - CU];
    acc += w[2] * s[i - CU + 1];
    acc += w[3] * s[i - 1];
    acc += w[4] * s[i];
    acc += w[5] * s[i + 1];
    acc += w[6] * s[i + CU - 1];
    acc += w[7] * s[i + CU];
    acc += w[8] * s[i + CU + 1];
    return acc;
  };

  // d_0 on the tile + halo nl (zero off the interior and outside the grid); the rest of the
  // staged region is zeroed so later layers read zeros there
  {
    const int h = nl;
    for (int i = tid; i < RU * CU; i += kHThreads) {
      const int y = i / CU, x = i - y * CU;
      const bool inr = y >= kHHalo - h && y < kHHalo + kHT + h && x >= kHHalo - h && x < kHHalo + TW + h;
      T d = T(0);
      if (inr && interior(y, x)) {
        d = jac(y, x) - su[i];
      } else if (inr && a.u_raw) {  // boundary node inside the grid: Dirichlet value - caller's value
        const int r = gy0 + y, c = gx0 + x;
        if (r >= 0 && r < H && c >= 0 && c < W) d = su[i] - a.u_raw[boff + gidx(r, c)];
      }
      sd0[i] = d;
      sd1[i] = T(0);
    }
  }
  __syncthreads();
  T* src = sd0;
  T* dst = sd1;
  for (int k = 0; k < nl; ++k) {
    const int h = nl - 1 - k;  // halo of layer k's output
    const int rows = kHT + 2 * h, cols = TW + 2 * h;
    for (int q = tid; q < rows * cols; q += kHThreads) {
      const int y = kHHalo - h + q / cols, x = kHHalo - h + q % cols;
      const int i = y * CU + x;
      dst[i] = interior(y, x) ? conv(src, i, hw + 9 * k) : T(0);
    }
    __syncthreads();
    T* t = src;
    src = dst;
    dst = t;
  }
  // out = j + d_nl on the tile's interior nodes
  for (int q = tid; q < kHT * TW; q += kHThreads) {
    const int y = kHHalo + q / TW, x = kHHalo + q % TW;
    if (!interior(y, x)) continue;
    const T j = jac(y, x);
    ob[gidx(gy0 + y, gx0 + x)] = j + (nl > 0 ? src[y * CU + x] : T(0));
  }
}

}  // namespace fea

using namespace fea;

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
    HArgs<T> a{u, u_raw, f, out, pid, ktab, omd, hw, ntab, nlayers, H, W, ld, bs};                           \
    const dim3 grid((unsigned)((W - 2 + HTile<T>::TW - 1) / HTile<T>::TW), (unsigned)((H - 2 + kHT - 1) / kHT), \
                    (unsigned)B);                                                                            \
    hipStream_t s = (hipStream_t)stream;                                                                     \
    const bool multi = ntab > 1;                                                                             \
    if (!u) {                                                                                                \
      if (multi) k_mg_hsweep<T, true, true><<<grid, kHThreads, 0, s>>>(a);                                   \
      else k_mg_hsweep<T, false, true><<<grid, kHThreads, 0, s>>>(a);                                        \
    } else {                                                                                                 \
      if (multi) k_mg_hsweep<T, true, false><<<grid, kHThreads, 0, s>>>(a);                                  \
      else k_mg_hsweep<T, false, false><<<grid, kHThreads, 0, s>>>(a);                                       \
    }                                                                                                        \
    FEA_LAUNCH_CHECK();                                                                                      \
  }

FEA_HNET_API(f32, float)
FEA_HNET_API(f64, double)
