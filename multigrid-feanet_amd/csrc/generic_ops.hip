// generic_ops.hip — FEANet operators on contiguous NCHW tensors (the drop-in operator
// boundary behind FEANet.model / FEANet.jacobi / FEANet.multigrid shims).
//
// These kernels take arbitrary contiguous user tensors (row pitch = W, any alignment), so they
// are written one-output-per-lane with the 3x3 neighbourhood read through L1/L2; the
// bandwidth-optimised path for the V-cycle is framed_ops.hip (solver-owned aligned buffers).
#include "fea_common.h"

namespace fea {

constexpr int kBX = 64, kBY = 4;  // one wave per block row

template <typename T>
__device__ __forceinline__ void load_table(T* dst, const T* src, int n) {
  for (int i = threadIdx.y * blockDim.x + threadIdx.x; i < n; i += blockDim.x * blockDim.y) dst[i] = src[i];
}

// y = K u  (FEANet/model.py:22-30): weight of neighbour j is ktab[pid(j)][d], zero padding.
template <typename T>
__global__ __launch_bounds__(256) void k_knet(const T* __restrict__ u, T* __restrict__ y,
                                              const uint8_t* __restrict__ pid, const T* __restrict__ ktab,
                                              int ntab, int H, int W) {
  __shared__ T tab[FEA_MAX_PATTERNS * 9];
  load_table(tab, ktab, ntab * 9);
  __syncthreads();
  const int c = blockIdx.x * kBX + threadIdx.x, r = blockIdx.y * kBY + threadIdx.y;
  if (r >= H || c >= W) return;
  const long long HW = (long long)H * W;
  const T* ub = u + blockIdx.z * HW;
  T acc = 0;
#pragma unroll
  for (int dr = 0; dr < 3; ++dr) {
    const int rr = r + dr - 1;
    if (rr < 0 || rr >= H) continue;
#pragma unroll
    for (int dc = 0; dc < 3; ++dc) {
      const int cc = c + dc - 1;
      if (cc < 0 || cc >= W) continue;
      const int p = pid ? pid[rr * W + cc] : 0;
      acc += tab[p * 9 + dr * 3 + dc] * ub[(long long)rr * W + cc];
    }
  }
  y[blockIdx.z * HW + (long long)r * W + c] = acc;
}

// xs[b, p] = (pid == p) ? x[b] : 0  (FEANet/model.py:37-47)
template <typename T>
__global__ __launch_bounds__(256) void k_split(const T* __restrict__ x, T* __restrict__ xs,
                                               const uint8_t* __restrict__ pid, int C, int H, int W) {
  const int c = blockIdx.x * kBX + threadIdx.x, r = blockIdx.y * kBY + threadIdx.y;
  if (r >= H || c >= W) return;
  const long long HW = (long long)H * W, i = (long long)r * W + c;
  const T v = x[blockIdx.z * HW + i];
  const int p = pid ? pid[i] : 0;
  T* o = xs + (long long)blockIdx.z * C * HW + i;
  for (int ch = 0; ch < C; ++ch) o[ch * HW] = (ch == p) ? v : T(0);
}

template <typename T>
__device__ __forceinline__ T reset_at(const T* geo, const T* bc, long long gi, long long bi, T v, int r, int c,
                                      int H, int W) {
  const T g = geo ? geo[gi] : T((r > 0 && r < H - 1 && c > 0 && c < W - 1) ? 1 : 0);
  const T b = bc ? bc[bi] : T(0);
  return v * g + b;
}

// One weighted-Jacobi sweep (FEANet/jacobi.py:39-47) with reset_boundary (:27-29) on both sides.
template <typename T>
__global__ __launch_bounds__(256) void k_jacobi(const T* __restrict__ u, const T* __restrict__ f,
                                                T* __restrict__ out, const uint8_t* __restrict__ pid,
                                                const T* __restrict__ ktab, const T* __restrict__ omd, int ntab,
                                                const T* __restrict__ geo, long long geo_bs,
                                                const T* __restrict__ bc, long long bc_bs, int H, int W) {
  __shared__ T tab[FEA_MAX_PATTERNS * 10];
  for (int i = threadIdx.y * blockDim.x + threadIdx.x; i < ntab * 10; i += blockDim.x * blockDim.y)
    tab[i] = (i % 10 == 9) ? omd[i / 10] : ktab[(i / 10) * 9 + (i % 10)];
  __syncthreads();
  const int c = blockIdx.x * kBX + threadIdx.x, r = blockIdx.y * kBY + threadIdx.y;
  if (r >= H || c >= W) return;
  const long long HW = (long long)H * W;
  const int b = blockIdx.z;
  const T* ub = u + b * HW;
  const T* gb = geo ? geo + b * geo_bs : nullptr;
  const T* bb = bc ? bc + b * bc_bs : nullptr;
  T acc = 0, u0c = 0;
#pragma unroll
  for (int dr = 0; dr < 3; ++dr) {
    const int rr = r + dr - 1;
    if (rr < 0 || rr >= H) continue;
#pragma unroll
    for (int dc = 0; dc < 3; ++dc) {
      const int cc = c + dc - 1;
      if (cc < 0 || cc >= W) continue;
      const long long j = (long long)rr * W + cc;
      const T v0 = reset_at(gb, bb, j, j, ub[j], rr, cc, H, W);
      if (dr == 1 && dc == 1) u0c = v0;
      const int p = pid ? pid[j] : 0;
      acc += tab[p * 10 + dr * 3 + dc] * v0;
    }
  }
  const long long i = (long long)r * W + c;
  const int p = pid ? pid[i] : 0;
  const T res = f[b * HW + i] - acc;
  const T u1 = tab[p * 10 + 9] * res + u0c;
  out[b * HW + i] = reset_at(gb, bb, i, i, u1, r, c, H, W);
}

// Periodic weighted-Jacobi sweep (JacobiBlockPBC.jacobi_convolution, FEANet/jacobi.py:86-97) on the
// N x N node grid with period n = N - 1.  The reference extends u circularly to (n+3)^2
// (pbc_boundary :72-79), convolves with K (zero padding never reaches the kept rows), crops
// [1:-1, 1:-1] and adds reset_boundary(u) (:81-84, the circular (n+1)^2 copy):
//   out(a, b) = omd * (f(a+1, b+1) - sum_d W[d] u((a+dy) mod n, (b+dx) mod n)) + u(a mod n, b mod n)
// with f the (N+2)^2 forcing term the reference's drivers build (FNet of the periodic extension).
// Single pattern only ("currently only for homogeneous problems", jacobi.py:51).
template <typename T>
__global__ __launch_bounds__(256) void k_jacobi_pbc(const T* __restrict__ u, const T* __restrict__ f,
                                                    T* __restrict__ out, const T* __restrict__ ktab,
                                                    const T* __restrict__ omd, int N) {
  const int c = blockIdx.x * kBX + threadIdx.x, r = blockIdx.y * kBY + threadIdx.y;
  if (r >= N || c >= N) return;
  const int n = N - 1, M = N + 2;
  const int b = blockIdx.z;
  const T* ub = u + (long long)b * N * N;
  auto wrap = [n](int x) { return x < 0 ? x + n : (x >= n ? x - n : x); };
  T acc = 0;
#pragma unroll
  for (int dr = 0; dr < 3; ++dr) {
    const long long row = (long long)wrap(r + dr - 1) * N;
#pragma unroll
    for (int dc = 0; dc < 3; ++dc) acc += ktab[dr * 3 + dc] * ub[row + wrap(c + dc - 1)];
  }
  const T res = f[(long long)b * M * M + (long long)(r + 1) * M + (c + 1)] - acc;
  out[(long long)b * N * N + (long long)r * N + c] = omd[0] * res + ub[(long long)wrap(r) * N + wrap(c)];
}

// Circular extension of the periodic part u[:-1, :-1] (period n = N - 1) to (n + lo + hi)^2:
// dst(i, j) = u((i - lo) mod n, (j - lo) mod n).  lo = 1, hi = 2: pbc_boundary (jacobi.py:72-79);
// lo = 0, hi = 1: reset_boundary (:81-84).
template <typename T>
__global__ __launch_bounds__(256) void k_pbc_pad(const T* __restrict__ u, T* __restrict__ dst, int N, int lo,
                                                 int M) {
  const int c = blockIdx.x * kBX + threadIdx.x, r = blockIdx.y * kBY + threadIdx.y;
  if (r >= M || c >= M) return;
  const int n = N - 1;
  const int b = blockIdx.z;
  const int sr = ((r - lo) % n + n) % n, sc = ((c - lo) % n + n) % n;
  dst[(long long)b * M * M + (long long)r * M + c] = u[(long long)b * N * N + (long long)sr * N + sc];
}

template <typename T>
__global__ __launch_bounds__(256) void k_residual(const T* __restrict__ u, const T* __restrict__ f,
                                                  T* __restrict__ res, const uint8_t* __restrict__ pid,
                                                  const T* __restrict__ ktab, int ntab, int H, int W) {
  __shared__ T tab[FEA_MAX_PATTERNS * 9];
  load_table(tab, ktab, ntab * 9);
  __syncthreads();
  const int c = blockIdx.x * kBX + threadIdx.x, r = blockIdx.y * kBY + threadIdx.y;
  if (r >= H || c >= W) return;
  const long long HW = (long long)H * W;
  const T* ub = u + blockIdx.z * HW;
  T acc = 0;
#pragma unroll
  for (int dr = 0; dr < 3; ++dr) {
    const int rr = r + dr - 1;
    if (rr < 0 || rr >= H) continue;
#pragma unroll
    for (int dc = 0; dc < 3; ++dc) {
      const int cc = c + dc - 1;
      if (cc < 0 || cc >= W) continue;
      const int p = pid ? pid[rr * W + cc] : 0;
      acc += tab[p * 9 + dr * 3 + dc] * ub[(long long)rr * W + cc];
    }
  }
  const long long i = blockIdx.z * HW + (long long)r * W + c;
  res[i] = f[i] - acc;
}

// fc = w0 * pad0(conv2d(x[..,1:-1,1:-1], R, stride 2)); C>1: split input, channel kernels.
template <typename T>
__global__ __launch_bounds__(256) void k_restrict(const T* __restrict__ x, int C, T* __restrict__ fc,
                                                  const uint8_t* __restrict__ pid, const T* __restrict__ rtab,
                                                  int ntab, T w0, int H, int W) {
  __shared__ T tab[FEA_MAX_PATTERNS * 9];
  load_table(tab, rtab, ntab * 9);
  __syncthreads();
  const int Hc = (H + 1) / 2, Wc = (W + 1) / 2;
  const int J = blockIdx.x * kBX + threadIdx.x, I = blockIdx.y * kBY + threadIdx.y;
  if (I >= Hc || J >= Wc) return;
  const long long HW = (long long)H * W;
  T acc = 0;
  if (I > 0 && I < Hc - 1 && J > 0 && J < Wc - 1) {
    const T* xb = x + (long long)blockIdx.z * C * HW;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const long long j = (long long)(2 * I - 1 + ky) * W + (2 * J - 1 + kx);
        if (C == 1) {
          const int p = pid ? pid[j] : 0;
          acc += tab[p * 9 + ky * 3 + kx] * xb[j];
        } else {
          for (int ch = 0; ch < C; ++ch) acc += tab[ch * 9 + ky * 3 + kx] * xb[ch * HW + j];
        }
      }
    }
    acc = w0 * acc;
  }
  fc[(long long)blockIdx.z * Hc * Wc + (long long)I * Wc + J] = acc;
}

// out = add + w1 * conv_transpose2d(e, P, stride 2, pad 1)
template <typename T>
__global__ __launch_bounds__(256) void k_prolong(const T* __restrict__ e, int C, T* __restrict__ out,
                                                 const T* __restrict__ add, const uint8_t* __restrict__ pidc,
                                                 const T* __restrict__ ptab, int ntab, T w1, int Hc, int Wc) {
  __shared__ T tab[FEA_MAX_PATTERNS * 9];
  load_table(tab, ptab, ntab * 9);
  __syncthreads();
  const int H = 2 * Hc - 1, W = 2 * Wc - 1;
  const int x = blockIdx.x * kBX + threadIdx.x, y = blockIdx.y * kBY + threadIdx.y;
  if (y >= H || x >= W) return;
  const long long HWc = (long long)Hc * Wc;
  const T* eb = e + (long long)blockIdx.z * C * HWc;
  T acc = 0;
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
    const int ty = y + 1 - ky;
    if (ty & 1) continue;
    const int a = ty >> 1;
    if (a < 0 || a >= Hc) continue;
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      const int tx = x + 1 - kx;
      if (tx & 1) continue;
      const int bb = tx >> 1;
      if (bb < 0 || bb >= Wc) continue;
      const long long j = (long long)a * Wc + bb;
      if (C == 1) {
        const int p = pidc ? pidc[j] : 0;
        acc += tab[p * 9 + ky * 3 + kx] * eb[j];
      } else {
        for (int ch = 0; ch < C; ++ch) acc += tab[ch * 9 + ky * 3 + kx] * eb[ch * HWc + j];
      }
    }
  }
  const long long i = (long long)blockIdx.z * H * W + (long long)y * W + x;
  const T v = w1 * acc;
  out[i] = add ? add[i] + v : v;
}

// Per-block partial sums of r^2 over the interior; r = f - K u (or u itself when f == NULL).
template <typename T>
__global__ __launch_bounds__(256) void k_norm_partial(const T* __restrict__ u, const T* __restrict__ f,
                                                      const uint8_t* __restrict__ pid,
                                                      const T* __restrict__ ktab, int ntab,
                                                      double* __restrict__ part, int H, int W) {
  __shared__ T tab[FEA_MAX_PATTERNS * 9];
  __shared__ double wsum[4];
  if (ktab) load_table(tab, ktab, ntab * 9);
  __syncthreads();
  const int c = blockIdx.x * kBX + threadIdx.x, r = blockIdx.y * kBY + threadIdx.y;
  double s = 0.0;
  if (r > 0 && r < H - 1 && c > 0 && c < W - 1) {
    const long long HW = (long long)H * W;
    const T* ub = u + blockIdx.z * HW;
    T v;
    if (f) {
      T acc = 0;
#pragma unroll
      for (int dr = 0; dr < 3; ++dr)
#pragma unroll
        for (int dc = 0; dc < 3; ++dc) {
          const long long j = (long long)(r + dr - 1) * W + (c + dc - 1);
          const int p = pid ? pid[j] : 0;
          acc += tab[p * 9 + dr * 3 + dc] * ub[j];
        }
      v = f[blockIdx.z * HW + (long long)r * W + c] - acc;
    } else {
      v = ub[(long long)r * W + c];
    }
    s = (double)v * (double)v;
  }
  s = wave_sum(s);
  if (lane_id() == 0) wsum[threadIdx.y] = s;
  __syncthreads();
  if (threadIdx.x == 0 && threadIdx.y == 0) {
    const long long nb = (long long)gridDim.x * gridDim.y;
    part[blockIdx.z * nb + (long long)blockIdx.y * gridDim.x + blockIdx.x] = ((wsum[0] + wsum[1]) + wsum[2]) + wsum[3];
  }
}

// ---------------------------------------------------------------------------
// Adjoints for autograd (MultiGrid.forward / qm training, FEANet/multigrid.py:132-157)
// ---------------------------------------------------------------------------
// K^T g: y = K u has y[i] = sum_d W_{p(i+d)}[d] u[i+d], so (K^T g)[j] = sum_d W_{p(j)}[d] g[j-d].
template <typename T>
__global__ __launch_bounds__(256) void k_knet_adj(const T* __restrict__ g, T* __restrict__ out,
                                                  const uint8_t* __restrict__ pid, const T* __restrict__ ktab,
                                                  int ntab, int H, int W) {
  __shared__ T tab[FEA_MAX_PATTERNS * 9];
  load_table(tab, ktab, ntab * 9);
  __syncthreads();
  const int c = blockIdx.x * kBX + threadIdx.x, r = blockIdx.y * kBY + threadIdx.y;
  if (r >= H || c >= W) return;
  const long long HW = (long long)H * W;
  const T* gb = g + blockIdx.z * HW;
  const int p = pid ? pid[(long long)r * W + c] : 0;
  T acc = 0;
#pragma unroll
  for (int dr = 0; dr < 3; ++dr) {
    const int rr = r - (dr - 1);
    if (rr < 0 || rr >= H) continue;
#pragma unroll
    for (int dc = 0; dc < 3; ++dc) {
      const int cc = c - (dc - 1);
      if (cc < 0 || cc >= W) continue;
      acc += tab[p * 9 + dr * 3 + dc] * gb[(long long)rr * W + cc];
    }
  }
  out[blockIdx.z * HW + (long long)r * W + c] = acc;
}

// Jacobi-sweep adjoint (k_jacobi above; bc carries no gradient).  With g' = geo . g:
//   grad_f = omd . g'          grad_u = geo . (g' - K^T grad_f)
template <typename T>
__global__ __launch_bounds__(256) void k_jacobi_adj(const T* __restrict__ g, T* __restrict__ gu, T* __restrict__ gf,
                                                    const uint8_t* __restrict__ pid, const T* __restrict__ ktab,
                                                    const T* __restrict__ omd, int ntab, const T* __restrict__ geo,
                                                    long long geo_bs, int H, int W) {
  __shared__ T tab[FEA_MAX_PATTERNS * 10];
  for (int i = threadIdx.y * blockDim.x + threadIdx.x; i < ntab * 10; i += blockDim.x * blockDim.y)
    tab[i] = (i % 10 == 9) ? omd[i / 10] : ktab[(i / 10) * 9 + (i % 10)];
  __syncthreads();
  const int c = blockIdx.x * kBX + threadIdx.x, r = blockIdx.y * kBY + threadIdx.y;
  if (r >= H || c >= W) return;
  const long long HW = (long long)H * W;
  const T* gb = g + blockIdx.z * HW;
  const T* geob = geo ? geo + blockIdx.z * geo_bs : nullptr;
  auto gm = [&](long long j, int rr, int cc) -> T {
    return geob ? geob[j] : T((rr > 0 && rr < H - 1 && cc > 0 && cc < W - 1) ? 1 : 0);
  };
  const long long i = (long long)r * W + c;
  const int p = pid ? pid[i] : 0;
  T acc = 0;
#pragma unroll
  for (int dr = 0; dr < 3; ++dr) {
    const int rr = r - (dr - 1);
    if (rr < 0 || rr >= H) continue;
#pragma unroll
    for (int dc = 0; dc < 3; ++dc) {
      const int cc = c - (dc - 1);
      if (cc < 0 || cc >= W) continue;
      const long long j = (long long)rr * W + cc;
      const int q = pid ? pid[j] : 0;
      acc += tab[p * 10 + dr * 3 + dc] * (tab[q * 10 + 9] * (gm(j, rr, cc) * gb[j]));
    }
  }
  const T gi = gm(i, r, c);
  const T g1 = gi * gb[i];
  gu[blockIdx.z * HW + i] = gi * (g1 - acc);
  if (gf) gf[blockIdx.z * HW + i] = tab[p * 10 + 9] * g1;
}

// Restriction adjoint w.r.t. its (split, C-channel) input: gx[ch][y][x] = w0 * sum over interior coarse
// (I, J) whose 3x3 window holds (y, x) of R_ch[y-2I+1][x-2J+1] * g[I][J]  (C == 1: kernel by pid).
template <typename T>
__global__ __launch_bounds__(256) void k_restrict_adj(const T* __restrict__ g, int C, T* __restrict__ gx,
                                                      const uint8_t* __restrict__ pid, const T* __restrict__ rtab,
                                                      int ntab, T w0, int H, int W) {
  __shared__ T tab[FEA_MAX_PATTERNS * 9];
  load_table(tab, rtab, ntab * 9);
  __syncthreads();
  const int Hc = (H + 1) / 2, Wc = (W + 1) / 2;
  const int x = blockIdx.x * kBX + threadIdx.x, y = blockIdx.y * kBY + threadIdx.y;
  if (y >= H || x >= W) return;
  const long long HW = (long long)H * W;
  const T* gb = g + (long long)blockIdx.z * Hc * Wc;
  const int p = (C == 1 && pid) ? pid[(long long)y * W + x] : 0;
  for (int ch = 0; ch < C; ++ch) {
    const int t = C == 1 ? p : ch;
    T acc = 0;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int ty = y + 1 - ky;  // = 2I
      if (ty & 1) continue;
      const int I = ty >> 1;
      if (I < 1 || I > Hc - 2) continue;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int tx = x + 1 - kx;
        if (tx & 1) continue;
        const int J = tx >> 1;
        if (J < 1 || J > Wc - 2) continue;
        acc += tab[t * 9 + ky * 3 + kx] * gb[(long long)I * Wc + J];
      }
    }
    gx[((long long)blockIdx.z * C + ch) * HW + (long long)y * W + x] = w0 * acc;
  }
}

// Prolongation adjoint w.r.t. its (split, C-channel) input: ge[ch][a][b] = w1 * sum_k P_ch[k] *
// g[2a-1+ky][2b-1+kx] over fine nodes inside the grid  (C == 1: kernel by the coarse pid).
template <typename T>
__global__ __launch_bounds__(256) void k_prolong_adj(const T* __restrict__ g, int C, T* __restrict__ ge,
                                                     const uint8_t* __restrict__ pidc, const T* __restrict__ ptab,
                                                     int ntab, T w1, int Hc, int Wc) {
  __shared__ T tab[FEA_MAX_PATTERNS * 9];
  load_table(tab, ptab, ntab * 9);
  __syncthreads();
  const int H = 2 * Hc - 1, W = 2 * Wc - 1;
  const int b = blockIdx.x * kBX + threadIdx.x, a = blockIdx.y * kBY + threadIdx.y;
  if (a >= Hc || b >= Wc) return;
  const long long HWc = (long long)Hc * Wc;
  const T* gb = g + (long long)blockIdx.z * H * W;
  const int p = (C == 1 && pidc) ? pidc[(long long)a * Wc + b] : 0;
  for (int ch = 0; ch < C; ++ch) {
    const int t = C == 1 ? p : ch;
    T acc = 0;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int y = 2 * a - 1 + ky;
      if (y < 0 || y >= H) continue;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int x = 2 * b - 1 + kx;
        if (x < 0 || x >= W) continue;
        acc += tab[t * 9 + ky * 3 + kx] * gb[(long long)y * W + x];
      }
    }
    ge[((long long)blockIdx.z * C + ch) * HWc + (long long)a * Wc + b] = w1 * acc;
  }
}

// Gradient of the 3x3 inter-grid kernels: per block partial sums of
//   gw[ch][k] = sum_{(a, b)} cf[chc][a][b] * ff[chf][2a-1+ky][2b-1+kx]
// over coarse (a, b) in [a0, Hc-a0) x [a0, Wc-a0) (a0 = 1: restriction interior, 0: prolongation),
// fine indices outside the grid contribute 0; chc = ch if c_split else 0, chf likewise.
template <typename T>
__global__ __launch_bounds__(256) void k_tapgrad_partial(const T* __restrict__ cf, int c_split,
                                                         const T* __restrict__ ff, int f_split, int C, int a0,
                                                         int Hc, int Wc, double* __restrict__ part) {
  __shared__ double red[kBY][FEA_MAX_PATTERNS * 9];
  const int H = 2 * Hc - 1, W = 2 * Wc - 1;
  const int b = blockIdx.x * kBX + threadIdx.x, a = blockIdx.y * kBY + threadIdx.y;
  const bool in = a >= a0 && a < Hc - a0 && b >= a0 && b < Wc - a0;
  const long long HWc = (long long)Hc * Wc, HW = (long long)H * W;
  for (int ch = 0; ch < C; ++ch) {
    const T* cb = cf + ((long long)blockIdx.z * (c_split ? C : 1) + (c_split ? ch : 0)) * HWc;
    const T* fb = ff + ((long long)blockIdx.z * (f_split ? C : 1) + (f_split ? ch : 0)) * HW;
    const double cv = in ? (double)cb[(long long)a * Wc + b] : 0.0;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const int y = 2 * a - 1 + k / 3, x = 2 * b - 1 + k % 3;
      double v = 0.0;
      if (in && y >= 0 && y < H && x >= 0 && x < W) v = cv * (double)fb[(long long)y * W + x];
      v = wave_sum(v);
      if (lane_id() == 0) red[threadIdx.y][ch * 9 + k] = v;
    }
  }
  __syncthreads();
  const int tid = threadIdx.y * kBX + threadIdx.x;
  const long long nb = (long long)gridDim.x * gridDim.y * gridDim.z;
  const long long blk = ((long long)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
  for (int i = tid; i < C * 9; i += kBX * kBY)
    part[(long long)i * nb + blk] = ((red[0][i] + red[1][i]) + red[2][i]) + red[3][i];
}

// Gradient of the per-pattern stencils of y = K u (k_knet): per block partial sums of
//   gw[p][d] = sum_i g[i] * u[i+d] * [pid(i+d) == p]      (zero padding; pid == NULL: p = 0)
// Also the weight gradient of conv3x3 (FNet, HNet layers): ntab = 1, no pid.
template <typename T>
__global__ __launch_bounds__(256) void k_stencil_wgrad_partial(const T* __restrict__ g, const T* __restrict__ u,
                                                               const uint8_t* __restrict__ pid, int ntab, int H,
                                                               int W, double* __restrict__ part) {
  __shared__ double red[kBY][FEA_MAX_PATTERNS * 9];
  const int c = blockIdx.x * kBX + threadIdx.x, r = blockIdx.y * kBY + threadIdx.y;
  const bool in = r < H && c < W;
  const long long HW = (long long)H * W;
  const T* gb = g + blockIdx.z * HW;
  const T* ub = u + blockIdx.z * HW;
  const double gi = in ? (double)gb[(long long)r * W + c] : 0.0;
#pragma unroll
  for (int d = 0; d < 9; ++d) {
    const int rr = r + d / 3 - 1, cc = c + d % 3 - 1;
    const bool ok = in && rr >= 0 && rr < H && cc >= 0 && cc < W;
    const long long j = (long long)rr * W + cc;
    const double v = ok ? gi * (double)ub[j] : 0.0;
    const int pj = (ok && pid) ? pid[j] : 0;
    for (int p = 0; p < ntab; ++p) {
      const double s = wave_sum(pj == p ? v : 0.0);
      if (lane_id() == 0) red[threadIdx.y][p * 9 + d] = s;
    }
  }
  __syncthreads();
  const int tid = threadIdx.y * kBX + threadIdx.x;
  const long long nb = (long long)gridDim.x * gridDim.y * gridDim.z;
  const long long blk = ((long long)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
  for (int i = tid; i < ntab * 9; i += kBX * kBY)
    part[(long long)i * nb + blk] = ((red[0][i] + red[1][i]) + red[2][i]) + red[3][i];
}

// Fixed-order sum of the partials of each of the n outputs (one block per output).
template <typename T>
__global__ __launch_bounds__(256) void k_tapgrad_final(const double* __restrict__ part, long long nb, T scale,
                                                       T* __restrict__ out) {
  __shared__ double sh[256];
  const double* p = part + blockIdx.x * nb;
  double s = 0.0;
  for (long long i = threadIdx.x; i < nb; i += 256) s += p[i];
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) sh[threadIdx.x] += sh[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[blockIdx.x] = (T)((double)scale * sh[0]);
}

}  // namespace fea

using namespace fea;

static inline dim3 grid_for(int H, int W, int B) { return dim3((W + kBX - 1) / kBX, (H + kBY - 1) / kBY, B); }
static inline bool bad_shape(int B, int H, int W) { return B <= 0 || H <= 0 || W <= 0 || B > 65535; }

#define FEA_GENERIC_API(SUF, T)                                                                          \
  extern "C" int fea_knet_apply_##SUF(const T* u, T* y, const uint8_t* pid, const T* ktab, int ntab, int B, \
                                      int H, int W, void* stream) {                                      \
    if (!u || !y || !ktab || ntab < 1 || ntab > FEA_MAX_PATTERNS || bad_shape(B, H, W)) return FEA_EINVAL; \
    k_knet<T><<<grid_for(H, W, B), dim3(kBX, kBY), 0, (hipStream_t)stream>>>(u, y, pid, ktab, ntab, H, W); \
    FEA_LAUNCH_CHECK();                                                                                  \
  }                                                                                                      \
  extern "C" int fea_split_x_##SUF(const T* x, T* xs, const uint8_t* pid, int C, int B, int H, int W,   \
                                   void* stream) {                                                       \
    if (!x || !xs || C < 1 || bad_shape(B, H, W)) return FEA_EINVAL;                                     \
    k_split<T><<<grid_for(H, W, B), dim3(kBX, kBY), 0, (hipStream_t)stream>>>(x, xs, pid, C, H, W);       \
    FEA_LAUNCH_CHECK();                                                                                  \
  }                                                                                                      \
  extern "C" int fea_jacobi_sweep_##SUF(const T* u, const T* f, T* out, const uint8_t* pid, const T* ktab, \
                                        const T* omd, int ntab, const T* geo, long long geo_bs,          \
                                        const T* bc, long long bc_bs, int B, int H, int W, void* stream) { \
    if (!u || !f || !out || !ktab || !omd || ntab < 1 || ntab > FEA_MAX_PATTERNS || bad_shape(B, H, W))  \
      return FEA_EINVAL;                                                                                 \
    if (out == u) return FEA_EINVAL;                                                                     \
    k_jacobi<T><<<grid_for(H, W, B), dim3(kBX, kBY), 0, (hipStream_t)stream>>>(u, f, out, pid, ktab, omd, \
                                                                                ntab, geo, geo_bs, bc,   \
                                                                                bc_bs, H, W);            \
    FEA_LAUNCH_CHECK();                                                                                  \
  }                                                                                                      \
  extern "C" int fea_jacobi_sweep_pbc_##SUF(const T* u, const T* f, T* out, const T* ktab, const T* omd,  \
                                            int B, int N, void* stream) {                                \
    if (!u || !f || !out || !ktab || !omd || out == u || bad_shape(B, N, N)) return FEA_EINVAL;          \
    k_jacobi_pbc<T><<<grid_for(N, N, B), dim3(kBX, kBY), 0, (hipStream_t)stream>>>(u, f, out, ktab, omd, N); \
    FEA_LAUNCH_CHECK();                                                                                  \
  }                                                                                                      \
  extern "C" int fea_pbc_pad_##SUF(const T* u, T* dst, int B, int N, int lo, int hi, void* stream) {     \
    if (!u || !dst || lo < 0 || hi < 0 || lo + hi > 64 || bad_shape(B, N, N)) return FEA_EINVAL;         \
    const int M = N - 1 + lo + hi;                                                                       \
    k_pbc_pad<T><<<grid_for(M, M, B), dim3(kBX, kBY), 0, (hipStream_t)stream>>>(u, dst, N, lo, M);        \
    FEA_LAUNCH_CHECK();                                                                                  \
  }                                                                                                      \
  extern "C" int fea_residual_##SUF(const T* u, const T* f, T* r, const uint8_t* pid, const T* ktab,    \
                                    int ntab, int B, int H, int W, void* stream) {                       \
    if (!u || !f || !r || !ktab || ntab < 1 || ntab > FEA_MAX_PATTERNS || bad_shape(B, H, W))            \
      return FEA_EINVAL;                                                                                 \
    k_residual<T><<<grid_for(H, W, B), dim3(kBX, kBY), 0, (hipStream_t)stream>>>(u, f, r, pid, ktab, ntab, \
                                                                                  H, W);                 \
    FEA_LAUNCH_CHECK();                                                                                  \
  }                                                                                                      \
  extern "C" int fea_restrict_##SUF(const T* x, int C, T* fc, const uint8_t* pid, const T* rtab, int ntab, \
                                    T w0, int B, int H, int W, void* stream) {                           \
    if (!x || !fc || !rtab || C < 1 || bad_shape(B, H, W) || H < 3 || W < 3 || !(H & 1) || !(W & 1))      \
      return FEA_EINVAL;                                                                                 \
    if ((C == 1 && (ntab < 1 || ntab > FEA_MAX_PATTERNS)) || (C > 1 && (ntab != C || C > FEA_MAX_PATTERNS))) \
      return FEA_EINVAL;                                                                                 \
    const int Hc = (H + 1) / 2, Wc = (W + 1) / 2;                                                        \
    k_restrict<T><<<grid_for(Hc, Wc, B), dim3(kBX, kBY), 0, (hipStream_t)stream>>>(x, C, fc, pid, rtab,  \
                                                                                    ntab, w0, H, W);     \
    FEA_LAUNCH_CHECK();                                                                                  \
  }                                                                                                      \
  extern "C" int fea_prolong_##SUF(const T* e, int C, T* out, const T* add, const uint8_t* pidc,          \
                                   const T* ptab, int ntab, T w1, int B, int Hc, int Wc, void* stream) { \
    if (!e || !out || !ptab || C < 1 || bad_shape(B, Hc, Wc) || Hc < 2 || Wc < 2) return FEA_EINVAL;     \
    if ((C == 1 && (ntab < 1 || ntab > FEA_MAX_PATTERNS)) || (C > 1 && (ntab != C || C > FEA_MAX_PATTERNS))) \
      return FEA_EINVAL;                                                                                 \
    k_prolong<T><<<grid_for(2 * Hc - 1, 2 * Wc - 1, B), dim3(kBX, kBY), 0, (hipStream_t)stream>>>(       \
        e, C, out, add, pidc, ptab, ntab, w1, Hc, Wc);                                                   \
    FEA_LAUNCH_CHECK();                                                                                  \
  }                                                                                                      \
  extern "C" int fea_residual_norm_##SUF(const T* u, const T* f, const uint8_t* pid, const T* ktab,     \
                                         int ntab, double* out, double* ws, int B, int H, int W,         \
                                         void* stream) {                                                 \
    if (!u || !out || !ws || bad_shape(B, H, W) || H < 3 || W < 3) return FEA_EINVAL;                     \
    if (f && (!ktab || ntab < 1 || ntab > FEA_MAX_PATTERNS)) return FEA_EINVAL;                           \
    const dim3 g = grid_for(H, W, B);                                                                    \
    k_norm_partial<T><<<g, dim3(kBX, kBY), 0, (hipStream_t)stream>>>(u, f, pid, f ? ktab : nullptr, ntab, \
                                                                      ws, H, W);                         \
    k_norm_final<<<B, 256, 0, (hipStream_t)stream>>>(ws, (long long)g.x * g.y, out);                  \
    FEA_LAUNCH_CHECK();                                                                                  \
  }

#define FEA_ADJOINT_API(SUF, T)                                                                          \
  extern "C" int fea_knet_apply_adj_##SUF(const T* g, T* out, const uint8_t* pid, const T* ktab, int ntab,  \
                                          int B, int H, int W, void* stream) {                           \
    if (!g || !out || !ktab || ntab < 1 || ntab > FEA_MAX_PATTERNS || bad_shape(B, H, W) || g == out)     \
      return FEA_EINVAL;                                                                                 \
    k_knet_adj<T><<<grid_for(H, W, B), dim3(kBX, kBY), 0, (hipStream_t)stream>>>(g, out, pid, ktab, ntab,  \
                                                                                  H, W);                 \
    FEA_LAUNCH_CHECK();                                                                                  \
  }                                                                                                      \
  extern "C" int fea_jacobi_sweep_adj_##SUF(const T* g, T* gu, T* gf, const uint8_t* pid, const T* ktab,    \
                                            const T* omd, int ntab, const T* geo, long long geo_bs, int B,   \
                                            int H, int W, void* stream) {                                    \
    if (!g || !gu || !ktab || !omd || ntab < 1 || ntab > FEA_MAX_PATTERNS || bad_shape(B, H, W) || g == gu ||  \
        g == gf)                                                                                            \
      return FEA_EINVAL;                                                                                     \
    k_jacobi_adj<T><<<grid_for(H, W, B), dim3(kBX, kBY), 0, (hipStream_t)stream>>>(g, gu, gf, pid, ktab, omd,  \
                                                                                    ntab, geo, geo_bs, H, W); \
    FEA_LAUNCH_CHECK();                                                                                      \
  }                                                                                                          \
  extern "C" int fea_restrict_adj_##SUF(const T* g, int C, T* gx, const uint8_t* pid, const T* rtab,     \
                                        int ntab, T w0, int B, int H, int W, void* stream) {             \
    if (!g || !gx || !rtab || C < 1 || bad_shape(B, H, W) || H < 3 || W < 3 || !(H & 1) || !(W & 1))      \
      return FEA_EINVAL;                                                                                 \
    if ((C == 1 && (ntab < 1 || ntab > FEA_MAX_PATTERNS)) || (C > 1 && (ntab != C || C > FEA_MAX_PATTERNS))) \
      return FEA_EINVAL;                                                                                 \
    k_restrict_adj<T><<<grid_for(H, W, B), dim3(kBX, kBY), 0, (hipStream_t)stream>>>(g, C, gx, pid, rtab, \
                                                                                      ntab, w0, H, W);   \
    FEA_LAUNCH_CHECK();                                                                                  \
  }                                                                                                      \
  extern "C" int fea_prolong_adj_##SUF(const T* g, int C, T* ge, const uint8_t* pidc, const T* ptab,     \
                                       int ntab, T w1, int B, int Hc, int Wc, void* stream) {            \
    if (!g || !ge || !ptab || C < 1 || bad_shape(B, Hc, Wc) || Hc < 2 || Wc < 2) return FEA_EINVAL;      \
    if ((C == 1 && (ntab < 1 || ntab > FEA_MAX_PATTERNS)) || (C > 1 && (ntab != C || C > FEA_MAX_PATTERNS))) \
      return FEA_EINVAL;                                                                                 \
    k_prolong_adj<T><<<grid_for(Hc, Wc, B), dim3(kBX, kBY), 0, (hipStream_t)stream>>>(g, C, ge, pidc, ptab, \
                                                                                      ntab, w1, Hc, Wc); \
    FEA_LAUNCH_CHECK();                                                                                  \
  }                                                                                                      \
  extern "C" int fea_transfer_weight_grad_##SUF(const T* cf, int c_split, const T* ff, int f_split, int C,  \
                                                int interior, T scale, T* gw, double* ws, int B, int Hc,   \
                                                int Wc, void* stream) {                                  \
    if (!cf || !ff || !gw || !ws || C < 1 || C > FEA_MAX_PATTERNS || bad_shape(B, Hc, Wc) || Hc < 2 || Wc < 2) \
      return FEA_EINVAL;                                                                                 \
    const dim3 gr = grid_for(Hc, Wc, B);                                                                 \
    k_tapgrad_partial<T><<<gr, dim3(kBX, kBY), 0, (hipStream_t)stream>>>(cf, c_split, ff, f_split, C,    \
                                                                          interior ? 1 : 0, Hc, Wc, ws);  \
    k_tapgrad_final<T><<<C * 9, 256, 0, (hipStream_t)stream>>>(ws, (long long)gr.x * gr.y * gr.z, scale, gw); \
    FEA_LAUNCH_CHECK();                                                                                  \
  }                                                                                                      \
  extern "C" int fea_stencil_weight_grad_##SUF(const T* g, const T* u, const uint8_t* pid, int ntab, T scale, \
                                               T* gw, double* ws, int B, int H, int W, void* stream) {      \
    if (!g || !u || !gw || !ws || ntab < 1 || ntab > FEA_MAX_PATTERNS || bad_shape(B, H, W)) return FEA_EINVAL; \
    const dim3 gr = grid_for(H, W, B);                                                                   \
    k_stencil_wgrad_partial<T><<<gr, dim3(kBX, kBY), 0, (hipStream_t)stream>>>(g, u, pid, ntab, H, W, ws); \
    k_tapgrad_final<T><<<ntab * 9, 256, 0, (hipStream_t)stream>>>(ws, (long long)gr.x * gr.y * gr.z, scale, gw); \
    FEA_LAUNCH_CHECK();                                                                                  \
  }                                                                                                      \
  extern "C" size_t fea_stencil_weight_grad_ws_bytes_##SUF(int ntab, int B, int H, int W) {              \
    const dim3 gr = grid_for(H, W, B);                                                                   \
    return (size_t)ntab * 9 * gr.x * gr.y * gr.z * sizeof(double);                                       \
  }                                                                                                      \
  extern "C" size_t fea_transfer_weight_grad_ws_bytes_##SUF(int C, int B, int Hc, int Wc) {              \
    const dim3 gr = grid_for(Hc, Wc, B);                                                                 \
    return (size_t)C * 9 * gr.x * gr.y * gr.z * sizeof(double);                                          \
  }

FEA_GENERIC_API(f32, float)
FEA_GENERIC_API(f64, double)
FEA_ADJOINT_API(f32, float)
FEA_ADJOINT_API(f64, double)
