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
#ifdef FEA_TAIL_TRACE
#define FEA_TAIL_TRACE_ON
#endif
#include "fea_common.h"

#ifdef FEA_TAIL_TRACE_ON  // lab builds only (tools/lab/tail_lab.py): a timestamp after every barrier
namespace fea {
__device__ long long g_tail_trace[256];
}  // namespace fea
#define FEA_TAIL_SYNC()                                                                     \
  do {                                                                                      \
    __syncthreads();                                                                        \
    if (threadIdx.x == 0 && blockIdx.x == 0 && nph < 256) fea::g_tail_trace[nph] = clock64(); \
    ++nph;                                                                                  \
  } while (0)
#endif
#include "tail_core.h"

namespace fea {

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
#ifdef FEA_TAIL_TRACE_ON
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
    if (MULTI) FEA_TAIL_SYNC();
    tail_fast<T, MULTI, 65, 6>(a, va, fs, ktb, rtb, ptb, pl, wv, lane, TailOut<T>{(int)blockIdx.x}
#ifdef FEA_TAIL_TRACE_ON
                               , nph
#endif
    );
    return;
  } else if (fast) {
    if (MULTI || nlev == 1) FEA_TAIL_SYNC();
    tail_fast<T, MULTI>(a, va, fs, ktb, rtb, ptb, pl, wv, lane, TailOut<T>{(int)blockIdx.x}
#ifdef FEA_TAIL_TRACE_ON
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

#ifdef FEA_TAIL_TRACE_ON
extern "C" int fea_tail_trace_read(long long* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_tail_trace), sizeof(long long) * 256, 0, hipMemcpyDeviceToHost);
}
#endif
