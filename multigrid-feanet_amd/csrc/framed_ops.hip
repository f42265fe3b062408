// framed_ops.hip — bandwidth-optimised multigrid level kernels on solver-owned FRAMED buffers.
//
// Layout (see include/feanet_hip.h): node (r, c) of sample b at
//     base[b*bstride + (r+1)*ld + OFF + c],   OFF = A-1,  A = 128/sizeof(T)
// so interior column 1 starts a 128-byte line and every 16-byte lane vector is aligned.
//
// Work decomposition ("column strip x row march", one wave = one independent task):
//   * a wave owns a strip of SW = 64*VEC fine columns starting at c0 = 1 + s*SW (lane l holds
//     columns c0 + VEC*l .. +VEC-1, VEC = 16/sizeof(T): one 16-byte load per lane per row, the
//     whole row segment is one 1 KiB coalesced request);
//   * it marches down RB rows keeping a 3-row window of the field in registers, so every input
//     byte is read from HBM once (plus a 2-row / 2-line halo per task);
//   * x-neighbours come from the adjacent lane via DPP wave_shr:1 / wave_shl:1; the two lanes at
//     the strip edges take them from a 16-byte halo load (a line the neighbouring wave of the same
//     block also reads, so it is an L1/L2 hit);
//   * no LDS, no barriers in the stencil path (LDS only holds the <=16-pattern coefficient tables
//     of the two-material problem), 4 independent waves per 256-thread block, XCD-aware block
//     order so row-adjacent tasks share an L2.
// Roofline: these kernels are HBM-bound (~0.9 flop/byte in fp64); algorithmic bytes per fine node
// are documented in DESIGN.md (sweep 24 B, residual+restrict 18 B, prolong+sweep 26 B in fp64).
#include <cstdlib>

#include "fea_common.h"

#include <type_traits>
#include <utility>

namespace fea {

template <typename T>
struct Frame {
  static constexpr int A = 128 / (int)sizeof(T);
  static constexpr int OFF = A - 1;
  static constexpr int VEC = 16 / (int)sizeof(T);
  static constexpr int SW = kWave * VEC;
};
constexpr int kRB = 32;     // fine rows per task (even: tasks start on odd rows)
constexpr int kWaves = 4;   // waves (tasks) per block
constexpr int kTabStride = 10;  // LDS table row: 9 stencil weights + omega/d
// Pattern windows (PRow, CRow::o, the prolongation's pe) hold BYTE offsets of a pattern's LDS table row
// (pattern * kTabStride * sizeof(T)), so a table read is one ds_read at that address
// plus the tap as an immediate offset, with no per-read index scaling
template <typename T>
__host__ __device__ constexpr int tab_row_bytes() { return kTabStride * (int)sizeof(T); }
template <typename T>
__device__ __forceinline__ T tabv(const T* t, int off, int d) {
  return *reinterpret_cast<const T*>(reinterpret_cast<const char*>(t) + off + d * (int)sizeof(T));
}
// The restricted field f_c (a quarter of the level's bytes) is stored with normal stores even when
// the level's own stores stream past the caches: the next kernel (the coarse level's restriction)
// reads it straight back, from the Infinity Cache instead of HBM.
#ifndef FEA_COARSE_NT
#define FEA_COARSE_NT 0
#endif
constexpr bool kCoarseNT = FEA_COARSE_NT != 0;

static inline int div_up(int a, int b) { return (a + b - 1) / b; }

template <typename T>
static inline int mg_nstrips(int W) { return div_up(W - 2, Frame<T>::SW); }

// row pitch (elements) of a framed grid with W columns
template <typename T>
static inline int mg_ld(int W) {
  using F = Frame<T>;
  // room for the last strip's loads: plain strips (k * SW + halo) and the overlapped strips of
  // k_mg_sweep_restrict / k_mg_cycle_join (start <= W - 2, 64*VEC columns)
  // (any strip starts at a column <= W - 2, so W + 2*SW columns cover every variant's last loads)
  const int need = F::OFF + 2 + std::max(mg_nstrips<T>(W) * F::SW + F::VEC, W + 2 * F::SW);
  return div_up(need, F::A) * F::A;
}

// sample pitch of an H x W framed grid: H rows plus the ghost rows -1 and H
template <typename T>
static inline long long mg_bstride(int H, int W) { return (long long)(H + 2) * mg_ld<T>(W); }

// ---------------------------------------------------------------------------
// vector access helpers
// ---------------------------------------------------------------------------
template <typename T, int V>
struct VecOf;
template <>
struct VecOf<double, 2> { typedef double type __attribute__((ext_vector_type(2))); };
template <>
struct VecOf<float, 4> { typedef float type __attribute__((ext_vector_type(4))); };
template <>
struct VecOf<float, 2> { typedef float type __attribute__((ext_vector_type(2))); };

template <typename T, int V, bool NTL = false>
__device__ __forceinline__ void vload(const T* p, T (&x)[V]) {
  if constexpr (V == 1) {
    x[0] = *p;
  } else {
    const auto* q = reinterpret_cast<const typename VecOf<T, V>::type*>(p);
    typename VecOf<T, V>::type v;
    if constexpr (NTL)
      v = __builtin_nontemporal_load(q);
    else
      v = *q;
#pragma unroll
    for (int k = 0; k < V; ++k) x[k] = v[k];
  }
}

// NT: nontemporal (streaming) store — used on levels too large to be re-read from cache.  A
// compile-time flag: with a runtime flag the two stores are merged before inlining and the
// nontemporal hint is lost.
template <typename T, int V, bool NT = false>
__device__ __forceinline__ void vstore(T* p, const T (&x)[V]) {
  constexpr bool nt = NT;
  if constexpr (V == 1) {
    if constexpr (nt)
      __builtin_nontemporal_store(x[0], p);
    else
      *p = x[0];
  } else {
    typename VecOf<T, V>::type v;
#pragma unroll
    for (int k = 0; k < V; ++k) v[k] = x[k];
    auto* q = reinterpret_cast<typename VecOf<T, V>::type*>(p);
    if constexpr (nt)
      __builtin_nontemporal_store(v, q);
    else
      *q = v;
  }
}

// V pattern bytes -> ints
template <int V>
__device__ __forceinline__ void pload(const uint8_t* p, int (&o)[V]) {
  if constexpr (V == 1) {
    o[0] = p[0];
  } else if constexpr (V == 2) {
    const unsigned v = *reinterpret_cast<const unsigned short*>(p);
    o[0] = v & 0xff;
    o[1] = v >> 8;
  } else {
    const unsigned v = *reinterpret_cast<const unsigned*>(p);
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = (v >> (8 * k)) & 0xff;
  }
}

// A row segment of one lane: a[0] = column c-1 (L), a[1..V] = own columns, a[V+1] = c+V (R),
// a[V+2] = c+V+1 (RR).
template <typename T, int V>
struct Row {
  T a[V + 3];
};
template <int V>
struct PRow {  // LDS table row byte offsets (pattern * tab_row_bytes<T>()) for the same columns
  int a[V + 3];
};

// Rows are loaded in two halves so a load can be issued one iteration ahead of its use:
// raw_*() issues the 16-byte vector load of the lane's columns plus the 16-byte halo load
// (lane 0: columns c0-V..c0-1, lane 63: c0+SW..), finish() builds the window row with DPP.
template <typename T, int V>
struct RawRow {
  T x[V], h[V];
};
template <int V>
struct RawP {
  int x[V], h[V];
};

template <typename T, int V, bool NTL = false>
__device__ __forceinline__ RawRow<T, V> raw_row(const T* __restrict__ rp, int lane) {
  RawRow<T, V> r;
  vload<T, V, NTL>(rp + V * lane, r.x);
  // halo: only the two edge lanes load (exec-masked), the other lanes' h is never read
#pragma unroll
  for (int k = 0; k < V; ++k) r.h[k] = T(0);
  if (lane == 0 || lane == kWave - 1) vload<T, V>(rp + (lane == 0 ? -V : kWave * V), r.h);
  return r;
}

template <typename T, int V>
__device__ __forceinline__ Row<T, V> finish(const RawRow<T, V>& r) {
  Row<T, V> w;
#pragma unroll
  for (int k = 0; k < V; ++k) w.a[k + 1] = r.x[k];
  w.a[0] = shr1(r.x[V - 1], r.h[V - 1]);
  w.a[V + 1] = shl1(r.x[0], r.h[0]);
  w.a[V + 2] = shl1(r.x[1 % V], r.h[1 % V]);
  return w;
}

template <int V>
__device__ __forceinline__ RawP<V> raw_prow(const uint8_t* __restrict__ pp, int lane) {
  RawP<V> r;
  pload<V>(pp + V * lane, r.x);
#pragma unroll
  for (int k = 0; k < V; ++k) r.h[k] = 0;
  if (lane == 0 || lane == kWave - 1) pload<V>(pp + (lane == 0 ? -V : kWave * V), r.h);
  return r;
}

template <typename T, int V>
__device__ __forceinline__ PRow<V> finish_p(const RawP<V>& r) {
  PRow<V> w;
#pragma unroll
  for (int k = 0; k < V; ++k) w.a[k + 1] = r.x[k] * tab_row_bytes<T>();
  w.a[0] = shr1(r.x[V - 1], r.h[V - 1]) * tab_row_bytes<T>();
  w.a[V + 1] = shl1(r.x[0], r.h[0]) * tab_row_bytes<T>();
  w.a[V + 2] = shl1(r.x[1 % V], r.h[1 % V]) * tab_row_bytes<T>();
  return w;
}

// (K u) at own column k (k = 0..V, k = V is the R column) from the 3-row window.
// Two-material (MULTI): KNet applies tap t with the weight of the NEIGHBOUR's pattern (split, then convolve:
// FEANet/model.py:22-30); K is a symmetric FE stiffness, so that weight is bit for bit the mirrored tap 8 - t of the
// CENTRE's pattern (stencil_table(); MultigridSolver checks it on every level's map, mesh_setup
// .stencil_mirror_mismatches).  All nine weights then come from one table row — one base address, adjacent
// offsets — instead of three rows picked by the window's neighbour patterns; taps are summed in the same order, so
// every value is the same bits as before.
#ifndef FEA_KSYM
#define FEA_KSYM 1
#endif
template <typename T, int V, bool MULTI>
__device__ __forceinline__ T kapply(const Row<T, V>& w0, const Row<T, V>& w1, const Row<T, V>& w2,
                                    const PRow<V>& p0, const PRow<V>& p1, const PRow<V>& p2, int k,
                                    const T (&ks)[9], const T* tab) {
  T acc;
  if constexpr (MULTI && FEA_KSYM) {
    const int pc = p1.a[k + 1];
    acc = tabv(tab, pc, 8) * w0.a[k];
    acc += tabv(tab, pc, 7) * w0.a[k + 1];
    acc += tabv(tab, pc, 6) * w0.a[k + 2];
    acc += tabv(tab, pc, 5) * w1.a[k];
    acc += tabv(tab, pc, 4) * w1.a[k + 1];
    acc += tabv(tab, pc, 3) * w1.a[k + 2];
    acc += tabv(tab, pc, 2) * w2.a[k];
    acc += tabv(tab, pc, 1) * w2.a[k + 1];
    acc += tabv(tab, pc, 0) * w2.a[k + 2];
  } else if constexpr (!MULTI) {
    acc = ks[0] * w0.a[k];
    acc += ks[1] * w0.a[k + 1];
    acc += ks[2] * w0.a[k + 2];
    acc += ks[3] * w1.a[k];
    acc += ks[4] * w1.a[k + 1];
    acc += ks[5] * w1.a[k + 2];
    acc += ks[6] * w2.a[k];
    acc += ks[7] * w2.a[k + 1];
    acc += ks[8] * w2.a[k + 2];
  } else {
    acc = tabv(tab, p0.a[k], 0) * w0.a[k];
    acc += tabv(tab, p0.a[k + 1], 1) * w0.a[k + 1];
    acc += tabv(tab, p0.a[k + 2], 2) * w0.a[k + 2];
    acc += tabv(tab, p1.a[k], 3) * w1.a[k];
    acc += tabv(tab, p1.a[k + 1], 4) * w1.a[k + 1];
    acc += tabv(tab, p1.a[k + 2], 5) * w1.a[k + 2];
    acc += tabv(tab, p2.a[k], 6) * w2.a[k];
    acc += tabv(tab, p2.a[k + 1], 7) * w2.a[k + 1];
    acc += tabv(tab, p2.a[k + 2], 8) * w2.a[k + 2];
  }
  return acc;
}

template <typename T>
struct MgArgs {
  const T* u;
  const T* f;
  T* out;
  T* out2;
  const T* ec;
  const uint8_t* pid;
  const uint8_t* pidc;
  const T* ktab;
  const T* omd;
  const T* rtab;
  const T* ptab;
  double* part;
  int ntab, nrtab, nptab;
  T w;
  T w2;  // second ratio (cycle join: w1 of the prolongation)
  int H, W, ld;  // rows, columns of the (local) grid
  long long bs;
  int Hc, Wc, ldc;
  long long bsc;
  int Hc2, Wc2, ldc2;  // the level below the coarse one (k_mg_zero_restrict2: its right-hand side in out2;
  long long bsc2;      //   k_mg_prolong2: its correction in ec2, its pattern map in pidc2)
  const T* ec2;
  const uint8_t* pidc2;
  int nstrips, ntr;  // strips per row, row tasks per sample
  int rb;            // fine rows per row task (even)
  int rlo, rhi;      // row range of the residual norm
  int clo, chi;      // column range of the residual norm
  int nt;            // 1: nontemporal stores (level larger than FEANET_NT_BYTES); 2: also loads (sweep, join)
  int rev;           // decode_task_lin: deal the launch's tasks in reverse order (last task first)
  int flip;          // cycle join: every task streams in the other direction (even tasks bottom-up, odd top-down)
  // cycle join over up to 4 rectangles (nrect > 0; a domain-decomposed rank's border strips, then its interior):
  // rectangle r = coarse rows [rI0[r], rI1[r]) x fine columns [rc0[r], rc1[r]) (odd bounds, coarse column J owned
  // with its fine columns 2J-1, 2J), its nstrips rns[r], its row tasks rnt[r]; the launch's tasks per sample are
  // rectangle by rectangle, rt[r] the first of rectangle r
  int nrect;
  int rI0[4], rI1[4], rc0[4], rc1[4], rns[4], rt[5];
  // zero-guess restrictions of a domain-decomposed rank (k_mg_zero_restrict, k_mg_zero_restrict2): the output level's
  // block [gr0, gr1) x [gc0, gc1) (local rows / columns) also goes to gsend[b][r - gr0][c - gc0] — the all-gather's
  // send buffer of the agglomeration, written by the kernel that computes it instead of a copy launch after it
  T* gsend;
  int gr0, gr1, gc0, gc1;
};

// the agglomeration send-buffer store of a zero-guess restriction (MgArgs::gsend), node (r, c) of the output level
template <typename T>
__device__ __forceinline__ void gather_store(const MgArgs<T>& g, int b, int r, int c, T v) {
  if (g.gsend && r >= g.gr0 && r < g.gr1 && c >= g.gc0 && c < g.gc1)
    g.gsend[((long long)b * (g.gr1 - g.gr0) + (r - g.gr0)) * (g.gc1 - g.gc0) + (c - g.gc0)] = v;
}

struct TaskId {
  int b, s, t;
  bool valid;
};

__device__ __forceinline__ TaskId decode_task(int nstrips, int ntr) {
  const int nsg = (nstrips + kWaves - 1) / kWaves;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int per_b = ntr * nsg;
  TaskId id;
  id.b = bid / per_b;
  const int rem = bid - id.b * per_b;
  id.t = rem / nsg;
  const int sg = rem - id.t * nsg;
  id.s = sg * kWaves + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));  // wave-uniform: scalar
  id.valid = id.s < nstrips;
  return id;
}

// Linear task order for the overlapped-strip kernels (cycle join, sweep+restriction), whose strip count
// per row is ragged (35 at 4097 wide in fp64, 5 at 1025 in fp32): a workgroup's four waves take the next
// four (row task, strip) pairs of one sample instead of four strips of one row task, so no wave slot is
// left empty (5 strips in two 4-wave groups idled 3 of 8 slots).  Workgroups never mix samples (the
// fused norm partials stay per sample); only a sample's last workgroup may hold idle waves.
// the launch's logical block: XCD-remapped (each XCD a contiguous band), in reverse when `rev` (every XCD then
// walks its band from the end)
__device__ __forceinline__ int lin_block(int rev) {
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  return rev ? (int)gridDim.x - 1 - bid : bid;
}

__device__ __forceinline__ TaskId decode_task_lin(int nstrips, int ntr, int rev = 0) {
  const int per = ntr * nstrips;
  const int wpb = (per + kWaves - 1) / kWaves;  // workgroups per sample
  const int bid = lin_block(rev);
  TaskId id;
  id.b = bid / wpb;
  // the wave index is wave-uniform: keep the task coordinates in scalar registers
  const int w = (bid - id.b * wpb) * kWaves + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  id.t = w / nstrips;
  id.s = w - id.t * nstrips;
  id.valid = w < per;
  return id;
}

// Fused residual norm of a launch (kernels with a NORM variant): every wave's partial sum of squares
// goes to part[remapped block * kWaves + wave] (waves without a task write 0); k_norm_append, launched
// right after on the same stream, sums each sample's partials in index order — deterministic, the same
// order every launch — and appends sqrt(sum) as history row cnt[1].  (A last-workgroup reduction inside
// the kernel would need a device-scope release per workgroup, i.e. an L2 write-back on every one of
// them; the kernel boundary gives the same visibility once.)
template <typename T>
__device__ __forceinline__ void norm_partial(const MgArgs<T>& g, double ssq) {
  ssq = wave_sum(ssq);
  const int bid = lin_block(g.rev);  // the slot of the block's tasks, whatever order they were dealt in
  if (lane_id() == 0) g.part[(long long)bid * kWaves + (threadIdx.x >> 6)] = ssq;
}

// One workgroup: for r < nrows, hist[(row0 + r) * B + b] = sqrt(sum of part[r * stride + b * per + i],
// i < per) with row0 = cnt[1]; then cnt[1] = row0 + nrows.
__global__ __launch_bounds__(256) void k_norm_append(const double* __restrict__ part, long long stride, long long per,
                                                    int B, int nrows, double* __restrict__ hist,
                                                    unsigned* __restrict__ cnt) {
  __shared__ double red[256];
  const unsigned row0 = cnt[1];
  for (int r = 0; r < nrows; ++r)
    for (int b = 0; b < B; ++b) {
      const double* p = part + r * stride + b * per;
      double s = 0.0;
      for (long long i = threadIdx.x; i < per; i += 256) s += p[i];
      red[threadIdx.x] = s;
      __syncthreads();
      for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
      }
      if (threadIdx.x == 0) hist[(long long)(row0 + r) * B + b] = sqrt(red[0]);
      __syncthreads();
    }
  if (threadIdx.x == 0) cnt[1] = row0 + nrows;
}

// Loads ktab/omd (stride 10) and optionally a second 9-wide table into LDS.
template <typename T>
__device__ __forceinline__ void load_tables(T* tab, const T* ktab, const T* omd, int ntab, T* tab2,
                                            const T* t2, int n2) {
  for (int i = threadIdx.x; i < ntab * kTabStride; i += blockDim.x) {
    const int p = i / kTabStride, d = i - p * kTabStride;
    tab[i] = (d == 9) ? (omd ? omd[p] : T(0)) : ktab[p * 9 + d];
  }
  if (tab2)
    for (int i = threadIdx.x; i < n2 * kTabStride; i += blockDim.x) {
      const int p = i / kTabStride, d = i - p * kTabStride;
      tab2[i] = (d == 9) ? T(0) : t2[p * 9 + d];
    }
}

template <typename T, int V, bool NT>
__device__ __forceinline__ void store_masked(T* p, const T (&o)[V], int cl, int W) {
  if (cl + V - 1 <= W - 2) {
    vstore<T, V, NT>(p, o);
  } else {
#pragma unroll
    for (int k = 0; k < V; ++k)
      if (cl + k <= W - 2) p[k] = o[k];
  }
}

// ---------------------------------------------------------------------------
// Kernel A: interior Jacobi sweep  out = J(u, f);  ZERO: u == 0  ->  out = omd * f
// ---------------------------------------------------------------------------
// NTL: nontemporal loads of u and f too — on fields larger than the Infinity Cache (nt_policy: nothing of
// them can be re-read from it; 8193^2 fp64 sweep 321 -> 310 us, 256 x 1025^2 fp32 700 -> 667 us, same-process
// A/B, profiles/r03_stream/ntl_ab.txt; at 4097^2 it costs 64 -> 78 us, the fields being partly resident)
template <typename T, bool MULTI, bool ZERO, bool NT, bool NTL = false>
__global__ __launch_bounds__(256) void k_mg_sweep(MgArgs<T> g) {
  using F = Frame<T>;
  constexpr int V = F::VEC;
  __shared__ T tab[MULTI ? FEA_MAX_PATTERNS * kTabStride : 1];
  if constexpr (MULTI) {
    load_tables<T>(tab, g.ktab, g.omd, g.ntab, nullptr, nullptr, 0);
    __syncthreads();
  }
  const TaskId id = decode_task(g.nstrips, g.ntr);
  if (!id.valid) return;
  const int lane = lane_id();
  const int H = g.H, W = g.W;
  const int c0 = 1 + id.s * F::SW;
  const int r0 = 1 + id.t * g.rb;
  const int r1 = min(r0 + g.rb, H - 1);
  const int cl = c0 + V * lane;  // first own column
  T ks[9];
  T om = 0;
  if constexpr (!MULTI) {
#pragma unroll
    for (int d = 0; d < 9; ++d) ks[d] = g.ktab[d];
    om = g.omd[0];
  }
  const long long poff = F::OFF + c0;
  const long long boff = (long long)id.b * g.bs + poff;
  const T* __restrict__ ub = g.u + boff;
  const T* __restrict__ fb = g.f + boff;
  T* __restrict__ ob = g.out + boff;
  const uint8_t* __restrict__ pb = MULTI ? g.pid + poff : nullptr;  // pattern maps: one per mesh
  const int ld = g.ld;
  auto rowo = [&](int r) -> long long { return (long long)(min(r, H) + 1) * ld; };

  if constexpr (ZERO) {
    for (int r = r0; r < r1; ++r) {
      const long long ro = rowo(r) + V * lane;
      T fv[V], o[V];
      vload<T, V, NTL>(fb + ro, fv);
      int pv[V];
      if constexpr (MULTI) pload<V>(pb + ro, pv);
#pragma unroll
      for (int k = 0; k < V; ++k) o[k] = (MULTI ? tab[pv[k] * kTabStride + 9] : om) * fv[k];
      store_masked<T, V, NT>(ob + ro, o, cl, W);
    }
  } else {
    Row<T, V> w0 = finish(raw_row<T, V, NTL>(ub + rowo(r0 - 1), lane));
    Row<T, V> w1 = finish(raw_row<T, V, NTL>(ub + rowo(r0), lane));
    RawRow<T, V> nx = raw_row<T, V, NTL>(ub + rowo(r0 + 1), lane);
    T fx[V];
    vload<T, V, NTL>(fb + rowo(r0) + V * lane, fx);
    PRow<V> p0{}, p1{}, p2{};
    RawP<V> px{};
    if constexpr (MULTI) {
      p0 = finish_p<T>(raw_prow<V>(pb + rowo(r0 - 1), lane));
      p1 = finish_p<T>(raw_prow<V>(pb + rowo(r0), lane));
      px = raw_prow<V>(pb + rowo(r0 + 1), lane);
    }
    for (int r = r0; r < r1; ++r) {
      // issue next iteration's loads before this row's arithmetic
      const RawRow<T, V> nn = raw_row<T, V, NTL>(ub + rowo(r + 2), lane);
      T fn[V];
      vload<T, V, NTL>(fb + rowo(r + 1) + V * lane, fn);
      RawP<V> pn{};
      if constexpr (MULTI) pn = raw_prow<V>(pb + rowo(r + 2), lane);
      const Row<T, V> w2 = finish(nx);
      if constexpr (MULTI) p2 = finish_p<T>(px);
      T o[V];
#pragma unroll
      for (int k = 0; k < V; ++k) {
        const T acc = kapply<T, V, MULTI>(w0, w1, w2, p0, p1, p2, k, ks, tab);
        const T omk = MULTI ? tabv(tab, p1.a[k + 1], 9) : om;
        o[k] = omk * (fx[k] - acc) + w1.a[k + 1];
      }
      store_masked<T, V, NT>(ob + rowo(r) + V * lane, o, cl, W);
      w0 = w1;
      w1 = w2;
      nx = nn;
#pragma unroll
      for (int k = 0; k < V; ++k) fx[k] = fn[k];
      if constexpr (MULTI) {
        p0 = p1;
        p1 = p2;
        px = pn;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Kernel B: fused residual + restriction (+ optional zero-guess pre-sweep).
//   task = (strip s, coarse rows [I0, I1)), fine rows 2I0-2 .. 2I1 are read.
// ---------------------------------------------------------------------------
// residual + restriction: coarse-row iterations (2 fine rows each) whose loads are in flight at once
#ifndef FEA_RR_AHEAD
#define FEA_RR_AHEAD 2
#endif
constexpr int kRRAhead = FEA_RR_AHEAD;
static_assert(kRRAhead >= 1 && kRRAhead <= 4, "residual-restriction ring of 1..4 iterations");

#ifdef FEA_RR_TRACE
__device__ long long g_rr_trace[2 * 8192];
extern "C" int fea_rr_trace_read(long long* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_rr_trace), sizeof(long long) * 2 * 8192, 0,
                                  hipMemcpyDeviceToHost);
}
#endif
template <typename T, bool MULTI, bool ZERO, bool NT>
__global__ __launch_bounds__(256) void k_mg_resid_restrict(MgArgs<T> g) {
  using F = Frame<T>;
  constexpr int V = F::VEC;
  constexpr int Q = V / 2;  // coarse outputs per lane
  __shared__ T tab[MULTI ? FEA_MAX_PATTERNS * kTabStride : 1];
  __shared__ T rtb[MULTI ? FEA_MAX_PATTERNS * kTabStride : 1];
  if constexpr (MULTI) {
    load_tables<T>(tab, g.ktab, g.omd, g.ntab, rtb, g.rtab, g.nrtab);
    __syncthreads();
  }
  const TaskId id = decode_task(g.nstrips, g.ntr);
  if (!id.valid) return;
#ifdef FEA_RR_TRACE  // lab builds only (tools/lab/rr_trace.py): per-wave start / end, s_memrealtime (100 MHz)
  const int trace_w = blockIdx.x * kWaves + (threadIdx.x >> 6);
  if ((threadIdx.x & 63) == 0 && trace_w < 8192) g_rr_trace[trace_w] = (long long)__builtin_amdgcn_s_memrealtime();
  struct TraceEnd {
    int w;
    __device__ ~TraceEnd() {
      if ((threadIdx.x & 63) == 0 && w < 8192) g_rr_trace[8192 + w] = (long long)__builtin_amdgcn_s_memrealtime();
    }
  } trace_end{trace_w};
#endif
  const int lane = lane_id();
  const int H = g.H, W = g.W, Hc = g.Hc, Wc = g.Wc;
  const int c0 = 1 + id.s * F::SW;
  const int I0 = 1 + id.t * (g.rb / 2);
  const int I1 = min(I0 + g.rb / 2, Hc - 1);
  const int cl = c0 + V * lane;
  T ks[9], rs[9];
  T om = 0;
  if constexpr (!MULTI) {
#pragma unroll
    for (int d = 0; d < 9; ++d) {
      ks[d] = g.ktab[d];
      rs[d] = g.rtab[d];
    }
    om = g.omd ? g.omd[0] : T(0);
  }
  const T w0 = g.w;
  // interior mask of the lane's V+3 window columns (ZERO mode derives v = omd*f inside only)
  bool cin[V + 3];
#pragma unroll
  for (int j = 0; j < V + 3; ++j) {
    const int c = cl + j - 1;
    cin[j] = c >= 1 && c <= W - 2;
  }
  const long long poff = F::OFF + c0;
  const long long boff = (long long)id.b * g.bs + poff;
  const T* __restrict__ ub = ZERO ? nullptr : g.u + boff;
  const T* __restrict__ fb = g.f + boff;
  T* __restrict__ vb = (ZERO && g.out2) ? g.out2 + boff : nullptr;
  const uint8_t* __restrict__ pb = MULTI ? g.pid + poff : nullptr;
  const int ld = g.ld;
  const int bc0 = (c0 + 1) / 2;  // coarse column of lane 0's first output
  T* __restrict__ cb = g.out + (long long)id.b * g.bsc + F::OFF + bc0 + Q * lane;
  const int Jl = bc0 + Q * lane;
  auto rowo = [&](int r) -> long long { return (long long)(min(r, H) + 1) * ld; };

  // a window row: the field K acts on (u, or v = omd*f in ZERO mode), the f row, pattern offsets
  struct RawW {
    RawRow<T, V> u, f;
    RawP<V> p;
  };
  struct WRow {
    Row<T, V> u, f;
    PRow<V> p;
  };
  auto raw_w = [&](int y) {
    RawW w;
    const long long ro = rowo(y);
    if constexpr (MULTI) w.p = raw_prow<V>(pb + ro, lane);
    w.f = raw_row<T, V>(fb + ro, lane);
    if constexpr (!ZERO) w.u = raw_row<T, V>(ub + ro, lane);
    return w;
  };
  auto fin_w = [&](const RawW& r, int y) {
    WRow w;
    if constexpr (MULTI) w.p = finish_p<T>(r.p);
    w.f = finish(r.f);
    if constexpr (ZERO) {
      const bool rin = y >= 1 && y <= H - 2;
#pragma unroll
      for (int j = 0; j < V + 3; ++j) {
        const T omj = MULTI ? tabv(tab, w.p.a[j], 9) : om;
        w.u.a[j] = (rin && cin[j]) ? omj * w.f.a[j] : T(0);
      }
    } else {
      w.u = finish(r.u);
    }
    return w;
  };
  auto resid = [&](const WRow& a, const WRow& b, const WRow& c, T (&r)[V + 1]) {
#pragma unroll
    for (int k = 0; k <= V; ++k) r[k] = b.f.a[k + 1] - kapply<T, V, MULTI>(a.u, b.u, c.u, a.p, b.p, c.p, k, ks, tab);
  };
  auto store_v = [&](int y, const WRow& w) {
    if constexpr (ZERO) {
      if (!vb) return;  // v not kept: the prolongation recomputes it from f (k_mg_prolong ZU)
      const bool own = y >= 2 * I0 - 1 && (y < 2 * I1 - 1 || I1 == Hc - 1) && y <= H - 2;
      if (own) {
        T o[V];
#pragma unroll
        for (int k = 0; k < V; ++k) o[k] = w.u.a[k + 1];
        store_masked<T, V, NT>(vb + rowo(y) + V * lane, o, cl, W);
      }
    }
  };

  const int y0 = 2 * I0 - 1;
  WRow W0 = fin_w(raw_w(y0 - 1), y0 - 1);
  WRow W1 = fin_w(raw_w(y0), y0);
  WRow W2 = fin_w(raw_w(y0 + 1), y0 + 1);
  // the fine rows of the next D coarse rows are in flight, in a D-slot ring indexed by the
  // iteration's parity (compile-time after the unroll below): a slot is consumed in place and
  // refilled at once, so no in-flight register is ever copied (a copy waits for its load)
  constexpr int D = kRRAhead;
  RawW ring[D][2];
#pragma unroll
  for (int d = 0; d < D; ++d) {
    ring[d][0] = raw_w(2 * I0 + 1 + 2 * d);
    ring[d][1] = raw_w(2 * I0 + 2 + 2 * d);
  }
  T Ra[V + 1], Rb[V + 1], Rc[V + 1];
  PRow<V> Pa = W1.p, Pb, Pc;
  resid(W0, W1, W2, Ra);
  store_v(y0, W1);
  auto iter = [&](int I, auto slot) {
    constexpr int S = decltype(slot)::value;
    // fine row 2I
    W0 = W1;
    W1 = W2;
    W2 = fin_w(ring[S][0], 2 * I + 1);
    ring[S][0] = raw_w(2 * I + 1 + 2 * D);
    resid(W0, W1, W2, Rb);
    Pb = W1.p;
    store_v(2 * I, W1);
    // fine row 2I+1
    W0 = W1;
    W1 = W2;
    W2 = fin_w(ring[S][1], 2 * I + 2);
    ring[S][1] = raw_w(2 * I + 2 + 2 * D);
    resid(W0, W1, W2, Rc);
    Pc = W1.p;
    store_v(2 * I + 1, W1);
    // coarse row I: outputs q use fine columns 2q, 2q+1, 2q+2 of the residual rows
    T o[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      T acc;
      if constexpr (!MULTI) {
        acc = rs[0] * Ra[2 * q];
        acc += rs[1] * Ra[2 * q + 1];
        acc += rs[2] * Ra[2 * q + 2];
        acc += rs[3] * Rb[2 * q];
        acc += rs[4] * Rb[2 * q + 1];
        acc += rs[5] * Rb[2 * q + 2];
        acc += rs[6] * Rc[2 * q];
        acc += rs[7] * Rc[2 * q + 1];
        acc += rs[8] * Rc[2 * q + 2];
      } else {
        acc = tabv(rtb, Pa.a[2 * q + 1], 0) * Ra[2 * q];
        acc += tabv(rtb, Pa.a[2 * q + 2], 1) * Ra[2 * q + 1];
        acc += tabv(rtb, Pa.a[2 * q + 3], 2) * Ra[2 * q + 2];
        acc += tabv(rtb, Pb.a[2 * q + 1], 3) * Rb[2 * q];
        acc += tabv(rtb, Pb.a[2 * q + 2], 4) * Rb[2 * q + 1];
        acc += tabv(rtb, Pb.a[2 * q + 3], 5) * Rb[2 * q + 2];
        acc += tabv(rtb, Pc.a[2 * q + 1], 6) * Rc[2 * q];
        acc += tabv(rtb, Pc.a[2 * q + 2], 7) * Rc[2 * q + 1];
        acc += tabv(rtb, Pc.a[2 * q + 3], 8) * Rc[2 * q + 2];
      }
      o[q] = w0 * acc;
    }
    T* cp = cb + (long long)(I + 1) * g.ldc;
    if (Jl + Q - 1 <= Wc - 2) {
      vstore<T, Q, kCoarseNT && NT>(cp, o);
    } else {
#pragma unroll
      for (int q = 0; q < Q; ++q)
        if (Jl + q <= Wc - 2) cp[q] = o[q];
    }
#pragma unroll
    for (int k = 0; k <= V; ++k) Ra[k] = Rc[k];
    Pa = Pc;
  };
  int I = I0;
  for (; I + D - 1 < I1; I += D) {
    iter(I, std::integral_constant<int, 0>{});
    if constexpr (D > 1) iter(I + 1, std::integral_constant<int, 1 % D>{});
    if constexpr (D > 2) iter(I + 2, std::integral_constant<int, 2 % D>{});
    if constexpr (D > 3) iter(I + 3, std::integral_constant<int, 3 % D>{});
  }
  if constexpr (D > 1)
    if (I < I1) iter(I, std::integral_constant<int, 0>{});
  if constexpr (D > 2)
    if (I + 1 < I1) iter(I + 1, std::integral_constant<int, 1 % D>{});
  if constexpr (D > 3)
    if (I + 2 < I1) iter(I + 2, std::integral_constant<int, 2 % D>{});
}

// ---------------------------------------------------------------------------
// Kernel E: fused pre-smooth + residual + restriction on a level with a given iterate
// (temporal blocking of FEANet/multigrid.py:165 then :168-170):
//   u' = J(u, f)  (stored, interior)     f_c = w0 R(f - K u')
// One pass reads u and f once instead of twice.  OVERLAPPED STRIPS: a wave loads 64*VEC columns
// starting VEC columns left of the S it owns (S = 122 fp64, 248 fp32) and computes u' and the
// residual on all of them; the values its two edge lanes get wrong (missing neighbours) are never
// stored, so there is no edge-lane recomputation and no halo load (5 % of the columns are loaded
// twice instead).  Rounding is the same per node as every other kernel (fp-contract=on).
// ---------------------------------------------------------------------------
template <typename T>
struct Ovl {
  static constexpr int V = Frame<T>::VEC;
  static constexpr int S = ((63 * V - 3) / V) * V;  // owned fine columns per strip (mult. of V)
  static constexpr int OWN = S / V;                 // owning lanes: 1 .. OWN
};
template <typename T, int V>
__device__ __forceinline__ Row<T, V> own_row(const T (&x)[V]) {  // window L, own.., R from own values
  Row<T, V> w;
#pragma unroll
  for (int k = 0; k < V; ++k) w.a[k + 1] = x[k];
  w.a[0] = shr1z(x[V - 1]);
  w.a[V + 1] = shl1z(x[0]);
  return w;
}
template <typename T, int V>
__device__ __forceinline__ PRow<V> own_prow(const int (&x)[V]) {
  PRow<V> w;
#pragma unroll
  for (int k = 0; k < V; ++k) w.a[k + 1] = x[k] * tab_row_bytes<T>();
  w.a[0] = shr1z(x[V - 1]) * tab_row_bytes<T>();
  w.a[V + 1] = shl1z(x[0]) * tab_row_bytes<T>();
  return w;
}

// One row task of the sweep + restriction (below).  NORM: also accumulates, into ssq, the squared
// residual f - K u of the INPUT iterate over the task's owned interior nodes (the sweep forms it):
// the drivers' initial residual norm (M-FEANet-mg_test.ipynb:27428-27429) at no extra pass.
template <typename T, bool MULTI, bool NT, bool NORM>
__device__ __forceinline__ void sweep_restrict_task(const MgArgs<T>& g, const TaskId& id, const T* tab,
                                                    const T* rtb, double& ssq) {
  using F = Frame<T>;
  using O = Ovl<T>;
  constexpr int V = F::VEC;
  constexpr int Q = V / 2;
  const int lane = lane_id();
  const int H = g.H, W = g.W, Hc = g.Hc, Wc = g.Wc;
  const int c0 = 1 + id.s * O::S;  // first owned fine column
  const int cs = c0 - V;           // first loaded column (16-byte aligned)
  const int cl = cs + V * lane;    // lane's first column
  const int I0 = 1 + id.t * (g.rb / 2);
  const int I1 = min(I0 + g.rb / 2, Hc - 1);
  T ks[9], rs[9];
  T om = 0;
  if constexpr (!MULTI) {
#pragma unroll
    for (int d = 0; d < 9; ++d) {
      ks[d] = g.ktab[d];
      rs[d] = g.rtab[d];
    }
    om = g.omd[0];
  }
  const T w0 = g.w;
  bool cin[V];
#pragma unroll
  for (int k = 0; k < V; ++k) cin[k] = cl + k >= 1 && cl + k <= W - 2;
  const bool own = lane >= 1 && lane <= O::OWN;
  const int J0 = (cl + 1) / 2;  // coarse column of the lane's first (2J-1, 2J, 2J+1) window
  const long long boff = (long long)id.b * g.bs + F::OFF + cs;
  const T* __restrict__ ub = g.u + boff;
  const T* __restrict__ fb = g.f + boff;
  T* __restrict__ ob = g.out2 + boff;
  const uint8_t* __restrict__ pb = MULTI ? g.pid + F::OFF + cs : nullptr;
  T* __restrict__ cb = g.out + (long long)id.b * g.bsc + F::OFF + J0;
  const int ld = g.ld;
  // lanes past the grid's last column (W - 1) load the last needed lane's columns again: the last
  // strip of a row can be mostly outside the grid (stores are masked by column anyway)
  const int ll = min(lane, (W - 1 - cs) / V);
  auto rowo = [&](int r) -> long long { return (long long)(min(max(r, -1), H) + 1) * ld + V * ll; };

  struct In {  // a raw input row: u and f own values (+ pattern ids)
    T u[V], f[V];
    int p[V];
  };
  auto load = [&](int y) {
    In r;
    const long long o = rowo(y);
    vload<T, V>(ub + o, r.u);
    vload<T, V>(fb + o, r.f);
    if constexpr (MULTI) pload<V>(pb + o, r.p);
    return r;
  };
  struct Wn {  // an input row in use: u window, f own, pattern window
    Row<T, V> u;
    T f[V];
    PRow<V> p;
  };
  auto mk = [&](const In& r) {
    Wn w;
    w.u = own_row<T, V>(r.u);
#pragma unroll
    for (int k = 0; k < V; ++k) w.f[k] = r.f[k];
    if constexpr (MULTI) w.p = own_prow<T, V>(r.p);
    return w;
  };
  auto owns = [&](int y) { return own && y >= 2 * I0 - 1 && (y < 2 * I1 - 1 || I1 == Hc - 1) && y <= H - 2; };
  // u'(y) on the lane's own columns (boundary rows / columns keep u)
  auto usweep = [&](const Wn& a, const Wn& b, const Wn& c, int y, T (&o)[V]) {
    const bool rin = y >= 1 && y <= H - 2;
    const bool count = NORM && owns(y);
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const T acc = kapply<T, V, MULTI>(a.u, b.u, c.u, a.p, b.p, c.p, k, ks, tab);
      const T omk = MULTI ? tabv(tab, b.p.a[k + 1], 9) : om;
      const T rr = b.f[k] - acc;
      const T v = omk * rr + b.u.a[k + 1];
      o[k] = (rin && cin[k]) ? v : b.u.a[k + 1];
      if constexpr (NORM)
        if (count && rin && cin[k]) ssq += (double)rr * (double)rr;
    }
  };
  auto store_u = [&](int y, const T (&o)[V]) {
    if (owns(y)) store_masked<T, V, NT>(ob + rowo(y), o, cl, W);
  };
  // residual row y (u' windows a, b, c; f and patterns of row y) -> restriction row ky into acc
  auto racc = [&](const Row<T, V>& a, const Row<T, V>& b, const Row<T, V>& c, const Wn& sy, const Wn& pa,
                  const Wn& pc, int ky, T (&acc)[Q], bool init) {
    T r[V + 1];
#pragma unroll
    for (int k = 0; k < V; ++k) r[k] = sy.f[k] - kapply<T, V, MULTI>(a, b, c, pa.p, sy.p, pc.p, k, ks, tab);
    r[V] = shl1z(r[0]);  // column cl+V from the next lane
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      T t;
      if constexpr (!MULTI) {
        t = rs[ky * 3 + 0] * r[2 * q];
        t += rs[ky * 3 + 1] * r[2 * q + 1];
        t += rs[ky * 3 + 2] * r[2 * q + 2];
      } else {
        t = tabv(rtb, sy.p.a[2 * q + 1], ky * 3 + 0) * r[2 * q];
        t += tabv(rtb, sy.p.a[2 * q + 2], ky * 3 + 1) * r[2 * q + 1];
        t += tabv(rtb, sy.p.a[2 * q + 3], ky * 3 + 2) * r[2 * q + 2];
      }
      acc[q] = init ? t : acc[q] + t;
    }
  };
  auto store_c = [&](int I, const T (&acc)[Q]) {
    T o[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) o[q] = w0 * acc[q];
    if (!own) return;
    T* cp = cb + (long long)(I + 1) * g.ldc;
    if (J0 + Q - 1 <= Wc - 2) {
      vstore<T, Q, kCoarseNT && NT>(cp, o);
    } else {
#pragma unroll
      for (int q = 0; q < Q; ++q)
        if (J0 + q <= Wc - 2) cp[q] = o[q];
    }
  };

  const int ya = 2 * I0 - 1;  // first residual row
  Wn X0 = mk(load(ya - 2)), X1 = mk(load(ya - 1)), X2 = mk(load(ya)), X3 = mk(load(ya + 1));
  In nB = load(ya + 3);  // row 2I0+2, consumed in the first half of the first iteration
  Wn X4 = mk(load(ya + 2));
  T o[V];
  usweep(X0, X1, X2, ya - 1, o);  // u'(ya-1), not stored (row of the task above or boundary)
  const Row<T, V> Up = own_row<T, V>(o);
  usweep(X1, X2, X3, ya, o);
  store_u(ya, o);
  Row<T, V> Uc = own_row<T, V>(o);
  usweep(X2, X3, X4, ya + 1, o);
  store_u(ya + 1, o);
  Row<T, V> Un = own_row<T, V>(o);
  T acc[Q];
  racc(Up, Uc, Un, X2, X1, X3, 0, acc, true);  // residual row ya -> coarse I0, ky = 0
  // loop state for coarse row I: u' rows 2I-1 (Uc), 2I (Un); input rows 2I-1 (X2), 2I (X3),
  // 2I+1 (X4); raw row 2I+2 (nB) in flight
  for (int I = I0; I < I1; ++I) {
    const In m1 = load(2 * I + 3);  // consumed in the second half of this iteration
    const Wn X5 = mk(nB);           // row 2I+2
    usweep(X3, X4, X5, 2 * I + 1, o);
    store_u(2 * I + 1, o);
    const Row<T, V> U1 = own_row<T, V>(o);
    racc(Uc, Un, U1, X3, X2, X4, 1, acc, false);  // residual row 2I
    const In m2 = load(2 * I + 4);  // consumed in the first half of the next iteration
    const Wn X6 = mk(m1);           // row 2I+3
    usweep(X4, X5, X6, 2 * I + 2, o);
    store_u(2 * I + 2, o);
    const Row<T, V> U2 = own_row<T, V>(o);
    racc(Un, U1, U2, X4, X3, X5, 2, acc, false);  // residual row 2I+1: ky = 2 for I ...
    store_c(I, acc);
    racc(Un, U1, U2, X4, X3, X5, 0, acc, true);   // ... and ky = 0 for I+1
    Uc = U1;
    Un = U2;
    X2 = X4;
    X3 = X5;
    X4 = X6;
    nB = m2;
  }
}

template <typename T, bool MULTI, bool NORM, bool NT>
__global__ __launch_bounds__(256) void k_mg_sweep_restrict(MgArgs<T> g) {
  __shared__ T tab[MULTI ? FEA_MAX_PATTERNS * kTabStride : 1];
  __shared__ T rtb[MULTI ? FEA_MAX_PATTERNS * kTabStride : 1];
  if constexpr (MULTI) {
    load_tables<T>(tab, g.ktab, g.omd, g.ntab, rtb, g.rtab, g.nrtab);
    __syncthreads();
  }
  const TaskId id = decode_task_lin(g.nstrips, g.ntr);
  double ssq = 0.0;
  if (id.valid) sweep_restrict_task<T, MULTI, NT, NORM>(g, id, tab, rtb, ssq);
  if constexpr (NORM) norm_partial<T>(g, ssq);
}

// ---------------------------------------------------------------------------
// Kernel B0: zero-guess residual + restriction on OVERLAPPED strips (levels >= 1 going down, v not kept):
//   v = omd f (interior, 0 on the boundary),   f_c = w0 R(f - K v)
// k_mg_resid_restrict<ZERO> with v_out = NULL, restated: v is local to its node, so a wave forms it on
// all 64*VEC columns it loads and takes the window neighbours by DPP — no halo loads, K applied at VEC
// instead of VEC+1 columns per lane and v formed at VEC instead of VEC+3 (the residual of column
// cl+VEC comes from the next lane).  The per-node expressions and the restriction's 9-term order are
// those of k_mg_resid_restrict, so f_c is bitwise the same (tests/test_gpu_mg.py::test_mg_transfer).
// ---------------------------------------------------------------------------
template <typename T, bool MULTI, bool NT>
__global__ __launch_bounds__(256) void k_mg_zero_restrict(MgArgs<T> g) {
  using F = Frame<T>;
  using O = Ovl<T>;
  constexpr int V = F::VEC;
  constexpr int Q = V / 2;
  __shared__ T tab[MULTI ? FEA_MAX_PATTERNS * kTabStride : 1];
  __shared__ T rtb[MULTI ? FEA_MAX_PATTERNS * kTabStride : 1];
  if constexpr (MULTI) {
    load_tables<T>(tab, g.ktab, g.omd, g.ntab, rtb, g.rtab, g.nrtab);
    __syncthreads();
  }
  const TaskId id = decode_task_lin(g.nstrips, g.ntr);
  if (!id.valid) return;
  const int lane = lane_id();
  const int H = g.H, W = g.W, Hc = g.Hc, Wc = g.Wc;
  const int c0 = 1 + id.s * O::S;  // first owned fine column
  const int cs = c0 - V;           // first loaded column
  const int cl = cs + V * lane;
  const int I0 = 1 + id.t * (g.rb / 2);
  const int I1 = min(I0 + g.rb / 2, Hc - 1);
  T ks[9], rs[9];
  T om = 0;
  if constexpr (!MULTI) {
#pragma unroll
    for (int d = 0; d < 9; ++d) {
      ks[d] = g.ktab[d];
      rs[d] = g.rtab[d];
    }
    om = g.omd[0];
  }
  const T w0 = g.w;
  bool cin[V];
#pragma unroll
  for (int k = 0; k < V; ++k) cin[k] = cl + k >= 1 && cl + k <= W - 2;
  const bool own = lane >= 1 && lane <= O::OWN;
  const int J0 = (cl + 1) / 2;
  const long long boff = (long long)id.b * g.bs + F::OFF + cs;
  const T* __restrict__ fb = g.f + boff;
  const uint8_t* __restrict__ pb = MULTI ? g.pid + F::OFF + cs : nullptr;
  T* __restrict__ cb = g.out + (long long)id.b * g.bsc + F::OFF + J0;
  const int ld = g.ld;
  const int ll = min(lane, (W - 1 - cs) / V);  // lanes past the grid re-read the last needed line
  auto rowo = [&](int r) -> long long { return (long long)(min(max(r, -1), H) + 1) * ld + V * ll; };

  struct In {
    T f[V];
    int p[V];
  };
  struct Wn {  // v window (L, own.., R), f own, pattern window
    Row<T, V> v;
    T f[V];
    PRow<V> p;
  };
  auto load = [&](int y) {
    In r;
    const long long o = rowo(y);
    vload<T, V>(fb + o, r.f);
    if constexpr (MULTI) pload<V>(pb + o, r.p);
    return r;
  };
  auto mk = [&](const In& r, int y) {
    Wn w;
    const bool rin = y >= 1 && y <= H - 2;
    T x[V];
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const T omk = MULTI ? tab[r.p[k] * kTabStride + 9] : om;
      x[k] = (rin && cin[k]) ? omk * r.f[k] : T(0);
      w.f[k] = r.f[k];
    }
    w.v = own_row<T, V>(x);
    if constexpr (MULTI) w.p = own_prow<T, V>(r.p);
    return w;
  };
  auto resid = [&](const Wn& a, const Wn& b, const Wn& c, T (&r)[V + 1]) {
#pragma unroll
    for (int k = 0; k < V; ++k) r[k] = b.f[k] - kapply<T, V, MULTI>(a.v, b.v, c.v, a.p, b.p, c.p, k, ks, tab);
    r[V] = shl1z(r[0]);  // column cl+V from the next lane
  };

  const int y0 = 2 * I0 - 1;
  Wn X0 = mk(load(y0 - 1), y0 - 1);
  Wn X1 = mk(load(y0), y0);
  Wn X2 = mk(load(y0 + 1), y0 + 1);
  constexpr int D = kRRAhead;
  In ring[D][2];
#pragma unroll
  for (int d = 0; d < D; ++d) {
    ring[d][0] = load(2 * I0 + 1 + 2 * d);
    ring[d][1] = load(2 * I0 + 2 + 2 * d);
  }
  T Ra[V + 1], Rb[V + 1], Rc[V + 1];
  PRow<V> Pa = X1.p, Pb, Pc;
  resid(X0, X1, X2, Ra);
  auto iter = [&](int I, auto slot) {
    constexpr int S = decltype(slot)::value;
    X0 = X1;  // fine row 2I
    X1 = X2;
    X2 = mk(ring[S][0], 2 * I + 1);
    ring[S][0] = load(2 * I + 1 + 2 * D);
    resid(X0, X1, X2, Rb);
    Pb = X1.p;
    X0 = X1;  // fine row 2I+1
    X1 = X2;
    X2 = mk(ring[S][1], 2 * I + 2);
    ring[S][1] = load(2 * I + 2 + 2 * D);
    resid(X0, X1, X2, Rc);
    Pc = X1.p;
    T o[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      T acc;
      if constexpr (!MULTI) {
        acc = rs[0] * Ra[2 * q];
        acc += rs[1] * Ra[2 * q + 1];
        acc += rs[2] * Ra[2 * q + 2];
        acc += rs[3] * Rb[2 * q];
        acc += rs[4] * Rb[2 * q + 1];
        acc += rs[5] * Rb[2 * q + 2];
        acc += rs[6] * Rc[2 * q];
        acc += rs[7] * Rc[2 * q + 1];
        acc += rs[8] * Rc[2 * q + 2];
      } else {
        acc = tabv(rtb, Pa.a[2 * q + 1], 0) * Ra[2 * q];
        acc += tabv(rtb, Pa.a[2 * q + 2], 1) * Ra[2 * q + 1];
        acc += tabv(rtb, Pa.a[2 * q + 3], 2) * Ra[2 * q + 2];
        acc += tabv(rtb, Pb.a[2 * q + 1], 3) * Rb[2 * q];
        acc += tabv(rtb, Pb.a[2 * q + 2], 4) * Rb[2 * q + 1];
        acc += tabv(rtb, Pb.a[2 * q + 3], 5) * Rb[2 * q + 2];
        acc += tabv(rtb, Pc.a[2 * q + 1], 6) * Rc[2 * q];
        acc += tabv(rtb, Pc.a[2 * q + 2], 7) * Rc[2 * q + 1];
        acc += tabv(rtb, Pc.a[2 * q + 3], 8) * Rc[2 * q + 2];
      }
      o[q] = w0 * acc;
    }
    if (own) {
      T* cp = cb + (long long)(I + 1) * g.ldc;
      if (J0 + Q - 1 <= Wc - 2) {
        vstore<T, Q, kCoarseNT && NT>(cp, o);
      } else {
#pragma unroll
        for (int q = 0; q < Q; ++q)
          if (J0 + q <= Wc - 2) cp[q] = o[q];
      }
      if (g.gsend) {
#pragma unroll
        for (int q = 0; q < Q; ++q)
          if (J0 + q <= Wc - 2) gather_store(g, id.b, I, J0 + q, o[q]);
      }
    }
#pragma unroll
    for (int k = 0; k <= V; ++k) Ra[k] = Rc[k];
    Pa = Pc;
  };
  int I = I0;
  for (; I + D - 1 < I1; I += D) {
    iter(I, std::integral_constant<int, 0>{});
    if constexpr (D > 1) iter(I + 1, std::integral_constant<int, 1 % D>{});
    if constexpr (D > 2) iter(I + 2, std::integral_constant<int, 2 % D>{});
    if constexpr (D > 3) iter(I + 3, std::integral_constant<int, 3 % D>{});
  }
  if constexpr (D > 1)
    if (I < I1) iter(I, std::integral_constant<int, 0>{});
  if constexpr (D > 2)
    if (I + 1 < I1) iter(I + 1, std::integral_constant<int, 1 % D>{});
  if constexpr (D > 3)
    if (I + 2 < I1) iter(I + 2, std::integral_constant<int, 2 % D>{});
}

// ---------------------------------------------------------------------------
// Two zero-guess restrictions in one pass (levels l and l+1 going down, both below the tail-free top):
//   v = omd f_l;  f_{l+1} = w0 R(f_l - K v);  v' = omd f_{l+1};  f_{l+2} = w0 R(f_{l+1} - K v')
// Overlapped strips as k_mg_zero_restrict, with a second stage on the coarse values the first one leaves
// in registers (one per lane in fp64, two in fp32; neighbours by DPP): f_{l+1} is still stored (the up
// pass recomputes v' from it) but never re-read, and the level-(l+1) launch disappears.  Each strip
// loads HLc = max(V, 4) columns left of the S2 it owns, so the second stage's values are exact on its owned
// columns; a row task owns rb/4 rows of f_{l+2} and recomputes the 3 rows of f_{l+1} above and the 1 below
// them.  Every node value is the same expression, in the same order, as the two single-level launches
// (bitwise: tests/test_gpu_mg.py::test_zero_restrict2_bitwise).
// ---------------------------------------------------------------------------
template <typename T>
struct Ovl2 {
  static constexpr int V = Frame<T>::VEC;
  static constexpr int Q = V / 2;
  static constexpr int HLC = V > 4 ? V : 4;                  // left halo columns (a multiple of V)
  static constexpr int S = ((64 * V - 6 - HLC) / 4) * 4;     // owned fine columns per strip (fp64 116, fp32 244)
};

// ZR2 ALT: odd row tasks stream bottom-up, so two vertically adjacent tasks reach the fine rows both load
// (3 + 1 rows of the intermediate level are recomputed per task) at the same moment — both at their start
// or both at their end — and the second read of those rows is an L2 hit (k_mg_cycle_join does the same).
#ifndef FEA_ZR2_ALT
#define FEA_ZR2_ALT 1
#endif
constexpr bool kZr2Alternate = FEA_ZR2_ALT != 0;

// One row task of k_mg_zero_restrict2.  REV: rows are streamed bottom-up (row step S = -1); every node value
// is the same expression as in the forward task: stencil windows are passed in grid order, and each
// restriction sums its three residual rows in grid order (ky = 0, 1, 2) once all three are formed.
template <typename T, bool MULTI, bool REV>
__device__ __forceinline__ void zr2_task(const MgArgs<T>& g, const TaskId& id, const T* tab, const T* rtb) {
  using F = Frame<T>;
  using O = Ovl2<T>;
  constexpr int V = F::VEC;
  constexpr int Q = O::Q;
  constexpr int S = REV ? -1 : 1;  // row step
  const int lane = lane_id();
  const int H = g.H, W = g.W, Hc = g.Hc, Wc = g.Wc, Hc2 = g.Hc2, Wc2 = g.Wc2;
  const int c0 = 1 + id.s * O::S;  // first owned fine column
  const int cs = c0 - O::HLC;      // first loaded column
  const int cl = cs + V * lane;
  const int J0 = (cl + 1) / 2;     // the lane's first coarse column (level l+1)
  // owned columns of f_{l+1} and f_{l+2}, owned rows of f_{l+2}
  const int Jlo = id.s * (O::S / 2) + 1, Jhi = Jlo + O::S / 2;
  const int Mlo = id.s * (O::S / 4) + 1, Mhi = Mlo + O::S / 4;
  const int K0 = 1 + id.t * (g.rb / 4);
  const int K1 = min(K0 + g.rb / 4, Hc2 - 1);
  const int Ilo = 2 * K0 - 1, Ihi = K1 == Hc2 - 1 ? Hc - 1 : 2 * K1 - 1;  // owned rows of f_{l+1}
  T ks[9], rs[9];
  T om = 0;
  if constexpr (!MULTI) {
#pragma unroll
    for (int d = 0; d < 9; ++d) {
      ks[d] = g.ktab[d];
      rs[d] = g.rtab[d];
    }
    om = g.omd[0];
  }
  const T w0 = g.w;
  bool cin[V];
#pragma unroll
  for (int k = 0; k < V; ++k) cin[k] = cl + k >= 1 && cl + k <= W - 2;
  bool jin[Q];
#pragma unroll
  for (int q = 0; q < Q; ++q) jin[q] = J0 + q >= 1 && J0 + q <= Wc - 2;
  const long long boff = (long long)id.b * g.bs + F::OFF + cs;
  const T* __restrict__ fb = g.f + boff;
  const uint8_t* __restrict__ pb = MULTI ? g.pid + F::OFF + cs : nullptr;
  const uint8_t* __restrict__ pcb = MULTI ? g.pidc + F::OFF + J0 : nullptr;
  T* __restrict__ cb = g.out + (long long)id.b * g.bsc + F::OFF + J0;
  T* __restrict__ cb2 = g.out2 + (long long)id.b * g.bsc2 + F::OFF;
  const int ld = g.ld;
  const int ll = min(lane, (W - 1 - cs) / V);  // lanes past the grid re-read the last needed line
  auto rowo = [&](int r) -> long long { return (long long)(min(max(r, -1), H) + 1) * ld + V * ll; };

  // ---- stage 1 (level l): the rows of k_mg_zero_restrict
  struct In {
    T f[V];
    int p[V];
  };
  struct Wn {
    Row<T, V> v;
    T f[V];
    PRow<V> p;
  };
  auto load = [&](int y) {
    In r;
    const long long o = rowo(y);
    vload<T, V>(fb + o, r.f);
    if constexpr (MULTI) pload<V>(pb + o, r.p);
    return r;
  };
  auto mk = [&](const In& r, int y) {
    Wn w;
    const bool rin = y >= 1 && y <= H - 2;
    T x[V];
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const T omk = MULTI ? tab[r.p[k] * kTabStride + 9] : om;
      x[k] = (rin && cin[k]) ? omk * r.f[k] : T(0);
      w.f[k] = r.f[k];
    }
    w.v = own_row<T, V>(x);
    if constexpr (MULTI) w.p = own_prow<T, V>(r.p);
    return w;
  };
  // residual of the window's middle row; x0 is the oldest row streamed (the top one unless REV)
  auto resid = [&](const Wn& x0, const Wn& x1, const Wn& x2, T (&r)[V + 1]) {
    const Wn& a = REV ? x2 : x0;
    const Wn& c = REV ? x0 : x2;
#pragma unroll
    for (int k = 0; k < V; ++k) r[k] = x1.f[k] - kapply<T, V, MULTI>(a.v, x1.v, c.v, a.p, x1.p, c.p, k, ks, tab);
    r[V] = shl1z(r[0]);
  };

  // ---- stage 2 (level l+1): v' window rows (streaming order, Va oldest); residual rows of f_{l+2}'s row pair
  Row<T, Q> Va{}, Vb{}, Vc{};
  PRow<Q> Qa{}, Qb{}, Qc{};
  T fp2[Q];  // f_{l+1} of the previous row pushed
  Row<T, Q> Ro{}, Re{};  // the last odd / even residual rows of level l+1
  PRow<Q> So{}, Se{};    // their patterns
#pragma unroll
  for (int q = 0; q < Q; ++q) fp2[q] = T(0);

  // push f_{l+1} row I (all lanes, exact on the valid ones); n = rows pushed before it
  // ODD: parity of I, a compile-time constant (the first row is even), so the residual-row rotation is static
  auto push = [&](int I, const T (&o)[Q], int n, auto odd_c) {
    constexpr bool ODD = decltype(odd_c)::value;
    int pq[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) pq[q] = 0;
    if constexpr (MULTI) {
      const int Ic = min(max(I, -1), Hc);
      pload<Q>(pcb + (long long)(Ic + 1) * g.ldc, pq);
    }
    T x[Q];
    const bool iin = I >= 1 && I <= Hc - 2;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const T omk = MULTI ? tab[pq[q] * kTabStride + 9] : om;
      x[q] = (iin && jin[q]) ? omk * o[q] : T(0);
    }
    Va = Vb;
    Vb = Vc;
    Vc = own_row<T, Q>(x);
    if constexpr (MULTI) {
      Qa = Qb;
      Qb = Qc;
      Qc = own_prow<T, Q>(pq);
    }
    if (n >= 2) {
      // residual row j = I - S of level l+1 (k_mg_zero_restrict's resid on the coarse values)
      T r[Q];
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        if constexpr (REV) r[q] = fp2[q] - kapply<T, Q, MULTI>(Vc, Vb, Va, Qc, Qb, Qa, q, ks, tab);
        else r[q] = fp2[q] - kapply<T, Q, MULTI>(Va, Vb, Vc, Qa, Qb, Qc, q, ks, tab);
      }
      const Row<T, Q> R = own_row<T, Q>(r);
      const int j = I - S;  // residual row index (odd when I is even)
      if constexpr (!ODD) {
        // j = 2K + S closes f_{l+2} row K: residual rows 2K-1, 2K, 2K+1 (Ro and R in streaming order)
        const int K = (j - S) / 2;
        if (K >= K0 && K < K1) {
          // one output column per lane: fp64 the lane's own column when it is even, fp32 its second one
          constexpr int B0 = Q == 1 ? 0 : 1;     // window index of column 2M-1
          const int Jm = J0 + (Q == 1 ? 0 : 1);  // column 2M
          const int M = Jm / 2;
          const Row<T, Q>& r0 = REV ? R : Ro;  // row 2K-1
          const Row<T, Q>& r2 = REV ? Ro : R;  // row 2K+1
          T acc;
          if constexpr (!MULTI) {
            acc = rs[0] * r0.a[B0];
            acc += rs[1] * r0.a[B0 + 1];
            acc += rs[2] * r0.a[B0 + 2];
            acc += rs[3] * Re.a[B0];
            acc += rs[4] * Re.a[B0 + 1];
            acc += rs[5] * Re.a[B0 + 2];
            acc += rs[6] * r2.a[B0];
            acc += rs[7] * r2.a[B0 + 1];
            acc += rs[8] * r2.a[B0 + 2];
          } else {
            const PRow<Q>& p0 = REV ? Qb : So;
            const PRow<Q>& p2 = REV ? So : Qb;
            acc = tabv(rtb, p0.a[B0], 0) * r0.a[B0];
            acc += tabv(rtb, p0.a[B0 + 1], 1) * r0.a[B0 + 1];
            acc += tabv(rtb, p0.a[B0 + 2], 2) * r0.a[B0 + 2];
            acc += tabv(rtb, Se.a[B0], 3) * Re.a[B0];
            acc += tabv(rtb, Se.a[B0 + 1], 4) * Re.a[B0 + 1];
            acc += tabv(rtb, Se.a[B0 + 2], 5) * Re.a[B0 + 2];
            acc += tabv(rtb, p2.a[B0], 6) * r2.a[B0];
            acc += tabv(rtb, p2.a[B0 + 1], 7) * r2.a[B0 + 1];
            acc += tabv(rtb, p2.a[B0 + 2], 8) * r2.a[B0 + 2];
          }
          if (!(Jm & 1) && M >= Mlo && M < Mhi && M <= Wc2 - 2) {
            const T o2 = w0 * acc;
            cb2[(long long)(K + 1) * g.ldc2 + M] = o2;
            gather_store(g, id.b, K, M, o2);
          }
        }
        Ro = R;
        if constexpr (MULTI) So = Qb;
      } else {
        Re = R;
        if constexpr (MULTI) Se = Qb;
      }
    }
#pragma unroll
    for (int q = 0; q < Q; ++q) fp2[q] = o[q];
  };

  const int Ia = 2 * K0 - 2, Ib = 2 * K1;  // f_{l+1} rows computed (Ia .. Ib inclusive)
  const int Is = REV ? Ib : Ia;            // first row streamed
  Wn X0 = mk(load(2 * Is - 2 * S), 2 * Is - 2 * S);
  Wn X1 = mk(load(2 * Is - S), 2 * Is - S);
  Wn X2 = mk(load(2 * Is), 2 * Is);
  T Rp[V + 1], Rm[V + 1], Rn[V + 1];  // residual rows 2I - S (carried), 2I, 2I + S of the current row I
  PRow<V> Pp = X1.p, Pm, Pn;
  resid(X0, X1, X2, Rp);
  // the two fine rows 2I + S, 2I + 2S of a coarse row are loaded two coarse rows ahead, in ring slots indexed
  // by the row's parity (compile-time), as in k_mg_zero_restrict
  In ring[2][2];
#pragma unroll
  for (int d = 0; d < 2; ++d) {
    ring[d][0] = load(2 * Is + S + 2 * d * S);
    ring[d][1] = load(2 * Is + 2 * S + 2 * d * S);
  }
  auto row = [&](int I, int n, auto odd_c) {
    constexpr int SL = decltype(odd_c)::value ? 1 : 0;
    X0 = X1;  // window centred on fine row 2I
    X1 = X2;
    X2 = mk(ring[SL][0], 2 * I + S);
    ring[SL][0] = load(2 * I + 5 * S);
    resid(X0, X1, X2, Rm);
    Pm = X1.p;
    X0 = X1;  // window centred on fine row 2I + S
    X1 = X2;
    X2 = mk(ring[SL][1], 2 * I + 2 * S);
    ring[SL][1] = load(2 * I + 6 * S);
    resid(X0, X1, X2, Rn);
    Pn = X1.p;
    // rows 2I-1 (Ra), 2I (Rm), 2I+1 (Rc) in grid order
    const T(&Ra)[V + 1] = REV ? Rn : Rp;
    const T(&Rc)[V + 1] = REV ? Rp : Rn;
    const PRow<V>& Pa = REV ? Pn : Pp;
    const PRow<V>& Pc = REV ? Pp : Pn;
    T o[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      T acc;
      if constexpr (!MULTI) {
        acc = rs[0] * Ra[2 * q];
        acc += rs[1] * Ra[2 * q + 1];
        acc += rs[2] * Ra[2 * q + 2];
        acc += rs[3] * Rm[2 * q];
        acc += rs[4] * Rm[2 * q + 1];
        acc += rs[5] * Rm[2 * q + 2];
        acc += rs[6] * Rc[2 * q];
        acc += rs[7] * Rc[2 * q + 1];
        acc += rs[8] * Rc[2 * q + 2];
      } else {
        acc = tabv(rtb, Pa.a[2 * q + 1], 0) * Ra[2 * q];
        acc += tabv(rtb, Pa.a[2 * q + 2], 1) * Ra[2 * q + 1];
        acc += tabv(rtb, Pa.a[2 * q + 3], 2) * Ra[2 * q + 2];
        acc += tabv(rtb, Pm.a[2 * q + 1], 3) * Rm[2 * q];
        acc += tabv(rtb, Pm.a[2 * q + 2], 4) * Rm[2 * q + 1];
        acc += tabv(rtb, Pm.a[2 * q + 3], 5) * Rm[2 * q + 2];
        acc += tabv(rtb, Pc.a[2 * q + 1], 6) * Rc[2 * q];
        acc += tabv(rtb, Pc.a[2 * q + 2], 7) * Rc[2 * q + 1];
        acc += tabv(rtb, Pc.a[2 * q + 3], 8) * Rc[2 * q + 2];
      }
      o[q] = w0 * acc;
    }
    // f_{l+1}: owned rows and columns only
    if (I >= Ilo && I < Ihi) {
      T* cp = cb + (long long)(I + 1) * g.ldc;
#pragma unroll
      for (int q = 0; q < Q; ++q)
        if (J0 + q >= Jlo && J0 + q < Jhi && J0 + q <= Wc - 2) cp[q] = o[q];
    }
    push(I, o, n, odd_c);
#pragma unroll
    for (int k = 0; k <= V; ++k) Rp[k] = Rn[k];
    Pp = Pn;
  };
  // Ib - Ia + 1 = 2 (K1 - K0) + 3 rows: pairs (even, odd), then the last (even) row
  int n = 0, I = Is;
  for (; REV ? I - 1 >= Ia : I + 1 <= Ib; I += 2 * S, n += 2) {
    row(I, n, std::false_type{});
    row(I + S, n + 1, std::true_type{});
  }
  row(I, n, std::false_type{});
}

template <typename T, bool MULTI>
__global__ __launch_bounds__(256) void k_mg_zero_restrict2(MgArgs<T> g) {
  __shared__ T tab[MULTI ? FEA_MAX_PATTERNS * kTabStride : 1];
  __shared__ T rtb[MULTI ? FEA_MAX_PATTERNS * kTabStride : 1];
  if constexpr (MULTI) {
    load_tables<T>(tab, g.ktab, g.omd, g.ntab, rtb, g.rtab, g.nrtab);
    __syncthreads();
  }
  const TaskId id = decode_task_lin(g.nstrips, g.ntr);
  if (!id.valid) return;
  if (kZr2Alternate && (id.t & 1)) zr2_task<T, MULTI, true>(g, id, tab, rtb);
  else zr2_task<T, MULTI, false>(g, id, tab, rtb);
}

// Kernel C: fused prolongation + correction (+ post-sweep):
//   v = u + w1 * P(ec)   (P kernel of the coarse node);   out = SWEEP ? J(v, f) : v
// ZU (with SWEEP): the level's iterate is its zero-guess pre-sweep u = omd*f (interior, 0 on the
// boundary) — recomputed from the f rows the sweep reads anyway instead of being stored by the
// restriction and re-read here (bitwise the same product; 16 B per node less traffic in fp64).
// ---------------------------------------------------------------------------
template <typename T, int V>
struct CRow {  // coarse row at coarse columns b_base-1 .. b_base+V/2 (V/2+2 values)
  T e[V / 2 + 2];
  int o[V / 2 + 2];
};
template <typename T, int V>
struct RawC {
  T x[V / 2];
  T h;
  int px[V / 2];
  int ph;
};

// lq: the lane whose columns this lane loads (lane itself, or the last lane that holds a needed column
// when the strip runs past the grid: the lanes beyond then re-read one line instead of streaming
// columns nothing uses)
template <typename T, int V, bool MULTI>
__device__ __forceinline__ RawC<T, V> raw_crow(const T* __restrict__ ep, const uint8_t* __restrict__ pp, int lane,
                                               int lq) {
  constexpr int Q = V / 2;
  RawC<T, V> c;
  vload<T, Q>(ep + Q * lq, c.x);
  c.h = ep[lane < 32 ? -1 : kWave * Q];
  if constexpr (MULTI) {
#pragma unroll
    for (int q = 0; q < Q; ++q) c.px[q] = pp[Q * lq + q];
    c.ph = pp[lane < 32 ? -1 : kWave * Q];
  }
  return c;
}
template <typename T, int V, bool MULTI>
__device__ __forceinline__ RawC<T, V> raw_crow(const T* __restrict__ ep, const uint8_t* __restrict__ pp, int lane) {
  return raw_crow<T, V, MULTI>(ep, pp, lane, lane);
}

template <typename T, int V, bool MULTI>
__device__ __forceinline__ CRow<T, V> finish_c(const RawC<T, V>& r) {
  constexpr int Q = V / 2;
  CRow<T, V> c;
#pragma unroll
  for (int q = 0; q < Q; ++q) c.e[q + 1] = r.x[q];
  c.e[0] = shr1(r.x[Q - 1], r.h);
  c.e[Q + 1] = shl1(r.x[0], r.h);
  if constexpr (MULTI) {
#pragma unroll
    for (int q = 0; q < Q; ++q) c.o[q + 1] = r.px[q] * tab_row_bytes<T>();
    c.o[0] = shr1(r.px[Q - 1], r.ph) * tab_row_bytes<T>();
    c.o[Q + 1] = shl1(r.px[0], r.ph) * tab_row_bytes<T>();
  }
  return c;
}

// coarse row contribution sum_b P[pc(a,b)][ky][kx] e(a,b) at window column j (k = j-1)
template <typename T, int V, bool MULTI>
__device__ __forceinline__ T crow_term(const CRow<T, V>& c, int j, int ky, const T (&ps)[9], const T* ptb) {
  const int k = j - 1;
  if ((k & 1) != 0) {  // even fine column: one coarse node, kx = 1
    const int i = (k + 1) / 2;
    return (MULTI ? tabv(ptb, c.o[i], ky * 3 + 1) : ps[ky * 3 + 1]) * c.e[i];
  } else {  // odd fine column: coarse nodes k/2 (kx = 2) and k/2+1 (kx = 0)
    const int i = k / 2;
    T t = (MULTI ? tabv(ptb, c.o[i], ky * 3 + 2) : ps[ky * 3 + 2]) * c.e[i];
    t += (MULTI ? tabv(ptb, c.o[i + 1], ky * 3 + 0) : ps[ky * 3 + 0]) * c.e[i + 1];
    return t;
  }
}

template <typename T, int V, bool MULTI>
__device__ __forceinline__ void correct_even(Row<T, V>& u, const CRow<T, V>& ca, T w1, const T (&ps)[9],
                                             const T* ptb) {
#pragma unroll
  for (int j = 0; j <= V + 1; ++j) u.a[j] += w1 * crow_term<T, V, MULTI>(ca, j, 1, ps, ptb);
}

template <typename T, int V, bool MULTI>
__device__ __forceinline__ void correct_odd(Row<T, V>& u, const CRow<T, V>& ca, const CRow<T, V>& cb, T w1,
                                            const T (&ps)[9], const T* ptb) {
#pragma unroll
  for (int j = 0; j <= V + 1; ++j) {
    const T t = crow_term<T, V, MULTI>(ca, j, 2, ps, ptb) + crow_term<T, V, MULTI>(cb, j, 0, ps, ptb);
    u.a[j] += w1 * t;
  }
}

// prolongation(+sweep): iterations (2 fine rows each) whose loads are in flight at once
#ifndef FEA_PROLONG_AHEAD
#define FEA_PROLONG_AHEAD 2
#endif
constexpr int kProlongAhead = FEA_PROLONG_AHEAD;
static_assert(kProlongAhead >= 1 && kProlongAhead <= 4, "prolongation ring of 1..4 iterations");

template <typename T, bool MULTI, bool SWEEP, bool NT, bool ZU = false>
__global__ __launch_bounds__(256) void k_mg_prolong(MgArgs<T> g) {
  static_assert(!ZU || SWEEP, "ZU needs the sweep's f rows");
  using F = Frame<T>;
  constexpr int V = F::VEC;
  __shared__ T tab[MULTI ? FEA_MAX_PATTERNS * kTabStride : 1];
  __shared__ T ptb[MULTI ? FEA_MAX_PATTERNS * kTabStride : 1];
  if constexpr (MULTI) {
    load_tables<T>(tab, SWEEP ? g.ktab : g.ptab, SWEEP ? g.omd : nullptr, SWEEP ? g.ntab : 0, ptb, g.ptab,
                   g.nptab);
    __syncthreads();
  }
  const TaskId id = decode_task(g.nstrips, g.ntr);
  if (!id.valid) return;
  const int lane = lane_id();
  const int H = g.H, Hc = g.Hc, W = g.W;
  const int c0 = 1 + id.s * F::SW;
  const int r0 = 1 + id.t * g.rb;  // odd
  const int r1 = min(r0 + g.rb, H - 1);
  const int cl = c0 + V * lane;
  T ks[9], ps[9];
  T om = 0;
  if constexpr (!MULTI) {
#pragma unroll
    for (int d = 0; d < 9; ++d) {
      ks[d] = SWEEP ? g.ktab[d] : T(0);
      ps[d] = g.ptab[d];
    }
    om = SWEEP ? g.omd[0] : T(0);
  }
  const T w1 = g.w;
  const int ld = g.ld, ldc = g.ldc;
  const long long poff = F::OFF + c0;
  const long long boff = (long long)id.b * g.bs + poff;
  const T* __restrict__ fb = SWEEP ? g.f + boff : nullptr;
  const T* __restrict__ ub = ZU ? fb : g.u + boff;
  T* __restrict__ ob = g.out + boff;
  const uint8_t* __restrict__ pb = (MULTI && SWEEP) ? g.pid + poff : nullptr;
  // ZU: interior mask of the lane's window columns
  bool cin[V + 3];
#pragma unroll
  for (int j = 0; j < V + 3; ++j) {
    const int c = cl + j - 1;
    cin[j] = c >= 1 && c <= W - 2;
  }
  const int bc0 = (c0 + 1) / 2;
  const long long pcoff = F::OFF + bc0;
  const T* __restrict__ eb = g.ec + (long long)id.b * g.bsc + pcoff;
  const uint8_t* __restrict__ pcb = MULTI ? g.pidc + pcoff : nullptr;
  auto rowo = [&](int r) -> long long { return (long long)(min(r, H) + 1) * ld; };
  auto crowo = [&](int a) -> long long { return (long long)(min(a, Hc) + 1) * ldc; };

  auto rc = [&](int a) { return raw_crow<T, V, MULTI>(eb + crowo(a), MULTI ? pcb + crowo(a) : nullptr, lane); };
  auto ru = [&](int y) { return raw_row<T, V>(ub + rowo(y), lane); };
  auto rp = [&](int y) {
    RawP<V> p{};
    if constexpr (MULTI && SWEEP) p = raw_prow<V>(pb + rowo(y), lane);
    return p;
  };
  auto fp = [&](const RawP<V>& r) {
    PRow<V> p{};
    if constexpr (MULTI && SWEEP) p = finish_p<T>(r);
    return p;
  };
  auto rf = [&](int y, T (&fv)[V]) {
    if constexpr (SWEEP && !ZU) vload<T, V>(fb + rowo(y) + V * lane, fv);
  };
  // window row of the iterate from a loaded row: u itself, or (ZU) omd*f with f's own columns kept
  auto mk = [&](const RawRow<T, V>& raw, int y, const PRow<V>& p, T (&fo)[V]) {
    Row<T, V> r = finish(raw);
    if constexpr (ZU) {
      const bool rin = y >= 1 && y <= H - 2;
#pragma unroll
      for (int k = 0; k < V; ++k) fo[k] = r.a[k + 1];
#pragma unroll
      for (int j = 0; j < V + 3; ++j) {
        const T omj = MULTI ? tabv(tab, p.a[j], 9) : om;
        r.a[j] = (rin && cin[j]) ? omj * r.a[j] : T(0);
      }
    }
    return r;
  };
  auto emit = [&](int y, const Row<T, V>& a, const Row<T, V>& b, const Row<T, V>& c, const PRow<V>& pa,
                  const PRow<V>& pbb, const PRow<V>& pc, const T (&fv)[V]) {
    T o[V];
    if constexpr (SWEEP) {
#pragma unroll
      for (int k = 0; k < V; ++k) {
        const T acc = kapply<T, V, MULTI>(a, b, c, pa, pbb, pc, k, ks, tab);
        const T omk = MULTI ? tabv(tab, pbb.a[k + 1], 9) : om;
        o[k] = omk * (fv[k] - acc) + b.a[k + 1];
      }
    } else {
#pragma unroll
      for (int k = 0; k < V; ++k) o[k] = b.a[k + 1];
    }
    store_masked<T, V, NT>(ob + rowo(y) + V * lane, o, cl, W);
  };

  // window rows r0-1 (even, coarse a0) and r0 (odd, coarse a0, a0+1)
  const int a0 = (r0 - 1) / 2;
  CRow<T, V> C0 = finish_c<T, V, MULTI>(rc(a0));
  CRow<T, V> C1 = finish_c<T, V, MULTI>(rc(a0 + 1));
  PRow<V> Pp = fp(rp(r0 - 1)), Pc = fp(rp(r0));
  T fq[V], f0[V];  // ZU: f's own columns of rows r0-1 (unused), r0 (f0)
  Row<T, V> Vp = mk(ru(r0 - 1), r0 - 1, Pp, fq), Vc = mk(ru(r0), r0, Pc, f0);
  correct_even<T, V, MULTI>(Vp, C0, w1, ps, ptb);
  correct_odd<T, V, MULTI>(Vc, C0, C1, w1, ps, ptb);
  // Iteration y (odd) emits rows y and y+1 from fine rows y+1, y+2, coarse row (y+3)/2 and (not ZU)
  // f rows y, y+1.  Those loads are in flight kProlongAhead iterations ahead, in a ring of slots
  // indexed by the iteration's position (compile-time after the unroll below): a slot is consumed in
  // place and refilled at once, so no in-flight register is ever copied (a copy waits for its load).
  constexpr int D = kProlongAhead;
  struct Slot {
    RawRow<T, V> u1, u2;
    RawC<T, V> c;
    RawP<V> p1, p2;
    T f0[V], f1[V];
  };
  Slot ring[D];
  auto fill = [&](Slot& sl, int y) {
    sl.u1 = ru(y + 1);
    sl.u2 = ru(y + 2);
    sl.c = rc((y + 3) / 2);
    sl.p1 = rp(y + 1);
    sl.p2 = rp(y + 2);
    rf(y, sl.f0);
    rf(y + 1, sl.f1);
  };
#pragma unroll
  for (int d = 0; d < D; ++d) fill(ring[d], r0 + 2 * d);
  // ZU: f's own columns of row y come from the previous iteration's window row (f0 above)
  auto iter = [&](int y, auto slot) {
    Slot& sl = ring[decltype(slot)::value];
    T fa[V], fb1[V];  // f's own columns of rows y, y+1 (ZU: fb1 is filled from the window row)
#pragma unroll
    for (int k = 0; k < V; ++k) {
      if constexpr (ZU) {
        fa[k] = f0[k];
      } else {
        fa[k] = sl.f0[k];
        fb1[k] = sl.f1[k];
      }
    }
    // row y+1 (even, coarse (y+1)/2 = C1)
    const PRow<V> Pn = fp(sl.p1);
    Row<T, V> Vn = mk(sl.u1, y + 1, Pn, fb1);
    correct_even<T, V, MULTI>(Vn, C1, w1, ps, ptb);
    emit(y, Vp, Vc, Vn, Pp, Pc, Pn, fa);
    if (y + 1 < r1) {
      // row y+2 (odd, coarse (y+1)/2 and (y+3)/2)
      const CRow<T, V> C2 = finish_c<T, V, MULTI>(sl.c);
      const PRow<V> Pnn = fp(sl.p2);
      T g0[V];
      Row<T, V> Vnn = mk(sl.u2, y + 2, Pnn, g0);
      correct_odd<T, V, MULTI>(Vnn, C1, C2, w1, ps, ptb);
      emit(y + 1, Vc, Vn, Vnn, Pc, Pn, Pnn, fb1);
      Vp = Vn;
      Vc = Vnn;
      Pp = Pn;
      Pc = Pnn;
      C1 = C2;
#pragma unroll
      for (int k = 0; k < V; ++k) f0[k] = g0[k];
    }
    fill(sl, y + 2 * D);
  };
  int y = r0;
  for (; y + 2 * (D - 1) < r1; y += 2 * D) {
    iter(y, std::integral_constant<int, 0>{});
    if constexpr (D > 1) iter(y + 2, std::integral_constant<int, 1 % D>{});
    if constexpr (D > 2) iter(y + 4, std::integral_constant<int, 2 % D>{});
    if constexpr (D > 3) iter(y + 6, std::integral_constant<int, 3 % D>{});
  }
  if constexpr (D > 1)
    if (y < r1) iter(y, std::integral_constant<int, 0>{});
  if constexpr (D > 2)
    if (y + 2 < r1) iter(y + 2, std::integral_constant<int, 1 % D>{});
  if constexpr (D > 3)
    if (y + 4 < r1) iter(y + 4, std::integral_constant<int, 2 % D>{});
}

// ---------------------------------------------------------------------------
// Kernel C0: k_mg_prolong<SWEEP, ZU> (levels >= 1 going up) on OVERLAPPED strips:
//   x = omd f + w1 P(ec)  (interior),   out = J(x, f)
// x of a node needs only its own f and the coarse nodes left of and under it, so a wave forms x on the
// columns it loads (the coarse left neighbour by DPP) and takes the sweep's window neighbours by DPP: no
// halo loads, the correction at VEC instead of VEC+2 columns per lane and omd f at VEC instead of VEC+3.
// Lanes 1..OWN store.  Same per-node expressions (crow_term, correction order, sweep) as k_mg_prolong,
// so the output is bitwise the same.
// ---------------------------------------------------------------------------
template <typename T, bool MULTI, bool NT>
__global__ __launch_bounds__(256) void k_mg_prolong_zu_ovl(MgArgs<T> g) {
  using F = Frame<T>;
  using O = Ovl<T>;
  constexpr int V = F::VEC;
  constexpr int Q = V / 2;
  __shared__ T tab[MULTI ? FEA_MAX_PATTERNS * kTabStride : 1];
  __shared__ T ptb[MULTI ? FEA_MAX_PATTERNS * kTabStride : 1];
  if constexpr (MULTI) {
    load_tables<T>(tab, g.ktab, g.omd, g.ntab, ptb, g.ptab, g.nptab);
    __syncthreads();
  }
  const TaskId id = decode_task_lin(g.nstrips, g.ntr);
  if (!id.valid) return;
  const int lane = lane_id();
  const int H = g.H, Hc = g.Hc, W = g.W;
  const int c0 = 1 + id.s * O::S;  // first owned fine column
  const int cs = c0 - V;           // first loaded column
  const int cl = cs + V * lane;    // odd
  const int r0 = 1 + id.t * g.rb;  // odd
  const int r1 = min(r0 + g.rb, H - 1);
  T ks[9], ps[9];
  T om = 0;
  if constexpr (!MULTI) {
#pragma unroll
    for (int d = 0; d < 9; ++d) {
      ks[d] = g.ktab[d];
      ps[d] = g.ptab[d];
    }
    om = g.omd[0];
  }
  const T w1 = g.w;
  const int ld = g.ld, ldc = g.ldc;
  bool cin[V];
#pragma unroll
  for (int k = 0; k < V; ++k) cin[k] = cl + k >= 1 && cl + k <= W - 2;
  const bool own = lane >= 1 && lane <= O::OWN;
  const int ll = min(lane, (W - 1 - cs) / V);  // lanes past the grid re-read the last needed line
  const long long boff = (long long)id.b * g.bs + F::OFF + cs;
  const T* __restrict__ fb = g.f + boff;
  T* __restrict__ ob = g.out + boff;
  const uint8_t* __restrict__ pb = MULTI ? g.pid + F::OFF + cs : nullptr;
  const int jc = (cs + 1) / 2;  // coarse column of lane 0's first own coarse node
  const long long pcoff = F::OFF + jc;
  const T* __restrict__ eb = g.ec + (long long)id.b * g.bsc + pcoff;
  const uint8_t* __restrict__ pcb = MULTI ? g.pidc + pcoff : nullptr;
  auto rowo = [&](int r) -> long long { return (long long)(min(max(r, -1), H) + 1) * ld + V * ll; };
  auto crowo = [&](int a) -> long long { return (long long)(min(a, Hc) + 1) * ldc + Q * ll; };

  struct In {
    T f[V];
    int p[V];
  };
  struct RC {
    T x[Q];
    int p[Q];
  };
  struct XR {  // window row of the corrected iterate x, its pattern window, f's own columns
    Row<T, V> x;
    PRow<V> p;
    T f[V];
  };
  auto ld_f = [&](int y) {
    In r;
    const long long o = rowo(y);
    vload<T, V>(fb + o, r.f);
    if constexpr (MULTI) pload<V>(pb + o, r.p);
    return r;
  };
  auto ld_c = [&](int a) {
    RC r;
    const long long o = crowo(a);
    vload<T, Q>(eb + o, r.x);
    if constexpr (MULTI) {
#pragma unroll
      for (int q = 0; q < Q; ++q) r.p[q] = pcb[o + q];
    }
    return r;
  };
  auto fin_c = [&](const RC& r) {  // e[0] = the left lane's last coarse node, e[1..Q] own (e[Q+1] unused)
    CRow<T, V> c{};
#pragma unroll
    for (int q = 0; q < Q; ++q) c.e[q + 1] = r.x[q];
    c.e[0] = shr1z(r.x[Q - 1]);
    if constexpr (MULTI) {
#pragma unroll
      for (int q = 0; q < Q; ++q) c.o[q + 1] = r.p[q] * tab_row_bytes<T>();
      c.o[0] = shr1z(r.p[Q - 1]) * tab_row_bytes<T>();
    }
    return c;
  };
  // omd f of row y on the lane's own columns, then the correction of an even (ky = 1) or odd row
  auto zero_iterate = [&](const In& r, int y, T (&x)[V]) {
    const bool rin = y >= 1 && y <= H - 2;
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const T omk = MULTI ? tab[r.p[k] * kTabStride + 9] : om;
      x[k] = (rin && cin[k]) ? omk * r.f[k] : T(0);
    }
  };
  auto finish_x = [&](const In& r, const T (&x)[V]) {
    XR w;
    w.x = own_row<T, V>(x);
    if constexpr (MULTI) w.p = own_prow<T, V>(r.p);
#pragma unroll
    for (int k = 0; k < V; ++k) w.f[k] = r.f[k];
    return w;
  };
  auto row_even = [&](const In& r, int y, const CRow<T, V>& ca) {
    T x[V];
    zero_iterate(r, y, x);
#pragma unroll
    for (int k = 0; k < V; ++k) x[k] += w1 * crow_term<T, V, MULTI>(ca, k + 1, 1, ps, ptb);
    return finish_x(r, x);
  };
  auto row_odd = [&](const In& r, int y, const CRow<T, V>& ca, const CRow<T, V>& cb) {
    T x[V];
    zero_iterate(r, y, x);
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const T t = crow_term<T, V, MULTI>(ca, k + 1, 2, ps, ptb) + crow_term<T, V, MULTI>(cb, k + 1, 0, ps, ptb);
      x[k] += w1 * t;
    }
    return finish_x(r, x);
  };
  auto emit = [&](int y, const XR& a, const XR& b, const XR& c) {
    T o[V];
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const T acc = kapply<T, V, MULTI>(a.x, b.x, c.x, a.p, b.p, c.p, k, ks, tab);
      const T omk = MULTI ? tabv(tab, b.p.a[k + 1], 9) : om;
      o[k] = omk * (b.f[k] - acc) + b.x.a[k + 1];
    }
    if (own) store_masked<T, V, NT>(ob + rowo(y), o, cl, W);
  };

  // window rows r0-1 (even, coarse a0) and r0 (odd, coarse a0, a0+1)
  const int a0 = (r0 - 1) / 2;
  const CRow<T, V> C0 = fin_c(ld_c(a0));
  CRow<T, V> C1 = fin_c(ld_c(a0 + 1));
  XR Xp = row_even(ld_f(r0 - 1), r0 - 1, C0);
  XR Xc = row_odd(ld_f(r0), r0, C0, C1);
  // iteration y (odd) emits rows y and y+1 from fine rows y+1, y+2 and coarse row (y+3)/2, whose loads
  // are in flight kProlongAhead iterations ahead (ring slots consumed in place, refilled at once)
  constexpr int D = kProlongAhead;
  struct Slot {
    In u1, u2;
    RC c;
  };
  Slot ring[D];
  auto fill = [&](Slot& sl, int y) {
    sl.u1 = ld_f(y + 1);
    sl.u2 = ld_f(y + 2);
    sl.c = ld_c((y + 3) / 2);
  };
#pragma unroll
  for (int d = 0; d < D; ++d) fill(ring[d], r0 + 2 * d);
  auto iter = [&](int y, auto slot) {
    Slot& sl = ring[decltype(slot)::value];
    const XR Xn = row_even(sl.u1, y + 1, C1);  // row y+1 (even, coarse (y+1)/2 = C1)
    emit(y, Xp, Xc, Xn);
    if (y + 1 < r1) {  // row y+2 (odd, coarse (y+1)/2 and (y+3)/2)
      const CRow<T, V> C2 = fin_c(sl.c);
      const XR Xnn = row_odd(sl.u2, y + 2, C1, C2);
      emit(y + 1, Xc, Xn, Xnn);
      Xp = Xn;
      Xc = Xnn;
      C1 = C2;
    }
    fill(sl, y + 2 * D);
  };
  int y = r0;
  for (; y + 2 * (D - 1) < r1; y += 2 * D) {
    iter(y, std::integral_constant<int, 0>{});
    if constexpr (D > 1) iter(y + 2, std::integral_constant<int, 1 % D>{});
    if constexpr (D > 2) iter(y + 4, std::integral_constant<int, 2 % D>{});
    if constexpr (D > 3) iter(y + 6, std::integral_constant<int, 3 % D>{});
  }
  if constexpr (D > 1)
    if (y < r1) iter(y, std::integral_constant<int, 0>{});
  if constexpr (D > 2)
    if (y + 2 < r1) iter(y + 2, std::integral_constant<int, 1 % D>{});
  if constexpr (D > 3)
    if (y + 4 < r1) iter(y + 4, std::integral_constant<int, 2 % D>{});
}

// ---------------------------------------------------------------------------
// Two recomputed-iterate prolongations in one pass (levels l+1 and l going up, below the multi-level launch):
//   x' = omd f_{l+1} + w1 P(e_{l+2});  u' = J(x', f_{l+1});  x = omd f_l + w1 P(u');  out = J(x, f_l)
// k_mg_prolong_zu_ovl on level l, whose coarse correction rows u' come from a second stage on the coarse
// values in registers (one per lane in fp64, two in fp32; neighbours by DPP) instead of a separate launch:
// u' is never stored.  Each strip loads three lanes left of the S it owns, so the coarse stage is exact on
// every lane the fine one reads; the coarse stage advances one row per two fine rows, its inputs in the same
// prefetch ring.  Same per-node expressions and order as the two single-level launches (bitwise:
// tests/test_gpu_mg.py::test_prolong2_bitwise).
// ---------------------------------------------------------------------------
template <typename T>
struct Ovl4 {
  static constexpr int V = Frame<T>::VEC;
  static constexpr int HL = 3;          // lanes of left halo; owning lanes HL .. 61
  static constexpr int S = 59 * V;      // owned fine columns per strip (fp64 118, fp32 236)
};

// PROLONG2 ALT: odd row tasks stream bottom-up (REV), so vertically adjacent tasks read the rows they share (the
// fine halo row, the coarse stage's extra rows) at the same moment and the second read is an L2 hit.
#ifndef FEA_PROLONG2_ALT
#define FEA_PROLONG2_ALT 1
#endif
constexpr bool kProlong2Alternate = FEA_PROLONG2_ALT != 0;

template <typename T, bool MULTI, bool REV>
__device__ __forceinline__ void prolong2_task(const MgArgs<T>& g, const TaskId& id, const T* tab, const T* ptb) {
  using F = Frame<T>;
  using O = Ovl4<T>;
  constexpr int V = F::VEC;
  constexpr int Q = V / 2;
  const int lane = lane_id();
  const int H = g.H, Hc = g.Hc, W = g.W, Wc = g.Wc, Hc2 = g.Hc2, Wc2 = g.Wc2;
  const int c0 = 1 + id.s * O::S;  // first owned fine column
  const int cs = c0 - O::HL * V;   // first loaded column (odd)
  const int cl = cs + V * lane;
  const int r0 = 1 + id.t * g.rb;  // odd
  const int r1 = min(r0 + g.rb, H - 1);
  T ks[9], ps[9];
  T om = 0;
  if constexpr (!MULTI) {
#pragma unroll
    for (int d = 0; d < 9; ++d) {
      ks[d] = g.ktab[d];
      ps[d] = g.ptab[d];
    }
    om = g.omd[0];
  }
  const T w1 = g.w;
  const int ld = g.ld, ldc = g.ldc, ldc2 = g.ldc2;
  bool cin[V];
#pragma unroll
  for (int k = 0; k < V; ++k) cin[k] = cl + k >= 1 && cl + k <= W - 2;
  const bool own = lane >= O::HL && lane < 64 - 2;
  const int ll = min(lane, (W - 1 - cs) / V);  // lanes past the grid re-read the last needed line
  const long long boff = (long long)id.b * g.bs + F::OFF + cs;
  const T* __restrict__ fb = g.f + boff;
  T* __restrict__ ob = g.out + boff;
  const uint8_t* __restrict__ pb = MULTI ? g.pid + F::OFF + cs : nullptr;
  const int jc = (cs + 1) / 2;   // coarse column of lane 0's first own coarse node
  const int J0 = jc + Q * ll;    // this lane's first coarse column (the loaded one)
  const T* __restrict__ f2b = g.ec + (long long)id.b * g.bsc + F::OFF + J0;  // f_{l+1} (in ec)
  const uint8_t* __restrict__ p2b = MULTI ? g.pidc + F::OFF + J0 : nullptr;
  bool jin[Q];
#pragma unroll
  for (int q = 0; q < Q; ++q) jin[q] = J0 + q >= 1 && J0 + q <= Wc - 2;
  // level l+2 columns KL, KL+1 feed this lane's coarse columns (odd J: (J-1)/2, (J+1)/2; even J: J/2)
  const int KL = min((J0 - 1) >> 1, Wc2 - 2);
  const T* __restrict__ e3b = g.ec2 + (long long)id.b * g.bsc2 + F::OFF + KL;
  const uint8_t* __restrict__ p3b = MULTI ? g.pidc2 + F::OFF + KL : nullptr;
  auto rowo = [&](int r) -> long long { return (long long)(min(max(r, -1), H) + 1) * ld + V * ll; };
  auto crowo = [&](int a) -> long long { return (long long)(min(max(a, -1), Hc) + 1) * ldc; };
  auto c2rowo = [&](int a) -> long long { return (long long)(min(max(a, -1), Hc2) + 1) * ldc2; };

  // ---- coarse stage (level l+1): x' and u' rows ----
  struct In2 {  // inputs of x' row b: f_{l+1} (own coarse columns), patterns, e_{l+2} rows b>>1, (b>>1)+1
    T f[Q];
    int p[Q];
    T e[2][2];
    int pe[2][2];
  };
  auto ld2 = [&](int b) {
    In2 r;
    vload<T, Q>(f2b + crowo(b), r.f);
    if constexpr (MULTI) pload<Q>(p2b + crowo(b), r.p);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const long long o = c2rowo((b >> 1) + h);
      r.e[h][0] = e3b[o];
      r.e[h][1] = e3b[o + 1];
      if constexpr (MULTI) {
        r.pe[h][0] = p3b[o] * tab_row_bytes<T>();
        r.pe[h][1] = p3b[o + 1] * tab_row_bytes<T>();
      }
    }
    return r;
  };
  // crow_term on level l+2 values for coarse column Jq (bitwise k_mg_prolong_zu_ovl's coarse term)
  auto term2 = [&](const T (&e)[2], const int (&pe)[2], int Jq, int ky) -> T {
    if (Jq & 1) {  // odd: (Jq-1)/2 (kx = 2) and (Jq+1)/2 (kx = 0) — KL and KL+1
      T t = (MULTI ? tabv(ptb, pe[0], ky * 3 + 2) : ps[ky * 3 + 2]) * e[0];
      t += (MULTI ? tabv(ptb, pe[1], ky * 3 + 0) : ps[ky * 3 + 0]) * e[1];
      return t;
    }
    return (MULTI ? tabv(ptb, pe[1], ky * 3 + 1) : ps[ky * 3 + 1]) * e[1];  // even: Jq/2 = KL+1
  };
  struct X2 {
    Row<T, Q> x;
    PRow<Q> p;
    T f[Q];
  };
  auto mkx2 = [&](const In2& r, int b) {
    const bool bin = b >= 1 && b <= Hc - 2;
    T x[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const T omk = MULTI ? tab[r.p[q] * kTabStride + 9] : om;
      x[q] = (bin && jin[q]) ? omk * r.f[q] : T(0);
    }
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int Jq = J0 + q;
      if (b & 1) {
        const T t = term2(r.e[0], r.pe[0], Jq, 2) + term2(r.e[1], r.pe[1], Jq, 0);
        x[q] += w1 * t;
      } else {
        x[q] += w1 * term2(r.e[0], r.pe[0], Jq, 1);
      }
    }
    X2 w;
    w.x = own_row<T, Q>(x);
    if constexpr (MULTI) w.p = own_prow<T, Q>(r.p);
#pragma unroll
    for (int q = 0; q < Q; ++q) w.f[q] = r.f[q];
    return w;
  };
  // u' row a from x' rows a-1, a, a+1 -> the fine stage's coarse row (e[0] = left lane's last, e[1..Q] own)
  auto mku2 = [&](const X2& a_, const X2& b_, const X2& c_, int a) {
    const bool ain = a >= 1 && a <= Hc - 2;
    T o[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const T acc = kapply<T, Q, MULTI>(a_.x, b_.x, c_.x, a_.p, b_.p, c_.p, q, ks, tab);
      const T omk = MULTI ? tabv(tab, b_.p.a[q + 1], 9) : om;
      const T u = omk * (b_.f[q] - acc) + b_.x.a[q + 1];
      o[q] = (ain && jin[q]) ? u : T(0);
    }
    CRow<T, V> c{};
#pragma unroll
    for (int q = 0; q < Q; ++q) c.e[q + 1] = o[q];
    c.e[0] = shr1z(o[Q - 1]);
    if constexpr (MULTI) {
#pragma unroll
      for (int q = 0; q < Q; ++q) c.o[q + 1] = b_.p.a[q + 1];
      c.o[0] = b_.p.a[0];
    }
    return c;
  };

  // ---- fine stage (level l): k_mg_prolong_zu_ovl ----
  struct In {
    T f[V];
    int p[V];
  };
  struct XR {
    Row<T, V> x;
    PRow<V> p;
    T f[V];
  };
  auto ld_f = [&](int y) {
    In r;
    const long long o = rowo(y);
    vload<T, V>(fb + o, r.f);
    if constexpr (MULTI) pload<V>(pb + o, r.p);
    return r;
  };
  auto zero_iterate = [&](const In& r, int y, T (&x)[V]) {
    const bool rin = y >= 1 && y <= H - 2;
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const T omk = MULTI ? tab[r.p[k] * kTabStride + 9] : om;
      x[k] = (rin && cin[k]) ? omk * r.f[k] : T(0);
    }
  };
  auto finish_x = [&](const In& r, const T (&x)[V]) {
    XR w;
    w.x = own_row<T, V>(x);
    if constexpr (MULTI) w.p = own_prow<T, V>(r.p);
#pragma unroll
    for (int k = 0; k < V; ++k) w.f[k] = r.f[k];
    return w;
  };
  auto row_even = [&](const In& r, int y, const CRow<T, V>& ca) {
    T x[V];
    zero_iterate(r, y, x);
#pragma unroll
    for (int k = 0; k < V; ++k) x[k] += w1 * crow_term<T, V, MULTI>(ca, k + 1, 1, ps, ptb);
    return finish_x(r, x);
  };
  auto row_odd = [&](const In& r, int y, const CRow<T, V>& ca, const CRow<T, V>& cb) {
    T x[V];
    zero_iterate(r, y, x);
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const T t = crow_term<T, V, MULTI>(ca, k + 1, 2, ps, ptb) + crow_term<T, V, MULTI>(cb, k + 1, 0, ps, ptb);
      x[k] += w1 * t;
    }
    return finish_x(r, x);
  };
  auto emit = [&](int y, const XR& a, const XR& b, const XR& c) {
    T o[V];
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const T acc = kapply<T, V, MULTI>(a.x, b.x, c.x, a.p, b.p, c.p, k, ks, tab);
      const T omk = MULTI ? tabv(tab, b.p.a[k + 1], 9) : om;
      o[k] = omk * (b.f[k] - acc) + b.x.a[k + 1];
    }
    if (own) store_masked<T, V, false>(ob + rowo(y), o, cl, W);
  };

  if constexpr (!REV) {
    // coarse stage start: x' rows a0-1 .. a0+2 -> u' rows a0 (C0), a0+1 (C1)
    const int a0 = (r0 - 1) / 2;
    X2 Xa = mkx2(ld2(a0 - 1), a0 - 1);
    X2 Xb = mkx2(ld2(a0), a0);
    X2 Xc2 = mkx2(ld2(a0 + 1), a0 + 1);
    const CRow<T, V> C0 = mku2(Xa, Xb, Xc2, a0);
    Xa = Xb;
    Xb = Xc2;
    Xc2 = mkx2(ld2(a0 + 2), a0 + 2);
    CRow<T, V> C1 = mku2(Xa, Xb, Xc2, a0 + 1);
    XR Xp = row_even(ld_f(r0 - 1), r0 - 1, C0);
    XR Xc = row_odd(ld_f(r0), r0, C0, C1);
    // iteration y (odd) emits fine rows y, y+1 from fine rows y+1, y+2 and u' row (y+3)/2, which needs x' row
    // (y+5)/2: those loads are in flight kProlongAhead iterations ahead (ring slots consumed in place)
    constexpr int D = kProlongAhead;
    struct Slot {
      In u1, u2;
      In2 c;
    };
    Slot ring[D];
    auto fill = [&](Slot& sl, int y) {
      sl.u1 = ld_f(y + 1);
      sl.u2 = ld_f(y + 2);
      sl.c = ld2((y + 5) / 2);
    };
  #pragma unroll
    for (int d = 0; d < D; ++d) fill(ring[d], r0 + 2 * d);
    auto iter = [&](int y, auto slot) {
      Slot& sl = ring[decltype(slot)::value];
      const XR Xn = row_even(sl.u1, y + 1, C1);  // row y+1 (even, coarse (y+1)/2 = C1)
      emit(y, Xp, Xc, Xn);
      if (y + 1 < r1) {  // row y+2 (odd, coarse (y+1)/2 and (y+3)/2)
        Xa = Xb;
        Xb = Xc2;
        Xc2 = mkx2(sl.c, (y + 5) / 2);
        const CRow<T, V> C2 = mku2(Xa, Xb, Xc2, (y + 3) / 2);
        const XR Xnn = row_odd(sl.u2, y + 2, C1, C2);
        emit(y + 1, Xc, Xn, Xnn);
        Xp = Xn;
        Xc = Xnn;
        C1 = C2;
      }
      fill(sl, y + 2 * D);
    };
    int y = r0;
    for (; y + 2 * (D - 1) < r1; y += 2 * D) {
      iter(y, std::integral_constant<int, 0>{});
      if constexpr (D > 1) iter(y + 2, std::integral_constant<int, 1 % D>{});
      if constexpr (D > 2) iter(y + 4, std::integral_constant<int, 2 % D>{});
      if constexpr (D > 3) iter(y + 6, std::integral_constant<int, 3 % D>{});
    }
    if constexpr (D > 1)
      if (y < r1) iter(y, std::integral_constant<int, 0>{});
    if constexpr (D > 2)
      if (y + 2 < r1) iter(y + 2, std::integral_constant<int, 1 % D>{});
    if constexpr (D > 3)
      if (y + 4 < r1) iter(y + 4, std::integral_constant<int, 2 % D>{});
  } else {
    // bottom-up: pairs of fine rows (y + 1 even, then y odd) for odd y from the last one down; entering the pair
    // of y the window holds x(y + 2), x(y + 1), the coarse stage u'((y + 1) / 2) and x' rows (y+3)/2 .. (y-1)/2
    const int yl = r1 - 1;
    const int yt = (yl & 1) ? yl : yl - 1;  // first (bottom) pair
    const int A = (yt + 1) / 2;
    X2 Xa = mkx2(ld2(A + 2), A + 2);
    X2 Xb = mkx2(ld2(A + 1), A + 1);
    X2 Xc2 = mkx2(ld2(A), A);
    const CRow<T, V> Chi1 = mku2(Xc2, Xb, Xa, A + 1);  // u'(A + 1)
    Xa = Xb;
    Xb = Xc2;
    Xc2 = mkx2(ld2(A - 1), A - 1);
    CRow<T, V> Chi = mku2(Xc2, Xb, Xa, A);  // u'(A)
    XR R0 = row_odd(ld_f(yt + 2), yt + 2, Chi, Chi1);  // x(yt + 2)
    XR R1 = row_even(ld_f(yt + 1), yt + 1, Chi);       // x(yt + 1)
    // pair y's inputs (f rows y, y - 1 and the x' row (y - 3) / 2) in flight kProlongAhead pairs ahead
    constexpr int D = kProlongAhead;
    struct Slot {
      In u1, u2;
      In2 c;
    };
    Slot ring[D];
    auto fill = [&](Slot& sl, int y) {
      sl.u1 = ld_f(y);
      sl.u2 = ld_f(y - 1);
      sl.c = ld2((y - 3) / 2);
    };
#pragma unroll
    for (int d = 0; d < D; ++d) fill(ring[d], yt - 2 * d);
    auto iter = [&](int y, auto slot) {
      Slot& sl = ring[decltype(slot)::value];
      Xa = Xb;  // x' rows (y+1)/2, (y-1)/2, (y-3)/2 -> u'((y - 1) / 2)
      Xb = Xc2;
      Xc2 = mkx2(sl.c, (y - 3) / 2);
      const CRow<T, V> Clo = mku2(Xc2, Xb, Xa, (y - 1) / 2);
      const XR Xy = row_odd(sl.u1, y, Clo, Chi);  // x(y)
      if (y + 1 < r1) emit(y + 1, Xy, R1, R0);
      const XR Xm = row_even(sl.u2, y - 1, Clo);  // x(y - 1)
      emit(y, Xm, Xy, R1);
      R0 = Xy;
      R1 = Xm;
      Chi = Clo;
      fill(sl, y - 2 * D);
    };
    int y = yt;
    for (; y - 2 * (D - 1) >= r0; y -= 2 * D) {
      iter(y, std::integral_constant<int, 0>{});
      if constexpr (D > 1) iter(y - 2, std::integral_constant<int, 1 % D>{});
      if constexpr (D > 2) iter(y - 4, std::integral_constant<int, 2 % D>{});
      if constexpr (D > 3) iter(y - 6, std::integral_constant<int, 3 % D>{});
    }
    if constexpr (D > 1)
      if (y >= r0) iter(y, std::integral_constant<int, 0>{});
    if constexpr (D > 2)
      if (y - 2 >= r0) iter(y - 2, std::integral_constant<int, 1 % D>{});
    if constexpr (D > 3)
      if (y - 4 >= r0) iter(y - 4, std::integral_constant<int, 2 % D>{});
  }
}

template <typename T, bool MULTI>
__global__ __launch_bounds__(256) void k_mg_prolong2(MgArgs<T> g) {
  __shared__ T tab[MULTI ? FEA_MAX_PATTERNS * kTabStride : 1];
  __shared__ T ptb[MULTI ? FEA_MAX_PATTERNS * kTabStride : 1];
  if constexpr (MULTI) {
    load_tables<T>(tab, g.ktab, g.omd, g.ntab, ptb, g.ptab, g.nptab);
    __syncthreads();
  }
  const TaskId id = decode_task_lin(g.nstrips, g.ntr);
  if (!id.valid) return;
  // fp64 only: the reversed task body needs ~150 VGPRs (fp32 forward: 100, 4 waves per SIMD), which costs the
  // batched fp32 cycles (C5: 52 instead of 42 us) more than the L2 reuse gains; fp64 gains 1 us at 4097^2
  if constexpr (kProlong2Alternate && sizeof(T) == 8) {
    if (id.t & 1) {
      prolong2_task<T, MULTI, true>(g, id, tab, ptb);
      return;
    }
  }
  prolong2_task<T, MULTI, false>(g, id, tab, ptb);
}

// ---------------------------------------------------------------------------
// Kernel F: cycle join — the post-smooth of V-cycle k and the pre-smooth + residual + restriction
// of V-cycle k+1 on one level in ONE pass (temporal blocking across the cycle boundary):
//   x = u + w1 P(ec)        (FEANet/multigrid.py:177-180, prolongation + correction)
//   v = J(x, f)             (:181, post-smooth of cycle k — never stored)
//   w = J(v, f)             (:165, pre-smooth of cycle k+1 — stored)
//   f_c = w0 R(f - K w)     (:168-170, restriction of cycle k+1)
// Reads u, f, ec once and writes w, f_c: 28 instead of 52 B per fine node for the two passes it
// replaces.  Overlapped strips with a 2*VEC-column left halo (S = 120 fp64 / 244 fp32 owned
// columns per 64*VEC loaded); a row task streams its rows through the four stages skewed by one
// row each.  Per-node arithmetic is exactly that of fea_mg_prolong_sweep then fea_mg_sweep_restrict,
// so the result is bitwise the unfused sequence.
// ---------------------------------------------------------------------------
template <int SECOND, typename X>
__device__ __forceinline__ X& pick(X& a, X& b) {
  if constexpr (SECOND) return b;
  else return a;
}

// cycle join: input rows in flight per wave (2 or 4) and the occupancy the register budget is held to
// (0: the compiler's choice).  A/B on MI355X (tools/lab/ab_bench.sh, V-cycle): 2 rows, free budget
// (144 VGPRs, 3 waves/SIMD) 196.6 us; 4 rows at 3 waves (spills) 199.3 us; 4 rows at 2 waves 206.0 us.
#ifndef FEA_JOIN_AHEAD
#define FEA_JOIN_AHEAD 2
#endif
#ifndef FEA_JOIN_WAVES
#define FEA_JOIN_WAVES 0
#endif
static_assert(FEA_JOIN_AHEAD == 2 || FEA_JOIN_AHEAD == 4, "join prefetch ring of 2 or 4 rows");
#ifndef FEA_JOIN_UNROLL
#define FEA_JOIN_UNROLL 4
#endif
constexpr int kJoinUnroll = FEA_JOIN_UNROLL;
// FEA_JOIN_PEEL: fp32 joins peel the pipeline fill (compile-time stage flags); fp64 keeps runtime flags
#ifndef FEA_JOIN_PEEL
#define FEA_JOIN_PEEL 1
#endif
constexpr bool kJoinPeel = FEA_JOIN_PEEL != 0;
static_assert(kJoinUnroll % FEA_JOIN_AHEAD == 0 && kJoinUnroll % 2 == 0, "join unroll: a multiple of the ring");
// f(integral_constant<int, i>) for i = 0 .. N-1, in order (compile-time step positions)
template <int N, typename Fn, int... I>
__device__ __forceinline__ void unroll_steps_(Fn&& fn, std::integer_sequence<int, I...>) {
  (fn(std::integral_constant<int, I>{}), ...);
}
template <int N, typename Fn>
__device__ __forceinline__ void unroll_steps(Fn&& fn) {
  unroll_steps_<N>(fn, std::make_integer_sequence<int, N>{});
}
// FEA_JOIN_NTL: nontemporal loads of the iterate u in the join on levels above the NT threshold
#ifndef FEA_JOIN_NTL
#define FEA_JOIN_NTL 1
#endif
constexpr bool kJoinNTL = FEA_JOIN_NTL != 0;
// NTF (template flag of the join): nontemporal loads of the right-hand side f too, on levels whose fields of
// ONE sample exceed the Infinity Cache (8193^2 fp64 join 397 -> 371 us; with many small samples, C5, it
// costs 953 -> 980 us; same-process A/B, profiles/r03_stream/ntl_ab.txt)
// FEA_JOIN_ALT: odd row tasks stream bottom-up (see join_task).  FEA_JOIN_SHARED: the rows two tasks
// share are loaded through the cache instead of nontemporally (with FEA_JOIN_NTL).  Same-lease A/B at
// 4097^2 fp64 (profiles/r02_ab): ALT=1 join 82.6 us, 348 MB read per launch; ALT=0 84.3 us, 385 MB;
// ALT=1 SHARED=1 95 us, 336 MB (the cached rows evict the right-hand side, like NTL=0).
#ifndef FEA_JOIN_ALT
#define FEA_JOIN_ALT 1
#endif
#ifndef FEA_JOIN_SHARED
#define FEA_JOIN_SHARED 0
#endif
constexpr bool kJoinAlternate = FEA_JOIN_ALT != 0;
// FEA_JOIN_INNER (lab): interior tasks take a join_task instantiation without boundary selects / clamps (measured
// in the ISA only: the kernel holding both instantiations needs 203-209 VGPRs, two waves per SIMD instead of three).
// FEA_JOIN_OMZ: a sweep keeps a boundary node's value through a zero omega/d (v = 0 * r + b) instead of a select of
// the result; the select was compiled as an exec-mask branch per node and stage (fp64 join: 3090 -> 2025 SALU,
// 428 -> 167 branches in the kernel, 154 -> 145 VGPRs; metric V-cycle 136.8 -> 135.5 us, join 80.0 -> 79.1 us,
// same-lease A/B twice, profiles/r05_ab/join_omz.txt).  Bitwise: on a boundary node b == the kept value (x = u + w1 P e
// with every coarse value P reads there on the coarse boundary, i.e. zero), up to the sign of a zero.
#ifndef FEA_JOIN_INNER
#define FEA_JOIN_INNER 0
#endif
// lab builds (-DFEA_LAB_JREV): every second join launch deals its tasks in reverse order (decode_task_lin's rev) —
// measured slower (+1.5 us per V-cycle, profiles/r05_ab/join_omz.txt)
#ifdef FEA_LAB_JREV
#define FEA_LAB_JOIN_REV(g) { static int flip = 0; (g).rev = flip = !flip; }
#elif defined(FEA_LAB_JFLIP)
#define FEA_LAB_JOIN_REV(g) { static int fl = 0; (g).flip = fl; fl ^= 1; }
#else
#define FEA_LAB_JOIN_REV(g)
#endif
#ifndef FEA_JOIN_OMZ
#define FEA_JOIN_OMZ 1
#endif
constexpr bool kJoinInner = FEA_JOIN_INNER != 0;
constexpr bool kJoinOmz = FEA_JOIN_OMZ != 0;
#define REV_SHARED_LOADS (FEA_JOIN_SHARED != 0)

template <typename T>
struct Ovl3 {
  static constexpr int V = Frame<T>::VEC;
  static constexpr int HL = 2 * V;                       // left halo columns (keeps 16-B alignment)
  static constexpr int S = ((64 * V - 4 - HL) / V) * V;  // owned fine columns per strip
  static constexpr int L0 = HL / V;                      // first owning lane
  static constexpr int OWN = S / V;                      // owning lanes L0 .. L0 + OWN - 1
};

// One row task of the cycle join (below).  NORM: also accumulates, into ssq, the squared residual
// f - K v of the post-smoothed iterate v (the end-of-cycle iterate the reference drivers measure,
// M-FEANet-mg_test.ipynb:27428-27429) over the task's owned interior nodes — the pre-smooth of the
// next cycle forms exactly that residual, so the norm costs no extra pass.
//
// REV: the task streams its rows bottom-up.  Odd row tasks run reversed, so two vertically adjacent
// tasks reach the 7 rows they share (input rows each recomputes) at the same moment — both at their
// start or both at their end — and the second read of those rows comes from the L2 (37 MB less HBM
// traffic per launch at 4097^2 fp64, measured; nontemporal loads still allocate there).  Every node value
// is the same expression as in the forward task: windows are passed to the stencil in grid order and
// a coarse row's three restriction terms are summed in the forward order (ky = 0, 1, 2).
// the part of the grid a join task covers: sample b, coarse rows [I0, I1), fine columns from c0 (the strip's first
// owned one) up to cmax (exclusive; the rectangle's right edge)
struct JoinTask {
  int b, t, I0, I1, c0, cmax;
};

// EDGE = false: an interior task (join_interior): every row it streams and every column its lanes load lies inside
// the grid, so the boundary selects, the row clamps, the lane clamps and the partial stores drop out at compile
// time (same per-node expressions: bitwise the general task).
template <typename T, bool MULTI, bool NT, bool NORM, bool REV, bool NTF, bool EDGE = true>
__device__ __forceinline__ void join_task(const MgArgs<T>& g, const JoinTask& jt, const T* tab, const T* rtb,
                                          const T* ptb, double& ssq) {
  constexpr int kJoinAhead = MULTI ? 2 : FEA_JOIN_AHEAD;
  constexpr int S = REV ? -1 : 1;  // row step
  using F = Frame<T>;
  using O = Ovl3<T>;
  constexpr int V = F::VEC;
  constexpr int Q = V / 2;
  const int lane = lane_id();
  const int H = g.H, W = g.W, Hc = g.Hc, Wc = g.Wc;
  // stores stop at the rectangle's right edge (fine columns < cmax, coarse columns J <= (cmax - 1) / 2)
  const int Ws = min(W, jt.cmax + 1), Wcs = min(Wc, (jt.cmax + 3) / 2);
  const int c0 = jt.c0;            // first owned fine column (odd)
  const int cs = c0 - O::HL;       // first loaded column (odd)
  const int cl = cs + V * lane;    // lane's first column (odd)
  const int I0 = jt.I0;
  const int I1 = jt.I1;
  T ks[9], rs[9], ps[9];
  T om = 0;
  if constexpr (!MULTI) {
#pragma unroll
    for (int d = 0; d < 9; ++d) {
      ks[d] = g.ktab[d];
      rs[d] = g.rtab[d];
      ps[d] = g.ptab[d];
    }
    om = g.omd[0];
  }
  const T w0 = g.w, w1 = g.w2;
  bool cin[V];
#pragma unroll
  for (int k = 0; k < V; ++k) cin[k] = !EDGE || (cl + k >= 1 && cl + k <= W - 2);
  const bool own = lane >= O::L0 && lane < O::L0 + O::OWN;
  const int J0 = (cl + 1) / 2;
  const long long boff = (long long)jt.b * g.bs + F::OFF + cs;
  const T* __restrict__ ub = g.u + boff;
  const T* __restrict__ fb = g.f + boff;
  T* __restrict__ ob = g.out2 + boff;
  const uint8_t* __restrict__ pb = MULTI ? g.pid + F::OFF + cs : nullptr;
  const long long cboff = F::OFF + (cs + 1) / 2;  // coarse column of lane 0's first value
  const T* __restrict__ eb = g.ec + (long long)jt.b * g.bsc + cboff;
  const uint8_t* __restrict__ pcb = MULTI ? g.pidc + cboff : nullptr;
  T* __restrict__ cb = g.out + (long long)jt.b * g.bsc + F::OFF + J0;
  const int ld = g.ld, ldc = g.ldc;
  // lanes past the grid's last fine column W - 1 (coarse: Wc - 1) load the last needed lane's columns
  // again instead of streaming columns nothing uses: the last strip of a row can be mostly outside
  // the grid (25 % of the loaded columns at 1025 wide in fp32); stores are masked by column anyway
  const int ll = EDGE ? min(lane, (W - 1 - cs) / V) : lane;
  const int llc = EDGE ? min(lane, (Wc - 1 - (cs + 1) / 2) / Q) : lane;
  auto rowo = [&](int r) -> long long {
    if constexpr (EDGE) r = min(max(r, -1), H);
    return (long long)(r + 1) * ld + V * ll;
  };
  auto crowo = [&](int a) -> long long { return (long long)(min(max(a, -1), Hc) + 1) * ldc; };
  auto rc = [&](int a) {
    return raw_crow<T, V, MULTI>(eb + crowo(a), MULTI ? pcb + crowo(a) : nullptr, lane, llc);
  };

  // ---- pipeline state (rows relative to the step's y, s = +1 forward / -1 reversed)
  Row<T, V> Xa{}, Xb{}, Xc{};  // x windows of rows y-2s, y-s, y
  Row<T, V> Va{}, Vb{}, Vc{};  // v windows of rows y-3s, y-2s, y-s
  Row<T, V> Wa{}, Wb{}, Wc_{}; // w windows of rows y-4s, y-3s, y-2s
  PRow<V> P4{}, P3{}, P2{}, P1{}, P0{};  // pattern windows of rows y-4s .. y
  T f1[V], f2[V], f3[V];       // f of rows y-2s, y-3s, y-4s (after the rotation at the step's end: y-s ..)
  T um1[V];                    // u (uncorrected) of row y-s: v keeps it on boundary nodes
  T acc[Q], t2[Q];             // forward: restriction partial sum; reversed: the ky=1 and ky=2 terms
#pragma unroll
  for (int k = 0; k < V; ++k) f1[k] = f2[k] = f3[k] = um1[k] = T(0);
#pragma unroll
  for (int q = 0; q < Q; ++q) acc[q] = t2[q] = T(0);

  const int ys = 2 * I0 - 4, ye = 2 * I1 + 2;
  const int yb = REV ? ye : ys;  // first row streamed
  // shared input rows (recomputed by the neighbouring task too) are loaded through the cache
  auto shared_row = [&](int y) { return y <= ys + 6 || y >= ye - 6; };
  auto load_u = [&](int y, T (&x)[V]) {
    if constexpr (kJoinNTL && NT && REV_SHARED_LOADS) {
      if (shared_row(y)) vload<T, V>(ub + rowo(y), x);
      else vload<T, V, true>(ub + rowo(y), x);
    } else {
      vload<T, V, kJoinNTL && NT>(ub + rowo(y), x);
    }
  };
  // inputs u(y), f(y-s), pid(y) in flight kJoinAhead steps ahead, in a ring of buffers indexed by the
  // step's position mod kJoinAhead (compile-time), so no in-flight register is ever copied (a copy
  // would force the wait for its load at once) — the join runs 3 waves per SIMD and needs the
  // latency cover: 4 rows x 2 KiB of u and f per wave in flight
  T ub_[kJoinAhead][V], fb_[kJoinAhead][V];
  int pb_[kJoinAhead][V];
#pragma unroll
  for (int q = 0; q < kJoinAhead; ++q) {
    load_u(yb + S * q, ub_[q]);
    vload<T, V, NTF>(fb + rowo(yb + S * (q - 1)), fb_[q]);
    if constexpr (MULTI) pload<V>(pb + rowo(yb + S * q), pb_[q]);
  }
  // coarse rows: Ca = the row an even step uses, Cb = the next one in streaming order
  CRow<T, V> Ca = finish_c<T, V, MULTI>(rc(yb / 2));
  CRow<T, V> Cb = finish_c<T, V, MULTI>(rc(yb / 2 + S));
  RawC<T, V> nC = rc(yb / 2 + 2 * S);

  // count: add the squared residual of the input row y to ssq (NORM; the row and lane own y)
  auto sweep_own = [&](const Row<T, V>& a, const Row<T, V>& b, const Row<T, V>& c, const PRow<V>& pa,
                       const PRow<V>& pb_, const PRow<V>& pc, const T (&fy)[V], const T (&keep)[V], int y,
                       T (&o)[V], bool count) {
    const bool rin = !EDGE || (y >= 1 && y <= H - 2);
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const T acck = kapply<T, V, MULTI>(a, b, c, pa, pb_, pc, k, ks, tab);
      const T omk = MULTI ? tabv(tab, pb_.a[k + 1], 9) : om;
      const T rr = fy[k] - acck;
      if constexpr (kJoinOmz) {
        // boundary nodes: 0 * r + b = b, and b == keep there (the prolonged correction of a boundary node is a
        // sum of coarse boundary values, all zero, so x = u exactly)
        const T omz = (rin && cin[k]) ? omk : T(0);
        o[k] = omz * rr + b.a[k + 1];
      } else {
        const T v = omk * rr + b.a[k + 1];
        o[k] = (rin && cin[k]) ? v : keep[k];
      }
      if constexpr (NORM)
        if (count && rin && cin[k]) ssq += (double)rr * (double)rr;
    }
  };
  // the stencil takes its three rows in grid order (row i-1, i, i+1)
  auto sweep3 = [&](const Row<T, V>& a, const Row<T, V>& b, const Row<T, V>& c, const PRow<V>& pa,
                    const PRow<V>& pb_, const PRow<V>& pc, const T (&fy)[V], const T (&keep)[V], int y, T (&o)[V],
                    bool count) {
    if constexpr (REV) sweep_own(c, b, a, pc, pb_, pa, fy, keep, y, o, count);
    else sweep_own(a, b, c, pa, pb_, pc, fy, keep, y, o, count);
  };

  // nn: the step index where it is < kFill (the pipeline's fill steps run stages 2 .. 4 only from step 2, 4, 6
  // on, and the first residual row closes no coarse row), kFill or more for every later step.  Peeled (fp32):
  // a compile-time constant, so the steady-state steps carry no stage branches; fp64 passes the runtime step
  // index (the peeled fp64 body needs 180 VGPRs, 2 waves per SIMD instead of 3: 16 us slower at 4097^2)
  constexpr int kFill = 7;
  auto step = [&](int y, auto par, auto nn) {
    constexpr int SLOT = decltype(par)::value % kJoinAhead;  // step index mod kJoinAhead
    constexpr int ODD = decltype(par)::value & 1;            // y odd (yb is even)
    const int NN = nn;
    // this step's inputs; refill the slot with the rows kJoinAhead steps ahead
    T(&bu)[V] = ub_[SLOT];
    T(&bf)[V] = fb_[SLOT];
    int(&bp)[V] = pb_[SLOT];
    T u0[V], fy1[V];
    int p0[V];
#pragma unroll
    for (int k = 0; k < V; ++k) {
      u0[k] = bu[k];
      fy1[k] = bf[k];
      if constexpr (MULTI) p0[k] = bp[k];
    }
    load_u(y + S * kJoinAhead, bu);
    vload<T, V, NTF>(fb + rowo(y + S * (kJoinAhead - 1)), bf);
    if constexpr (MULTI) pload<V>(pb + rowo(y + S * kJoinAhead), bp);
    // 1. x(y) = u(y) + w1 P(ec) on the own columns (correct_even / correct_odd of Kernel C)
    T x[V];
#pragma unroll
    for (int k = 0; k < V; ++k) {
      T t;
      if constexpr (!ODD) {
        t = crow_term<T, V, MULTI>(Ca, k + 1, 1, ps, ptb);
      } else if constexpr (!REV) {  // coarse rows (y-1)/2 = Ca (ky = 2), (y+1)/2 = Cb (ky = 0)
        t = crow_term<T, V, MULTI>(Ca, k + 1, 2, ps, ptb) + crow_term<T, V, MULTI>(Cb, k + 1, 0, ps, ptb);
      } else {  // coarse rows (y-1)/2 = Cb (ky = 2), (y+1)/2 = Ca (ky = 0)
        t = crow_term<T, V, MULTI>(Cb, k + 1, 2, ps, ptb) + crow_term<T, V, MULTI>(Ca, k + 1, 0, ps, ptb);
      }
      x[k] = u0[k] + w1 * t;
    }
    if constexpr (ODD) {  // the next (even) step uses coarse row (y+s)/2 = Cb; prefetch the one after
      Ca = Cb;
      Cb = finish_c<T, V, MULTI>(nC);
      nC = rc((y + S) / 2 + 2 * S);
    }
    Xa = Xb;
    Xb = Xc;
    Xc = own_row<T, V>(x);
    P4 = P3;
    P3 = P2;
    P2 = P1;
    P1 = P0;
    if constexpr (MULTI) P0 = own_prow<T, V>(p0);
    // 2. v(y-s) = J(x) (boundary nodes keep u)
    if (NN >= 2) {
      T v[V];
      sweep3(Xa, Xb, Xc, P2, P1, P0, fy1, um1, y - S, v, false);
      Va = Vb;
      Vb = Vc;
      Vc = own_row<T, V>(v);
      // 3. w(y-2s) = J(v) (boundary nodes keep v)
      if (NN >= 4) {
        T keep[V], w[V];
#pragma unroll
        for (int k = 0; k < V; ++k) keep[k] = Vb.a[k + 1];
        const int yw = y - 2 * S;
        const bool ownr = yw >= 2 * I0 - 1 && (yw < 2 * I1 - 1 || I1 == Hc - 1) && yw <= H - 2;
        sweep3(Va, Vb, Vc, P3, P2, P1, f1, keep, yw, w, own && ownr);
        if constexpr (EDGE) {
          if (own && ownr) store_masked<T, V, NT>(ob + rowo(yw), w, cl, Ws);
        } else {
          if (own && ownr) vstore<T, V, NT>(ob + rowo(yw), w);
        }
        Wa = Wb;
        Wb = Wc_;
        Wc_ = own_row<T, V>(w);
        // 4. residual row y-3s -> restriction
        if (NN >= 6) {
          T r[V + 1];
#pragma unroll
          for (int k = 0; k < V; ++k) {
            if constexpr (REV) r[k] = f2[k] - kapply<T, V, MULTI>(Wc_, Wb, Wa, P2, P3, P4, k, ks, tab);
            else r[k] = f2[k] - kapply<T, V, MULTI>(Wa, Wb, Wc_, P4, P3, P2, k, ks, tab);
          }
          r[V] = shl1z(r[0]);
          auto term = [&](int q, int ky) -> T {
            T t;
            if constexpr (!MULTI) {
              t = rs[ky * 3 + 0] * r[2 * q];
              t += rs[ky * 3 + 1] * r[2 * q + 1];
              t += rs[ky * 3 + 2] * r[2 * q + 2];
            } else {
              t = tabv(rtb, P3.a[2 * q + 1], ky * 3 + 0) * r[2 * q];
              t += tabv(rtb, P3.a[2 * q + 2], ky * 3 + 1) * r[2 * q + 1];
              t += tabv(rtb, P3.a[2 * q + 3], ky * 3 + 2) * r[2 * q + 2];
            }
            return t;
          };
          const int yr = y - 3 * S;
          auto put = [&](int I, const T (&o)[Q]) {
            if (own) {
              T* cp = cb + (long long)(I + 1) * ldc;
              if (!EDGE || J0 + Q - 1 <= Wcs - 2) {
                vstore<T, Q, kCoarseNT && NT>(cp, o);
              } else {
#pragma unroll
                for (int q = 0; q < Q; ++q)
                  if (J0 + q <= Wcs - 2) cp[q] = o[q];
              }
            }
          };
          if constexpr (!REV) {
            if constexpr (!ODD) {  // yr odd = 2I+1: ky = 2 closes coarse row I, ky = 0 opens I+1
              if (NN > 6) {  // (yr > 2 I0 - 1)
                T o[Q];
#pragma unroll
                for (int q = 0; q < Q; ++q) o[q] = w0 * (acc[q] + term(q, 2));
                put((yr - 1) / 2, o);
              }
#pragma unroll
              for (int q = 0; q < Q; ++q) acc[q] = term(q, 0);
            } else {  // yr even = 2I: ky = 1
#pragma unroll
              for (int q = 0; q < Q; ++q) acc[q] = acc[q] + term(q, 1);
            }
          } else {
            if constexpr (!ODD) {  // yr odd = 2I-1: ky = 0 closes coarse row I, ky = 2 opens I-1
              if (NN > 6) {  // (yr < 2 I1 - 1)
                T o[Q];
#pragma unroll
                for (int q = 0; q < Q; ++q) o[q] = w0 * ((term(q, 0) + acc[q]) + t2[q]);
                put((yr + 1) / 2, o);
              }
#pragma unroll
              for (int q = 0; q < Q; ++q) t2[q] = term(q, 2);
            } else {  // yr even = 2I: ky = 1
#pragma unroll
              for (int q = 0; q < Q; ++q) acc[q] = term(q, 1);
            }
          }
        }
      }
    }
    // rotate f and u rows
#pragma unroll
    for (int k = 0; k < V; ++k) {
      f3[k] = f2[k];
      f2[k] = f1[k];
      f1[k] = fy1[k];
      um1[k] = u0[k];
    }
  };

  // ye - ys + 1 steps (odd); the ring slot is a template argument, so the loop is unrolled by a multiple of
  // the ring: FEA_JOIN_UNROLL = 4, or 6 (= the 3-row window period x the 2-slot ring: every window rotation
  // is a register renaming inside the body and the loop's back edge needs no moves)
  if constexpr (kJoinPeel && sizeof(T) == 4) {
    constexpr int U = kJoinUnroll;
    using Full = std::integral_constant<int, kFill>;
    // the kFill fill steps (>= 9 steps per task: rb >= 2), then the steady state in blocks of U (the step
    // index parity after the fill is kFill's: pass positions kFill .. kFill + U - 1 so slot and parity stay exact)
    unroll_steps<kFill>([&](auto i) { step(REV ? ye - decltype(i)::value : ys + decltype(i)::value, i, i); });
    int y = REV ? ye - kFill : ys + kFill;
    if constexpr (!REV) {
      for (; y + U - 1 <= ye; y += U)
        unroll_steps<U>([&](auto i) { step(y + decltype(i)::value, std::integral_constant<int, kFill + decltype(i)::value>{}, Full{}); });
      unroll_steps<U - 1>([&](auto i) {
        if (y + decltype(i)::value <= ye)
          step(y + decltype(i)::value, std::integral_constant<int, kFill + decltype(i)::value>{}, Full{});
      });
    } else {
      for (; y - (U - 1) >= ys; y -= U)
        unroll_steps<U>([&](auto i) { step(y - decltype(i)::value, std::integral_constant<int, kFill + decltype(i)::value>{}, Full{}); });
      unroll_steps<U - 1>([&](auto i) {
        if (y - decltype(i)::value >= ys)
          step(y - decltype(i)::value, std::integral_constant<int, kFill + decltype(i)::value>{}, Full{});
      });
    }
  } else {
    int y = yb;
    for (; REV ? y - 3 >= ys : y + 3 <= ye; y += 4 * S)
      unroll_steps<4>([&](auto i) { step(y + S * decltype(i)::value, i, S * (y - yb) + decltype(i)::value); });
    unroll_steps<3>([&](auto i) {
      if (REV ? y - decltype(i)::value >= ys : y + decltype(i)::value <= ye)
        step(y + S * decltype(i)::value, i, S * (y - yb) + decltype(i)::value);
    });
  }
}

template <typename T, bool MULTI, bool NORM, bool NT, bool NTF = false>
__global__ __launch_bounds__(256)
#if FEA_JOIN_WAVES > 0
__attribute__((amdgpu_waves_per_eu(FEA_JOIN_WAVES)))
#endif
void k_mg_cycle_join(MgArgs<T> g) {
  __shared__ T tab[MULTI ? FEA_MAX_PATTERNS * kTabStride : 1];
  __shared__ T rtb[MULTI ? FEA_MAX_PATTERNS * kTabStride : 1];
  __shared__ T ptb[MULTI ? FEA_MAX_PATTERNS * kTabStride : 1];
  if constexpr (MULTI) {
    load_tables<T>(tab, g.ktab, g.omd, g.ntab, rtb, g.rtab, g.nrtab);
    load_tables<T>(ptb, g.ptab, nullptr, g.nptab, nullptr, nullptr, 0);
    __syncthreads();
  }
  JoinTask jt;
  bool valid;
  if (g.nrect == 0) {
    const TaskId id = decode_task_lin(g.nstrips, g.ntr, g.rev);
    valid = id.valid;
    jt.b = id.b;
    jt.t = id.t;
    jt.I0 = 1 + id.t * (g.rb / 2);
    jt.I1 = min(jt.I0 + g.rb / 2, g.Hc - 1);
    jt.c0 = 1 + id.s * Ovl3<T>::S;
    jt.cmax = g.W - 1;
  } else {  // rectangles: tasks of a sample rectangle by rectangle, four per workgroup (wave-uniform, scalar)
    const int per = g.rt[g.nrect];
    const int wpb = (per + kWaves - 1) / kWaves;
    const int bid = xcd_remap(blockIdx.x, gridDim.x);
    jt.b = bid / wpb;
    const int w = (bid - jt.b * wpb) * kWaves + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    valid = w < per;
    int r = 0;
    while (r + 1 < g.nrect && w >= g.rt[r + 1]) ++r;
    const int lw = w - g.rt[r];
    jt.t = lw / g.rns[r];
    const int sx = lw - jt.t * g.rns[r];
    jt.I0 = g.rI0[r] + jt.t * (g.rb / 2);
    jt.I1 = min(jt.I0 + g.rb / 2, g.rI1[r]);
    jt.c0 = g.rc0[r] + sx * Ovl3<T>::S;
    jt.cmax = g.rc1[r];
  }
  double ssq = 0.0;
  if (valid) {
    // interior task: rows 2 I0 - 4 .. 2 I1 + 2 inside [1, H - 2] (loads reach 2 rows further, still in the frame) and
    // every loaded column inside [1, W - 2]
    const int cs = jt.c0 - Ovl3<T>::HL;
    const bool inner = kJoinInner && g.nrect == 0 && 2 * jt.I0 - 4 >= 1 && 2 * jt.I1 + 2 <= g.H - 2 && cs >= 1 &&
                       cs + kWave * Frame<T>::VEC - 1 <= g.W - 2;
    if ((kJoinAlternate && (jt.t & 1)) != (g.flip != 0)) {
      if (inner) join_task<T, MULTI, NT, NORM, true, NTF, false>(g, jt, tab, rtb, ptb, ssq);
      else join_task<T, MULTI, NT, NORM, true, NTF, true>(g, jt, tab, rtb, ptb, ssq);
    } else {
      if (inner) join_task<T, MULTI, NT, NORM, false, NTF, false>(g, jt, tab, rtb, ptb, ssq);
      else join_task<T, MULTI, NT, NORM, false, NTF, true>(g, jt, tab, rtb, ptb, ssq);
    }
  }
  if constexpr (NORM) norm_partial<T>(g, ssq);
}

// ---------------------------------------------------------------------------
// Kernel D: per-task partial sums of (f - K u)^2 over the interior (deterministic).
// ---------------------------------------------------------------------------
template <typename T, bool MULTI>
__global__ __launch_bounds__(256) void k_mg_resnorm(MgArgs<T> g) {
  using F = Frame<T>;
  constexpr int V = F::VEC;
  __shared__ T tab[MULTI ? FEA_MAX_PATTERNS * kTabStride : 1];
  if constexpr (MULTI) {
    load_tables<T>(tab, g.ktab, nullptr, g.ntab, nullptr, nullptr, 0);
    __syncthreads();
  }
  const TaskId id = decode_task(g.nstrips, g.ntr);
  if (!id.valid) return;
  const int lane = lane_id();
  const int H = g.H, W = g.W;
  const int c0 = 1 + id.s * F::SW;
  const int r0 = g.rlo + id.t * g.rb;
  const int r1 = min(r0 + g.rb, g.rhi);
  const int cl = c0 + V * lane;
  T ks[9];
  if constexpr (!MULTI) {
#pragma unroll
    for (int d = 0; d < 9; ++d) ks[d] = g.ktab[d];
  }
  const long long poff = F::OFF + c0;
  const long long boff = (long long)id.b * g.bs + poff;
  const T* __restrict__ ub = g.u + boff;
  const T* __restrict__ fb = g.f + boff;
  const uint8_t* __restrict__ pb = MULTI ? g.pid + poff : nullptr;
  const int ld = g.ld;
  auto rowo = [&](int r) -> long long { return (long long)(min(r, H) + 1) * ld; };
  Row<T, V> w0 = finish(raw_row<T, V>(ub + rowo(r0 - 1), lane));
  Row<T, V> w1 = finish(raw_row<T, V>(ub + rowo(r0), lane));
  RawRow<T, V> nx = raw_row<T, V>(ub + rowo(r0 + 1), lane);
  PRow<V> p0{}, p1{}, p2{};
  RawP<V> px{};
  if constexpr (MULTI) {
    p0 = finish_p<T>(raw_prow<V>(pb + rowo(r0 - 1), lane));
    p1 = finish_p<T>(raw_prow<V>(pb + rowo(r0), lane));
    px = raw_prow<V>(pb + rowo(r0 + 1), lane);
  }
  double s = 0.0;
  for (int r = r0; r < r1; ++r) {
    const RawRow<T, V> nn = raw_row<T, V>(ub + rowo(r + 2), lane);
    RawP<V> pn{};
    if constexpr (MULTI) pn = raw_prow<V>(pb + rowo(r + 2), lane);
    T fv[V];
    vload<T, V>(fb + rowo(r) + V * lane, fv);
    const Row<T, V> w2 = finish(nx);
    if constexpr (MULTI) p2 = finish_p<T>(px);
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const T rr = fv[k] - kapply<T, V, MULTI>(w0, w1, w2, p0, p1, p2, k, ks, tab);
      if (cl + k >= g.clo && cl + k < g.chi) s += (double)rr * (double)rr;
    }
    w0 = w1;
    w1 = w2;
    nx = nn;
    if constexpr (MULTI) {
      p0 = p1;
      p1 = p2;
      px = pn;
    }
  }
  s = wave_sum(s);
  if (lane == 0) g.part[(long long)id.b * g.ntr * g.nstrips + (long long)id.t * g.nstrips + id.s] = s;
}

// ---------------------------------------------------------------------------
// pack / unpack between contiguous [B,1,H,W] and the framed layout
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void k_mg_pack(const T* __restrict__ src, T* __restrict__ dst,
                                                 const T* __restrict__ geo, long long geo_bs,
                                                 const T* __restrict__ bc, long long bc_bs, int H, int W, int ld,
                                                 long long bs) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), r = blockIdx.y * 4 + (threadIdx.x >> 6), b = blockIdx.z;
  if (r >= H || c >= W) return;
  const long long i = (long long)r * W + c;
  const T v = src ? src[(long long)b * H * W + i] : T(0);
  const T gv = geo ? geo[b * geo_bs + i]
                   : T((geo_bs < 0 || (r > 0 && r < H - 1 && c > 0 && c < W - 1)) ? 1 : 0);
  const T bv = bc ? bc[b * bc_bs + i] : T(0);
  dst[(long long)b * bs + (long long)(r + 1) * ld + Frame<T>::OFF + c] = v * gv + bv;
}

template <typename T>
__global__ __launch_bounds__(256) void k_mg_unpack(const T* __restrict__ src, T* __restrict__ dst, int H, int W,
                                                   int ld, long long bs) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), r = blockIdx.y * 4 + (threadIdx.x >> 6), b = blockIdx.z;
  if (r >= H || c >= W) return;
  dst[(long long)b * H * W + (long long)r * W + c] = src[(long long)b * bs + (long long)(r + 1) * ld + Frame<T>::OFF + c];
}

}  // namespace fea

using namespace fea;

// Grid sizes: H, W >= 3; the intergrid kernels additionally need odd H and W (coarse (H+1)/2).
static inline bool mg_dim_ok(int n) { return n >= 3 && n <= (1 << 20) + 1; }
static inline bool mg_dims_ok(int H, int W) { return mg_dim_ok(H) && mg_dim_ok(W); }
static inline bool mg_odd(int H, int W) { return (H & 1) && (W & 1); }

// Rows per wave task: the largest even count (<= kRB) that still gives >= kTargetWaves waves, so small
// levels are spread over the chip instead of being marched row by row by a few waves (1024 / 4096 / 8192
// measured slower than 2048 on levels 1-2, profiles/r02_ab).
constexpr int kTargetWaves = 2048;  // 8 waves per CU
static int target_waves() { return kTargetWaves; }
static inline int pick_rb(int B, int nstrips, int rows, int maxrb = kRB) {
  const int tw = target_waves();
  for (int rb = maxrb; rb > 2; rb /= 2)
    if ((long long)B * nstrips * div_up(rows, rb) >= tw) return rb;
  return 2;
}

static int num_cus() {
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

// Row tasks of the compute-heavier row-pair kernels (sweep+restriction, cycle join), whose 4-wave
// workgroups run a few per CU at once: choose the task height so the workgroup count fills the CUs
// evenly (ceil(WGs / CUs) decides the slowest CU), counting the `halo` rows each task re-streams,
// with at least target_waves() waves in flight.  e.g. 4097^2 fp64: 504 workgroups of 74 rows
// (2 per CU) instead of 576 of 64 (2.25 per CU: a quarter of the CUs run 3).  Results are bitwise
// independent of the task height.  Same-process A/B against the power-of-two height
// (profiles/r03_stream/balance_ab.txt): join -13.5 % at 4097^2, -3 % at 8193^2, -6 % on C3, -11 % at 2049^2
// fp32; sweep+restriction -2 .. -12 %.  Batches of many samples are the exception (cycle_join_rb).
static int balanced_rb(int B, int nstrips, int rows_c, int halo, int rb_pow2, int min_waves = kTargetWaves) {
  if (rows_c < 2) return rb_pow2;
  const long long ncu = num_cus();
  const long long min_wg = std::max<long long>(1, min_waves / kWaves);
  long long best_cost = -1;
  int best = rb_pow2;
  for (int rbc = 1; rbc <= rows_c && 2 * rbc <= 4 * rb_pow2; ++rbc) {
    const long long ntr = div_up(rows_c, rbc), wgs = (long long)B * div_up(ntr * nstrips, kWaves);  // linear order
    if (wgs < min_wg) break;  // larger tasks only lower the count further
    const long long cost = div_up(wgs, ncu) * (2 * rbc + halo);
    if (best_cost < 0 || cost < best_cost) {
      best_cost = cost;
      best = 2 * rbc;
    }
  }
  return best;
}

// Levels whose fields exceed this many bytes stream their stores past the caches (measured on the
// 4097^2 fp64 sweep: 64.8 us with nontemporal stores vs 84.6 us without).  64 MiB: the three fields
// of a 2049^2 fp64 level (~36 MB each) stay in the 256 MiB Infinity Cache between the level's
// restriction and prolongation (V-cycle 201 -> 196 us with 64 instead of 32 MiB, A/B on MI355X).
static long long nt_bytes() {
  const char* e = getenv("FEANET_NT_BYTES");
  return e ? atoll(e) : (64ll << 20);
}

// Fields larger than the 256 MiB Infinity Cache cannot be re-read from it between launches: there the sweep
// and (for one sample's field) the cycle join also load nontemporally (g.nt = 2, see k_mg_sweep / the join).
// Tied to the store threshold (4 x 64 MiB by default) so the tests' FEANET_NT_BYTES=0 runs both paths.
static long long nt_load_bytes() { return 4 * nt_bytes(); }

// Prolongation + sweep of a recomputed zero-guess iterate (levels >= 1 going up): on overlapped strips
// (k_mg_prolong_zu_ovl, bitwise k_mg_prolong<ZU>) on levels of at most a quarter of the nontemporal-store
// threshold (16 MiB by default): there the shorter per-wave chain pays (1025^2 fp64: 6.1 -> 5.5 us); on
// larger levels the fine output dominates and the owned strips (122 of 128 columns) split 128-byte lines
// between two waves' stores (2049^2: 14.6 -> 15.0 us; line-aligned owned strips of 112 columns: no gain;
// same-lease A/B, profiles/r02_ab/prolong_ovl).  Tied to FEANET_NT_BYTES so the tests' FEANET_NT_BYTES=0
// runs select the other kernel on the same level (bitwise comparison of the two).
static bool zu_ovl(long long level_bytes) { return level_bytes <= nt_bytes() / 4; }

// rows per task cap of the cycle-join kernel (its stages recompute 7 rows per task)
constexpr int kJoinMaxRB = 64;
static int join_max_rb() { return kJoinMaxRB; }

template <typename T>
static MgArgs<T> mg_args(int H, int W, int ld, long long bs, int B) {
  MgArgs<T> g{};
  g.nt = (long long)B * bs * (long long)sizeof(T) > nt_bytes();
  g.H = H;
  g.W = W;
  g.ld = ld;
  g.bs = bs;
  g.nstrips = mg_nstrips<T>(W);
  g.rb = pick_rb(B, g.nstrips, H - 2);
  g.ntr = div_up(H - 2, g.rb);
  g.rlo = 1;
  g.rhi = H - 1;
  g.clo = 1;
  g.chi = W - 1;
  return g;
}

template <typename T>
static inline bool layout_ok(int H, int W, int ld, long long bs) {
  return mg_dims_ok(H, W) && ld >= mg_ld<T>(W) && ld % Frame<T>::A == 0 && bs >= (long long)(H + 2) * ld;
}

// coarse grid of an intergrid kernel: (H+1)/2 x (W+1)/2 with its own framed layout
template <typename T>
static inline bool coarse_ok(int H, int W, int ldc, long long bsc) {
  if (!mg_odd(H, W)) return false;
  const int Hc = (H + 1) / 2, Wc = (W + 1) / 2;
  return Hc >= 3 && Wc >= 3 && ldc >= mg_ld<T>(Wc) && ldc % Frame<T>::A == 0 && bsc >= (long long)(Hc + 2) * ldc;
}

static inline dim3 mg_grid_lin(int B, int ntr, int nstrips) {  // decode_task_lin launches
  return dim3((unsigned)(B * div_up(ntr * nstrips, kWaves)));
}
static inline dim3 mg_grid(int B, int ntr, int nstrips) {
  return dim3((unsigned)(B * ntr * div_up(nstrips, kWaves)));
}

extern "C" int fea_abi_version(void) { return 3; }

extern "C" int fea_mg_layout(int H, int W, int elem_size, int* ld, long long* bstride) {
  if (!mg_dims_ok(H, W) || !ld || !bstride) return FEA_EINVAL;
  if (elem_size == 8) {
    *ld = mg_ld<double>(W);
    *bstride = mg_bstride<double>(H, W);
  } else if (elem_size == 4) {
    *ld = mg_ld<float>(W);
    *bstride = mg_bstride<float>(H, W);
  } else {
    return FEA_EINVAL;
  }
  return 0;
}

extern "C" size_t fea_norm_workspace_bytes(int B, int H, int W) {
  if (B <= 0 || H <= 0 || W <= 0) return 0;
  // generic: one partial per 64x4 block; framed: one per (strip, row task) at the fp32 strip width
  const long long gen = (long long)div_up(W, 64) * div_up(H, 4);
  const long long frm = (long long)div_up(W, 64) * div_up(H, 2);
  // fused norms of the cycle join: one partial per wave of its grid (>= 2 fine rows per task, overlapped
  // strips of >= 120 owned columns, 4 waves per workgroup)
  const long long join = (long long)std::max(1, (H + 1) / 2 - 2) * div_up(div_up(std::max(W - 2, 1), 120), kWaves) *
                         kWaves;
  return (size_t)B * (size_t)std::max(std::max(gen, frm), join) * sizeof(double);
}

// launch configuration of the cycle join (overlapped strips, balanced row tasks)
// Batches of >= 16 samples keep the power-of-two task height (64 rows): many short tasks balance better
// than few long balanced ones there (256 x 1025^2 fp32 join 899 -> 843 us, 16 x 1025^2 59.4 -> 57.3 us;
// 8 x 2049^2 fp64 prefers balanced, 201 vs 207 us; profiles/r03_stream/balance_ab.txt).
constexpr int kJoinBatchPow2 = 16;
// The fewest waves a cycle-join launch may have: 1536 (the balance rule then picks 20-row tasks on 2049^2, 1854
// waves: C3 join 40.5 -> 32.0 us, the 2049^2 Poisson join 24.6 -> 21.9 us; 4097^2 72-row tasks, 1995 waves: 79.1 ->
// 77.1 us).  The two-material fp64 join runs two waves per SIMD (230 VGPRs), 2048 wave slots: its old 2646-wave
// launch needed a second round on most CUs.  Same-lease A/B, profiles/r06_ab/join_minw.txt.
#ifndef FEA_JOIN_MINW
#define FEA_JOIN_MINW 1536
#endif
constexpr int kJoinMinWaves = FEA_JOIN_MINW;
template <typename T>
static void join_config(int B, int H, int W, MgArgs<T>& g) {
  g.nstrips = div_up(W - 2, Ovl3<T>::S);
  const int rb_pow2 = pick_rb(B, g.nstrips, H - 2, join_max_rb());
  g.rb = B >= kJoinBatchPow2 ? rb_pow2 : balanced_rb(B, g.nstrips, (H + 1) / 2 - 2, 7, rb_pow2, kJoinMinWaves);
#ifdef FEA_LAB_JOIN_RB  // lab builds: a fixed task height (fine rows, even) for A/B runs
  g.rb = FEA_LAB_JOIN_RB;
#endif
  g.ntr = div_up((H + 1) / 2 - 2, g.rb / 2);
}

extern "C" long long fea_mg_join_norm_parts(int B, int H, int W, int elem_size) {
  if (B <= 0 || !mg_dims_ok(H, W) || !mg_odd(H, W)) return -1;
  MgArgs<double> gd{};
  MgArgs<float> gf{};
  if (elem_size == 8) {
    join_config<double>(B, H, W, gd);
    return (long long)div_up(gd.ntr * gd.nstrips, kWaves) * kWaves;
  }
  if (elem_size == 4) {
    join_config<float>(B, H, W, gf);
    return (long long)div_up(gf.ntr * gf.nstrips, kWaves) * kWaves;
  }
  return -1;
}

extern "C" int fea_norm_append(const double* ws, long long stride, long long per, int B, int nrows, double* hist,
                               unsigned* cnt, void* stream) {
  if (!ws || !hist || !cnt || B <= 0 || nrows <= 0 || per <= 0 || (nrows > 1 && stride < B * per)) return FEA_EINVAL;
  k_norm_append<<<1, 256, 0, (hipStream_t)stream>>>(ws, stride, per, B, nrows, hist, cnt);
  FEA_LAUNCH_CHECK();
}

#define FEA_NT_LAUNCH(K, TARGS)                                   \
  {                                                               \
    if (g.nt) K<TARGS, true><<<grid, 256, 0, s>>>(g);             \
    else K<TARGS, false><<<grid, 256, 0, s>>>(g);                 \
  }

// three streaming policies (g.nt: 0 cached, 1 nontemporal stores, 2 also nontemporal loads)
#define FEA_NT3_LAUNCH(K, TARGS)                                  \
  {                                                               \
    if (g.nt == 2) K<TARGS, true, true><<<grid, 256, 0, s>>>(g);  \
    else if (g.nt) K<TARGS, true, false><<<grid, 256, 0, s>>>(g); \
    else K<TARGS, false, false><<<grid, 256, 0, s>>>(g);          \
  }

#define FEA_NT_LAUNCH_ZU(K, TARGS)                                \
  {                                                               \
    if (g.nt) K<TARGS, true, true><<<grid, 256, 0, s>>>(g);       \
    else K<TARGS, false, true><<<grid, 256, 0, s>>>(g);           \
  }

#define FEA_MG_API(SUF, T)                                                                                   \
  extern "C" int fea_mg_pack_##SUF(const T* src, T* dst, const T* geo, long long geo_bs, const T* bc,         \
                                   long long bc_bs, int B, int H, int W, int ld, long long bs, void* stream) { \
    if (!dst || B <= 0 || B > 65535 || !layout_ok<T>(H, W, ld, bs)) return FEA_EINVAL;                        \
    k_mg_pack<T><<<dim3(div_up(W, 64), div_up(H, 4), B), 256, 0, (hipStream_t)stream>>>(src, dst, geo, geo_bs, \
                                                                                       bc, bc_bs, H, W, ld, bs); \
    FEA_LAUNCH_CHECK();                                                                                      \
  }                                                                                                          \
  extern "C" int fea_mg_unpack_##SUF(const T* src, T* dst, int B, int H, int W, int ld, long long bs,         \
                                     void* stream) {                                                         \
    if (!src || !dst || B <= 0 || B > 65535 || !layout_ok<T>(H, W, ld, bs)) return FEA_EINVAL;                \
    k_mg_unpack<T><<<dim3(div_up(W, 64), div_up(H, 4), B), 256, 0, (hipStream_t)stream>>>(src, dst, H, W, ld, \
                                                                                         bs);                \
    FEA_LAUNCH_CHECK();                                                                                      \
  }                                                                                                          \
  extern "C" int fea_mg_sweep_##SUF(const T* u, const T* f, T* out, const uint8_t* pid, const T* ktab,         \
                                    const T* omd, int ntab, int B, int H, int W, int ld, long long bs,         \
                                    void* stream) {                                                          \
    if (!f || !out || !ktab || !omd || B <= 0 || !layout_ok<T>(H, W, ld, bs)) return FEA_EINVAL;              \
    if (ntab < 1 || ntab > FEA_MAX_PATTERNS || (ntab > 1 && !pid) || out == u) return FEA_EINVAL;             \
    MgArgs<T> g = mg_args<T>(H, W, ld, bs, B);                                                               \
    g.u = u; g.f = f; g.out = out; g.pid = pid; g.ktab = ktab; g.omd = omd; g.ntab = ntab;                   \
    if (g.nt && (long long)B * bs * (long long)sizeof(T) > nt_load_bytes()) g.nt = 2;                      \
    const dim3 grid = mg_grid(B, g.ntr, g.nstrips);                                                          \
    hipStream_t s = (hipStream_t)stream;                                                                     \
    const bool multi = ntab > 1;                                                                             \
    if (!u) {                                                                                                \
      if (multi) FEA_NT3_LAUNCH(k_mg_sweep, T COMMA true COMMA true)                                          \
      else FEA_NT3_LAUNCH(k_mg_sweep, T COMMA false COMMA true)                                               \
    } else {                                                                                                 \
      if (multi) FEA_NT3_LAUNCH(k_mg_sweep, T COMMA true COMMA false)                                         \
      else FEA_NT3_LAUNCH(k_mg_sweep, T COMMA false COMMA false)                                              \
    }                                                                                                        \
    FEA_LAUNCH_CHECK();                                                                                      \
  }                                                                                                          \
  extern "C" int fea_mg_residual_restrict_##SUF(const T* u, const T* f, T* v_out, T* fc, const uint8_t* pid, \
                                                const T* ktab, const T* omd, int ntab, const T* rtab,          \
                                                int nrtab, T w0, int B, int H, int W, int ld, long long bs,    \
                                                int ldc, long long bsc, void* stream) {                        \
    if (!f || !fc || !ktab || !rtab || B <= 0 || !layout_ok<T>(H, W, ld, bs)) return FEA_EINVAL;               \
    if (!coarse_ok<T>(H, W, ldc, bsc)) return FEA_EINVAL;                                                    \
    if (ntab < 1 || ntab > FEA_MAX_PATTERNS || (ntab > 1 && !pid)) return FEA_EINVAL;                         \
    if (nrtab != ntab && nrtab != 1) return FEA_EINVAL;                                                      \
    if (!u && !omd) return FEA_EINVAL;                                                                       \
    MgArgs<T> g = mg_args<T>(H, W, ld, bs, B);                                                               \
    g.u = u; g.f = f; g.out = fc; g.out2 = v_out; g.pid = pid; g.ktab = ktab; g.omd = omd; g.ntab = ntab;     \
    g.rtab = rtab; g.nrtab = nrtab; g.w = w0; g.Hc = (H + 1) / 2; g.Wc = (W + 1) / 2; g.ldc = ldc;            \
    g.bsc = bsc;                                                                                             \
    g.ntr = div_up(g.Hc - 2, g.rb / 2);                                                                      \
    hipStream_t s = (hipStream_t)stream;                                                                     \
    const bool multi = ntab > 1;                                                                             \
    if (multi && nrtab == 1) return FEA_EINVAL;                                                              \
    if (!u && !v_out) { /* zero guess, v not kept: overlapped strips (k_mg_zero_restrict) */                \
      g.nstrips = div_up(W - 2, Ovl<T>::S);                                                                  \
      g.rb = pick_rb(B, g.nstrips, H - 2);                                                                   \
      g.ntr = div_up(g.Hc - 2, g.rb / 2);                                                                    \
      const dim3 grid = mg_grid_lin(B, g.ntr, g.nstrips);                                                    \
      if (multi) FEA_NT_LAUNCH(k_mg_zero_restrict, T COMMA true)                                             \
      else FEA_NT_LAUNCH(k_mg_zero_restrict, T COMMA false)                                                  \
      FEA_LAUNCH_CHECK();                                                                                    \
    }                                                                                                        \
    const dim3 grid = mg_grid(B, g.ntr, g.nstrips);                                                          \
    if (!u) {                                                                                                \
      if (multi) FEA_NT_LAUNCH(k_mg_resid_restrict, T COMMA true COMMA true)                                 \
      else FEA_NT_LAUNCH(k_mg_resid_restrict, T COMMA false COMMA true)                                      \
    } else {                                                                                                 \
      if (multi) FEA_NT_LAUNCH(k_mg_resid_restrict, T COMMA true COMMA false)                                \
      else FEA_NT_LAUNCH(k_mg_resid_restrict, T COMMA false COMMA false)                                     \
    }                                                                                                        \
    FEA_LAUNCH_CHECK();                                                                                      \
  }                                                                                                          \
  extern "C" int fea_mg_zero_restrict_send_##SUF(const T* f, T* fc, const uint8_t* pid, const T* ktab,           \
                                                 const T* omd, int ntab, const T* rtab, int nrtab, T w0, int B,  \
                                                 int H, int W, int ld, long long bs, int ldc, long long bsc,     \
                                                 T* send, int r0, int r1, int c0, int c1, void* stream) {        \
    if (!f || !fc || !ktab || !rtab || !omd || !send || B <= 0 || !layout_ok<T>(H, W, ld, bs)) return FEA_EINVAL; \
    if (!coarse_ok<T>(H, W, ldc, bsc)) return FEA_EINVAL;                                                    \
    if (ntab < 1 || ntab > FEA_MAX_PATTERNS || (ntab > 1 && !pid)) return FEA_EINVAL;                         \
    if (nrtab != ntab && nrtab != 1) return FEA_EINVAL;                                                      \
    const bool multi = ntab > 1;                                                                             \
    if (multi && nrtab == 1) return FEA_EINVAL;                                                              \
    MgArgs<T> g = mg_args<T>(H, W, ld, bs, B);                                                               \
    g.f = f; g.out = fc; g.pid = pid; g.ktab = ktab; g.omd = omd; g.ntab = ntab;                              \
    g.rtab = rtab; g.nrtab = nrtab; g.w = w0; g.Hc = (H + 1) / 2; g.Wc = (W + 1) / 2; g.ldc = ldc;            \
    g.bsc = bsc;                                                                                             \
    if (r0 < 0 || r1 <= r0 || c0 < 0 || c1 <= c0 || r1 > g.Hc || c1 > g.Wc) return FEA_EINVAL;               \
    g.gsend = send; g.gr0 = r0; g.gr1 = r1; g.gc0 = c0; g.gc1 = c1;                                          \
    g.nstrips = div_up(W - 2, Ovl<T>::S);                                                                    \
    g.rb = pick_rb(B, g.nstrips, H - 2);                                                                     \
    g.ntr = div_up(g.Hc - 2, g.rb / 2);                                                                      \
    const dim3 grid = mg_grid_lin(B, g.ntr, g.nstrips);                                                      \
    hipStream_t s = (hipStream_t)stream;                                                                     \
    if (multi) FEA_NT_LAUNCH(k_mg_zero_restrict, T COMMA true)                                               \
    else FEA_NT_LAUNCH(k_mg_zero_restrict, T COMMA false)                                                    \
    FEA_LAUNCH_CHECK();                                                                                      \
  }                                                                                                          \
  extern "C" int fea_mg_sweep_restrict_##SUF(const T* u, const T* f, T* u_out, T* fc, const uint8_t* pid,       \
                                             const T* ktab, const T* omd, int ntab, const T* rtab, int nrtab,    \
                                             T w0, int B, int H, int W, int ld, long long bs, int ldc,          \
                                             long long bsc, double* norm_ws, double* norm_hist,                 \
                                             unsigned* norm_cnt, void* stream) {                                \
    if (!u || !f || !u_out || !fc || !ktab || !omd || !rtab || B <= 0 || !layout_ok<T>(H, W, ld, bs) ||       \
        u_out == u)                                                                                          \
      return FEA_EINVAL;                                                                                     \
    const bool norm = norm_hist != nullptr;                                                                  \
    if (norm && (!norm_ws || !norm_cnt)) return FEA_EINVAL;                                                  \
    if (!coarse_ok<T>(H, W, ldc, bsc)) return FEA_EINVAL;                                                    \
    if (ntab < 1 || ntab > FEA_MAX_PATTERNS || (ntab > 1 && !pid) || (nrtab != ntab && nrtab != 1))          \
      return FEA_EINVAL;                                                                                     \
    if (ntab > 1 && nrtab == 1) return FEA_EINVAL;                                                           \
    MgArgs<T> g = mg_args<T>(H, W, ld, bs, B);                                                               \
    g.u = u; g.f = f; g.out = fc; g.out2 = u_out; g.pid = pid; g.ktab = ktab; g.omd = omd; g.ntab = ntab;     \
    g.rtab = rtab; g.nrtab = nrtab; g.w = w0; g.Hc = (H + 1) / 2; g.Wc = (W + 1) / 2; g.ldc = ldc;            \
    g.bsc = bsc;                                                                                             \
    g.nstrips = div_up(W - 2, Ovl<T>::S);  /* overlapped strips */                                           \
    g.rb = balanced_rb(B, g.nstrips, g.Hc - 2, 3, pick_rb(B, g.nstrips, H - 2, 2 * kRB));                    \
    g.ntr = div_up(g.Hc - 2, g.rb / 2);                                                                      \
    g.part = norm_ws;                                                                                        \
    const dim3 grid = mg_grid_lin(B, g.ntr, g.nstrips);                                                      \
    hipStream_t s = (hipStream_t)stream;                                                                     \
    if (norm && (long long)grid.x * kWaves * 8 > (long long)fea_norm_workspace_bytes(B, H, W))               \
      return FEA_EINVAL;                                                                                     \
    if (ntab > 1) {                                                                                          \
      if (norm) FEA_NT_LAUNCH(k_mg_sweep_restrict, T COMMA true COMMA true)                                  \
      else FEA_NT_LAUNCH(k_mg_sweep_restrict, T COMMA true COMMA false)                                      \
    } else {                                                                                                 \
      if (norm) FEA_NT_LAUNCH(k_mg_sweep_restrict, T COMMA false COMMA true)                                 \
      else FEA_NT_LAUNCH(k_mg_sweep_restrict, T COMMA false COMMA false)                                     \
    }                                                                                                        \
    if (norm)                                                                                                \
      k_norm_append<<<1, 256, 0, s>>>(norm_ws, 0, (long long)(grid.x / B) * kWaves, B, 1, norm_hist, norm_cnt); \
    FEA_LAUNCH_CHECK();                                                                                      \
  }                                                                                                          \
  static int mg_prolong_##SUF(const T* u, const T* ec, const T* f, T* out, const uint8_t* pid,               \
                              const uint8_t* pidc, const T* ktab, const T* omd, int ntab, const T* ptab,      \
                              int nptab, T w1, int B, int H, int W, int ld, long long bs, int ldc,           \
                              long long bsc, void* stream, bool sweep) {                                     \
    if ((!u && !sweep) || !ec || !out || !ptab || B <= 0 || !layout_ok<T>(H, W, ld, bs) || out == u)         \
      return FEA_EINVAL;                                                                                     \
    if (!u && out == f) return FEA_EINVAL;                                                                   \
    if (!coarse_ok<T>(H, W, ldc, bsc)) return FEA_EINVAL;                                                    \
    if (nptab < 1 || nptab > FEA_MAX_PATTERNS || (nptab > 1 && !pidc)) return FEA_EINVAL;                    \
    if (sweep && (!f || !ktab || !omd || ntab < 1 || ntab > FEA_MAX_PATTERNS || (ntab > 1 && !pid)))          \
      return FEA_EINVAL;                                                                                     \
    const bool multi = nptab > 1 || (sweep && ntab > 1);                                                     \
    if (multi && ((sweep && (!pid || ntab == 1)) || !pidc || nptab == 1)) return FEA_EINVAL;                 \
    MgArgs<T> g = mg_args<T>(H, W, ld, bs, B);                                                               \
    g.u = u; g.ec = ec; g.f = f; g.out = out; g.pid = pid; g.pidc = pidc; g.ktab = ktab; g.omd = omd;         \
    g.ntab = ntab; g.ptab = ptab; g.nptab = nptab; g.w = w1; g.Hc = (H + 1) / 2; g.Wc = (W + 1) / 2;          \
    g.ldc = ldc; g.bsc = bsc;                                                                                \
    hipStream_t s = (hipStream_t)stream;                                                                     \
    if (sweep && !u && zu_ovl((long long)B * bs * (long long)sizeof(T))) { /* overlapped strips */           \
      g.nstrips = div_up(W - 2, Ovl<T>::S);                                                                  \
      g.rb = pick_rb(B, g.nstrips, H - 2);                                                                   \
      g.ntr = div_up(H - 2, g.rb);                                                                           \
      const dim3 grid = mg_grid_lin(B, g.ntr, g.nstrips);                                                    \
      if (multi) FEA_NT_LAUNCH(k_mg_prolong_zu_ovl, T COMMA true)                                            \
      else FEA_NT_LAUNCH(k_mg_prolong_zu_ovl, T COMMA false)                                                 \
      FEA_LAUNCH_CHECK();                                                                                    \
    }                                                                                                        \
    const dim3 grid = mg_grid(B, g.ntr, g.nstrips);                                                          \
    if (sweep && !u) {                                                                                       \
      if (multi) FEA_NT_LAUNCH_ZU(k_mg_prolong, T COMMA true COMMA true)                                     \
      else FEA_NT_LAUNCH_ZU(k_mg_prolong, T COMMA false COMMA true)                                          \
    } else if (sweep) {                                                                                      \
      if (multi) FEA_NT_LAUNCH(k_mg_prolong, T COMMA true COMMA true)                                        \
      else FEA_NT_LAUNCH(k_mg_prolong, T COMMA false COMMA true)                                             \
    } else {                                                                                                 \
      if (multi) FEA_NT_LAUNCH(k_mg_prolong, T COMMA true COMMA false)                                       \
      else FEA_NT_LAUNCH(k_mg_prolong, T COMMA false COMMA false)                                            \
    }                                                                                                        \
    FEA_LAUNCH_CHECK();                                                                                      \
  }                                                                                                          \
  extern "C" int fea_mg_prolong_sweep_##SUF(const T* u, const T* ec, const T* f, T* out, const uint8_t* pid,  \
                                            const uint8_t* pidc, const T* ktab, const T* omd, int ntab,       \
                                            const T* ptab, int nptab, T w1, int B, int H, int W, int ld,     \
                                            long long bs, int ldc, long long bsc, void* stream) {             \
    return mg_prolong_##SUF(u, ec, f, out, pid, pidc, ktab, omd, ntab, ptab, nptab, w1, B, H, W, ld, bs, ldc, \
                            bsc, stream, true);                                                              \
  }                                                                                                          \
  extern "C" int fea_mg_prolong_add_##SUF(const T* u, const T* ec, T* out, const uint8_t* pidc, const T* ptab, \
                                          int nptab, T w1, int B, int H, int W, int ld, long long bs, int ldc, \
                                          long long bsc, void* stream) {                                     \
    return mg_prolong_##SUF(u, ec, nullptr, out, nullptr, pidc, nullptr, nullptr, 0, ptab, nptab, w1, B, H,  \
                            W, ld, bs, ldc, bsc, stream, false);                                             \
  }                                                                                                          \
  extern "C" int fea_mg_cycle_join_##SUF(const T* u, const T* ec, const T* f, T* u_out, T* fc, const uint8_t* pid, \
                                         const uint8_t* pidc, const T* ktab, const T* omd, int ntab, const T* ptab, \
                                         int nptab, const T* rtab, int nrtab, T w1, T w0, int B, int H, int W,     \
                                         int ld, long long bs, int ldc, long long bsc, double* norm_ws,          \
                                         double* norm_hist, unsigned* norm_cnt, void* stream) {                  \
    if (!u || !ec || !f || !u_out || !fc || !ktab || !omd || !ptab || !rtab || B <= 0 || u_out == u)          \
      return FEA_EINVAL;                                                                                     \
    const bool norm = norm_ws != nullptr, append = norm_hist != nullptr;                                      \
    if (append && (!norm_ws || !norm_cnt)) return FEA_EINVAL;                                                \
    if (!layout_ok<T>(H, W, ld, bs) || !coarse_ok<T>(H, W, ldc, bsc)) return FEA_EINVAL;                     \
    if (ntab < 1 || ntab > FEA_MAX_PATTERNS || (nrtab != ntab && nrtab != 1) || (nptab != ntab && nptab != 1)) \
      return FEA_EINVAL;                                                                                     \
    const bool multi = ntab > 1;                                                                             \
    if (multi && (!pid || !pidc || nrtab == 1 || nptab == 1)) return FEA_EINVAL;                             \
    MgArgs<T> g = mg_args<T>(H, W, ld, bs, B);                                                               \
    g.u = u; g.ec = ec; g.f = f; g.out = fc; g.out2 = u_out; g.pid = pid; g.pidc = pidc; g.ktab = ktab;       \
    g.omd = omd; g.ntab = ntab; g.ptab = ptab; g.nptab = nptab; g.rtab = rtab; g.nrtab = nrtab; g.w = w0;     \
    g.w2 = w1; g.Hc = (H + 1) / 2; g.Wc = (W + 1) / 2; g.ldc = ldc; g.bsc = bsc;                              \
    join_config<T>(B, H, W, g);                                                                              \
    if (g.nt && bs * (long long)sizeof(T) > nt_load_bytes()) g.nt = 2;                                         \
    FEA_LAB_JOIN_REV(g);                                                                                     \
    g.part = norm_ws;                                                                                        \
    const dim3 grid = mg_grid_lin(B, g.ntr, g.nstrips);                                                      \
    hipStream_t s = (hipStream_t)stream;                                                                     \
    if (norm && (long long)grid.x * kWaves * 8 > (long long)fea_norm_workspace_bytes(B, H, W))               \
      return FEA_EINVAL;                                                                                     \
    if (multi) {                                                                                             \
      if (norm) FEA_NT3_LAUNCH(k_mg_cycle_join, T COMMA true COMMA true)                                      \
      else FEA_NT3_LAUNCH(k_mg_cycle_join, T COMMA true COMMA false)                                          \
    } else {                                                                                                 \
      if (norm) FEA_NT3_LAUNCH(k_mg_cycle_join, T COMMA false COMMA true)                                     \
      else FEA_NT3_LAUNCH(k_mg_cycle_join, T COMMA false COMMA false)                                         \
    }                                                                                                        \
    if (append)                                                                                              \
      k_norm_append<<<1, 256, 0, s>>>(norm_ws, 0, (long long)(grid.x / B) * kWaves, B, 1, norm_hist, norm_cnt); \
    FEA_LAUNCH_CHECK();                                                                                      \
  }                                                                                                          \
  extern "C" int fea_mg_residual_norm_##SUF(const T* u, const T* f, const uint8_t* pid, const T* ktab,        \
                                            int ntab, double* out, double* ws, int B, int H, int W, int ld,   \
                                            long long bs, int rlo, int rhi, int clo, int chi, void* stream) {\
    if (!u || !f || !ktab || !out || !ws || B <= 0 || !layout_ok<T>(H, W, ld, bs)) return FEA_EINVAL;         \
    if (ntab < 1 || ntab > FEA_MAX_PATTERNS || (ntab > 1 && !pid)) return FEA_EINVAL;                         \
    if (rlo == 0 && rhi == 0) {                                                                              \
      rlo = 1;                                                                                               \
      rhi = H - 1;                                                                                           \
    }                                                                                                        \
    if (rlo < 1 || rhi > H - 1 || rhi < rlo) return FEA_EINVAL;                                              \
    if (clo == 0 && chi == 0) {                                                                              \
      clo = 1;                                                                                               \
      chi = W - 1;                                                                                           \
    }                                                                                                        \
    if (clo < 1 || chi > W - 1 || chi < clo) return FEA_EINVAL;                                              \
    MgArgs<T> g = mg_args<T>(H, W, ld, bs, B);                                                               \
    g.u = u; g.f = f; g.pid = pid; g.ktab = ktab; g.ntab = ntab; g.part = ws;                                \
    g.rlo = rlo; g.rhi = rhi; g.clo = clo; g.chi = chi;                                                      \
    g.rb = 2;                                                                                                \
    while (g.rb < kRB && (long long)B * g.nstrips * div_up(rhi - rlo, g.rb * 2) >= target_waves()) g.rb *= 2; \
    g.ntr = std::max(div_up(rhi - rlo, g.rb), 1);                                                            \
    const dim3 grid = mg_grid(B, g.ntr, g.nstrips);                                                          \
    hipStream_t s = (hipStream_t)stream;                                                                     \
    if (rhi == rlo) {                                                                                        \
      (void)hipMemsetAsync(ws, 0, sizeof(double) * (size_t)B * g.nstrips, s);                                      \
      g.ntr = 1;                                                                                             \
    } else if (ntab > 1) {                                                                                   \
      k_mg_resnorm<T, true><<<grid, 256, 0, s>>>(g);                                                         \
    } else {                                                                                                 \
      k_mg_resnorm<T, false><<<grid, 256, 0, s>>>(g);                                                        \
    }                                                                                                        \
    k_norm_final<<<B, 256, 0, s>>>(ws, (long long)g.ntr * g.nstrips, out);                                   \
    FEA_LAUNCH_CHECK();                                                                                      \
  }

#define COMMA ,
FEA_MG_API(f32, float)
FEA_MG_API(f64, double)

// The cycle join over up to four rectangles of the grid in ONE launch (a domain-decomposed rank's border strips,
// whose nodes its halo exchange sends, ahead of the interior that runs while the messages are in flight).
// rects: nrect x {I0, I1, c0, c1}: coarse rows [I0, I1) with their fine rows 2I-1, 2I (and row H-2 when I1 = Hc-1),
// fine columns [c0, c1) with odd c0 and c1 odd or W-1 (coarse column J goes with fine columns 2J-1, 2J).  Every node is the same
// expression as in the whole-grid launch, so a cover of the grid by rectangles is bitwise fea_mg_cycle_join.
template <typename T>
static int cycle_join_rects(const T* u, const T* ec, const T* f, T* u_out, T* fc, const uint8_t* pid,
                            const uint8_t* pidc, const T* ktab, const T* omd, int ntab, const T* ptab, int nptab,
                            const T* rtab, int nrtab, T w1, T w0, int B, int H, int W, int ld, long long bs, int ldc,
                            long long bsc, int nrect, const int* rects, void* stream) {
  if (!u || !ec || !f || !u_out || !fc || !ktab || !omd || !ptab || !rtab || B <= 0 || u_out == u || !rects ||
      nrect < 1 || nrect > 4)
    return FEA_EINVAL;
  if (!layout_ok<T>(H, W, ld, bs) || !coarse_ok<T>(H, W, ldc, bsc)) return FEA_EINVAL;
  if (ntab < 1 || ntab > FEA_MAX_PATTERNS || (nrtab != ntab && nrtab != 1) || (nptab != ntab && nptab != 1))
    return FEA_EINVAL;
  const bool multi = ntab > 1;
  if (multi && (!pid || !pidc || nrtab == 1 || nptab == 1)) return FEA_EINVAL;
  MgArgs<T> g = mg_args<T>(H, W, ld, bs, B);
  g.u = u; g.ec = ec; g.f = f; g.out = fc; g.out2 = u_out; g.pid = pid; g.pidc = pidc; g.ktab = ktab;
  g.omd = omd; g.ntab = ntab; g.ptab = ptab; g.nptab = nptab; g.rtab = rtab; g.nrtab = nrtab; g.w = w0;
  g.w2 = w1; g.Hc = (H + 1) / 2; g.Wc = (W + 1) / 2; g.ldc = ldc; g.bsc = bsc;
  if (g.nt && bs * (long long)sizeof(T) > nt_load_bytes()) g.nt = 2;
  g.nrect = nrect;
  for (int r = 0; r < nrect; ++r) {
    const int I0 = rects[4 * r], I1 = rects[4 * r + 1], c0 = rects[4 * r + 2], c1 = rects[4 * r + 3];
    if (I0 < 1 || I1 > g.Hc - 1 || I0 >= I1 || c0 < 1 || c1 > W - 1 || c0 >= c1 || !(c0 & 1) ||
        (!(c1 & 1) && c1 != W - 1))
      return FEA_EINVAL;
    g.rI0[r] = I0; g.rI1[r] = I1; g.rc0[r] = c0; g.rc1[r] = c1;
    g.rns[r] = div_up(c1 - c0, Ovl3<T>::S);
  }
  // rows per task: the tallest (<= the join's cap) that still gives the launch target_waves() waves
  auto tasks = [&](int rb) {
    long long n = 0;
    for (int r = 0; r < nrect; ++r) n += (long long)div_up(g.rI1[r] - g.rI0[r], rb / 2) * g.rns[r];
    return n;
  };
  g.rb = join_max_rb();
  while (g.rb > 2 && (long long)B * tasks(g.rb) < target_waves()) g.rb /= 2;
  g.rt[0] = 0;
  for (int r = 0; r < nrect; ++r) g.rt[r + 1] = g.rt[r] + div_up(g.rI1[r] - g.rI0[r], g.rb / 2) * g.rns[r];
  const dim3 grid((unsigned)(B * div_up(g.rt[nrect], kWaves)));
  hipStream_t s = (hipStream_t)stream;
  if (multi) FEA_NT3_LAUNCH(k_mg_cycle_join, T COMMA true COMMA false)
  else FEA_NT3_LAUNCH(k_mg_cycle_join, T COMMA false COMMA false)
  FEA_LAUNCH_CHECK();
}

#define FEA_JOIN_RECTS_API(SUF, T)                                                                            \
  extern "C" int fea_mg_cycle_join_rects_##SUF(const T* u, const T* ec, const T* f, T* u_out, T* fc,            \
                                               const uint8_t* pid, const uint8_t* pidc, const T* ktab,          \
                                               const T* omd, int ntab, const T* ptab, int nptab, const T* rtab,  \
                                               int nrtab, T w1, T w0, int B, int H, int W, int ld, long long bs,  \
                                               int ldc, long long bsc, int nrect, const int* rects,             \
                                               void* stream) {                                                  \
    return cycle_join_rects<T>(u, ec, f, u_out, fc, pid, pidc, ktab, omd, ntab, ptab, nptab, rtab, nrtab, w1, w0, \
                               B, H, W, ld, bs, ldc, bsc, nrect, rects, stream);                               \
  }
FEA_JOIN_RECTS_API(f32, float)
FEA_JOIN_RECTS_API(f64, double)

// Rows per task of k_mg_zero_restrict2 (fine rows, a multiple of 4): the tallest power of two that still
// gives kZr2Waves waves, at least kZr2MinRb (each task recomputes 3 + 1 rows of the intermediate level).
// Lab A/B at 2049^2 fp64 (tools/lab/zr2_ab.py): 16 rows 14.3 us, 32 rows 16.2, 64 rows 19.1.
#ifndef FEA_ZR2_MINRB
#define FEA_ZR2_MINRB 4
#endif
#ifndef FEA_ZR2_WAVES
#define FEA_ZR2_WAVES 2048
#endif
constexpr int kZr2MinRb = FEA_ZR2_MINRB;
constexpr int kZr2Waves = FEA_ZR2_WAVES;

// Two-level kernels (zero_restrict2, prolong2): task height by the balanced rule (balanced_rb's cost: the slowest
// CU's workgroup count x the rows a task streams, u units of k fine rows + ovh recomputed rows), among heights
// that keep >= 2048 waves and are at most umax units tall; the power-of-two choice `fallback` when none does.  e.g. the 2049^2 fp64 level-pair
// prolongation: 662 workgroups of 14 rows (<= 3 per CU) instead of 576 of 16 (a quarter of the CUs ran 3 of the
// 2.25 average).
#ifndef FEA_BAL2
#define FEA_BAL2 1
#endif
// the fewest waves a two-level launch may have: 1024 (metric V-cycle 132.5 -> 131.0 us against 2048 — fewer,
// taller tasks re-stream fewer overlap rows; 3072 / 4096 measured +4 us, 512 / 768 +1.5 us; profiles/r06_ab)
#ifndef FEA_BAL2_WAVES
#define FEA_BAL2_WAVES 1024
#endif
static int balanced_units(int B, int nstrips, int rows_u, int k, int ovh, int fallback, int umax = 256) {
#if FEA_BAL2
  const long long ncu = num_cus();
  long long best = -1;
  int bu = fallback;
  for (int u = 1; u <= rows_u && u <= umax && k * u <= 256; ++u) {
    const long long ntr = div_up(rows_u, u), waves = (long long)B * nstrips * ntr;
    if (waves < FEA_BAL2_WAVES) break;
    const long long wgs = (long long)B * div_up(ntr * nstrips, kWaves);
    const long long cost = div_up(wgs, ncu) * (k * u + ovh);
    if (best < 0 || cost < best) best = cost, bu = u;
  }
  return bu;
#else
  (void)B; (void)nstrips; (void)rows_u; (void)k; (void)ovh; (void)umax;
  return fallback;
#endif
}

// send: the agglomeration's all-gather send buffer ([B, r1 - r0, c1 - c0]) that also receives f_{l+2}'s block
// [r0, r1) x [c0, c1) (nullptr: none)
template <typename T>
static int zero_restrict2(const T* f, T* fc, T* fc2, const uint8_t* pid, const uint8_t* pidc, const T* ktab,
                          const T* omd, int ntab, const T* rtab, int nrtab, T w0, int B, int H, int W, int ld,
                          long long bs, int ldc, long long bsc, int ldc2, long long bsc2, void* stream,
                          T* send = nullptr, int r0 = 0, int r1 = 0, int c0 = 0, int c1 = 0) {
  if (!f || !fc || !fc2 || !ktab || !omd || !rtab || B <= 0 || !layout_ok<T>(H, W, ld, bs)) return FEA_EINVAL;
  if (!coarse_ok<T>(H, W, ldc, bsc)) return FEA_EINVAL;
  const int Hc = (H + 1) / 2, Wc = (W + 1) / 2;
  if (!coarse_ok<T>(Hc, Wc, ldc2, bsc2)) return FEA_EINVAL;
  const bool multi = ntab > 1;
  if (ntab < 1 || ntab > FEA_MAX_PATTERNS || (multi && (!pid || !pidc))) return FEA_EINVAL;
  if (nrtab != ntab && nrtab != 1) return FEA_EINVAL;
  if (multi && nrtab == 1) return FEA_EINVAL;
  MgArgs<T> g = mg_args<T>(H, W, ld, bs, B);
  g.f = f; g.out = fc; g.out2 = fc2; g.pid = pid; g.pidc = pidc; g.ktab = ktab; g.omd = omd; g.ntab = ntab;
  g.rtab = rtab; g.nrtab = nrtab; g.w = w0;
  g.Hc = Hc; g.Wc = Wc; g.ldc = ldc; g.bsc = bsc;
  g.Hc2 = (Hc + 1) / 2; g.Wc2 = (Wc + 1) / 2; g.ldc2 = ldc2; g.bsc2 = bsc2;
  if (send) {
    if (r0 < 0 || r1 <= r0 || c0 < 0 || c1 <= c0 || r1 > g.Hc2 || c1 > g.Wc2) return FEA_EINVAL;
    g.gsend = send; g.gr0 = r0; g.gr1 = r1; g.gc0 = c0; g.gc1 = c1;
  }
  g.nstrips = div_up(W - 2, Ovl2<T>::S);
  g.rb = 2 * kRB;
  while (g.rb > kZr2MinRb && (long long)B * g.nstrips * div_up(g.Hc2 - 2, g.rb / 4) < kZr2Waves) g.rb /= 2;
  g.rb = 4 * balanced_units(B, g.nstrips, g.Hc2 - 2, 4, 8, g.rb / 4);
  g.ntr = div_up(g.Hc2 - 2, g.rb / 4);
  const dim3 grid = mg_grid_lin(B, g.ntr, g.nstrips);
  hipStream_t s = (hipStream_t)stream;
  if (multi) k_mg_zero_restrict2<T, true><<<grid, 256, 0, s>>>(g);
  else k_mg_zero_restrict2<T, false><<<grid, 256, 0, s>>>(g);
  FEA_LAUNCH_CHECK();
}

#define FEA_ZR2_API(SUF, T)                                                                                   \
  extern "C" int fea_mg_zero_restrict2_##SUF(const T* f, T* fc, T* fc2, const uint8_t* pid, const uint8_t* pidc, \
                                             const T* ktab, const T* omd, int ntab, const T* rtab, int nrtab,     \
                                             T w0, int B, int H, int W, int ld, long long bs, int ldc,          \
                                             long long bsc, int ldc2, long long bsc2, void* stream) {            \
    return zero_restrict2<T>(f, fc, fc2, pid, pidc, ktab, omd, ntab, rtab, nrtab, w0, B, H, W, ld, bs, ldc, bsc,  \
                             ldc2, bsc2, stream);                                                              \
  }                                                                                                           \
  extern "C" int fea_mg_zero_restrict2_send_##SUF(const T* f, T* fc, T* fc2, const uint8_t* pid,                \
                                                  const uint8_t* pidc, const T* ktab, const T* omd, int ntab,    \
                                                  const T* rtab, int nrtab, T w0, int B, int H, int W, int ld,   \
                                                  long long bs, int ldc, long long bsc, int ldc2, long long bsc2, \
                                                  T* send, int r0, int r1, int c0, int c1, void* stream) {       \
    if (!send) return FEA_EINVAL;                                                                             \
    return zero_restrict2<T>(f, fc, fc2, pid, pidc, ktab, omd, ntab, rtab, nrtab, w0, B, H, W, ld, bs, ldc, bsc,  \
                             ldc2, bsc2, stream, send, r0, r1, c0, c1);                                        \
  }
FEA_ZR2_API(f32, float)
FEA_ZR2_API(f64, double)

template <typename T>
static int prolong2(const T* fc, const T* ec2, const T* f, T* out, const uint8_t* pid, const uint8_t* pidc,
                    const uint8_t* pidc2, const T* ktab, const T* omd, int ntab, const T* ptab, int nptab, T w1, int B,
                    int H, int W, int ld, long long bs, int ldc, long long bsc, int ldc2, long long bsc2,
                    void* stream) {
  if (!fc || !ec2 || !f || !out || !ktab || !omd || !ptab || B <= 0 || !layout_ok<T>(H, W, ld, bs)) return FEA_EINVAL;
  if (!coarse_ok<T>(H, W, ldc, bsc)) return FEA_EINVAL;
  const int Hc = (H + 1) / 2, Wc = (W + 1) / 2;
  if (!coarse_ok<T>(Hc, Wc, ldc2, bsc2)) return FEA_EINVAL;
  const bool multi = ntab > 1;
  if (ntab < 1 || ntab > FEA_MAX_PATTERNS || (nptab != ntab && nptab != 1)) return FEA_EINVAL;
  if (multi && (!pid || !pidc || !pidc2 || nptab == 1)) return FEA_EINVAL;
  MgArgs<T> g = mg_args<T>(H, W, ld, bs, B);
  g.ec = fc; g.ec2 = ec2; g.f = f; g.out = out; g.pid = pid; g.pidc = pidc; g.pidc2 = pidc2; g.ktab = ktab;
  g.omd = omd; g.ntab = ntab; g.ptab = ptab; g.nptab = nptab; g.w = w1;
  g.Hc = Hc; g.Wc = Wc; g.ldc = ldc; g.bsc = bsc;
  g.Hc2 = (Hc + 1) / 2; g.Wc2 = (Wc + 1) / 2; g.ldc2 = ldc2; g.bsc2 = bsc2;
  g.nstrips = div_up(W - 2, Ovl4<T>::S);
  // (no taller tasks than the power-of-two choice: batched fp32 prolong2 at 1025^2 x 256 ran 41.7 -> 51.5 us with
  // half the waves)
  const int u2 = pick_rb(B, g.nstrips, H - 2) / 2;
  g.rb = 2 * balanced_units(B, g.nstrips, (H - 1) / 2, 2, 4, u2, u2);
  g.ntr = div_up(H - 2, g.rb);
  const dim3 grid = mg_grid_lin(B, g.ntr, g.nstrips);
  hipStream_t s = (hipStream_t)stream;
  if (multi) k_mg_prolong2<T, true><<<grid, 256, 0, s>>>(g);
  else k_mg_prolong2<T, false><<<grid, 256, 0, s>>>(g);
  FEA_LAUNCH_CHECK();
}

#define FEA_PROLONG2_API(SUF, T)                                                                              \
  extern "C" int fea_mg_prolong2_##SUF(const T* fc, const T* ec2, const T* f, T* out, const uint8_t* pid,      \
                                       const uint8_t* pidc, const uint8_t* pidc2, const T* ktab, const T* omd,  \
                                       int ntab, const T* ptab, int nptab, T w1, int B, int H, int W, int ld,   \
                                       long long bs, int ldc, long long bsc, int ldc2, long long bsc2,          \
                                       void* stream) {                                                        \
    return prolong2<T>(fc, ec2, f, out, pid, pidc, pidc2, ktab, omd, ntab, ptab, nptab, w1, B, H, W, ld, bs, ldc, \
                       bsc, ldc2, bsc2, stream);                                                               \
  }
FEA_PROLONG2_API(f32, float)
FEA_PROLONG2_API(f64, double)
