// dd_ops.hip — packing for the domain-decomposed V-cycle's halo exchange (feanet_amd.dd): the 2-D blocks of
// one or more exchanges (ghost rows, columns and corners of all their levels and buffers, all samples) copied
// between the framed level buffers and contiguous staging buffers in a single launch, so an exchange is
// pack -> one group of P2P messages (one per neighbour) -> unpack, whatever its number of blocks.
// The block table travels in the kernel arguments (a halo's blocks are few and tiny: the copy is latency-
// bound, and a table read from device memory would put one more dependent DRAM round trip in front of it).
#include "fea_common.h"

namespace fea {

struct DDBlock {       // (mirrors feanet_amd/dd.py _Staging records: 4 int64 words)
  long long frame;     // device address of the block's first element in the framed buffer
  long long stage;     // device address of the block in its staging buffer (rows x cols, row-major)
  long long ld;        // row pitch of the framed buffer, elements
  int rows, cols;
};

constexpr int kDDTable = 48;  // blocks per launch (1.5 KB of kernel arguments)

struct DDTable {
  DDBlock b[kDDTable];
};

template <typename T>
__global__ __launch_bounds__(256) void k_dd_copy_blocks(const DDTable tab, int to_stage) {
  const DDBlock b = tab.b[blockIdx.y];
  T* __restrict__ frame = reinterpret_cast<T*>(b.frame);
  T* __restrict__ st = reinterpret_cast<T*>(b.stage);
  const int n = b.rows * b.cols;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const int r = i / b.cols, c = i - r * b.cols;
    if (to_stage)
      st[i] = frame[(long long)r * b.ld + c];
    else
      frame[(long long)r * b.ld + c] = st[i];
  }
}

// Strided rectangle copies (the agglomeration's all-gather staging, the placement of the gathered blocks into the
// coarse field and the scatter of the coarse solution back): both sides strided, any number of rectangles in
// one launch.  Latency-bound like the halo pack, so the grid spreads a rectangle over up to 256 workgroups
// (one element per thread) instead of looping.
struct DDRect {     // (mirrors feanet_amd/dd.py _rect_records: 6 int64 words)
  long long dst, src;        // device addresses of the rectangles' first elements
  long long dst_ld, src_ld;  // row pitches, elements
  long long rows, cols;
};

constexpr int kDDRects = 32;  // rectangles per launch (1.5 KB of kernel arguments)

struct DDRectTable {
  DDRect r[kDDRects];
};

template <typename T>
__global__ __launch_bounds__(256) void k_dd_copy_rects(const DDRectTable tab) {
  const DDRect q = tab.r[blockIdx.y];
  T* __restrict__ dst = reinterpret_cast<T*>(q.dst);
  const T* __restrict__ src = reinterpret_cast<const T*>(q.src);
  const int cols = (int)q.cols;
  const int n = (int)(q.rows * q.cols);
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const int r = i / cols, c = i - r * cols;
    dst[r * q.dst_ld + c] = src[r * q.src_ld + c];
  }
}

}  // namespace fea

using namespace fea;

extern "C" int fea_dd_copy_rects(const void* rects, int nrects, int elem_size, void* stream) {
  if (!rects || nrects <= 0 || (elem_size != 4 && elem_size != 8)) return FEA_EINVAL;
  const DDRect* all = static_cast<const DDRect*>(rects);
  hipStream_t s = (hipStream_t)stream;
  for (int r0 = 0; r0 < nrects; r0 += kDDRects) {
    DDRectTable tab{};
    const int nr = std::min(kDDRects, nrects - r0);
    long long mx = 1;
    for (int i = 0; i < nr; ++i) {
      const DDRect& q = all[r0 + i];
      const long long n = q.rows * q.cols;
      if (q.rows < 0 || q.cols <= 0 || n >= (1ll << 31) || !q.dst || !q.src || q.dst_ld < q.cols ||
          q.src_ld < q.cols)
        return FEA_EINVAL;
      tab.r[i] = q;
      mx = std::max(mx, n);
    }
    const dim3 grid((unsigned)std::min<long long>((mx + 255) / 256, 256), (unsigned)nr);
    if (elem_size == 8)
      k_dd_copy_rects<double><<<grid, 256, 0, s>>>(tab);
    else
      k_dd_copy_rects<float><<<grid, 256, 0, s>>>(tab);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
  }
  return 0;
}

extern "C" int fea_dd_copy_blocks(const void* blocks, int nblocks, int elem_size, int to_stage, void* stream) {
  if (!blocks || nblocks <= 0 || (elem_size != 4 && elem_size != 8)) return FEA_EINVAL;
  const DDBlock* all = static_cast<const DDBlock*>(blocks);
  hipStream_t s = (hipStream_t)stream;
  for (int b0 = 0; b0 < nblocks; b0 += kDDTable) {
    DDTable tab{};
    const int nb = std::min(kDDTable, nblocks - b0);
    long long mx = 1;
    for (int i = 0; i < nb; ++i) {
      tab.b[i] = all[b0 + i];
      const long long n = (long long)tab.b[i].rows * tab.b[i].cols;
      if (tab.b[i].rows < 0 || tab.b[i].cols <= 0 || n >= (1ll << 31) || !tab.b[i].frame || !tab.b[i].stage)
        return FEA_EINVAL;
      mx = std::max(mx, n);
    }
    const dim3 grid((unsigned)std::min<long long>((mx + 255) / 256, 256), (unsigned)nb);
    if (elem_size == 8)
      k_dd_copy_blocks<double><<<grid, 256, 0, s>>>(tab, to_stage);
    else
      k_dd_copy_blocks<float><<<grid, 256, 0, s>>>(tab, to_stage);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
  }
  return 0;
}
