// dd_ops.hip — packing for the domain-decomposed V-cycle's halo exchange (feanet_amd.dd): every 2-D block of
// one exchange (the ghost rows, columns and corners of all its levels and buffers, all samples) copied
// between the framed level buffers and ONE contiguous staging buffer in a single launch, so an exchange is
// pack -> one group of P2P messages (one per neighbour) -> unpack, whatever its number of blocks.
#include "fea_common.h"

namespace fea {

struct DDBlock {       // (mirrors feanet_amd/dd.py _DD_BLOCK: 4 int64 words)
  long long base;      // device address of the block's first element in the framed buffer
  long long stage;     // element offset of the block in the staging buffer (rows x cols, row-major)
  long long ld;        // row pitch of the framed buffer, elements
  int rows, cols;
};

template <typename T>
__global__ __launch_bounds__(256) void k_dd_copy_blocks(const DDBlock* __restrict__ blocks, T* __restrict__ stage,
                                                        int to_stage) {
  const DDBlock b = blocks[blockIdx.y];
  T* __restrict__ frame = reinterpret_cast<T*>(b.base);
  T* __restrict__ st = stage + b.stage;
  const long long n = (long long)b.rows * b.cols;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const long long r = i / b.cols, c = i - r * b.cols;
    if (to_stage)
      st[i] = frame[r * b.ld + c];
    else
      frame[r * b.ld + c] = st[i];
  }
}

}  // namespace fea

using namespace fea;

extern "C" int fea_dd_copy_blocks(const void* blocks, int nblocks, long long max_elems, void* stage, int elem_size,
                                  int to_stage, void* stream) {
  if (!blocks || !stage || nblocks <= 0 || nblocks > 65535 || max_elems <= 0 || (elem_size != 4 && elem_size != 8))
    return FEA_EINVAL;
  const long long gx = std::min<long long>((max_elems + 255) / 256, 64);
  const dim3 grid((unsigned)gx, (unsigned)nblocks);
  hipStream_t s = (hipStream_t)stream;
  if (elem_size == 8)
    k_dd_copy_blocks<double><<<grid, 256, 0, s>>>(static_cast<const DDBlock*>(blocks), static_cast<double*>(stage),
                                                   to_stage);
  else
    k_dd_copy_blocks<float><<<grid, 256, 0, s>>>(static_cast<const DDBlock*>(blocks), static_cast<float*>(stage),
                                                  to_stage);
  FEA_LAUNCH_CHECK();
}
