// setup_ops.hip — on-device mesh set-up: the two-material node pattern map.
//
// FEANet/mesh.py builds MeshCenterInterface's per-node pattern ids with an O(N^4) Python search
// (place_circle / place_rect :62-76, identify_patterns :78-93, generate_global_pattern_map :95-101;
// ~64 h at 2049^2).  The map is a pure function of the node position, so one thread per node
// computes it here, with the reference's float32 geometry reproduced operation by operation:
//   x = linspace(size/2, -size/2, N) along columns, y = linspace(-size/2, size/2, N) along rows,
//       each evaluated like numpy (float64 i*step + start, last point = stop, then cast to float32);
//   element (r, c) centroid = float32 np.mean of its 4 points: ((p0 + p1) + p2) + p3, then / 4;
//   phase 1 inside the circle x^2 + y^2 < 0.5^2 (shape 0) or the square |x|, |y| < 0.5 (shape 1);
//   node (r, c) quadrants e1 = element (r-1, c), e2 = (r-1, c-1), e3 = (r, c-1), e4 = (r, c);
//   pattern id = the reference's ref_pattern_dict entry of [e1, e2, e3, e4]; boundary nodes 0.
// Every floating-point operation is an explicitly rounded intrinsic (no contraction), so the map is
// bit-identical to the reference's (tests/test_gpu_setup.py against feanet_amd.mesh_setup, which
// tests/test_setup.py pins to the reference's own maps).
#include "fea_common.h"

namespace fea {

// bits e1 + 2 e2 + 4 e3 + 8 e4 -> pattern id (inverse of FEANet/mesh.py:23-26)
__constant__ uint8_t kBitsToId[16] = {0, 4, 5, 7, 3, 11, 8, 12, 2, 9, 10, 13, 6, 15, 14, 1};

__device__ __forceinline__ float lin(int i, int N, double start, double stop) {
  if (i == N - 1) return (float)stop;
  const double step = __ddiv_rn(stop - start, (double)(N - 1));
  return (float)__dadd_rn(__dmul_rn((double)i, step), start);
}

// phase of element (er, ec): rows er, er+1 and columns ec, ec+1 of the node grid
__device__ __forceinline__ int elem_phase(int er, int ec, int N, double half, int shape) {
  const float x0 = lin(ec, N, half, -half), x1 = lin(ec + 1, N, half, -half);
  const float y0 = lin(er, N, -half, half), y1 = lin(er + 1, N, -half, half);
  // element points in the reference's cell order: (er,ec), (er,ec+1), (er+1,ec+1), (er+1,ec)
  const float cx = __fdiv_rn(__fadd_rn(__fadd_rn(__fadd_rn(x0, x1), x1), x0), 4.0f);
  const float cy = __fdiv_rn(__fadd_rn(__fadd_rn(__fadd_rn(y0, y0), y1), y1), 4.0f);
  if (shape == 0) {
    const float dx = __fsub_rn(cx, 0.0f), dy = __fsub_rn(cy, 0.0f);
    return __fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)) < 0.25f ? 1 : 0;
  }
  return (fabsf(__fsub_rn(cx, 0.0f)) < 0.5f && fabsf(__fsub_rn(cy, 0.0f)) < 0.5f) ? 1 : 0;
}

__global__ __launch_bounds__(256) void k_interface_pattern_map(uint8_t* __restrict__ out, long long ld, int N,
                                                               int shape, double half) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x, r = blockIdx.y;
  if (c >= N || r >= N) return;
  uint8_t p = 0;
  if (r >= 1 && r <= N - 2 && c >= 1 && c <= N - 2) {
    const int e1 = elem_phase(r - 1, c, N, half, shape), e2 = elem_phase(r - 1, c - 1, N, half, shape);
    const int e3 = elem_phase(r, c - 1, N, half, shape), e4 = elem_phase(r, c, N, half, shape);
    p = kBitsToId[e1 + 2 * e2 + 4 * e3 + 8 * e4];
  }
  out[(long long)r * ld + c] = p;
}

}  // namespace fea

using namespace fea;

extern "C" int fea_interface_pattern_map(uint8_t* out, long long ld, int N, int shape, double size, void* stream) {
  if (!out || N < 2 || N > (1 << 20) + 1 || ld < N || (shape != 0 && shape != 1) || !(size > 0)) return FEA_EINVAL;
  k_interface_pattern_map<<<dim3((N + 255) / 256, N), 256, 0, (hipStream_t)stream>>>(out, ld, N, shape, size / 2);
  FEA_LAUNCH_CHECK();
}
