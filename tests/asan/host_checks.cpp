// AddressSanitizer host build of the C ABI (tests/test_asan_host.py): every host-side path that runs
// without a GPU — layout and workspace queries, LDS sizing, and the argument checks every launcher
// performs before it touches the device (null pointers, impossible shapes, oversized tiles) — under
// -fsanitize=address on the host code (the kernels are not launched: this image has no GPU).
#include <stdio.h>
#include <stdlib.h>

#include "feanet_hip.h"

static int fails = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++fails;                                                     \
    }                                                              \
  } while (0)

int main() {
  CHECK(fea_abi_version() >= 3);
  // framed layout: aligned rows, ghost ring, every size class
  for (int H : {3, 5, 65, 1025, 4097, 8193})
    for (int W : {3, 9, 129, 4097}) {
      int ld = 0;
      long long bs = 0;
      CHECK(fea_mg_layout(H, W, 8, &ld, &bs) == 0 && ld % 16 == 0 && ld >= W + 16 && bs == (long long)(H + 2) * ld);
      CHECK(fea_mg_layout(H, W, 4, &ld, &bs) == 0 && ld % 32 == 0 && bs == (long long)(H + 2) * ld);
    }
  int ld = 0;
  long long bs = 0;
  CHECK(fea_mg_layout(2, 100, 8, &ld, &bs) != 0);
  CHECK(fea_mg_layout(100, 100, 2, &ld, &bs) != 0);
  CHECK(fea_mg_layout(100, 100, 8, nullptr, &bs) != 0);
  CHECK(fea_norm_workspace_bytes(2, 4097, 4097) >= (size_t)2 * 65 * 129 * 8);
  CHECK(fea_norm_workspace_bytes(0, 5, 5) == 0);
  CHECK(fea_mg_join_norm_parts(1, 4097, 4097, 8) > 0);
  CHECK(fea_mg_join_norm_parts(1, 4096, 4097, 8) < 0);
  // LDS sizing of the coarse tail and the multi-level launches
  CHECK(fea_mg_coarse_tail_lds_bytes(65, 65, 6, 8, 0) > 0);
  CHECK(fea_mg_coarse_tail_lds_bytes(65, 65, 9, 8, 0) == 0);
  CHECK(fea_mg_coarse_tail_lds_bytes(2, 65, 3, 8, 0) == 0);
  CHECK(fea_mg_mid_lds_bytes(0, 3, 4, 4, 8, 0) > 0);
  CHECK(fea_mg_mid_lds_bytes(1, 3, 32, 32, 8, 0) > 0);
  CHECK(fea_mg_mid_lds_bytes(0, 3, 64, 64, 8, 0) < 0);  // a region row must fit one wave
  CHECK(fea_mg_mid_lds_bytes(0, 5, 4, 4, 8, 0) < 0);
  CHECK(fea_stencil_weight_grad_ws_bytes_f64(2, 3, 65, 65) > 0);
  CHECK(fea_transfer_weight_grad_ws_bytes_f32(16, 2, 33, 33) > 0);
  // launchers reject bad arguments before any device call
  double d[16] = {0};
  const double* fl[5] = {d, d, d, d, d};
  CHECK(fea_knet_apply_f64(nullptr, d, nullptr, d, 1, 1, 5, 5, nullptr) != 0);
    CHECK(fea_mg_sweep_f64(d, nullptr, d, nullptr, d, d, 1, 1, 5, 5, 32, 7 * 32, nullptr) != 0);
  CHECK(fea_mg_coarse_tail_f64(nullptr, d, 65, 65, 6, 96, 96 * 67, nullptr, d, d, 1, d, d, 1.0, 1.0, 1, 1, 0, 1,
                               nullptr) != 0);
  CHECK(fea_mg_coarse_tail_f64(d, d, 64, 64, 6, 96, 96 * 67, nullptr, d, d, 1, d, d, 1.0, 1.0, 1, 1, 0, 1,
                               nullptr) != 0);  // 63 intervals do not coarsen
  CHECK(fea_mg_mid_down_f64(fl, nullptr, 0, 1, 513, 513, d, d, 1, d, 1, 1.0, 4, 4, nullptr) != 0);
  CHECK(fea_mg_mid_down_f64(fl, nullptr, 3, 1, 513, 513, d, d, 1, d, 1, 1.0, 64, 64, nullptr) != 0);
  CHECK(fea_mg_mid_up_f64(fl, d, d, nullptr, 3, 1, 513, 513, d, d, 1, d, 1, 1.0, 32, 32, nullptr) != 0);  // e == out
  CHECK(fea_interface_pattern_map(nullptr, 16, 5, 0, 0.5, nullptr) != 0);
  if (fails) return 1;
  printf("asan host checks ok\n");
  return 0;
}
