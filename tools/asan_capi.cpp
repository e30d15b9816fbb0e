// Host-side AddressSanitizer driver for the C ABI (the "-fsanitize=address
// debug build" of the host code).  Built by `make asan` (csrc/Makefile) against
// lib/asan/libaonerf_asan.so, whose host code -- argument validation, size queries, the error
// plumbing, packing tables -- is compiled with -fsanitize=address (host-only objects: no device
// code, so nothing here may launch a kernel).  Every call below must fail argument validation
// BEFORE touching the GPU and report it through aon_last_error(); ASan aborts the process on
// any out-of-bounds or use-after-free on the way.
#include <cstdio>
#include <cstring>

#include "aonerf.h"

static int failures = 0;

static void expect_invalid(int rc, const char* what) {
  const char* msg = aon_last_error();
  if (rc >= 0 || !msg || !msg[0]) {
    std::printf("FAIL %s: rc=%d msg=%s\n", what, rc, msg ? msg : "(null)");
    ++failures;
  } else {
    std::printf("ok   %s -> %s\n", what, msg);
  }
}

int main() {
  if (aon_abi_version() != AON_ABI_VERSION) {
    std::printf("FAIL abi version\n");
    return 1;
  }
  float c2w[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 4};
  float dummy[16];
  void* p = dummy;
  expect_invalid(aon_ray_directions(0, 4, 1.f, dummy, nullptr), "ray_directions H=0");
  expect_invalid(aon_get_rays(nullptr, 4, c2w, dummy, dummy, nullptr, 0, 0, nullptr, nullptr),
                 "get_rays null dirs");
  expect_invalid(aon_get_rays(dummy, 4, c2w, dummy, dummy, nullptr, 2, 2, dummy, nullptr),
                 "get_rays radii H=2");
  expect_invalid(aon_frame_rays(4, 4, 1.f, nullptr, 0, 16, dummy, dummy, nullptr, nullptr),
                 "frame_rays null c2w");
  expect_invalid(aon_sample_pdf(nullptr, 0, dummy, 4, 4, 1000, 128, dummy, 0, nullptr, 0, nullptr,
                                nullptr, dummy, nullptr, nullptr),
                 "sample_pdf nb > 256");
  expect_invalid(aon_composite_march(dummy + 1, dummy, dummy, 4, 65, 1, 0, dummy, 0, 128, dummy,
                                     dummy, nullptr, dummy, dummy, nullptr),
                 "composite_march misaligned raw");
  expect_invalid(aon_composite_march(dummy, dummy, dummy, 4, 300, 1, 0, dummy, 0, 128, dummy,
                                     dummy, nullptr, dummy, dummy, nullptr),
                 "composite_march S > 256");
  expect_invalid(aon_composite_fwd(dummy, 2, dummy, 1, dummy, dummy, 4, 8, 1, 0, dummy, dummy,
                                   nullptr, dummy, nullptr),
                 "composite_fwd rgb_stride < 3");
  expect_invalid(aon_mlp_pack(nullptr, AON_PREC_F16X3, p, nullptr), "mlp_pack null params");
  aon_mlp_params prm;
  std::memset(&prm, 0, sizeof(prm));
  expect_invalid(aon_mlp_pack(&prm, 7, p, nullptr), "mlp_pack bad precision");
  expect_invalid(aon_mlp_pack(&prm, AON_PREC_F16X3, p, nullptr), "mlp_pack no shapes");
  // the default geometry's shapes (ABI 9), null tensors: refused by the null check, no launch
  const int64_t shp[12][2] = {{256, 63},  {256, 256}, {256, 256}, {256, 256}, {256, 256}, {256, 319},
                              {256, 256}, {256, 256}, {1, 256},   {256, 256}, {128, 283}, {3, 128}};
  for (int i = 0; i < 12; ++i) {
    prm.w_rows[i] = shp[i][0];
    prm.w_cols[i] = shp[i][1];
    prm.b_len[i] = shp[i][0];
  }
  expect_invalid(aon_mlp_pack(&prm, AON_PREC_F16X3, p, nullptr), "mlp_pack null layer");
  // registration order (views_linear.0 in the density slot): refused by the shape check
  prm.w_rows[8] = 128;
  prm.w_cols[8] = 283;
  prm.b_len[8] = 128;
  expect_invalid(aon_mlp_pack(&prm, AON_PREC_F16X3, p, nullptr), "mlp_pack registration order");
  expect_invalid(aon_mlp_bwd_pack(&prm, p, nullptr), "mlp_bwd_pack registration order");
  aon_mlp_art_params aprm;
  std::memset(&aprm, 0, sizeof(aprm));
  expect_invalid(aon_mlp_art_pack(&aprm, p, nullptr), "mlp_art_pack no shapes");
  expect_invalid(aon_mlp_art_bwd_pack(&aprm, p, nullptr), "mlp_art_bwd_pack no shapes");
  uint32_t st = 0;
  expect_invalid(aon_mlp_read_status(p, 3, &st, nullptr), "read_status bad size");
  aon_gemm_args g;
  std::memset(&g, 0, sizeof(g));
  g.M = g.N = g.K = 16;
  g.A = g.B = dummy;
  g.C = dummy;
  g.lda = g.ldb = 16;
  g.a_kc = g.b_kc = 1;
  g.ldc = 8;  // < N
  g.a_scale = g.b_scale = 1.f;
  expect_invalid(aon_gemm(&g, nullptr, 0, nullptr), "gemm ldc < N");
  g.ldc = 16;
  g.a_scale = 0.f;
  expect_invalid(aon_gemm(&g, nullptr, 0, nullptr), "gemm zero scale");
  aon_adam_tensor t;
  std::memset(&t, 0, sizeof(t));
  expect_invalid(aon_adam_step(&t, 0, 1e-3, 0.9, 0.999, 1e-8, 1, nullptr), "adam count 0");
  // size queries: pure host arithmetic
  if (aon_mlp_packed_bytes(AON_PREC_F16X3) == 0 || aon_mlp_bwd_packed_bytes() == 0 ||
      aon_mlp_art_packed_bytes() == 0 || aon_colsum_workspace_bytes(1024, 256) == 0) {
    std::printf("FAIL size queries\n");
    ++failures;
  }
  std::printf("%s: %d failures\n", failures ? "FAILED" : "ASAN_CAPI_OK", failures);
  return failures ? 1 : 0;
}
