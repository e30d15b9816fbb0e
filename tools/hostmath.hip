// The library's transcendental restatements (aon_common.hpp: exp_sleef, exp_cr, sincos_cr)
// compiled for the HOST from the same source, so tests/test_transcendentals.py can pin them
// against torch's CPU results without a GPU.  Not part of the library.
#include "../articulated-object-nerf_amd/csrc/aon_common.hpp"

extern "C" {
// torch.sigmoid's form: 1 / (1 + exp(-x)) with SLEEF's exp
void aonh_sigmoid(const float* x, float* y, long n) {
  for (long i = 0; i < n; ++i) y[i] = 1.0f / (1.0f + aon::exp_sleef(-x[i]));
}
void aonh_exp_sleef(const float* x, float* y, long n) {
  for (long i = 0; i < n; ++i) y[i] = aon::exp_sleef(x[i]);
}
void aonh_exp_cr(const float* x, float* y, long n) {
  for (long i = 0; i < n; ++i) y[i] = aon::exp_cr(x[i]);
}
// qoff 0: sin, 1: cos (arguments below aon::kSinCrMax)
void aonh_sincos(const float* x, float* y, long n, int qoff) {
  for (long i = 0; i < n; ++i) y[i] = aon::sincos_cr(x[i], qoff);
}
}
