// The loss pass of the native CPU MLP-VAE step (cpu_mlp.cpp), in its own
// translation unit: it is the one loop that wants -ffast-math (glibc libmvec
// exp/log, a vectorised float reduction); the rest of the step, Adam in
// particular, keeps IEEE semantics.
#include <cmath>
#include <cstdint>

namespace mdt {

// sum over j of the reference's clamped BCE (F.binary_cross_entropy on
// sigmoid(t): -log clamped at 100) and t[j] <- sigmoid(t[j]) - x[j] (dlogits),
// branch-free, one exp and one log per element
float bce_dlogits_row(float* t, const float* x, int64_t n) {
  float rs = 0.f;
  for (int64_t j = 0; j < n; ++j) {
    const float tv = t[j], xv = x[j];
    const float e = std::exp(-std::fabs(tv));
    const float sp = std::fmax(tv, 0.f) + std::log(1.f + e);  // -log(1-p), stable
    const float sn = sp - tv;                                 // -log p
    rs += xv * std::fmin(sn, 100.f) + (1.f - xv) * std::fmin(sp, 100.f);
    const float inv = 1.f / (1.f + e);
    t[j] = (tv >= 0.f ? inv : e * inv) - xv;
  }
  return rs;
}

}  // namespace mdt
