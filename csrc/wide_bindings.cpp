// Torch op registrations of the wide BiLSTM cell kernels (csrc/kernels/lstm_wide.hip).
// Both ops update their output tensors in place (the per-step driver loop lives in ops/wide.py).
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>
#include <torch/library.h>

#include "ina_launch.h"

namespace {

using at::Tensor;

void chk(const Tensor& t, const char* name, at::ScalarType dt, int64_t numel) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "ina.lstm_wide: ", name, " must be a contiguous GPU tensor");
  TORCH_CHECK(t.scalar_type() == dt, "ina.lstm_wide: ", name, " has dtype ", t.scalar_type(), ", expected ", dt);
  TORCH_CHECK(t.numel() == numel, "ina.lstm_wide: ", name, " has ", t.numel(), " elements, expected ", numel);
}
uint32_t salt_of(int64_t seed, int64_t d) {
  return (uint32_t)((uint32_t)(seed & 0x7FFFFFFF) * 0x2545F491u + (uint32_t)d * 0x3C6EF372u + 0x1234567u);
}
void fill_drop(ina::LstmWideArgs& a, int64_t seed, double keep_prob) {
  a.salt0 = salt_of(seed, 0);
  a.salt1 = salt_of(seed, 1);
  const double t = keep_prob * 4294967296.0;
  a.thr = t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
  a.inv_kp = (float)(1.0 / keep_prob);
  a.drop = keep_prob < 1.0 ? 1 : 0;
}

void lstm_wide_fwd_step(const Tensor& gx, const Tensor& gh, const Tensor& c, const Tensor& hcur, const Tensor& hall,
                        const Tensor& call, const Tensor& acts, const Tensor& hout, int64_t tau, int64_t seed,
                        double keep_prob) {
  TORCH_CHECK(gx.dim() == 4 && gx.size(0) == 2, "ina.lstm_wide_fwd_step: gx must be [2, S, L, 4U]");
  const int64_t S = gx.size(1), L = gx.size(2), U = gx.size(3) / 4;
  TORCH_CHECK(tau >= 0 && tau < L, "ina.lstm_wide_fwd_step: step out of range");
  chk(gx, "gx", at::kFloat, 2 * S * L * 4 * U);
  chk(gh, "gh", at::kFloat, 2 * S * 4 * U);
  chk(c, "c", at::kFloat, 2 * S * U);
  chk(hcur, "hcur", at::kBFloat16, 2 * S * U);
  chk(hall, "hall", at::kBFloat16, 2 * S * L * U);
  const bool keep = call.numel() > 0;
  if (keep) {
    chk(call, "call", at::kFloat, 2 * S * L * U);
    chk(acts, "acts", at::kBFloat16, 2 * S * L * 4 * U);
  }
  chk(hout, "hout", at::kBFloat16, S * L * 2 * U);
  ina::LstmWideArgs a{};
  a.S = (int)S;
  a.L = (int)L;
  a.U = (int)U;
  a.gx = gx.data_ptr<float>();
  a.gh = gh.data_ptr<float>();
  a.c = c.data_ptr<float>();
  a.hcur = hcur.data_ptr();
  a.hall = hall.data_ptr();
  a.call = keep ? call.data_ptr<float>() : nullptr;
  a.acts = keep ? acts.data_ptr() : nullptr;
  a.hout = hout.data_ptr();
  fill_drop(a, seed, keep_prob);
  TORCH_CHECK(ina::lstm_wide_fwd_step(a, (int)tau, c10::hip::getCurrentHIPStream().stream()) == 0,
              "ina.lstm_wide_fwd_step: launch failed");
}

void lstm_wide_bwd_step(const Tensor& dH, const Tensor& dhrec, const Tensor& dcrec, const Tensor& call,
                        const Tensor& acts, const Tensor& dG, const Tensor& dGcur, int64_t tau, int64_t seed,
                        double keep_prob) {
  TORCH_CHECK(acts.dim() == 4 && acts.size(0) == 2, "ina.lstm_wide_bwd_step: acts must be [2, S, L, 4U]");
  const int64_t S = acts.size(1), L = acts.size(2), U = acts.size(3) / 4;
  TORCH_CHECK(tau >= 0 && tau < L, "ina.lstm_wide_bwd_step: step out of range");
  chk(dH, "dH", at::kBFloat16, S * L * 2 * U);
  chk(dhrec, "dhrec", at::kFloat, 2 * S * U);
  chk(dcrec, "dcrec", at::kFloat, 2 * S * U);
  chk(call, "call", at::kFloat, 2 * S * L * U);
  chk(acts, "acts", at::kBFloat16, 2 * S * L * 4 * U);
  chk(dG, "dG", at::kBFloat16, 2 * S * L * 4 * U);
  if (dGcur.numel() > 0) chk(dGcur, "dGcur", at::kBFloat16, 2 * S * 4 * U);   // empty: not written
  ina::LstmWideArgs a{};
  a.S = (int)S;
  a.L = (int)L;
  a.U = (int)U;
  a.dH = dH.data_ptr();
  a.dhrec = dhrec.data_ptr<float>();
  a.dcrec = dcrec.data_ptr<float>();
  a.call = call.data_ptr<float>();
  a.acts = acts.data_ptr();
  a.dG = dG.data_ptr();
  a.dGcur = dGcur.numel() > 0 ? dGcur.data_ptr() : nullptr;
  fill_drop(a, seed, keep_prob);
  TORCH_CHECK(ina::lstm_wide_bwd_step(a, (int)tau, c10::hip::getCurrentHIPStream().stream()) == 0,
              "ina.lstm_wide_bwd_step: launch failed");
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(ina, m) {
  m.def("lstm_wide_fwd_step", &lstm_wide_fwd_step);
  m.def("lstm_wide_bwd_step", &lstm_wide_bwd_step);
}
