// Torch op registrations of the wide BiLSTM cell kernels (csrc/kernels/lstm_wide.hip).
// Both ops update their output tensors in place (the per-step driver loop lives in ops/wide.py).
#include <cstdlib>
#include <algorithm>

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

// ---- persistent wide BiLSTM (one launch per pass; lstm_wide.hip lstm_wide_seq_*)
static int64_t wide_seq_pad(int64_t S) { return (S + 31) / 32 * 32; }
int64_t wide_up(int64_t U) { return (U + 31) / 32 * 32; }

// gx [S*L, 2 * 4UP] bf16 (x W_x of both directions, permuted + pre-scaled gate columns), bx [2, 4UP] fp32 biases, apk =
// pack_lstm_wide's forward fragments -> (hout [S, L, 2U] bf16, hprev [2, S, L, UP] bf16,
// acts [2, Sp*L, 4UP] bf16, cst [2, Sp*L, UP] fp16: tile-major, Sp = S rounded up to 32);
// the last three only when stash (training), else empty
// hdst (optional, stash only): the x rows [S*L, W] whose columns hcol .. hcol + 2 UP take the h_{t-1} stash (direction
// d at hcol + d UP), so one weight-gradient GEMM covers x and both directions' h; then hprev is returned empty
std::tuple<Tensor, Tensor, Tensor, Tensor> lstm_wide_seq_fwd(const Tensor& gx, const Tensor& bx, const Tensor& apk,
                                                             int64_t S, int64_t L, int64_t U, bool stash, int64_t seed,
                                                             double keep_prob, const Tensor& hdst, int64_t hcol) {
  TORCH_CHECK(ina::lstm_wide_seq_supported((int)U), "ina.lstm_wide_seq_fwd: U must be 64, 100 or 128");
  const int64_t UP = wide_up(U), G4 = 4 * UP, NW = UP / 16;
  chk(gx, "gx", at::kBFloat16, 2 * S * L * G4);
  chk(bx, "bx", at::kFloat, 2 * G4);
  chk(apk, "apk", at::kBFloat16, 2 * NW * 4 * (UP / 32) * 64 * 8);
  TORCH_CHECK(S * L * G4 < (1LL << 31) * 2, "ina.lstm_wide_seq_fwd: batch too large");
  auto bopt = gx.options().dtype(at::kBFloat16), hopt = gx.options().dtype(at::kHalf);
  auto hout = at::empty({S, L, 2 * U}, bopt);
  const bool into_x = stash && hdst.numel() > 0;
  if (into_x) {
    TORCH_CHECK(hdst.is_cuda() && hdst.is_contiguous() && hdst.scalar_type() == at::kBFloat16 && hdst.dim() == 2 &&
                    hdst.size(0) == S * L && hcol >= 0 && hcol % 8 == 0 && hcol + 2 * UP <= hdst.size(1) &&
                    hdst.size(1) % 8 == 0,
                "ina.lstm_wide_seq_fwd: hdst must be contiguous bf16 [S*L, W] with room for 2 UP columns at hcol");
    TORCH_CHECK(S * L * hdst.size(1) < (1LL << 31) * 2, "ina.lstm_wide_seq_fwd: hdst too large");
  }
  auto hprev = stash && !into_x ? at::empty({2, S, L, UP}, bopt) : at::empty({0}, bopt);
  const int64_t Sp = wide_seq_pad(S);   // tile-major stash: whole 32-sequence tiles
  auto acts = stash ? at::empty({2, Sp * L, G4}, bopt) : at::empty({0}, bopt);
  auto cst = stash ? at::empty({2, Sp * L, UP}, hopt) : at::empty({0}, hopt);
  if (S == 0) return {hout, hprev, acts, cst};
  ina::WideSeqArgs a{};
  a.S = (int)S;
  a.L = (int)L;
  a.U = (int)U;
  a.gx = gx.data_ptr();
  a.bx = bx.data_ptr<float>();
  a.apk = apk.data_ptr();
  a.hprev = !stash ? nullptr : into_x ? (void*)((unsigned short*)hdst.data_ptr() + hcol) : hprev.data_ptr();
  a.hld = into_x ? (int)hdst.size(1) : (int)UP;
  a.hdo = into_x ? (long)UP : (long)(S * L * UP);
  a.acts = stash ? acts.data_ptr() : nullptr;
  a.cst = stash ? cst.data_ptr() : nullptr;
  a.hout = hout.data_ptr();
  a.stash = stash ? 1 : 0;
  ina::LstmWideArgs d{};
  fill_drop(d, seed, keep_prob);
  a.salt0 = d.salt0;
  a.salt1 = d.salt1;
  a.thr = d.thr;
  a.inv_kp = d.inv_kp;
  a.drop = d.drop;
  TORCH_CHECK(ina::lstm_wide_seq_fwd(a, c10::hip::getCurrentHIPStream().stream()) == 0,
              "ina.lstm_wide_seq_fwd: launch failed");
  return {hout, hprev, acts, cst};
}

// dH [S, L, 2U] bf16 (gradient w.r.t. hout) + the forward's stash -> dG [S*L, 2 * 4UP] bf16 (both directions, permuted
// columns) and, with wpk ([2][4UP/32][64][8] bf16 W_pos^T fragments, ops/wide.py::pos_frags; empty: none), the
// input gradient's np position columns per direction dxp [2, S*L, np] fp32
std::tuple<Tensor, Tensor> lstm_wide_seq_bwd(const Tensor& dH, const Tensor& acts, const Tensor& cst, const Tensor& a2pk,
                                             int64_t S, int64_t L, int64_t U, int64_t seed, double keep_prob,
                                             const Tensor& wpk, int64_t np) {
  TORCH_CHECK(ina::lstm_wide_seq_supported((int)U), "ina.lstm_wide_seq_bwd: U must be 64, 100 or 128");
  const int64_t UP = wide_up(U), G4 = 4 * UP, NW = UP / 16;
  chk(dH, "dH", at::kBFloat16, S * L * 2 * U);
  chk(acts, "acts", at::kBFloat16, 2 * wide_seq_pad(S) * L * G4);
  chk(cst, "cst", at::kHalf, 2 * wide_seq_pad(S) * L * UP);
  chk(a2pk, "a2pk", at::kBFloat16, 2 * NW * (G4 / 32) * 64 * 8);
  auto dG = at::empty({S * L, 2 * G4}, dH.options());
  const bool pg = wpk.numel() > 0;
  if (pg) {
    chk(wpk, "wpk", at::kBFloat16, 2 * (G4 / 32) * 64 * 8);
    TORCH_CHECK(np >= 1 && np <= 16, "ina.lstm_wide_seq_bwd: 1 <= np <= 16 position columns");
  }
  auto dxp = at::empty({pg ? 2 : 0, S * L, pg ? np : 0}, dH.options().dtype(at::kFloat));
  if (S == 0) return {dG, dxp};
  ina::WideSeqArgs a{};
  a.S = (int)S;
  a.L = (int)L;
  a.U = (int)U;
  a.dH = dH.data_ptr();
  a.acts = acts.data_ptr();
  a.cst = cst.data_ptr();
  a.a2pk = a2pk.data_ptr();
  a.dG = dG.data_ptr();
  a.wpk = pg ? wpk.data_ptr() : nullptr;
  a.dxp = pg ? dxp.data_ptr<float>() : nullptr;
  a.np = pg ? (int)np : 0;
  ina::LstmWideArgs d{};
  fill_drop(d, seed, keep_prob);
  a.salt0 = d.salt0;
  a.salt1 = d.salt1;
  a.thr = d.thr;
  a.inv_kp = d.inv_kp;
  a.drop = d.drop;
  TORCH_CHECK(ina::lstm_wide_seq_bwd(a, c10::hip::getCurrentHIPStream().stream()) == 0,
              "ina.lstm_wide_seq_bwd: launch failed");
  return {dG, dxp};
}

bool lstm_wide_seq_ok(int64_t U) { return ina::lstm_wide_seq_supported((int)U); }

void chk_ids(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.scalar_type() == at::kInt, "ina.wide: ", name,
              " must be a contiguous int32 GPU tensor");
}

// Xb [S*L, E + 2PD] bf16 = [word row ; pos1 row ; pos2 row] of every token of the rows inst
// extra: columns appended to each row after the DP gathered ones (not written here: the BiLSTM forward's h_{t-1}
// stash, lstm_wide_seq_fwd hdst)
Tensor wide_x_gather(const Tensor& inst, const Tensor& word, const Tensor& pos1, const Tensor& pos2,
                     const Tensor& wemb, const Tensor& p1emb, const Tensor& p2emb, int64_t extra) {
  chk_ids(inst, "inst");
  chk_ids(word, "word");
  chk_ids(pos1, "pos1");
  chk_ids(pos2, "pos2");
  const bool wb = wemb.scalar_type() == at::kBFloat16;   // cached bf16 copy of a frozen word table
  chk(wemb, "wemb", wb ? at::kBFloat16 : at::kFloat, wemb.numel());
  chk(p1emb, "p1emb", at::kFloat, p1emb.numel());
  chk(p2emb, "p2emb", at::kFloat, p2emb.numel());
  const int64_t S = inst.size(0), L = word.size(1), E = wemb.size(1), PD = p1emb.size(1);
  TORCH_CHECK(pos1.sizes() == word.sizes() && pos2.sizes() == word.sizes() && p2emb.size(1) == PD,
              "ina.wide_x_gather: shapes");
  const int64_t DP = (E + 2 * PD + 1 + 31) / 32 * 32;   // + the ones column, K padded to 32 (packing.wide_x_cols)
  TORCH_CHECK(extra >= 0 && extra % 8 == 0, "ina.wide_x_gather: extra columns must be a multiple of 8");
  auto xb = at::empty({S * L, DP + extra}, p1emb.options().dtype(at::kBFloat16));
  TORCH_CHECK(ina::wide_x_gather(inst.data_ptr<int>(), (int)S, (int)L, word.data_ptr<int>(), pos1.data_ptr<int>(),
                                 pos2.data_ptr<int>(), wemb.data_ptr(), wb, (int)E, p1emb.data_ptr<float>(),
                                 p2emb.data_ptr<float>(), (int)PD, (int)DP, xb.data_ptr(), (int)(DP + extra),
                                 c10::hip::getCurrentHIPStream().stream()) == 0,
              "ina.wide_x_gather: launch failed");
  return xb;
}

// position-table gradients [2, P2, PD] from dX's position columns dxp [S*L, 2PD] or [2, S*L, 2PD] (the two
// directions' parts, summed) fp32 (shifted-arange ids)
Tensor wide_pos_grad(const Tensor& dxp, const Tensor& inst, const Tensor& pos1, const Tensor& pos2, int64_t P2) {
  chk_ids(inst, "inst");
  chk_ids(pos1, "pos1");
  chk_ids(pos2, "pos2");
  TORCH_CHECK(dxp.dim() == 2 || (dxp.dim() == 3 && dxp.size(0) == 2), "ina.wide_pos_grad: dxp [S*L, 2PD] or [2, S*L, 2PD]");
  const int64_t planes = dxp.dim() == 3 ? 2 : 1;
  const int64_t S = inst.size(0), L = pos1.size(1), PD = dxp.size(-1) / 2;
  chk(dxp, "dxp", at::kFloat, planes * S * L * 2 * PD);
  // sequence chunks (grid.y), cap 1024 (75 -> 45 us vs 256 at the paper configuration, profiles/r5_posc).  The cap
  // sets the partial sums' order, so it is a compile-time constant (A/B builds: -DINA_POSG_CHUNKS=n), not an
  // environment knob that would make two runs' gradients differ bitwise
#ifndef INA_POSG_CHUNKS
#define INA_POSG_CHUNKS 1024
#endif
  constexpr int64_t cap = INA_POSG_CHUNKS;
  const int64_t chunks = std::max<int64_t>(1, std::min<int64_t>(std::max<int64_t>(cap, 1), S / 16));
  auto part = at::empty({chunks, 2, P2, PD}, dxp.options());
  if (S == 0) return part.sum(0);
  TORCH_CHECK(ina::wide_pos_grad(dxp.data_ptr<float>(), inst.data_ptr<int>(), pos1.data_ptr<int>(), pos2.data_ptr<int>(),
                                 (int)S, (int)L, (int)PD, (int)P2, (int)chunks, (int)planes, part.data_ptr<float>(),
                                 c10::hip::getCurrentHIPStream().stream()) == 0,
              "ina.wide_pos_grad: launch failed");
  return part.sum(0);
}

}  // namespace

// ---- fused self-attention pooling over the wide BiLSTM output (attn_wide.hip)
static ina::WideAttnArgs attn_args(const Tensor& hin, const Tensor& inst, const Tensor& mask, const Tensor& w1t,
                                   const Tensor& b1, const Tensor& w2) {
  TORCH_CHECK(hin.dim() == 3, "ina.wide_attn: hin must be [S, L, H]");
  const int64_t S = hin.size(0), L = hin.size(1), H = hin.size(2), HP = ina::wide_attn_hp((int)H);
  TORCH_CHECK(HP > 0, "ina.wide_attn: H must be 128, 200 or 256");
  TORCH_CHECK(L >= 1 && L <= 256, "ina.wide_attn: L must be in [1, 256]");
  chk(hin, "hin", at::kBFloat16, S * L * H);
  chk(inst, "inst", at::kInt, S);
  TORCH_CHECK(mask.dim() == 2 && mask.size(1) == L, "ina.wide_attn: mask must be [rows, L]");
  chk(mask, "mask", at::kInt, mask.numel());
  chk(w1t, "w1t", at::kBFloat16, HP * HP);
  chk(b1, "b1", at::kFloat, HP);
  chk(w2, "w2", at::kFloat, HP);
  TORCH_CHECK(S * L * H < (1LL << 31), "ina.wide_attn: batch too large");
  ina::WideAttnArgs a{};
  a.S = (int)S;
  a.L = (int)L;
  a.H = (int)H;
  a.SB = ina::wide_attn_sb((int)L);
  a.hin = hin.data_ptr();
  a.inst = inst.data_ptr<int>();
  a.mask = mask.data_ptr<int>();
  a.w1t = w1t.data_ptr();
  a.b1 = b1.data_ptr<float>();
  a.w2 = w2.data_ptr<float>();
  return a;
}

static int attn_grid(const ina::WideAttnArgs& a, bool bwd) {
  TORCH_CHECK(ina::wide_attn_smem(a.H, a.L, bwd) <= 160 * 1024, "ina.wide_attn: L too long for LDS");
  const int g = ina::wide_attn_grid(a.H, a.L, a.S, bwd);
  TORCH_CHECK(g >= 0, "ina.wide_attn: occupancy query failed");
  return g;
}

// hin [S, L, H] bf16 -> (e [S, H] fp32, alpha [S, L] fp32)
std::tuple<Tensor, Tensor> wide_attn_fwd(const Tensor& hin, const Tensor& inst, const Tensor& mask, const Tensor& w1t,
                                         const Tensor& b1, const Tensor& w2) {
  auto a = attn_args(hin, inst, mask, w1t, b1, w2);
  const int grid = attn_grid(a, false);
  auto fopt = hin.options().dtype(at::kFloat);
  auto e = at::empty({a.S, a.H}, fopt), alpha = at::empty({a.S, a.L}, fopt);
  a.e = e.data_ptr<float>();
  a.alpha = alpha.data_ptr<float>();
  if (a.S > 0)
    TORCH_CHECK(ina::wide_attn_fwd(a, grid, c10::hip::getCurrentHIPStream().stream()) == 0,
                "ina.wide_attn_fwd: launch failed");
  return {e, alpha};
}

// + alpha [S, L], de [S, H] fp32 -> (dH [S, L, H] bf16, dZ [S*L, H] bf16, part [blocks, 2, HP] fp32: dw2, db1)
std::tuple<Tensor, Tensor, Tensor> wide_attn_bwd(const Tensor& hin, const Tensor& inst, const Tensor& mask,
                                                 const Tensor& w1t, const Tensor& w1, const Tensor& b1,
                                                 const Tensor& w2, const Tensor& alpha, const Tensor& de) {
  auto a = attn_args(hin, inst, mask, w1t, b1, w2);
  const int grid = attn_grid(a, true);
  const int64_t HP = ina::wide_attn_hp(a.H);
  chk(w1, "w1", at::kBFloat16, HP * HP);
  chk(alpha, "alpha", at::kFloat, (int64_t)a.S * a.L);
  chk(de, "de", at::kFloat, (int64_t)a.S * a.H);
  auto dH = at::empty({a.S, a.L, a.H}, hin.options());
  auto dZ = at::empty({(int64_t)a.S * a.L, a.H}, hin.options());
  auto part = at::zeros({std::max(grid, 1), 2, HP}, hin.options().dtype(at::kFloat));
  a.w1 = w1.data_ptr();
  a.alpha = alpha.data_ptr<float>();
  a.de = de.data_ptr<float>();
  a.dH = dH.data_ptr();
  a.dZ = dZ.data_ptr();
  a.part = part.data_ptr<float>();
  if (a.S > 0)
    TORCH_CHECK(ina::wide_attn_bwd(a, grid, c10::hip::getCurrentHIPStream().stream()) == 0,
                "ina.wide_attn_bwd: launch failed");
  return {dH, dZ, part};
}

bool wide_attn_ok(int64_t H, int64_t L) {
  return ina::wide_attn_hp((int)H) > 0 && L >= 1 && L <= 256 &&
         ina::wide_attn_smem((int)H, (int)L, true) <= 160 * 1024;
}

// ---------------------------------------------------------------- wide head (head_wide.hip)
bool routing_wide_ok(int64_t K, int64_t H, int64_t R) { return ina::routing_wide_supported((int)K, (int)H, (int)R); }

// eh [items * K, H] fp32 -> (cls [items, H] fp32, cls_bf [items, H] bf16)
std::tuple<Tensor, Tensor> routing_wide_fwd(const Tensor& eh, int64_t items, int64_t K, int64_t R) {
  TORCH_CHECK(eh.dim() == 2, "ina.routing_wide_fwd: eh must be [items * K, H]");
  const int64_t H = eh.size(1);
  TORCH_CHECK(ina::routing_wide_supported((int)K, (int)H, (int)R), "ina.routing_wide_fwd: unsupported K/H/R");
  chk(eh, "eh", at::kFloat, items * K * H);
  auto cls = at::empty({items, H}, eh.options());
  auto cls_bf = at::empty({items, H}, eh.options().dtype(at::kBFloat16));
  TORCH_CHECK(ina::routing_wide_fwd(eh.data_ptr<float>(), (int)items, (int)K, (int)H, (int)R, cls.data_ptr<float>(),
                                    cls_bf.data_ptr(), c10::hip::getCurrentHIPStream().stream()) == 0,
              "ina.routing_wide_fwd: launch failed");
  return {cls, cls_bf};
}

// eh [items * K, H], dcls [items, H] fp32 -> deh [items * K, H] fp32
Tensor routing_wide_bwd(const Tensor& eh, const Tensor& dcls, int64_t items, int64_t K, int64_t R) {
  TORCH_CHECK(eh.dim() == 2, "ina.routing_wide_bwd: eh must be [items * K, H]");
  const int64_t H = eh.size(1);
  TORCH_CHECK(ina::routing_wide_supported((int)K, (int)H, (int)R), "ina.routing_wide_bwd: unsupported K/H/R");
  chk(eh, "eh", at::kFloat, items * K * H);
  chk(dcls, "dcls", at::kFloat, items * H);
  auto deh = at::empty_like(eh);
  TORCH_CHECK(ina::routing_wide_bwd(eh.data_ptr<float>(), dcls.data_ptr<float>(), (int)items, (int)K, (int)H, (int)R,
                                    deh.data_ptr<float>(), c10::hip::getCurrentHIPStream().stream()) == 0,
              "ina.routing_wide_bwd: launch failed");
  return deh;
}

bool ntn_wide_epi_ok(int64_t N, bool paper) { return ina::ntn_wide_epi_supported((int)N, paper); }

static void epi_check(const Tensor& T, int64_t N, int64_t h, const Tensor& w, bool paper, const char* op) {
  TORCH_CHECK(T.is_cuda() && T.is_contiguous() && T.scalar_type() == at::kFloat, op, ": T must be contiguous fp32");
  TORCH_CHECK(N >= 1 && h >= 1 && T.numel() % (N * h) == 0, op, ": T is not [rows, N*h]");
  TORCH_CHECK(ina::ntn_wide_epi_supported((int)N, paper), op, ": unsupported N for this head");
  chk(w, "w", at::kFloat, paper ? h : h * N * N);
}

// T [rows, N*h] fp32 (column c*h + s) -> probs [rows, N]
Tensor ntn_wide_epi_fwd(const Tensor& T, int64_t N, int64_t h, const Tensor& w, const Tensor& b, bool paper) {
  epi_check(T, N, h, w, paper, "ina.ntn_wide_epi_fwd");
  chk(b, "b", at::kFloat, paper ? 1 : N);
  const int64_t rows = T.numel() / (N * h);
  auto probs = at::empty({rows, N}, T.options());
  TORCH_CHECK(ina::ntn_wide_epi_fwd(T.data_ptr<float>(), (long)rows, (int)N, (int)h, w.data_ptr<float>(),
                                    b.data_ptr<float>(), paper, probs.data_ptr<float>(),
                                    c10::hip::getCurrentHIPStream().stream()) == 0,
              "ina.ntn_wide_epi_fwd: launch failed");
  return probs;
}

// T (in: pre-ReLU, out: ReLU(T)), dz [rows, N] fp32, g: [] or [1] upstream scale -> (dT [rows, N*h] bf16, dzs)
std::tuple<Tensor, Tensor> ntn_wide_epi_bwd(Tensor T, int64_t N, int64_t h, const Tensor& w, const Tensor& dz,
                                            const Tensor& g, bool paper) {
  epi_check(T, N, h, w, paper, "ina.ntn_wide_epi_bwd");
  const int64_t rows = T.numel() / (N * h);
  chk(dz, "dz", at::kFloat, rows * N);
  TORCH_CHECK(g.numel() == 0 || (g.numel() == 1 && g.is_cuda() && g.scalar_type() == at::kFloat),
              "ina.ntn_wide_epi_bwd: g must be empty or one fp32 GPU scalar");
  auto dT = at::empty({rows, N * h}, T.options().dtype(at::kBFloat16));
  auto dzs = at::empty({rows, N}, T.options());
  TORCH_CHECK(ina::ntn_wide_epi_bwd(T.data_ptr<float>(), (long)rows, (int)N, (int)h, w.data_ptr<float>(),
                                    dz.data_ptr<float>(), g.numel() ? g.data_ptr<float>() : nullptr, paper,
                                    dT.data_ptr(), dzs.data_ptr<float>(),
                                    c10::hip::getCurrentHIPStream().stream()) == 0,
              "ina.ntn_wide_epi_bwd: launch failed");
  return {dT, dzs};
}

TORCH_LIBRARY_FRAGMENT(ina, m) {
  m.def("routing_wide_ok", &routing_wide_ok);
  m.def("routing_wide_fwd", &routing_wide_fwd);
  m.def("routing_wide_bwd", &routing_wide_bwd);
  m.def("ntn_wide_epi_ok", &ntn_wide_epi_ok);
  m.def("ntn_wide_epi_fwd", &ntn_wide_epi_fwd);
  m.def("ntn_wide_epi_bwd", &ntn_wide_epi_bwd);
  m.def("lstm_wide_fwd_step", &lstm_wide_fwd_step);
  m.def("lstm_wide_bwd_step", &lstm_wide_bwd_step);
  m.def("lstm_wide_seq_fwd", &lstm_wide_seq_fwd);
  m.def("lstm_wide_seq_bwd", &lstm_wide_seq_bwd);
  m.def("lstm_wide_seq_ok", &lstm_wide_seq_ok);
  m.def("wide_x_gather", &wide_x_gather);
  m.def("wide_pos_grad", &wide_pos_grad);
  m.def("wide_attn_fwd", &wide_attn_fwd);
  m.def("wide_attn_bwd", &wide_attn_bwd);
  m.def("wide_attn_ok", &wide_attn_ok);
}
