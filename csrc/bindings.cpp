// Torch op registrations for the Induction-Network gfx950 kernels (namespace torch.ops.ina).
//
// Every op validates device / dtype / contiguity / shapes on the host BEFORE launching, so a shape
// that the kernel grid does not assume never reaches the GPU.  Launches go to the current HIP
// stream (capturable into hipGraphs by the caller).  No op has a CPU implementation: the CPU path
// of the framework is the pure-PyTorch oracle in models/reference.py.
#include <map>
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>
#include <torch/library.h>

#include <tuple>

#include "ina_launch.h"

namespace {

using at::Tensor;

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check_cuda(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "ina: ", name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), "ina: ", name, " must be contiguous");
}
void check(const Tensor& t, const char* name, at::ScalarType dt) {
  check_cuda(t, name);
  TORCH_CHECK(t.scalar_type() == dt, "ina: ", name, " has dtype ", t.scalar_type(), ", expected ", dt);
}
void check_launch(int rc, const char* what) {
  TORCH_CHECK(rc == 0, "ina: ", what, " launch failed / unsupported configuration (rc=", rc, ")");
}
const float* dev_float(const std::optional<Tensor>& t, const char* name) {
  if (!t.has_value() || !t->defined() || t->numel() == 0) return nullptr;
  check(*t, name, at::kFloat);
  return t->data_ptr<float>();
}
const int* dev_int(const std::optional<Tensor>& t, const char* name) {
  if (!t.has_value() || !t->defined() || t->numel() == 0) return nullptr;
  check(*t, name, at::kInt);
  return t->data_ptr<int>();
}

// the optimizer's device skip counter, required together with a guard flag
int* guard_skips(const std::optional<Tensor>& guard, const std::optional<Tensor>& skips) {
  if (!guard.has_value() || !guard->defined() || guard->numel() == 0) return nullptr;
  TORCH_CHECK(skips.has_value() && skips->defined() && skips->numel() >= 1, "ina: a guard flag needs a skip counter");
  check(*skips, "skips", at::kInt);
  return skips->data_ptr<int>();
}

// ragged-tile arrays (ops/encoder.py): int32 device vectors of an exact length, or absent
const int* ragged_arg(const std::optional<Tensor>& t, int64_t n, const char* name) {
  if (!t.has_value() || !t->defined() || t->numel() == 0) return nullptr;
  check(*t, name, at::kInt);
  TORCH_CHECK(t->numel() == n, "ina: ", name, " must have ", n, " elements, got ", t->numel());
  return t->data_ptr<int>();
}

int64_t frag_elems(bool bf16) { return bf16 ? 8 : 1; }
uint32_t keep_threshold(double kp) {
  const double t = kp * 4294967296.0;
  return t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
}


// ------------------------------------------------------------------ LSTM
// Returns (hlane, cst, hnat, dmask, xg): hlane = raw recurrent h and cst = cell states, both in the
// lane-native tile layout [ceil(S/16), 2, L, U/4, 64] (only when store_c: the backward needs them);
// hnat = the DropoutWrapper output in natural layout [S, L, 2U] (the attention input); dmask = the
// dropout keep bits; xg (bf16 mode) = the gathered encoder input [tiles][L][64][NX] followed by the
// position ids [tiles][L][16] (x_gather_kernel; an input of lstm_bwd).
static std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor> lstm_fwd_impl(
    const Tensor& inst, const Tensor& word, const Tensor& pos1, const Tensor& pos2, const Tensor& wemb,
    const Tensor& p1emb, const Tensor& p2emb, const Tensor& apack, const Tensor& bias, int64_t U, int64_t NX, bool bf16,
    bool store_c, int64_t seed, double keep_prob, const std::optional<Tensor>& seed_dev,
    const std::optional<Tensor>& wrows, bool natural, const std::optional<Tensor>& tlen = std::nullopt,
    const std::optional<Tensor>& slen = std::nullopt, const std::optional<Tensor>& perm = std::nullopt,
    bool direct_x = false) {
  check(inst, "inst", at::kInt);
  check(word, "word", at::kInt);
  check(pos1, "pos1", at::kInt);
  check(pos2, "pos2", at::kInt);
  check(wemb, "wemb", at::kFloat);
  check(p1emb, "p1emb", at::kFloat);
  check(p2emb, "p2emb", at::kFloat);
  check(bias, "bias", at::kFloat);
  check(apack, "apack", bf16 ? at::kBFloat16 : at::kFloat);
  TORCH_CHECK(ina::lstm_supported((int)U, (int)NX), "ina.lstm_fwd: unsupported (U, NX) = (", U, ", ", NX, ")");
  const int64_t S = inst.size(0), L = word.size(1), E = wemb.size(1), PD = p1emb.size(1);
  TORCH_CHECK(word.sizes() == pos1.sizes() && word.sizes() == pos2.sizes(), "ina.lstm_fwd: token array shapes differ");
  TORCH_CHECK(E + 2 * PD <= 4 * NX, "ina.lstm_fwd: input dim ", E + 2 * PD, " > 4*NX");
  TORCH_CHECK(p1emb.size(0) >= 2 * L && p2emb.size(0) >= 2 * L, "ina.lstm_fwd: pos tables need 2L rows");
  TORCH_CHECK(bias.numel() == 2 * 4 * U, "ina.lstm_fwd: bias must be [2, 4U]");
  const int64_t U4 = U / 4, KPL = frag_elems(bf16), NKS = (U4 + NX + KPL - 1) / KPL;
  TORCH_CHECK(apack.numel() == 2 * U4 * NKS * 64 * KPL, "ina.lstm_fwd: apack has ", apack.numel(), " elems, expected ",
              2 * U4 * NKS * 64 * KPL);
  TORCH_CHECK(L * 2 * 16 * (int64_t)sizeof(int) * 4 <= 64 * 1024, "ina.lstm_fwd: L too large for the id stage");
  const bool drop = keep_prob < 1.0;
  auto hopt = word.options().dtype(bf16 ? at::kBFloat16 : at::kFloat);
  const int64_t ntiles = (S + 15) / 16;
  // bf16: hlane = the step records [tiles][2][L][2][U4][64] (h slot bf16, c slot fp16 bits; always
  // written -- the h slot is also the attention input) and cst is empty.  fp32: h / c stash (store_c)
  auto hlane = bf16 ? at::empty({ntiles, 2, L, 2, U4, 64}, hopt)
                    : (store_c ? at::empty({ntiles, 2, L, U4, 64}, hopt) : at::empty({0}, hopt));
  // hnat is allocated with 16 * ntiles rows so the kernel stores padding rows unconditionally
  // (no lane-divergent store branch); callers see the first S rows.
  // (bf16 without natural: the attention reads the step records directly; no natural copy)
  auto hnat_full = at::empty({(bf16 && !natural) ? 0 : ntiles * 16, L, 2 * U}, hopt);
  auto hnat = hnat_full.narrow(0, 0, (bf16 && !natural) ? 0 : S);
  auto copt = wemb.options().dtype(bf16 ? at::kHalf : at::kFloat);   // fp16 cell states in bf16 mode
  Tensor cst = (store_c && !bf16) ? at::empty({ntiles, 2, L, U4, 64}, copt) : at::empty({0}, copt);
  TORCH_CHECK(ntiles * 16 * L * 2 * U < (1LL << 31) && ntiles * 2 * L * U4 * 64 < (1LL << 32),
              "ina.lstm_fwd: batch too large for 32-bit offsets (split the episode batch)");
  TORCH_CHECK(wemb.size(0) < (1 << 24) && 2 * L < (1 << 16), "ina.lstm_fwd: table rows exceed 24-bit indexing");
  // dropout keep bits (one byte per lane-step): for the backward, and in bf16 mode for h_natural
  const bool want_mask = drop && (store_c || bf16);
  Tensor dmask = want_mask ? at::empty({ntiles, 2, L, 64}, word.options().dtype(at::kByte))
                           : at::empty({0}, word.options().dtype(at::kByte));
  TORCH_CHECK(ntiles * L * (64 * NX + 16) < (1LL << 31), "ina.lstm_fwd: batch too large for the x rows");
  // direct x (record path, NX == 4, shifted position ids, word rows): the recurrences read the word rows and
  // LDS position tables themselves; xg then holds only x_gather's position ids [tiles][L][16]
  const bool has_wrows = wrows.has_value() && wrows->defined() && wrows->numel() > 0;
  TORCH_CHECK(!direct_x || (bf16 && !natural && NX == 4 && has_wrows),
              "ina.lstm_fwd: direct x needs the bf16 record path, NX == 4 and word rows");
  // (direct x: [position ids][position tables 4 x 2 x 2L x 4 bf16], see lstm.hip xd_build)
  Tensor xg = bf16 ? at::empty({ntiles * L * ((direct_x ? 0 : 64 * NX) + 16) + (direct_x ? 64 * L : 0)},
                               word.options().dtype(at::kBFloat16))
                   : at::empty({0}, word.options().dtype(at::kBFloat16));
  if (S == 0) return {hlane, cst, hnat, dmask, xg};
  ina::LstmArgs a{};
  a.inst = inst.data_ptr<int>();
  a.S = (int)S;
  a.word = word.data_ptr<int>();
  a.pos1 = pos1.data_ptr<int>();
  a.pos2 = pos2.data_ptr<int>();
  a.L = (int)L;
  a.wemb = wemb.data_ptr<float>();
  a.E = (int)E;
  a.p1emb = p1emb.data_ptr<float>();
  a.p2emb = p2emb.data_ptr<float>();
  a.PD = (int)PD;
  a.apack = apack.data_ptr();
  a.bias = bias.data_ptr<float>();
  // non-null hraw / cst select the stash-writing kernel (bf16: c slots of the step records)
  a.hraw = store_c ? hlane.data_ptr() : nullptr;
  a.cst = store_c ? (bf16 ? hlane.data_ptr() : cst.data_ptr()) : nullptr;
  // bf16: the kernel writes its step records (hlane); h_natural transposes the h slots into hnat
  a.hdrop = bf16 ? hlane.data_ptr() : hnat.data_ptr();
  a.dmask = want_mask ? dmask.data_ptr<uint8_t>() : nullptr;
  a.seed_dev = dev_int(seed_dev, "seed_dev");
  a.seed = (uint32_t)seed;
  a.thr = keep_threshold(keep_prob);
  a.inv_kp = (float)(1.0 / keep_prob);
  a.drop = drop ? 1 : 0;
  a.wrows = nullptr;
  if (has_wrows) {
    check(*wrows, "wrows", at::kBFloat16);
    TORCH_CHECK(wrows->numel() == word.numel() * 8 && E <= 8, "ina.lstm_fwd: wrows must be bf16 [NI * L, 8] (E <= 8)");
    TORCH_CHECK(wrows->numel() * 2 < (1LL << 31), "ina.lstm_fwd: word rows exceed a buffer descriptor");
    a.wrows = wrows->data_ptr();
    a.wbytes = (uint32_t)(wrows->numel() * 2);
  }
  a.xd = direct_x ? 1 : 0;
  a.tlen = ragged_arg(tlen, ntiles, "tlen");
  a.slen = ragged_arg(slen, S, "slen");
  a.perm = ragged_arg(perm, S, "perm");
  TORCH_CHECK(!a.tlen || (bf16 && !natural), "ina.lstm_fwd: ragged tiles need the bf16 record path");
  TORCH_CHECK(!a.slen || a.tlen, "ina.lstm_fwd: slen needs tlen");
  if (bf16) {
    a.xg = direct_x ? nullptr : xg.data_ptr();
    a.posb = reinterpret_cast<const unsigned short*>(xg.data_ptr<at::BFloat16>() + (direct_x ? 0 : ntiles * L * 64 * NX));
    a.xdtab = direct_x ? (void*)(xg.data_ptr<at::BFloat16>() + ntiles * L * 16) : nullptr;
    check_launch(ina::x_gather(a, (int)U, (int)NX, cur_stream()), "x_gather");
  }
  check_launch(ina::lstm_fwd(a, (int)U, (int)NX, bf16, cur_stream()), "lstm_fwd");
  if (bf16 && natural)
    check_launch(ina::h_natural(hlane.data_ptr(), drop ? dmask.data_ptr<uint8_t>() : nullptr, (float)(1.0 / keep_prob),
                                (int)S, (int)L, (int)U, hnat_full.data_ptr(), cur_stream()),
                 "h_natural");
  return {hlane, cst, hnat, dmask, xg};
}

std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor> lstm_fwd(const Tensor& inst, const Tensor& word, const Tensor& pos1,
                                            const Tensor& pos2, const Tensor& wemb, const Tensor& p1emb,
                                            const Tensor& p2emb, const Tensor& apack, const Tensor& bias, int64_t U,
                                            int64_t NX, bool bf16, bool store_c, int64_t seed, double keep_prob,
                                            const std::optional<Tensor>& seed_dev,
                                            const std::optional<Tensor>& wrows) {
  return lstm_fwd_impl(inst, word, pos1, pos2, wemb, p1emb, p2emb, apack, bias, U, NX, bf16, store_c, seed, keep_prob,
                       seed_dev, wrows, true);
}

// bf16 encoder forward in three launches: x_gather, lstm_fwd, rec_attn_fwd (the self-attention forward
// straight from the step records, rec_attn.hip: no natural-layout copy of the LSTM output).  Returns
// lstm_fwd's outputs (hnat empty) plus (e, alphas).  Callers check rec_attn_ok first (else lstm_fwd +
// attn_fwd).  w1r = the record-order projection pack (ops/packing.py::pack_attn_rec).
std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor> lstm_attn_fwd(
    const Tensor& inst, const Tensor& word, const Tensor& pos1, const Tensor& pos2, const Tensor& wemb,
    const Tensor& p1emb, const Tensor& p2emb, const Tensor& apack, const Tensor& bias, int64_t U, int64_t NX,
    bool store_c, int64_t seed, double keep_prob, const std::optional<Tensor>& seed_dev,
    const std::optional<Tensor>& wrows, const Tensor& mask, const Tensor& w1r, const Tensor& b1, const Tensor& w2,
    const std::optional<Tensor>& tlen, const std::optional<Tensor>& perm, const std::optional<Tensor>& slen,
    bool direct_x) {
  check(mask, "mask", at::kInt);
  check(w1r, "w1r", at::kBFloat16);
  check(b1, "b1", at::kFloat);
  check(w2, "w2", at::kFloat);
  const int64_t L = word.size(1), S = inst.size(0);
  TORCH_CHECK(mask.size(1) == L, "ina.lstm_attn_fwd: mask length");
  TORCH_CHECK(b1.numel() == 2 * U && w2.numel() == 2 * U, "ina.lstm_attn_fwd: b1/w2 size");
  TORCH_CHECK(L >= 1 && L <= 64, "ina.lstm_attn_fwd: L must be in [1, 64]");
  const int64_t H2 = 2 * U, MT = (H2 + 15) / 16, NKR = (2 * (U / 4) + 7) / 8;
  TORCH_CHECK(w1r.numel() == MT * NKR * 64 * 8, "ina.lstm_attn_fwd: w1r pack size");
  const bool drop = keep_prob < 1.0;
  auto r = lstm_fwd_impl(inst, word, pos1, pos2, wemb, p1emb, p2emb, apack, bias, U, NX, true, store_c, seed, keep_prob,
                         seed_dev, wrows, false, tlen, slen, perm, direct_x);
  auto e = at::empty({S, 2 * U}, b1.options());
  auto alphas = at::empty({S, L}, b1.options());
  if (S == 0) return {std::get<0>(r), std::get<1>(r), std::get<2>(r), std::get<3>(r), std::get<4>(r), e, alphas};
  const Tensor& hlane = std::get<0>(r);
  const Tensor& dmask = std::get<3>(r);
  TORCH_CHECK(hlane.numel() == ((S + 15) / 16) * 2 * L * 2 * (U / 4) * 64, "ina.lstm_attn_fwd: step records");
  TORCH_CHECK(!drop || dmask.numel() == ((S + 15) / 16) * 2 * L * 64, "ina.lstm_attn_fwd: keep bits");
  ina::AttnArgs a{};
  a.inst = inst.data_ptr<int>();
  a.mask = mask.data_ptr<int>();
  a.S = (int)S;
  a.L = (int)L;
  a.w1pack = w1r.data_ptr();
  a.b1 = b1.data_ptr<float>();
  a.w2 = w2.data_ptr<float>();
  a.e = e.data_ptr<float>();
  a.alphas = alphas.data_ptr<float>();
  a.tlen = ragged_arg(tlen, (S + 15) / 16, "tlen");
  a.perm = ragged_arg(perm, S, "perm");
  check_launch(ina::rec_attn_fwd(hlane.data_ptr(), drop ? dmask.data_ptr<uint8_t>() : nullptr, (float)(1.0 / keep_prob),
                                 a, (int)U, cur_stream()),
               "rec_attn_fwd");
  return {std::get<0>(r), std::get<1>(r), std::get<2>(r), std::get<3>(r), std::get<4>(r), e, alphas};
}

bool rec_attn_ok(int64_t U, int64_t L) { return (U == 8 || U == 20 || U == 32) && L >= 1 && L <= 64; }

// bf16 attention backward from the step records (rec_attn.hip; e = the forward's output) -> (dHl [tiles, 2, L, U/4, 64] bf16 in
// lstm_bwd's lane layout, slab [blocks, H2*H2 + 2*H2] in attn_bwd's layout)
std::tuple<Tensor, Tensor> rec_attn_bwd(const Tensor& hlane, const Tensor& dmask, const Tensor& w1r, const Tensor& w1rt,
                                        const Tensor& b1, const Tensor& w2, const Tensor& de, const Tensor& e,
                                        const Tensor& alphas, int64_t U, double keep_prob, int64_t blocks,
                                        const std::optional<Tensor>& tlen, const std::optional<Tensor>& perm) {
  check(hlane, "hlane", at::kBFloat16);
  check(e, "e", at::kFloat);
  check(w1r, "w1r", at::kBFloat16);
  check(w1rt, "w1rt", at::kBFloat16);
  check(b1, "b1", at::kFloat);
  check(w2, "w2", at::kFloat);
  check(de, "de", at::kFloat);
  check(alphas, "alphas", at::kFloat);
  TORCH_CHECK(rec_attn_ok(U, alphas.size(1)), "ina.rec_attn_bwd: unsupported (U, L)");
  const int64_t S = de.size(0), L = alphas.size(1), H2 = 2 * U, U4 = U / 4, ntiles = (S + 15) / 16;
  TORCH_CHECK(de.size(1) == H2 && alphas.size(0) == S && e.sizes() == de.sizes(), "ina.rec_attn_bwd: de / e / alphas shape");
  TORCH_CHECK(hlane.numel() == ntiles * 2 * L * 2 * U4 * 64, "ina.rec_attn_bwd: step records shape");
  const int64_t MT = (H2 + 15) / 16, NKR = (2 * U4 + 7) / 8, NRT = (2 * U4 + 3) / 4, NKS2 = (4 * MT + 7) / 8;
  TORCH_CHECK(w1r.numel() == MT * NKR * 64 * 8 && w1rt.numel() == NRT * NKS2 * 64 * 8, "ina.rec_attn_bwd: pack sizes");
  const bool drop = keep_prob < 1.0;
  if (drop) {
    check(dmask, "dmask", at::kByte);
    TORCH_CHECK(dmask.numel() == ntiles * 2 * L * 64, "ina.rec_attn_bwd: keep bits shape");
  }
  if (blocks <= 0) {
    blocks = ina::rec_attn_bwd_resident_blocks((int)U);
    if (blocks <= 0) blocks = 1024;
  }
  blocks = std::max<int64_t>(1, std::min<int64_t>(blocks, (ntiles + 3) / 4));
  auto dH = at::empty({ntiles, 2, L, U4, 64}, de.options().dtype(at::kBFloat16));
  auto slab = at::empty({blocks, H2 * H2 + 2 * H2}, de.options());
  if (S == 0) {
    slab.zero_();
    return {dH, slab};
  }
  ina::AttnArgs a{};
  a.S = (int)S;
  a.L = (int)L;
  a.w1pack = w1r.data_ptr();
  a.w1tpack = w1rt.data_ptr();
  a.b1 = b1.data_ptr<float>();
  a.w2 = w2.data_ptr<float>();
  a.de = de.data_ptr<float>();
  a.e = const_cast<float*>(e.data_ptr<float>());   // read-only here: the forward's pooled output (sd = de . e)
  a.alphas = alphas.data_ptr<float>();
  a.dHraw = dH.data_ptr();
  a.slab = slab.data_ptr<float>();
  a.blocks = (int)blocks;
  a.tlen = ragged_arg(tlen, ntiles, "tlen");
  a.perm = ragged_arg(perm, S, "perm");
  check_launch(ina::rec_attn_bwd(hlane.data_ptr(), drop ? dmask.data_ptr<uint8_t>() : nullptr, (float)(1.0 / keep_prob),
                                 a, (int)U, cur_stream()),
               "rec_attn_bwd");
  return {dH, slab};
}

std::tuple<Tensor, Tensor, Tensor> lstm_bwd(
    const Tensor& inst, const Tensor& word, const Tensor& pos1, const Tensor& pos2, const Tensor& wemb,
    const Tensor& p1emb, const Tensor& p2emb, const Tensor& apack, const Tensor& a2pack, const Tensor& bias,
    const Tensor& hraw, const Tensor& cst, const Tensor& dH, const Tensor& dmask, const Tensor& xg, int64_t U, int64_t NX,
    bool bf16, bool word_grad, int64_t blocks, int64_t seed, double keep_prob, bool pos_shift,
    const std::optional<Tensor>& tlen, const std::optional<Tensor>& slen, const std::optional<Tensor>& wrows) {
  check(inst, "inst", at::kInt);
  check(word, "word", at::kInt);
  check(pos1, "pos1", at::kInt);
  check(pos2, "pos2", at::kInt);
  check(wemb, "wemb", at::kFloat);
  check(p1emb, "p1emb", at::kFloat);
  check(p2emb, "p2emb", at::kFloat);
  check(bias, "bias", at::kFloat);
  if (!bf16) check(cst, "cst", at::kFloat);   // bf16: the cell states are packed into hlane
  check(dH, "dH", bf16 ? at::kBFloat16 : at::kFloat);
  check(apack, "apack", bf16 ? at::kBFloat16 : at::kFloat);
  check(a2pack, "a2pack", bf16 ? at::kBFloat16 : at::kFloat);
  check(hraw, "hraw", bf16 ? at::kBFloat16 : at::kFloat);   // bf16: lstm_fwd's step records
  TORCH_CHECK(ina::lstm_supported((int)U, (int)NX), "ina.lstm_bwd: unsupported (U, NX)");
  const int64_t S = inst.size(0), L = word.size(1), E = wemb.size(1), PD = p1emb.size(1);
  const int64_t DIN = E + 2 * PD, NF = DIN + U + 1, U4 = U / 4, KPL = frag_elems(bf16);
  TORCH_CHECK(DIN <= 4 * NX, "ina.lstm_bwd: input dim too large");
  TORCH_CHECK(hraw.numel() == ((S + 15) / 16) * 2 * L * U4 * 64 * (bf16 ? 2 : 1), "ina.lstm_bwd: hlane shape");
  // dH: natural [S, L, 2U] (attn_bwd) or, bf16, the step-record lane layout [tiles, 2, L, U/4, 64] (rec_attn_bwd)
  const bool dh_lane = dH.dim() == 5;
  TORCH_CHECK(dh_lane ? (bf16 && dH.size(0) == (S + 15) / 16 && dH.size(1) == 2 && dH.size(2) == L &&
                         dH.size(3) == U / 4 && dH.size(4) == 64)
                      : (dH.dim() == 3 && dH.size(0) == S && dH.size(1) == L && dH.size(2) == 2 * U),
              "ina.lstm_bwd: dH shape");
  TORCH_CHECK(bf16 || cst.numel() == ((S + 15) / 16) * 2 * L * U4 * 64, "ina.lstm_bwd: cst shape");
  const bool drop_ = keep_prob < 1.0;
  if (drop_) {
    check(dmask, "dmask", at::kByte);
    TORCH_CHECK(dmask.numel() == ((S + 15) / 16) * 2 * L * 64, "ina.lstm_bwd: dmask (from lstm_fwd) shape");
  }
  const int64_t NSLOT = U4 + NX;
  TORCH_CHECK(a2pack.numel() == 2 * ((NSLOT + 3) / 4) * ((4 * U4 + KPL - 1) / KPL) * 64 * KPL, "ina.lstm_bwd: a2pack");
  TORCH_CHECK(ina::lstm_bwd_lds_bytes((int)U, (int)NX, bf16, (int)L, (int)PD) <= 160 * 1024, "ina.lstm_bwd: LDS budget");
  const int64_t ngroups = ((S + 15) / 16 + 3) / 4;
  // 768 workgroups per direction (the backward direction's first, longest-first order), back-filled by the
  // dispatcher: 23.79-23.81 vs 23.87-24.06 ms per 18 calls for 512, 25.5 for 640, 24.4 for 896 (profiles/r6_blocks).
  // (A grid of exactly the resident workgroups, ina::lstm_bwd_resident_blocks, measured slower in round 3:
  // 616 vs 580 us -- its critical path is the 7-group workgroups.)
  if (blocks <= 0) blocks = 768;
  blocks = std::max<int64_t>(1, std::min<int64_t>(blocks, ngroups));
  auto opt = wemb.options();
  auto dw_slab = at::empty({blocks, 2, 4 * U, NF}, opt);
  // bf16: pos gradients leave lstm_bwd as per-token rows and pos_grad reduces them -> [pblocks, 1, 2, 2L, PD]
  const int64_t ntiles = (S + 15) / 16;
  const int64_t pitems = ntiles * ((L + 1) / 2);
  const int64_t pblocks = std::max<int64_t>(1, std::min<int64_t>(1024, (pitems + 31) / 32));
  if (bf16) TORCH_CHECK(2 * PD <= 16 && 2 * L <= 128, "ina.lstm_bwd: bf16 path needs pos_dim <= 8 and L <= 64");
  // pos_shift (caller-checked pos[s][t] = pos[s][0] + t, pos[s][0] <= L): per-sequence one-hot GEMM -> ONE slab
  // (pos_shift_gemm addresses one direction of dxp through a 32-bit buffer offset: < 2 GiB, ~2M sequences at L=38)
  const bool shift = bf16 && pos_shift && (L + 1 + 15) / 16 <= 5 && ((S + 15) / 16) * L * (2 * PD + 1) * 32 < (1LL << 31);
  // (direct x: x_gather wrote only the t = 0 position ids -- the shifted-form reduction's per-sequence offsets)
  TORCH_CHECK(!(bf16 && xg.numel() == ((S + 15) / 16) * L * 16 + 64 * L) || shift,
              "ina.lstm_bwd: direct x needs the shifted-position gradient path");
  auto dpos_slab = shift ? at::empty({1, 1, 2, 2 * L, PD}, opt)
                         : (bf16 ? at::empty({pblocks, 1, 2, 2 * L, PD}, opt) : at::empty({blocks, 2, 2, 2 * L, PD}, opt));
  // [2 dir][tiles][L][2PD + 1][16] bf16 dx of the pos features (+ a trash row for the other lanes)
  Tensor dxp = bf16 ? at::empty({2 * (2 * PD + 1) * ntiles * L * 16}, opt.dtype(at::kBFloat16)) : at::empty({0}, opt);
  // direct x (lstm_attn_fwd with direct_x): xg holds only the position ids, x comes from the word rows
  const bool direct_x = bf16 && xg.numel() == ntiles * L * 16 + 64 * L;
  if (bf16) {
    check(xg, "xg", at::kBFloat16);
    TORCH_CHECK(direct_x || xg.numel() == ntiles * L * (64 * NX + 16), "ina.lstm_bwd: xg (from lstm_fwd) shape");
  }
  if (direct_x) {
    TORCH_CHECK(wrows.has_value() && wrows->defined() && wrows->numel() == word.numel() * 8,
                "ina.lstm_bwd: direct x needs the forward's word rows");
    check(*wrows, "wrows", at::kBFloat16);
    TORCH_CHECK(dh_lane && NX == 4 && wrows->numel() * 2 < (1LL << 31),
                "ina.lstm_bwd: direct x runs in the lean lane-layout BPTT only");
  }
  Tensor dwemb = word_grad ? at::zeros_like(wemb) : at::empty({0}, opt);
  if (S == 0) {
    dw_slab.zero_();
    dpos_slab.zero_();
    return {dw_slab, dpos_slab, dwemb};
  }
  ina::LstmArgs a{};
  a.inst = inst.data_ptr<int>();
  a.S = (int)S;
  a.word = word.data_ptr<int>();
  a.pos1 = pos1.data_ptr<int>();
  a.pos2 = pos2.data_ptr<int>();
  a.L = (int)L;
  a.wemb = wemb.data_ptr<float>();
  a.E = (int)E;
  a.p1emb = p1emb.data_ptr<float>();
  a.p2emb = p2emb.data_ptr<float>();
  a.PD = (int)PD;
  a.apack = apack.data_ptr();
  a.a2pack = a2pack.data_ptr();
  a.bias = bias.data_ptr<float>();
  a.hraw = hraw.data_ptr();
  a.cst = bf16 ? hraw.data_ptr() : cst.data_ptr();
  a.dH = dH.data_ptr();
  a.dw_slab = dw_slab.data_ptr<float>();
  a.dpos_slab = dpos_slab.data_ptr<float>();
  a.dwemb = word_grad ? dwemb.data_ptr<float>() : nullptr;
  // the FewRel / synthetic word tables end with the padding row BLANK = V + 1 (data/fewrel.py)
  a.wblank = word_grad ? (int)wemb.size(0) - 1 : -1;
  a.dmask = drop_ ? dmask.data_ptr<uint8_t>() : nullptr;
  a.bwd_blocks = (int)blocks;
  a.seed = (uint32_t)seed;
  a.thr = keep_threshold(keep_prob);
  a.inv_kp = (float)(1.0 / keep_prob);
  a.drop = keep_prob < 1.0 ? 1 : 0;
  a.dxp = bf16 ? dxp.data_ptr() : nullptr;
  a.dh_lane = dh_lane ? 1 : 0;
  a.tlen = ragged_arg(tlen, ntiles, "tlen");
  a.slen = ragged_arg(slen, S, "slen");
  TORCH_CHECK(!a.tlen || (bf16 && dh_lane), "ina.lstm_bwd: ragged tiles need the bf16 lane-layout dH path");
  TORCH_CHECK(!a.slen || a.tlen, "ina.lstm_bwd: slen needs tlen");
  a.xg = (bf16 && !direct_x) ? xg.data_ptr() : nullptr;
  a.posb = bf16 ? reinterpret_cast<const unsigned short*>(xg.data_ptr<at::BFloat16>() + (direct_x ? 0 : ntiles * L * 64 * NX))
                : nullptr;
  a.xd = direct_x ? 1 : 0;
  a.xdtab = direct_x ? (void*)(xg.data_ptr<at::BFloat16>() + ntiles * L * 16) : nullptr;
  a.wrows = direct_x ? wrows->data_ptr() : nullptr;
  a.wbytes = direct_x ? (uint32_t)(wrows->numel() * 2) : 0u;
  check_launch(ina::lstm_bwd(a, (int)U, (int)NX, bf16, cur_stream()), "lstm_bwd");
  if (shift) {
    Tensor gpart = at::empty({(int64_t)ina::pos_shift_workspace_floats((int)S, (int)L, (int)PD, nullptr, nullptr)}, opt);
    check_launch(ina::pos_grad_shift(a, gpart.data_ptr<float>(), dpos_slab.data_ptr<float>(), cur_stream()),
                 "pos_grad_shift");
  } else if (bf16) {
    check_launch(ina::pos_grad(a, (int)pblocks, dpos_slab.data_ptr<float>(), cur_stream()), "pos_grad");
  }
  return {dw_slab, dpos_slab, dwemb};
}


// ------------------------------------------------------------------ attention

std::tuple<Tensor, Tensor> attn_fwd(const Tensor& hraw, const Tensor& inst, const Tensor& mask, const Tensor& w1pack,
                                    const Tensor& b1, const Tensor& w2, int64_t U, bool bf16, int64_t blocks) {
  check(hraw, "hraw", bf16 ? at::kBFloat16 : at::kFloat);
  check(inst, "inst", at::kInt);
  check(mask, "mask", at::kInt);
  check(w1pack, "w1pack", bf16 ? at::kBFloat16 : at::kFloat);
  check(b1, "b1", at::kFloat);
  check(w2, "w2", at::kFloat);
  const int64_t S = hraw.size(0), L = hraw.size(1);
  TORCH_CHECK(hraw.size(2) == 2 * U, "ina.attn_fwd: hraw last dim must be 2U");
  TORCH_CHECK(mask.size(1) == L, "ina.attn_fwd: mask length");
  TORCH_CHECK(b1.numel() == 2 * U && w2.numel() == 2 * U, "ina.attn_fwd: b1/w2 size");
  const int64_t NT = (L + 15) / 16;
  TORCH_CHECK(NT >= 1 && NT <= 4, "ina.attn_fwd: L must be <= 64");
  auto e = at::empty({S, 2 * U}, b1.options());
  auto alphas = at::empty({S, L}, b1.options());
  if (S == 0) return {e, alphas};
  ina::AttnArgs a{};
  a.hraw = hraw.data_ptr();
  a.inst = inst.data_ptr<int>();
  a.mask = mask.data_ptr<int>();
  a.S = (int)S;
  a.L = (int)L;
  a.w1pack = w1pack.data_ptr();
  a.b1 = b1.data_ptr<float>();
  a.w2 = w2.data_ptr<float>();
  a.e = e.data_ptr<float>();
  a.alphas = alphas.data_ptr<float>();
  if (blocks <= 0) blocks = 2048;
  a.blocks = (int)std::max<int64_t>(1, std::min<int64_t>(blocks, (S + 3) / 4));
  check_launch(ina::attn_fwd(a, (int)U, (int)NT, bf16, cur_stream()), "attn_fwd");
  return {e, alphas};
}

std::tuple<Tensor, Tensor> attn_bwd(const Tensor& hraw, const Tensor& inst, const Tensor& w1pack, const Tensor& w1tpack,
                                    const Tensor& b1, const Tensor& w2, const Tensor& de, const Tensor& alphas,
                                    int64_t U, bool bf16, int64_t blocks) {
  check(hraw, "hraw", bf16 ? at::kBFloat16 : at::kFloat);
  check(inst, "inst", at::kInt);
  check(w1pack, "w1pack", bf16 ? at::kBFloat16 : at::kFloat);
  check(w1tpack, "w1tpack", bf16 ? at::kBFloat16 : at::kFloat);
  check(b1, "b1", at::kFloat);
  check(w2, "w2", at::kFloat);
  check(de, "de", at::kFloat);
  check(alphas, "alphas", at::kFloat);
  const int64_t S = hraw.size(0), L = hraw.size(1), H2 = 2 * U;
  TORCH_CHECK(de.size(0) == S && de.size(1) == H2, "ina.attn_bwd: de shape");
  TORCH_CHECK(alphas.size(0) == S && alphas.size(1) == L, "ina.attn_bwd: alphas shape");
  const int64_t NT = (L + 15) / 16;
  TORCH_CHECK(NT >= 1 && NT <= 4, "ina.attn_bwd: L must be <= 64");
  // 4-wave workgroups; bf16 (attn_bwd3, persistent): by default exactly the resident workgroups
  const int64_t wpb = 4;
  if (blocks <= 0) {
    blocks = ina::attn_bwd_resident_blocks((int)U, (int)NT, bf16);
    if (blocks <= 0) blocks = 1024;
  }
  blocks = std::max<int64_t>(1, std::min<int64_t>(blocks, (S + wpb - 1) / wpb));
  auto dH = at::empty({S, L, H2}, de.options().dtype(bf16 ? at::kBFloat16 : at::kFloat));
  auto slab = at::empty({blocks, H2 * H2 + 2 * H2}, de.options());
  if (S == 0) {
    slab.zero_();
    return {dH, slab};
  }
  ina::AttnArgs a{};
  a.hraw = hraw.data_ptr();
  a.inst = inst.data_ptr<int>();
  a.S = (int)S;
  a.L = (int)L;
  a.w1pack = w1pack.data_ptr();
  a.w1tpack = w1tpack.data_ptr();
  a.b1 = b1.data_ptr<float>();
  a.w2 = w2.data_ptr<float>();
  a.de = de.data_ptr<float>();
  a.alphas = alphas.data_ptr<float>();
  a.dHraw = dH.data_ptr();
  a.slab = slab.data_ptr<float>();
  a.blocks = (int)blocks;
  check_launch(ina::attn_bwd(a, (int)U, (int)NT, bf16, cur_stream()), "attn_bwd");
  return {dH, slab};
}

// ------------------------------------------------------------------ routing
void check_episode_rows(const Tensor& e, int64_t E, int64_t N, int64_t K, int64_t Q, const char* who) {
  TORCH_CHECK(e.dim() == 2 && e.size(0) == E * (N * K + N * Q), who, ": e must be [E*(N*K+N*Q), H]");
}

Tensor routing_fwd(const Tensor& e, const Tensor& Ws, int64_t E, int64_t N, int64_t K, int64_t Q, int64_t R,
                   int64_t blocks) {
  check(e, "e", at::kFloat);
  check(Ws, "W_s", at::kFloat);
  check_episode_rows(e, E, N, K, Q, "ina.routing_fwd");
  const int64_t H = e.size(1);
  TORCH_CHECK(Ws.size(0) == H && Ws.size(1) == H, "ina.routing_fwd: W_s must be [H, H]");
  TORCH_CHECK(ina::routing_lds_bytes((int)N, (int)K, (int)H, (int)R, false) <= 160 * 1024, "ina.routing_fwd: N*K too large");
  auto cls = at::empty({E, N, H}, e.options());
  if (E == 0) return cls;
  if (blocks <= 0) blocks = 8192;   // work items = (episode, class) pairs
  blocks = std::max<int64_t>(1, std::min<int64_t>(blocks, E * N));
  check_launch(ina::routing_fwd(e.data_ptr<float>(), Ws.data_ptr<float>(), (int)E, (int)N, (int)K, (int)Q, (int)R,
                                (int)H, cls.data_ptr<float>(), (int)blocks, cur_stream()),
               "routing_fwd");
  return cls;
}

Tensor routing_bwd(const Tensor& e, const Tensor& Ws, const Tensor& dcls, Tensor de, int64_t E, int64_t N, int64_t K,
                   int64_t Q, int64_t R, int64_t blocks) {
  check(e, "e", at::kFloat);
  check(Ws, "W_s", at::kFloat);
  check(dcls, "dcls", at::kFloat);
  check(de, "de", at::kFloat);
  check_episode_rows(e, E, N, K, Q, "ina.routing_bwd");
  const int64_t H = e.size(1);
  TORCH_CHECK(de.sizes() == e.sizes(), "ina.routing_bwd: de shape");
  TORCH_CHECK(dcls.numel() == E * N * H, "ina.routing_bwd: dcls shape");
  TORCH_CHECK(ina::routing_lds_bytes((int)N, (int)K, (int)H, (int)R, true) <= 160 * 1024, "ina.routing_bwd: N*K too large");
  if (blocks <= 0) blocks = ina::routing_bwd_default_blocks((int)N, (int)K, (int)H, (int)R);   // slab per block
  blocks = std::max<int64_t>(1, std::min<int64_t>(blocks, std::max<int64_t>(E * N, 1)));
  auto slab = at::empty({blocks, H, H}, e.options());   // every block writes its whole slab
  if (E == 0) return slab.zero_();
  check_launch(ina::routing_bwd(e.data_ptr<float>(), Ws.data_ptr<float>(), (int)E, (int)N, (int)K, (int)Q, (int)R,
                                (int)H, dcls.data_ptr<float>(), de.data_ptr<float>(), slab.data_ptr<float>(),
                                (int)blocks, cur_stream()),
               "routing_bwd");
  return slab;
}

// ------------------------------------------------------------------ NTN
// tile pack geometry (must match ops/packing.py::ntn_tile_geometry)
static void ntn_geometry(int64_t N, int64_t H, int64_t h, int64_t& SG, int64_t& ntile, int64_t& tpb) {
  const int64_t MTH = (H + 15) / 16;
  SG = ina::ntn_slices_per_tile((int)N);
  ntile = (h + SG - 1) / SG;
  tpb = SG * MTH * 16 * 128 + 1024;
}

static ina::NtnArgs ntn_args(const Tensor& cls, const Tensor& e, const Tensor& tiles, int64_t E, int64_t N, int64_t K,
                             int64_t Q, int64_t h, bool paper, int64_t blocks, const char* who) {
  check(cls, "cls", at::kFloat);
  check(e, "e", at::kFloat);
  check(tiles, "tiles", at::kBFloat16);
  check_episode_rows(e, E, N, K, Q, who);
  const int64_t H = e.size(1), MTH = (H + 15) / 16;
  TORCH_CHECK(N >= 1 && N <= 16 && N * Q <= 64, who, ": needs 1 <= N <= 16 and N*Q <= 64");
  TORCH_CHECK((MTH == 1 || MTH == 3 || MTH == 4) && H % 8 == 0, who, ": unsupported H ", H);
  TORCH_CHECK(cls.numel() == E * N * H, who, ": cls shape");
  int64_t SG, ntile, tpb;
  ntn_geometry(N, H, h, SG, ntile, tpb);
  TORCH_CHECK(tiles.numel() * 2 == ntile * tpb, who, ": tile pack size ", tiles.numel(), " != ", ntile * tpb / 2);
  ina::NtnArgs a{};
  a.cls = cls.data_ptr<float>();
  a.e = e.data_ptr<float>();
  a.E = (int)E;
  a.N = (int)N;
  a.K = (int)K;
  a.Q = (int)Q;
  a.H = (int)H;
  a.h = (int)h;
  a.tiles = tiles.data_ptr();
  a.G = ina::ntn_episodes_per_wave((int)N, (int)Q);
  a.SG = (int)SG;
  a.ntile = (int)ntile;
  a.tpb = (int)tpb;
  a.paper = paper ? 1 : 0;
  if (blocks <= 0) blocks = 65535;   // one workgroup per 8 waves x G episodes (grid-stride beyond)
  a.blocks = (int)std::max<int64_t>(1, std::min<int64_t>(blocks, 65535));
  a.split = ina::ntn_split((int)E, (int)N, (int)Q, (int)h);
  return a;
}

Tensor ntn_fwd(const Tensor& cls, const Tensor& e, const Tensor& tiles, const Tensor& bias, int64_t E, int64_t N,
               int64_t K, int64_t Q, int64_t h, bool paper, int64_t blocks) {
  check(bias, "bias", at::kFloat);
  TORCH_CHECK(bias.numel() == (paper ? 1 : N), "ina.ntn_fwd: bias must be [", paper ? 1 : N, "]");
  auto a = ntn_args(cls, e, tiles, E, N, K, Q, h, paper, blocks, "ina.ntn_fwd");
  auto probs = at::empty({E, N * Q, N}, e.options());
  if (E == 0) return probs;
  a.bias = bias.data_ptr<float>();
  a.probs = probs.data_ptr<float>();
  Tensor part;
  if (a.split > 1) {
    part = at::empty({a.split * E * N * Q * N}, e.options());
    a.part = part.data_ptr<float>();
  }
  check_launch(ina::ntn_fwd(a, cur_stream()), "ntn_fwd");
  return probs;
}

// -> (dcls [E, N, H], dP bf16 [Kp, h H], dw slab [ngroups, ntile * (SG N N | SG)], C bf16 [Kp, H]) with the
// class rows padded to Kp = E N rounded up to 64 (zero rows): dP and C are the operands of the dM reduction
// GEMM (gemm_tn_slab)
std::tuple<Tensor, Tensor, Tensor, Tensor> ntn_bwd(const Tensor& cls, const Tensor& e, const Tensor& tiles,
                                                   const Tensor& dz, Tensor de, int64_t E, int64_t N, int64_t K,
                                                   int64_t Q, int64_t h, bool paper, int64_t blocks,
                                                   const std::optional<Tensor>& gscale) {
  auto a = ntn_args(cls, e, tiles, E, N, K, Q, h, paper, blocks, "ina.ntn_bwd");
  check(dz, "dz", at::kFloat);
  check(de, "de", at::kFloat);
  const int64_t H = e.size(1), hH = h * H, rows = E * N, Kp = (rows + 63) / 64 * 64;
  TORCH_CHECK(dz.numel() == E * N * Q * N, "ina.ntn_bwd: dz shape");
  TORCH_CHECK(de.sizes() == e.sizes(), "ina.ntn_bwd: de shape");
  auto dcls = at::empty({E, N, H}, e.options());
  // dP: a trash tail past the padded rows takes the stores of lanes outside the valid (slice, class) / H
  // ranges (no exec-mask branches in the tile loop)
  auto dpf = at::empty({Kp * hH + 64}, e.options().dtype(at::kBFloat16));
  auto dp = dpf.narrow(0, 0, Kp * hH).view({Kp, hH});
  auto cbf = at::empty({Kp, H}, e.options().dtype(at::kBFloat16));
  if (Kp > rows) {
    dp.narrow(0, rows, Kp - rows).zero_();
    cbf.narrow(0, rows, Kp - rows).zero_();
  }
  const int64_t groups = ina::ntn_groups((int)E, (int)N, (int)Q);
  const int64_t dwe = paper ? a.SG : a.SG * N * N;
  auto dw = at::empty({groups, a.ntile * dwe}, e.options());
  if (E == 0) return {dcls, dp, dw, cbf};
  a.dz = dz.data_ptr<float>();
  a.dcls = dcls.data_ptr<float>();
  a.de = de.data_ptr<float>();
  a.dp_out = dp.data_ptr();
  a.dw_slab = dw.data_ptr<float>();
  a.gscale = dev_float(gscale, "gscale");
  a.cls_bf = cbf.data_ptr();
  Tensor pc, pq;
  if (a.split > 1) {
    pc = at::empty({a.split * E * N * H}, e.options());
    pq = at::empty({a.split * E * N * Q * H}, e.options());
    a.part = pc.data_ptr<float>();
    a.part2 = pq.data_ptr<float>();
  }
  check_launch(ina::ntn_bwd(a, cur_stream()), "ntn_bwd");
  return {dcls, dp, dw, cbf};
}

int64_t ntn_slices_per_tile(int64_t N) { return ina::ntn_slices_per_tile((int)N); }

// slab [splits, MI, NJ] fp32 = per-split sums over k of A[k, :MI]^T B[k, :NJ] (A [K, >= MI], B [K, >= NJ] bf16 rows
// with unit column stride, row strides multiples of 8, 16-byte aligned bases; K % 64 == 0)
Tensor gemm_tn_slab(const Tensor& A, const Tensor& B, int64_t MI, int64_t splits) {
  TORCH_CHECK(A.is_cuda() && B.is_cuda() && A.scalar_type() == at::kBFloat16 && B.scalar_type() == at::kBFloat16,
              "ina.gemm_tn_slab: bf16 GPU operands");
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A.size(0) == B.size(0), "ina.gemm_tn_slab: A [K, lda], B [K, NJ]");
  TORCH_CHECK(A.stride(1) == 1 && B.stride(1) == 1 && A.stride(0) % 8 == 0 && B.stride(0) % 8 == 0 &&
                  reinterpret_cast<uintptr_t>(A.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(B.data_ptr()) % 16 == 0,
              "ina.gemm_tn_slab: rows with unit column stride, strides % 8 == 0, 16-byte aligned");
  const int64_t K = A.size(0), NJ = B.size(1);
  TORCH_CHECK(K % 64 == 0 && MI % 8 == 0 && MI > 0 && MI <= 64 && MI <= A.size(1) && NJ % 8 == 0 && NJ >= 8,
              "ina.gemm_tn_slab: needs K % 64 == 0, MI % 8 == 0, MI <= 64, NJ % 8 == 0");
  if (splits <= 0) splits = ina::gemm_tn_splits((int)K, (int)MI, (int)NJ);
  auto slab = at::empty({splits, MI, NJ}, A.options().dtype(at::kFloat));
  static thread_local std::map<int, Tensor> zeros;
  const int dev = A.get_device();
  auto it = zeros.find(dev);
  if (it == zeros.end()) it = zeros.emplace(dev, at::zeros({64}, A.options())).first;
  check_launch(ina::gemm_tn_slab(A.data_ptr(), (int)A.stride(0), B.data_ptr(), (int)B.stride(0), (int)K, (int)MI,
                                 (int)NJ, it->second.data_ptr(), slab.data_ptr<float>(), (int)splits, cur_stream()),
               "gemm_tn_slab");
  return slab;
}

// ------------------------------------------------------------------ optim / misc
// lr: the scheduled rate (or lr_dev[0]); the kernel applies TF1's bias correction for the applied-step
// count t = (t_dev[0] if given else t_host) - skips[0] (skips: steps the guard skipped)
void adam_step(Tensor p, Tensor m, Tensor v, const Tensor& g, const std::optional<Tensor>& l2mask, double lr,
               int64_t t_host, double b1, double b2, double eps, double gscale, double l2,
               const std::optional<Tensor>& lr_dev, const std::optional<Tensor>& t_dev,
               const std::optional<Tensor>& guard, const std::optional<Tensor>& skips) {
  check(p, "p", at::kFloat);
  check(m, "m", at::kFloat);
  check(v, "v", at::kFloat);
  check(g, "g", at::kFloat);
  const int64_t n = p.numel();
  TORCH_CHECK(m.numel() == n && v.numel() == n && g.numel() == n, "ina.adam_step: size mismatch");
  const unsigned char* mk = nullptr;
  if (l2mask.has_value() && l2mask->defined() && l2mask->numel() > 0) {
    check(*l2mask, "l2mask", at::kByte);
    TORCH_CHECK(l2mask->numel() == n, "ina.adam_step: l2mask size");
    mk = l2mask->data_ptr<unsigned char>();
  }
  if (n == 0) return;
  check_launch(ina::adam_step(p.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), g.data_ptr<float>(), mk, n,
                              (float)lr, (int)t_host, (float)b1, (float)b2, (float)eps, (float)gscale, (float)l2,
                              dev_float(lr_dev, "lr_dev"), dev_int(t_dev, "t_dev"), dev_float(guard, "guard"),
                              guard_skips(guard, skips),
                              cur_stream()),
               "adam_step");
}

void adagrad_step(Tensor p, Tensor acc, const Tensor& g, const std::optional<Tensor>& l2mask, double lr, double gscale,
                  double l2, const std::optional<Tensor>& lr_dev, const std::optional<Tensor>& guard,
                  const std::optional<Tensor>& skips) {
  check(p, "p", at::kFloat);
  check(acc, "acc", at::kFloat);
  check(g, "g", at::kFloat);
  const int64_t n = p.numel();
  TORCH_CHECK(acc.numel() == n && g.numel() == n, "ina.adagrad_step: size mismatch");
  const unsigned char* mk = nullptr;
  if (l2mask.has_value() && l2mask->defined() && l2mask->numel() > 0) {
    check(*l2mask, "l2mask", at::kByte);
    mk = l2mask->data_ptr<unsigned char>();
  }
  if (n == 0) return;
  check_launch(ina::adagrad_step(p.data_ptr<float>(), acc.data_ptr<float>(), g.data_ptr<float>(), mk, n, (float)lr,
                                 (float)gscale, (float)l2, dev_float(lr_dev, "lr_dev"), dev_float(guard, "guard"),
                                 guard_skips(guard, skips), cur_stream()),
               "adagrad_step");
}

// NaN/Inf guard: flag[0] = 1 when any element of g (or the loss scalar) is not finite; flag must be 0
// before (it is the zeroed tail of the flat gradient buffer, ops/optim.py::FlatParams)
void nonfinite_flag(const Tensor& g, const std::optional<Tensor>& loss, Tensor flag) {
  check(g, "g", at::kFloat);
  check(flag, "flag", at::kFloat);
  TORCH_CHECK(flag.numel() >= 1, "ina.nonfinite_flag: flag needs 1 float");
  const float* lp = dev_float(loss, "loss");
  if (g.numel() == 0 && lp == nullptr) return;
  check_launch(ina::nonfinite_flag(g.data_ptr<float>(), g.numel(), lp, flag.data_ptr<float>(), cur_stream()),
               "nonfinite_flag");
}

void slab_reduce(const Tensor& slabs, Tensor out, bool accumulate) {
  check(slabs, "slabs", at::kFloat);
  check(out, "out", at::kFloat);
  const int64_t len = out.numel();
  TORCH_CHECK(len > 0 && slabs.numel() % len == 0, "ina.slab_reduce: slabs must be [k, out.numel()]");
  check_launch(ina::slab_reduce(slabs.data_ptr<float>(), slabs.numel() / len, len, out.data_ptr<float>(),
                                accumulate ? 1 : 0, cur_stream()),
               "slab_reduce");
}

std::tuple<Tensor, Tensor> sample_episodes(const Tensor& scopes, int64_t E, int64_t N, int64_t K, int64_t Q, int64_t seed,
                                           double nota_rate, const std::optional<Tensor>& seed_dev,
                                           const std::optional<Tensor>& fail) {
  check(scopes, "scopes", at::kInt);
  TORCH_CHECK(scopes.dim() == 2 && scopes.size(1) == 2, "ina.sample_episodes: scopes must be [R, 2]");
  const int64_t R = scopes.size(0);
  TORCH_CHECK(N <= R, "ina.sample_episodes: N > number of relations");
  TORCH_CHECK(ina::sampler_supported((int)N, (int)K, (int)Q), "ina.sample_episodes: N/K/Q too large");
  auto idx = at::empty({E, N * K + N * Q}, scopes.options());
  auto lab = at::empty({E, N * Q}, scopes.options());
  if (E == 0) return {idx, lab};
  check_launch(ina::sample_episodes(scopes.data_ptr<int>(), (int)R, (int)E, (int)N, (int)K, (int)Q, (uint32_t)seed,
                                    (float)nota_rate, idx.data_ptr<int>(), lab.data_ptr<int>(),
                                    dev_int(seed_dev, "seed_dev"), const_cast<int*>(dev_int(fail, "fail")),
                                    cur_stream()),
               "sample_episodes");
  return {idx, lab};
}

// per-step control block for HIP-graph replay (see optim.hip::step_control_kernel)
void step_control(Tensor ctl, Tensor lrt, int64_t seedA, int64_t seedB, double lr0, double decay_steps,
                  double decay_rate, bool staircase, bool constant, bool adam, double b1, double b2) {
  check(ctl, "ctl", at::kInt);
  check(lrt, "lrt", at::kFloat);
  TORCH_CHECK(ctl.numel() >= 5 && lrt.numel() >= 1, "ina.step_control: ctl needs 5 ints, lrt 1 float");
  check_launch(ina::step_control(ctl.data_ptr<int>(), lrt.data_ptr<float>(), (long long)seedA, (long long)seedB, lr0,
                                 decay_steps, decay_rate, staircase ? 1 : 0, constant ? 1 : 0, adam ? 1 : 0, b1, b2,
                                 cur_stream()),
               "step_control");
}

int64_t abi_version() { return 6; }

}  // namespace

TORCH_LIBRARY(ina, m) {
  m.def("abi_version", &abi_version);
  m.def("lstm_fwd", &lstm_fwd);
  m.def("lstm_bwd", &lstm_bwd);
  m.def("lstm_attn_fwd", &lstm_attn_fwd);
  m.def("rec_attn_ok", &rec_attn_ok);
  m.def("rec_attn_bwd", &rec_attn_bwd);
  m.def("attn_fwd", &attn_fwd);
  m.def("attn_bwd", &attn_bwd);
  m.def("routing_fwd", &routing_fwd);
  m.def("routing_bwd", &routing_bwd);
  m.def("ntn_fwd", &ntn_fwd);
  m.def("ntn_bwd", &ntn_bwd);
  m.def("ntn_slices_per_tile", &ntn_slices_per_tile);
  m.def("gemm_tn_slab", &gemm_tn_slab);
  m.def("adam_step", &adam_step);
  m.def("adagrad_step", &adagrad_step);
  m.def("nonfinite_flag", &nonfinite_flag);
  m.def("slab_reduce", &slab_reduce);
  m.def("sample_episodes", &sample_episodes);
  m.def("step_control", &step_control);
}
