// Torch op registrations of the BERT encoder kernels (csrc/kernels/bert.hip), namespace torch.ops.ina.
// Host-side validation of every shape / dtype the kernel grids assume happens here, before launch.
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>
#include <torch/library.h>

#include <map>
#include <tuple>

#include "ina_launch.h"

namespace {

using at::Tensor;

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

void chk(const Tensor& t, const char* name, at::ScalarType dt) {
  TORCH_CHECK(t.is_cuda(), "ina.bert: ", name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), "ina.bert: ", name, " must be contiguous");
  TORCH_CHECK(t.scalar_type() == dt, "ina.bert: ", name, " has dtype ", t.scalar_type(), ", expected ", dt);
}
void launched(int rc, const char* what) {
  TORCH_CHECK(rc == 0, "ina.bert: ", what, " launch failed / unsupported configuration (rc=", rc, ")");
}
uint32_t thr_of(double kp) {
  const double t = kp * 4294967296.0;
  return t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
}
// same recipe as dropout_salt() in ina_common.h / models/bert.py::keep_mask
uint32_t salt_of(int64_t seed, int64_t stream_id) {
  return (uint32_t)((uint32_t)(seed & 0x7FFFFFFF) * 0x2545F491u + (uint32_t)stream_id * 0x3C6EF372u + 0x1234567u);
}
void check_hd(int64_t HD) {
  TORCH_CHECK(HD % 256 == 0 && HD >= 256 && HD <= 1024, "ina.bert: hidden width must be 256/512/768/1024, got ",
              HD);
}

// ------------------------------------------------------------------ embeddings + LN
std::tuple<Tensor, Tensor> bert_embed_ln_fwd(const Tensor& inst, const Tensor& ids, const Tensor& wemb,
                                             const Tensor& pemb, const Tensor& temb, const Tensor& gamma,
                                             const Tensor& beta, int64_t seed, double p) {
  chk(inst, "inst", at::kInt);
  chk(ids, "ids", at::kInt);
  for (auto* t : {&wemb, &pemb, &temb, &gamma, &beta}) chk(*t, "table", at::kFloat);
  const int64_t S = inst.size(0), L = ids.size(1), HD = wemb.size(1);
  check_hd(HD);
  TORCH_CHECK(pemb.size(0) >= L && pemb.size(1) == HD && temb.size(1) == HD, "ina.bert_embed_ln_fwd: tables");
  TORCH_CHECK(gamma.numel() == HD && beta.numel() == HD, "ina.bert_embed_ln_fwd: LN params");
  TORCH_CHECK(S * L * HD < (1LL << 32), "ina.bert_embed_ln_fwd: batch too large");
  auto y = at::empty({S * L, HD}, wemb.options().dtype(at::kBFloat16));
  auto stats = at::empty({S * L, 2}, wemb.options());
  if (S == 0) return {y, stats};
  ina::BertEmbArgs a{};
  a.inst = inst.data_ptr<int>();
  a.ids = ids.data_ptr<int>();
  a.S = (int)S;
  a.L = (int)L;
  a.HD = (int)HD;
  a.wemb = wemb.data_ptr<float>();
  a.pemb = pemb.data_ptr<float>();
  a.temb = temb.data_ptr<float>();
  a.gamma = gamma.data_ptr<float>();
  a.beta = beta.data_ptr<float>();
  a.y = y.data_ptr();
  a.stats = stats.data_ptr<float>();
  a.salt = salt_of(seed, 16);
  a.thr = thr_of(1.0 - p);
  a.inv_kp = (float)(1.0 / (1.0 - p));
  a.drop = p > 0.0 ? 1 : 0;
  launched(ina::embed_ln_fwd(a, stream()), "embed_ln_fwd");
  return {y, stats};
}

std::tuple<Tensor, Tensor> bert_embed_ln_bwd(const Tensor& dy, const Tensor& inst, const Tensor& ids,
                                             const Tensor& wemb, const Tensor& pemb, const Tensor& temb,
                                             const Tensor& gamma, const Tensor& stats, int64_t seed, double p,
                                             int64_t blocks) {
  chk(dy, "dy", at::kBFloat16);
  chk(inst, "inst", at::kInt);
  chk(ids, "ids", at::kInt);
  for (auto* t : {&wemb, &pemb, &temb, &gamma, &stats}) chk(*t, "table", at::kFloat);
  const int64_t S = inst.size(0), L = ids.size(1), HD = wemb.size(1);
  check_hd(HD);
  TORCH_CHECK(dy.size(0) == S * L && dy.size(1) == HD && stats.size(0) == S * L, "ina.bert_embed_ln_bwd: shapes");
  blocks = std::max<int64_t>(1, std::min<int64_t>(blocks > 0 ? blocks : 1024, (S * L + 3) / 4));
  auto dx = at::empty({S * L, HD}, wemb.options());
  auto slab = at::zeros({blocks, 2, HD}, wemb.options());
  if (S == 0) return {dx, slab};
  ina::BertEmbArgs a{};
  a.inst = inst.data_ptr<int>();
  a.ids = ids.data_ptr<int>();
  a.S = (int)S;
  a.L = (int)L;
  a.HD = (int)HD;
  a.blocks = (int)blocks;
  a.wemb = wemb.data_ptr<float>();
  a.pemb = pemb.data_ptr<float>();
  a.temb = temb.data_ptr<float>();
  a.gamma = gamma.data_ptr<float>();
  a.stats = stats.data_ptr<float>();
  a.dy = dy.data_ptr();
  a.dx = dx.data_ptr<float>();
  a.slab = slab.data_ptr<float>();
  a.salt = salt_of(seed, 16);
  a.thr = thr_of(1.0 - p);
  a.inv_kp = (float)(1.0 / (1.0 - p));
  a.drop = p > 0.0 ? 1 : 0;
  launched(ina::embed_ln_bwd(a, stream()), "embed_ln_bwd");
  return {dx, slab};
}

// ------------------------------------------------------------------ residual + dropout + LN
std::tuple<Tensor, Tensor> bert_ln_res_fwd(const Tensor& a_, const Tensor& res, const Tensor& gamma,
                                           const Tensor& beta, int64_t seed, int64_t stream_id, double p) {
  chk(a_, "a", at::kBFloat16);
  chk(res, "res", at::kBFloat16);
  chk(gamma, "gamma", at::kFloat);
  chk(beta, "beta", at::kFloat);
  const int64_t T = a_.size(0), HD = a_.size(1);
  check_hd(HD);
  TORCH_CHECK(res.sizes() == a_.sizes() && gamma.numel() == HD && beta.numel() == HD, "ina.bert_ln_res_fwd: shapes");
  TORCH_CHECK(T * HD < (1LL << 32), "ina.bert_ln_res_fwd: batch too large");
  auto y = at::empty_like(a_);
  auto stats = at::empty({T, 2}, gamma.options());
  if (T == 0) return {y, stats};
  ina::BertLnArgs a{};
  a.a = a_.data_ptr();
  a.res = res.data_ptr();
  a.gamma = gamma.data_ptr<float>();
  a.beta = beta.data_ptr<float>();
  a.y = y.data_ptr();
  a.stats = stats.data_ptr<float>();
  a.T = (int)T;
  a.HD = (int)HD;
  a.salt = salt_of(seed, stream_id);
  a.thr = thr_of(1.0 - p);
  a.inv_kp = (float)(1.0 / (1.0 - p));
  a.drop = p > 0.0 ? 1 : 0;
  launched(ina::ln_res_fwd(a, stream()), "ln_res_fwd");
  return {y, stats};
}

std::tuple<Tensor, Tensor, Tensor> bert_ln_res_bwd(const Tensor& dy, const Tensor& a_, const Tensor& res,
                                                   const Tensor& gamma, const Tensor& stats, int64_t seed,
                                                   int64_t stream_id, double p, int64_t blocks) {
  chk(dy, "dy", at::kBFloat16);
  chk(a_, "a", at::kBFloat16);
  chk(res, "res", at::kBFloat16);
  chk(gamma, "gamma", at::kFloat);
  chk(stats, "stats", at::kFloat);
  const int64_t T = a_.size(0), HD = a_.size(1);
  check_hd(HD);
  TORCH_CHECK(dy.sizes() == a_.sizes() && res.sizes() == a_.sizes() && stats.size(0) == T,
              "ina.bert_ln_res_bwd: shapes");
  blocks = std::max<int64_t>(1, std::min<int64_t>(blocks > 0 ? blocks : 1024, (T + 3) / 4));
  auto dres = at::empty_like(a_);
  auto da = at::empty_like(a_);
  // [blocks][d gamma | d beta | column sums of da]; every block writes its whole row
  auto slab = T == 0 ? at::zeros({blocks, 3, HD}, gamma.options()) : at::empty({blocks, 3, HD}, gamma.options());
  if (T == 0) return {dres, da, slab};
  ina::BertLnArgs a{};
  a.a = a_.data_ptr();
  a.res = res.data_ptr();
  a.gamma = gamma.data_ptr<float>();
  a.stats = stats.data_ptr<float>();
  a.dy = dy.data_ptr();
  a.dres = dres.data_ptr();
  a.da = da.data_ptr();
  a.slab = slab.data_ptr<float>();
  a.T = (int)T;
  a.HD = (int)HD;
  a.blocks = (int)blocks;
  a.salt = salt_of(seed, stream_id);
  a.thr = thr_of(1.0 - p);
  a.inv_kp = (float)(1.0 / (1.0 - p));
  a.drop = p > 0.0 ? 1 : 0;
  launched(ina::ln_res_bwd(a, stream()), "ln_res_bwd");
  return {dres, da, slab};
}

// ------------------------------------------------------------------ bias + GELU
Tensor bert_bias_gelu_fwd(const Tensor& x, const Tensor& b) {
  chk(x, "x", at::kBFloat16);
  chk(b, "b", at::kFloat);
  const int64_t T = x.size(0), I = x.size(1);
  TORCH_CHECK(I % 8 == 0 && b.numel() == I, "ina.bert_bias_gelu_fwd: I must be a multiple of 8 and b [I]");
  auto y = at::empty_like(x);
  if (T == 0) return y;
  launched(ina::bias_gelu_fwd(x.data_ptr(), b.data_ptr<float>(), y.data_ptr(), T, (int)I, stream()), "bias_gelu_fwd");
  return y;
}

std::tuple<Tensor, Tensor> bert_bias_gelu_bwd(const Tensor& dy, const Tensor& x, const Tensor& b, int64_t blocks) {
  chk(dy, "dy", at::kBFloat16);
  chk(x, "x", at::kBFloat16);
  chk(b, "b", at::kFloat);
  const int64_t T = x.size(0), I = x.size(1);
  TORCH_CHECK(dy.sizes() == x.sizes() && I % 8 == 0 && I / 8 <= 1024 && b.numel() == I,
              "ina.bert_bias_gelu_bwd: shapes");
  blocks = std::max<int64_t>(1, std::min<int64_t>(blocks > 0 ? blocks : 1024, T));
  auto dx = at::empty_like(x);
  // every launched block writes its whole slab row
  auto slab = T == 0 ? at::zeros({blocks, I}, b.options()) : at::empty({blocks, I}, b.options());
  if (T == 0) return {dx, slab};
  launched(ina::bias_gelu_bwd(dy.data_ptr(), x.data_ptr(), b.data_ptr<float>(), dx.data_ptr(),
                              slab.data_ptr<float>(), (int)T, (int)I, (int)blocks, stream()),
           "bias_gelu_bwd");
  return {dx, slab};
}

// ------------------------------------------------------------------ own GEMM (gemm.hip)
// y = x W^T with epilogue epi: 0 -> (y [+ b]), 1 -> (gelu(y + b), pre-activation aux), 2 -> (y * gelu'(aux),
// bias-gradient column-sum slab [2 ceil(M/256)][N])
std::tuple<Tensor, Tensor> bert_gemm(const Tensor& x, const Tensor& w, const c10::optional<Tensor>& b,
                                     const c10::optional<Tensor>& aux, int64_t epi) {
  // x may be a column slice of wider rows (stride(1) == 1, row stride = lda)
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 2 && x.stride(1) == 1 &&
                  x.stride(0) >= x.size(1),
              "ina.bert_gemm: x must be a bf16 GPU matrix with unit column stride");
  chk(w, "w", at::kBFloat16);
  TORCH_CHECK(w.dim() == 2 && x.size(1) == w.size(1), "ina.bert_gemm: x [M, K], w [N, K]");
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0), lda = x.stride(0);
  TORCH_CHECK(N % 8 == 0 && K % 64 == 0 && K >= 64, "ina.bert_gemm: N must be a multiple of 8, K of 64");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && lda % 8 == 0,
              "ina.bert_gemm: x must start 16-byte aligned with a row stride that is a multiple of 8");
  TORCH_CHECK(M * lda * 2 < (1LL << 31) && N * K * 2 < (1LL << 31), "ina.bert_gemm: operand too large");
  TORCH_CHECK(epi >= 0 && epi <= 2, "ina.bert_gemm: epi must be 0, 1 or 2");
  const float* bp = nullptr;
  if (b.has_value() && b->defined()) {
    chk(*b, "b", at::kFloat);
    TORCH_CHECK(b->numel() == N, "ina.bert_gemm: b must be [N]");
    bp = b->data_ptr<float>();
  }
  TORCH_CHECK(epi != 1 || bp != nullptr, "ina.bert_gemm: epi 1 needs the bias");
  auto y = at::empty({M, N}, x.options());
  Tensor ax, slab;
  if (epi == 0) ax = at::empty({0}, x.options());
  if (epi == 1) ax = at::empty({M, N}, x.options());
  if (epi == 2) {
    TORCH_CHECK(aux.has_value() && aux->defined(), "ina.bert_gemm: epi 2 needs aux");
    ax = *aux;
    chk(ax, "aux", at::kBFloat16);
    TORCH_CHECK(ax.size(0) == M && ax.size(1) == N, "ina.bert_gemm: aux must be [M, N]");
    slab = at::empty({2 * ((M + 255) / 256), N}, x.options().dtype(at::kFloat));
  }
  if (M == 0) return {y, epi == 2 ? slab.zero_() : ax};
  launched(ina::gemm_bf16_nt(x.data_ptr(), (int)lda, w.data_ptr(), (int)K, (int)M, (int)N, (int)K, bp, y.data_ptr(),
                             (int)N, epi != 0 ? ax.data_ptr() : nullptr, (int)N,
                             slab.defined() ? slab.data_ptr<float>() : nullptr, (int)epi, stream()),
           "gemm_bf16_nt");
  return {y, epi == 2 ? slab : ax};
}

// zero bytes for the K-major operands' rows past K (one small buffer per device)
const void* zero16(const Tensor& like) {
  static thread_local std::map<int, Tensor> zeros;
  const int dev = like.get_device();
  auto it = zeros.find(dev);
  if (it == zeros.end()) it = zeros.emplace(dev, at::zeros({64}, like.options().dtype(at::kFloat))).first;
  return it->second.data_ptr();
}

// y = a b with b K-major (a [M, K], b [K, N]; dx = dy W for a torch-layout weight W [out][in]).  epi 0: plain;
// 2: y * gelu'(aux) with the column-sum slab [2 ceil(M/256)][N] (FFN dgrad); 4: y added into res IN PLACE (res
// is returned).  Returns (y, slab-or-empty).
std::tuple<Tensor, Tensor> gemm_nn(const Tensor& a, const Tensor& b, const c10::optional<Tensor>& aux,
                                   const c10::optional<Tensor>& res, int64_t epi) {
  chk(a, "a", at::kBFloat16);
  chk(b, "b", at::kBFloat16);
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && a.size(1) == b.size(0), "ina.gemm_nn: a [M, K], b [K, N]");
  const int64_t M = a.size(0), K = a.size(1), N = b.size(1);
  TORCH_CHECK(N % 8 == 0 && K % 64 == 0 && K >= 64, "ina.gemm_nn: N must be a multiple of 8, K of 64");
  TORCH_CHECK(M < (1LL << 31), "ina.gemm_nn: too many rows");
  TORCH_CHECK(epi == 0 || epi == 2 || epi == 4, "ina.gemm_nn: epi must be 0, 2 or 4");
  Tensor y, ax, slab;
  if (epi == 4) {
    TORCH_CHECK(res.has_value() && res->defined(), "ina.gemm_nn: epi 4 needs res");
    y = *res;
    chk(y, "res", at::kBFloat16);
    TORCH_CHECK(y.size(0) == M && y.size(1) == N, "ina.gemm_nn: res must be [M, N]");
  } else {
    y = at::empty({M, N}, a.options());
  }
  if (epi == 2) {
    TORCH_CHECK(aux.has_value() && aux->defined(), "ina.gemm_nn: epi 2 needs aux");
    ax = *aux;
    chk(ax, "aux", at::kBFloat16);
    TORCH_CHECK(ax.size(0) == M && ax.size(1) == N, "ina.gemm_nn: aux must be [M, N]");
    slab = at::empty({2 * ((M + 255) / 256), N}, a.options().dtype(at::kFloat));
  } else {
    slab = at::empty({0}, a.options().dtype(at::kFloat));
  }
  if (M == 0) return {y, epi == 2 ? slab.zero_() : slab};
  launched(ina::gemm_bf16(1, a.data_ptr(), (int)K, b.data_ptr(), (int)N, (int)M, (int)N, (int)K, nullptr,
                          y.data_ptr(), (int)N, epi == 2 ? ax.data_ptr() : nullptr, (int)N,
                          epi == 2 ? slab.data_ptr<float>() : nullptr, zero16(a), (int)epi, 1, stream()),
           "gemm_nn");
  return {y, slab};
}

// Weight-gradient split-K GEMM: slabs [splits, M, N] fp32 with slabs[s] = sum over the K rows of split s of
// a[k, :]^T b[k, :] (a [K, M], b [K, N] bf16, K = tokens; splits <= 0: one round of workgroups).  The caller sums
// the slabs in a fixed order (ina.slab_reduce straight into the flat gradient).
Tensor gemm_wgrad(const Tensor& a, const Tensor& b, int64_t splits) {
  TORCH_CHECK(a.is_cuda() && b.is_cuda() && a.scalar_type() == at::kBFloat16 && b.scalar_type() == at::kBFloat16,
              "ina.gemm_wgrad: bf16 GPU operands");
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && a.size(0) == b.size(0), "ina.gemm_wgrad: a [K, M], b [K, N]");
  TORCH_CHECK(a.stride(1) == 1 && b.stride(1) == 1, "ina.gemm_wgrad: unit column stride");
  const int64_t K = a.size(0), M = a.size(1), N = b.size(1), lda = a.stride(0), ldb = b.stride(0);
  TORCH_CHECK(M % 8 == 0 && N % 8 == 0 && M > 0 && N > 0, "ina.gemm_wgrad: M and N must be multiples of 8");
  TORCH_CHECK(lda % 8 == 0 && ldb % 8 == 0 && reinterpret_cast<uintptr_t>(a.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(b.data_ptr()) % 16 == 0,
              "ina.gemm_wgrad: 16-byte aligned rows");
  if (splits <= 0) splits = ina::gemm_wgrad_splits((int)M, (int)N, (int)K);
  const int64_t ks = (K + 63) / 64;
  if (splits > ks) splits = ks > 0 ? ks : 1;
  while (splits > 1 && (splits - 1) * ((ks + splits - 1) / splits) >= ks) --splits;
  auto out = at::empty({splits, M, N}, a.options().dtype(at::kFloat));
  if (K == 0) return out.zero_();
  launched(ina::gemm_bf16(2, a.data_ptr(), (int)lda, b.data_ptr(), (int)ldb, (int)M, (int)N, (int)K, nullptr,
                          out.data_ptr(), (int)N, nullptr, 0, nullptr, zero16(a), 5, (int)splits, stream()),
           "gemm_wgrad");
  return out;
}

// ------------------------------------------------------------------ fused attention
void mha_checks(const Tensor& qkv, const Tensor& inst, const Tensor& mask, int64_t L, int64_t nh) {
  chk(qkv, "qkv", at::kBFloat16);
  chk(inst, "inst", at::kInt);
  chk(mask, "mask", at::kInt);
  TORCH_CHECK(ina::mha_lp((int)L) > 0, "ina.bert_mha: L must be <= 128, got ", L);
  TORCH_CHECK(mask.size(1) == L, "ina.bert_mha: mask must be [NI, L]");
  TORCH_CHECK(qkv.size(0) == inst.size(0) * L && qkv.size(1) == 3 * 64 * nh, "ina.bert_mha: qkv must be [S*L, 3*nh*64]");
  TORCH_CHECK(inst.size(0) * nh * L * L < (1LL << 32), "ina.bert_mha: dropout index range");
}

std::tuple<Tensor, Tensor> bert_mha_fwd(const Tensor& qkv, const Tensor& inst, const Tensor& mask, int64_t L,
                                        int64_t nh, int64_t seed, int64_t stream_id, double p) {
  mha_checks(qkv, inst, mask, L, nh);
  const int64_t S = inst.size(0);
  const int LP = ina::mha_lp((int)L);
  auto ctx = at::empty({S * L, 64 * nh}, qkv.options());
  auto lse = at::empty({S, nh, LP}, qkv.options().dtype(at::kFloat));
  if (S == 0) return {ctx, lse};
  ina::BertMhaArgs a{};
  a.qkv = qkv.data_ptr();
  a.inst = inst.data_ptr<int>();
  a.mask = mask.data_ptr<int>();
  a.S = (int)S;
  a.L = (int)L;
  a.nh = (int)nh;
  a.ctx = ctx.data_ptr();
  a.lse = lse.data_ptr<float>();
  a.salt = salt_of(seed, stream_id);
  a.thr = thr_of(1.0 - p);
  a.inv_kp = (float)(1.0 / (1.0 - p));
  a.drop = p > 0.0 ? 1 : 0;
  launched(ina::mha_fwd(a, stream()), "mha_fwd");
  return {ctx, lse};
}

// -> (dqkv [S*L, 3*nh*64] bf16, bsum [S*nh, 3, 64] fp32 per-(sequence, head) column sums of dQ | dK | dV:
//     the QKV bias gradient is bsum.view(S, nh, 3, 64).sum(0).transpose(0, 1))
std::tuple<Tensor, Tensor> bert_mha_bwd(const Tensor& qkv, const Tensor& ctx, const Tensor& dctx, const Tensor& lse,
                                        const Tensor& inst, const Tensor& mask, int64_t L, int64_t nh, int64_t seed,
                                        int64_t stream_id, double p) {
  mha_checks(qkv, inst, mask, L, nh);
  chk(ctx, "ctx", at::kBFloat16);
  chk(dctx, "dctx", at::kBFloat16);
  chk(lse, "lse", at::kFloat);
  const int64_t S = inst.size(0);
  TORCH_CHECK(ctx.size(0) == S * L && ctx.size(1) == 64 * nh && dctx.sizes() == ctx.sizes(), "ina.bert_mha_bwd: ctx");
  TORCH_CHECK(lse.numel() == S * nh * ina::mha_lp((int)L), "ina.bert_mha_bwd: lse");
  auto dqkv = at::empty_like(qkv);
  auto bsum = (S == 0 ? at::zeros({S * nh, 3, 64}, lse.options()) : at::empty({S * nh, 3, 64}, lse.options()));
  if (S == 0) return {dqkv, bsum};
  ina::BertMhaArgs a{};
  a.qkv = qkv.data_ptr();
  a.inst = inst.data_ptr<int>();
  a.mask = mask.data_ptr<int>();
  a.S = (int)S;
  a.L = (int)L;
  a.nh = (int)nh;
  a.ctx = ctx.data_ptr();
  a.lse = lse.data_ptr<float>();
  a.dctx = dctx.data_ptr();
  a.dqkv = dqkv.data_ptr();
  a.bsum = bsum.data_ptr<float>();
  a.salt = salt_of(seed, stream_id);
  a.thr = thr_of(1.0 - p);
  a.inv_kp = (float)(1.0 / (1.0 - p));
  a.drop = p > 0.0 ? 1 : 0;
  launched(ina::mha_bwd(a, stream()), "mha_bwd");
  return {dqkv, bsum};
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(ina, m) {
  m.def("bert_embed_ln_fwd", &bert_embed_ln_fwd);
  m.def("bert_embed_ln_bwd", &bert_embed_ln_bwd);
  m.def("bert_ln_res_fwd", &bert_ln_res_fwd);
  m.def("bert_ln_res_bwd", &bert_ln_res_bwd);
  m.def("bert_bias_gelu_fwd", &bert_bias_gelu_fwd);
  m.def("bert_bias_gelu_bwd", &bert_bias_gelu_bwd);
  m.def("bert_gemm", &bert_gemm);
  m.def("gemm_nn", &gemm_nn);
  m.def("gemm_wgrad", &gemm_wgrad);
  m.def("bert_mha_fwd", &bert_mha_fwd);
  m.def("bert_mha_bwd", &bert_mha_bwd);
}
