// Torch op registrations of the step-glue kernels (csrc/kernels/glue.hip): one-launch weight
// packing, the fused loss / accuracy / loss-gradient kernel and the multi-slab gradient
// reduce-scatter into the flat gradient buffer.  Python side: ops/glue.py.
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>
#include <torch/library.h>

#include <algorithm>
#include <vector>

#include "ina_launch.h"

namespace {

using at::Tensor;

void need(const Tensor& t, const char* op, const char* name, at::ScalarType dt) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), op, ": ", name, " must be a contiguous GPU tensor");
  TORCH_CHECK(t.scalar_type() == dt, op, ": ", name, " has dtype ", t.scalar_type(), ", expected ", dt);
}
hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

// in [A, B, C] fp32 contiguous -> [A, C, B] (bf16 if bf16 else fp32): the last two dims transposed
Tensor transpose12(const Tensor& in, bool bf16) {
  TORCH_CHECK(in.is_cuda() && in.is_contiguous() && in.scalar_type() == at::kFloat && in.dim() == 3,
              "ina.transpose12: in must be a contiguous fp32 [A, B, C] GPU tensor");
  const int64_t A = in.size(0), B = in.size(1), C = in.size(2);
  auto out = at::empty({A, C, B}, in.options().dtype(bf16 ? at::kBFloat16 : at::kFloat));
  TORCH_CHECK(ina::transpose12(in.data_ptr<float>(), out.data_ptr(), (int)A, (int)B, (int)C, bf16,
                               c10::hip::getCurrentHIPStream().stream()) == 0,
              "ina.transpose12: launch failed");
  return out;
}

void gather_pack(const Tensor& src, const Tensor& idx, int64_t nb, Tensor out_bf16, Tensor out_f32) {
  const char* op = "ina.gather_pack";
  need(src, op, "src", at::kFloat);
  need(idx, op, "idx", at::kInt);
  need(out_bf16, op, "out_bf16", at::kBFloat16);
  need(out_f32, op, "out_f32", at::kFloat);
  const int64_t ntot = idx.numel();
  TORCH_CHECK(nb >= 0 && nb <= ntot && out_bf16.numel() == nb && out_f32.numel() == ntot - nb,
              op, ": output sizes must split idx into [nb | rest]");
  TORCH_CHECK(src.numel() < (int64_t)1 << 31, op, ": src too large for int32 indices");
  TORCH_CHECK(ina::gather_pack(src.data_ptr<float>(), idx.data_ptr<int>(), (long)nb, (long)ntot, out_bf16.data_ptr(),
                               out_f32.data_ptr<float>(), stream()) == 0, op, ": launch failed");
}

// the same gather with a per-element affine map ma [2][ntot] (out = v * ma[0][i] + ma[1][i]); the
// indices must lie inside src (checked here once per call against the plan's maximum)
void gather_pack_affine(const Tensor& src, const Tensor& idx, int64_t nb, Tensor out_bf16, Tensor out_f32,
                        const Tensor& ma, int64_t idx_max) {
  const char* op = "ina.gather_pack_affine";
  need(src, op, "src", at::kFloat);
  need(idx, op, "idx", at::kInt);
  need(out_bf16, op, "out_bf16", at::kBFloat16);
  need(out_f32, op, "out_f32", at::kFloat);
  need(ma, op, "ma", at::kFloat);
  const int64_t ntot = idx.numel();
  TORCH_CHECK(nb >= 0 && nb <= ntot && out_bf16.numel() == nb && out_f32.numel() == ntot - nb,
              op, ": output sizes must split idx into [nb | rest]");
  TORCH_CHECK(ma.numel() == 2 * ntot, op, ": ma must be [2, ntot]");
  TORCH_CHECK(idx_max < src.numel() && src.numel() < (int64_t)1 << 31, op, ": index plan exceeds src");
  TORCH_CHECK(ina::gather_pack(src.data_ptr<float>(), idx.data_ptr<int>(), (long)nb, (long)ntot, out_bf16.data_ptr(),
                               out_f32.data_ptr<float>(), stream(), ma.data_ptr<float>()) == 0, op, ": launch failed");
}

// ragged record plan: inst int32 [S] (dataset rows), lengths int32 [NI] (valid lengths, <= L) ->
// (inst_sorted, perm, tlen [ceil(S/16)], slen) = the stable argsort of lengths[inst] and its derivatives
std::tuple<Tensor, Tensor, Tensor, Tensor> ragged_sort(const Tensor& inst, const Tensor& lengths, int64_t L) {
  const char* op = "ina.ragged_sort";
  need(inst, op, "inst", at::kInt);
  need(lengths, op, "lengths", at::kInt);
  TORCH_CHECK(L >= 0 && L <= ina::ragged_max_len(), op, ": L must be in [0, ", ina::ragged_max_len(), "]");
  const int64_t S = inst.numel();
  auto io = inst.options();
  auto perm = at::empty({S}, io), inst_s = at::empty({S}, io), slen = at::empty({S}, io);
  auto tlen = at::empty({(S + 15) / 16}, io);
  auto ws = at::empty({std::max<int64_t>(1, 2 * (L + 1) * (int64_t)ina::ragged_blocks(S))}, io);
  TORCH_CHECK(ina::ragged_sort(inst.data_ptr<int>(), lengths.data_ptr<int>(), (long)S, (int)L, ws.data_ptr<int>(),
                               perm.data_ptr<int>(), inst_s.data_ptr<int>(), slen.data_ptr<int>(),
                               tlen.data_ptr<int>(), stream()) == 0,
              op, ": launch failed");
  return {inst_s, perm, tlen, slen};
}

// probs [rows, N] fp32, labels int32 [rows]; writes dz [rows, N] and out [N + 3] =
// (loss, accuracy, db[0..N), db_total); part: workspace [blocks * 18].  ce: 0 the reference MSE, 1 softmax
// cross-entropy over the pre-sigmoid scores, 2 the NOTA-aware cross-entropy (an extra class of logit 0)
void head_loss(const Tensor& probs, const Tensor& labels, double scale, Tensor dz, Tensor out, Tensor part,
               int64_t blocks, int64_t ce) {
  const char* op = "ina.head_loss";
  need(probs, op, "probs", at::kFloat);
  need(labels, op, "labels", at::kInt);
  need(dz, op, "dz", at::kFloat);
  need(out, op, "out", at::kFloat);
  need(part, op, "part", at::kFloat);
  const int64_t N = probs.size(-1), rows = probs.numel() / N;
  TORCH_CHECK(N >= 1 && N <= 16, op, ": N must be in [1, 16]");
  TORCH_CHECK(labels.numel() == rows && dz.numel() == probs.numel() && out.numel() >= N + 3, op, ": shapes");
  TORCH_CHECK(blocks >= 1 && part.numel() >= blocks * ina::head_loss_part_floats(), op, ": workspace too small");
  TORCH_CHECK(ce >= 0 && ce <= 2, op, ": ce must be 0 (mse), 1 (ce) or 2 (ce_nota)");
  TORCH_CHECK(ina::head_loss(probs.data_ptr<float>(), labels.data_ptr<int>(), (long)rows, (int)N, (float)scale,
                             (int)ce, dz.data_ptr<float>(), out.data_ptr<float>(), part.data_ptr<float>(), (int)blocks,
                             stream()) == 0,
              op, ": launch failed");
}

// dst[map_j[i]] += sum_b src_j[b][i] (* scale_j[0] when scale_j is non-empty); deterministic.
// Returns the workspace floats it needs when ws is too small (call again with a larger ws).
int64_t slab_scatter_add(Tensor dst, const std::vector<Tensor>& srcs, const std::vector<Tensor>& maps,
                         const std::vector<int64_t>& nblks, const std::vector<Tensor>& scales, Tensor ws) {
  const char* op = "ina.slab_scatter_add";
  need(dst, op, "dst", at::kFloat);
  need(ws, op, "ws", at::kFloat);
  const size_t J = srcs.size();
  TORCH_CHECK(J >= 1 && J <= (size_t)ina::SLAB_MAX_JOBS && maps.size() == J && nblks.size() == J && scales.size() == J,
              op, ": 1..8 jobs with matching srcs / maps / nblks / scales");
  ina::SlabJobs jobs{};
  jobs.njobs = (int)J;
  long wsb = 0, bb = 0, fb = 0;
  for (size_t j = 0; j < J; ++j) {
    need(srcs[j], op, "src", at::kFloat);
    need(maps[j], op, "map", at::kInt);
    const int64_t n = maps[j].numel();
    TORCH_CHECK(n >= 1 && nblks[j] >= 1 && srcs[j].numel() == nblks[j] * n, op, ": slab ", j,
                " must be [nblk, map.numel()]");
    TORCH_CHECK(dst.numel() < ((int64_t)1 << 31), op, ": dst too large for int32 maps");
    jobs.src[j] = srcs[j].data_ptr<float>();
    jobs.map[j] = maps[j].data_ptr<int>();
    jobs.n[j] = (long)n;
    jobs.nblk[j] = (int)nblks[j];
    // chunks of ~32 slab rows (8 per wave): ~sqrt(nblk) chunks gave the wide, short dM slabs (32 x 160,000) 3,750
    // workgroups of ~5 rows each (launch-bound: 33-36 us for ~50 MB at the headline step)
    jobs.nch[j] = (int)std::min<int64_t>(256, std::max<int64_t>(1, (nblks[j] + 31) / 32));
    if (scales[j].numel() > 0) {
      need(scales[j], op, "scale", at::kFloat);
      jobs.scale[j] = scales[j].data_ptr<float>();
    }
    const long ncol = (long)((n + 63) / 64);
    // float4 columns for the partial sums when every row (slab and workspace) is 16-byte aligned
    jobs.vec[j] = (n % 4 == 0 && ((uintptr_t)jobs.src[j] & 15) == 0 && wsb % 4 == 0) ? 1 : 0;
    const long ncolp = jobs.vec[j] ? (long)((n + 255) / 256) : ncol;
    jobs.wsbase[j] = wsb;
    jobs.bbase[j] = bb;
    jobs.fbase[j] = fb;
    wsb += (long)jobs.nch[j] * (long)n;
    bb += ncolp * jobs.nch[j];
    fb += (long)((n + 255) / 256);   // finish: one thread per column
  }
  jobs.bbase[J] = bb;
  jobs.fbase[J] = fb;
  if (ws.numel() < wsb) return (int64_t)wsb;
  TORCH_CHECK(ina::slab_scatter(jobs, dst.data_ptr<float>(), ws.data_ptr<float>(), stream()) == 0, op,
              ": launch failed");
  return 0;
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(ina, m) {
  m.def("gather_pack", &gather_pack);
  m.def("transpose12", &transpose12);
  m.def("head_loss", &head_loss);
  m.def("ragged_sort", &ragged_sort);
  m.def("gather_pack_affine", &gather_pack_affine);
  m.def("slab_scatter_add", &slab_scatter_add);
}
