// Step-glue kernels: everything between the model's big kernels that would otherwise be a string
// of ~80 small PyTorch launches per training step (weight re-packing, loss / accuracy / loss
// gradient, slab reductions, transposes and the adds into the flat gradient buffer).  At ~5 us of
// GPU time per tiny launch those cost ~15% of the BiLSTM step; here they are 5 launches.
//
//  gather_pack : every per-step MFMA weight pack (LSTM gate/transpose packs, attention W1 packs,
//                NTN M / w packs, stacked LSTM biases) in ONE gather from the flat parameter buffer
//                with a precomputed int32 index (-1 -> 0); bf16 region then fp32 region.
//  head_loss   : MSE loss vs one-hot labels (tf.one_hot semantics: NOTA -> zero row), accuracy
//                (first-max argmax == label), the pre-sigmoid gradient dz = dL/dp * p(1-p) for the
//                NTN backward and the bias gradient sum_rows dz (loss_type ce: softmax cross-entropy
//                over the relation scores instead).  Deterministic two-level reduce: per-block
//                partials, then a one-block launch sums them with a fixed shuffle tree.
//  slab_scatter: sum per-block gradient slabs over their blocks (chunked across workgroups, then
//                the chunk partials summed in chunk order by a second launch) and ADD the
//                result into the flat gradient at an int32 map (-1 = skip); transposes and pos-table
//                crops are encoded in the maps.  Up to 8 slabs per launch.
// Reference semantics: model/graph.py:88-95 (MSE on one-hot, accuracy), model/base.py (grads).
#include "ina_common.h"
#include "ina_launch.h"

using namespace ina;

namespace {

// ma (optional): [2][ntot] per-element affine map out = v * ma[i] + ma[ntot + i] (the wide path's
// exp2 gate pre-scales and the TF forget bias, ops/wide_packs.py)
__global__ __launch_bounds__(256) void gather_pack_kernel(const float* __restrict__ src, const int* __restrict__ idx,
                                                          long nb, long ntot, unsigned short* __restrict__ outb,
                                                          float* __restrict__ outf, const float* __restrict__ ma) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < ntot; i += (long)gridDim.x * 256) {
    const int k = idx[i];
    float v = k >= 0 ? src[k] : 0.f;
    if (ma != nullptr) v = v * ma[i] + ma[ntot + i];
    if (i < nb)
      outb[i] = f2bf(v);
    else
      outf[i - nb] = v;
  }
}

constexpr int HL_NMAX = 16;
constexpr int HL_PART = 2 + HL_NMAX;   // loss, correct, db[16]

constexpr float CE_ODDS_EPS = 1e-7f;   // models/reference.py::CE_ODDS_EPS
constexpr float CE_P_MIN = 1e-30f;     // models/reference.py::CE_P_MIN (z >= -69: no -inf / NaN)

// rows = E * NQ; probs/dz [rows][N]; labels int32 [rows] (N = NOTA).
// ce = 0: MSE on the sigmoid scores vs one-hot (reference).  ce = 1: softmax cross-entropy over the
// pre-sigmoid scores z = log p - log(1 - p) (models/reference.py::ce_loss); NOTA rows contribute 0.
// ce = 2: NOTA-aware cross-entropy (FewRel 2.0 training with none-of-the-above queries,
// models/reference.py::ce_nota_loss): the softmax runs over the N scores plus a NOTA class whose logit is
// fixed at 0 (the score 0.5); a NOTA row's target is that class, so it pushes every z_c below 0.  The
// accuracy counts a row as NOTA when its best score is below 0.5.
// NT: compile-time class count (0 = runtime N <= HL_NMAX): the 5-way instantiation loads each row's
// scores unconditionally and reduces 5 bias-gradient columns instead of 16
template <int NT>
__global__ __launch_bounds__(256) void head_loss_kernel(const float* __restrict__ probs,
                                                        const int* __restrict__ labels, long rows, int N,
                                                        float scale, int ce, float* __restrict__ dz,
                                                        float* __restrict__ part) {
  constexpr int HL_NMAX = NT > 0 ? NT : ::HL_NMAX;
  if constexpr (NT > 0) N = NT;
  __shared__ float red[4][HL_PART];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float ls = 0.f, cor = 0.f, db[HL_NMAX];
#pragma unroll
  for (int c = 0; c < HL_NMAX; ++c) db[c] = 0.f;
  for (long r = (long)blockIdx.x * 256 + threadIdx.x; r < rows; r += (long)gridDim.x * 256) {
    const int lab = labels[r];
    const float* pr = probs + r * N;
    float best = -1.f;
    int arg = 0;
    float pv[HL_NMAX];
#pragma unroll
    for (int c = 0; c < HL_NMAX; ++c) {
      pv[c] = c < N ? pr[c] : 0.f;
      if (c < N && pv[c] > best) {   // first maximum (torch.argmax)
        best = pv[c];
        arg = c;
      }
    }
    const bool nota = ce == 2;
    cor += ((nota && best < 0.5f ? N : arg) == lab) ? 1.f : 0.f;
    if (ce) {
      float z[HL_NMAX], zm = nota ? 0.f : -INFINITY, zl = 0.f;   // nota: the fixed NOTA logit 0 (zl if lab == N)
#pragma unroll
      for (int c = 0; c < HL_NMAX; ++c) {
        z[c] = c < N ? logf(fmaxf(pv[c], CE_P_MIN)) - logf(fmaxf(1.f - pv[c], CE_ODDS_EPS)) : -INFINITY;
        zm = fmaxf(zm, z[c]);
        if (c == lab) zl = z[c];
      }
      float s = nota ? expf(-zm) : 0.f;
#pragma unroll
      for (int c = 0; c < HL_NMAX; ++c) {
        z[c] = c < N ? expf(z[c] - zm) : 0.f;
        s += z[c];
      }
      const bool has = lab < N || nota;
      const float inv = 1.f / s;
#pragma unroll
      for (int c = 0; c < HL_NMAX; ++c) {
        if (c < N) {
          const float g = has ? scale * (z[c] * inv - (c == lab ? 1.f : 0.f)) : 0.f;
          dz[r * N + c] = g;
          db[c] += g;
        }
      }
      if (has) ls += logf(s) + zm - zl;   // -log softmax_lab
    } else {
#pragma unroll
      for (int c = 0; c < HL_NMAX; ++c) {
        if (c < N) {
          const float p = pv[c];
          const float d = p - (c == lab ? 1.f : 0.f);
          ls += d * d;
          const float g = 2.f * scale * d * p * (1.f - p);
          dz[r * N + c] = g;
          db[c] += g;
        }
      }
    }
  }
  ls = wave_sum(ls);
  cor = wave_sum(cor);
#pragma unroll
  for (int c = 0; c < HL_NMAX; ++c) db[c] = wave_sum(db[c]);
  if (lane == 0) {
    red[wave][0] = ls;
    red[wave][1] = cor;
#pragma unroll
    for (int c = 0; c < ::HL_NMAX; ++c) red[wave][2 + c] = c < HL_NMAX ? db[c < HL_NMAX ? c : 0] : 0.f;
  }
  __syncthreads();
  if (threadIdx.x < HL_PART)
    part[(long)blockIdx.x * HL_PART + threadIdx.x] =
        (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
}

// second launch (the kernel boundary orders it after every partial): per column, lane b loads block
// b's partial (nblocks <= 64: ONE load latency instead of a 64-long dependent chain) and a fixed
// shuffle tree sums them -- deterministic
__global__ __launch_bounds__(256) void head_loss_finish_kernel(const float* __restrict__ part, int nblocks, long rows,
                                                               int N, float scale, float* __restrict__ out) {
  __shared__ float tot[HL_PART];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int col = wave; col < HL_PART; col += 4) {
    float s = 0.f;
    for (int b = lane; b < nblocks; b += 64) s += part[(long)b * HL_PART + col];
    s = wave_sum(s);
    if (lane == 0) tot[col] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    out[0] = tot[0] * scale;
    out[1] = tot[1] / (float)(rows > 0 ? rows : 1);
    float t = 0.f;
    for (int c = 0; c < N; ++c) {
      out[2 + c] = tot[2 + c];
      t += tot[2 + c];
    }
    out[2 + N] = t;
  }
}

// slab_scatter: column sums of each job's [nblk][n] slab, added into dst at the job's map.
// Launch 1 (slab_partial): workgroup = (job, 64-column group, chunk of rows); its 4 waves take
// the chunk's rows round-robin (lanes = columns, coalesced 256-byte rows, 4 loads in flight per
// lane) and combine in wave order -> ws[wsbase + chunk * n + col].  Launch 2 (slab_finish):
// workgroup = (job, 64-column group); the waves split the chunk partials, combine in wave order,
// scale, and add at the map.  Fixed summation order everywhere: deterministic.  (Two launches
// rather than a last-block ticket: a device-scope fence per workgroup is an L2 write-back on
// gfx950.)
INA_DEVICE int find_job(const long* base, int njobs, long x) {
  int j = 0;
  while (j + 1 < njobs && x >= base[j + 1]) ++j;
  return j;
}

__global__ __launch_bounds__(256) void slab_partial_kernel(SlabJobs jobs, float* __restrict__ ws) {
  __shared__ float red[4][256];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long bid = blockIdx.x;
  const int j = find_job(jobs.bbase, jobs.njobs, bid);
  const long loc = bid - jobs.bbase[j];
  const bool vec = jobs.vec[j] != 0;   // uniform
  const int ncol = (int)((jobs.n[j] + (vec ? 255 : 63)) / (vec ? 256 : 64)), nch = jobs.nch[j];
  const int cg = (int)(loc % ncol), ch = (int)(loc / ncol);
  const long n = jobs.n[j];
  const int nb = jobs.nblk[j];
  const int b0 = (int)(((long)nb * ch) / nch), b1 = (int)(((long)nb * (ch + 1)) / nch);
  if (vec) {   // lane = 4 consecutive columns (16-byte loads: a wave reads 1 KiB per row), the same row order per column
    const long c4 = (long)cg * 256 + 4 * lane;
    f32x4_t a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0, a2 = a0, a3 = a0;
    if (c4 < n) {
      const float* s = jobs.src[j] + c4;
      int b = b0 + wave;
      for (; b + 12 < b1; b += 16) {
        a0 += *reinterpret_cast<const f32x4_t*>(s + (long)b * n);
        a1 += *reinterpret_cast<const f32x4_t*>(s + (long)(b + 4) * n);
        a2 += *reinterpret_cast<const f32x4_t*>(s + (long)(b + 8) * n);
        a3 += *reinterpret_cast<const f32x4_t*>(s + (long)(b + 12) * n);
      }
      for (; b < b1; b += 4) a0 += *reinterpret_cast<const f32x4_t*>(s + (long)b * n);
    }
    *reinterpret_cast<f32x4_t*>(&red[wave][4 * lane]) = (a0 + a1) + (a2 + a3);
    __syncthreads();
    if (wave == 0 && c4 < n) {
      const f32x4_t r0 = *reinterpret_cast<const f32x4_t*>(&red[0][4 * lane]);
      const f32x4_t r1 = *reinterpret_cast<const f32x4_t*>(&red[1][4 * lane]);
      const f32x4_t r2 = *reinterpret_cast<const f32x4_t*>(&red[2][4 * lane]);
      const f32x4_t r3 = *reinterpret_cast<const f32x4_t*>(&red[3][4 * lane]);
      *reinterpret_cast<f32x4_t*>(ws + jobs.wsbase[j] + (long)ch * n + c4) = (r0 + r1) + (r2 + r3);
    }
    return;
  }
  const long col = (long)cg * 64 + lane;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (col < n) {
    const float* s = jobs.src[j] + col;
    int b = b0 + wave;
    for (; b + 12 < b1; b += 16) {
      a0 += s[(long)b * n];
      a1 += s[(long)(b + 4) * n];
      a2 += s[(long)(b + 8) * n];
      a3 += s[(long)(b + 12) * n];
    }
    for (; b < b1; b += 4) a0 += s[(long)b * n];
  }
  red[wave][lane] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (wave == 0 && col < n)
    ws[jobs.wsbase[j] + (long)ch * n + col] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
}

__global__ __launch_bounds__(256) void slab_finish_kernel(SlabJobs jobs, const float* __restrict__ ws,
                                                          float* __restrict__ dst) {
  // one thread per column: its nch chunk partials in 4 interleaved accumulators (fixed order), then the
  // scatter-add (4-wave workgroups per 64 columns left 3 waves idle at the 1-2 chunks of the wide slabs)
  const long bid = blockIdx.x;
  const int j = find_job(jobs.fbase, jobs.njobs, bid);
  const long n = jobs.n[j];
  const long col = (bid - jobs.fbase[j]) * 256 + threadIdx.x;
  if (col >= n) return;
  const float* w = ws + jobs.wsbase[j] + col;
  const int nch = jobs.nch[j];
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int c = 0;
  for (; c + 3 < nch; c += 4) {
    a0 += w[(long)c * n];
    a1 += w[(long)(c + 1) * n];
    a2 += w[(long)(c + 2) * n];
    a3 += w[(long)(c + 3) * n];
  }
  for (; c < nch; ++c) a0 += w[(long)c * n];
  const int m = jobs.map[j][col];
  if (m >= 0) {
    float s = (a0 + a1) + (a2 + a3);
    if (jobs.scale[j]) s *= jobs.scale[j][0];
    dst[m] += s;
  }
}

// out[a][c][b] = in[a][b][c] (fp32 in, fp32 or bf16 out): the wide NTN head's M <-> M' layouts
// ([H][H][h] <-> [H][h][H]).  32 x 32 tiles through LDS (row stride 33: conflict-free column reads), coalesced
// reads along c and writes along b (torch's generic permute copy ran these at ~1.3 TB/s, 40 us per direction).
template <bool BF>
__global__ __launch_bounds__(256) void transpose12_kernel(const float* __restrict__ in, void* __restrict__ out, int B,
                                                          int C) {
  __shared__ float tile[32][33];
  const int a = blockIdx.z, b0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;   // 32 x 8
  const float* src = in + (size_t)a * B * C;
#pragma unroll
  for (int k = 0; k < 32; k += 8) {
    const int b = b0 + ty + k, c = c0 + tx;
    tile[ty + k][tx] = (b < B && c < C) ? src[(size_t)b * C + c] : 0.f;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 32; k += 8) {
    const int c = c0 + ty + k, b = b0 + tx;
    if (b < B && c < C) {
      const size_t o = (size_t)a * B * C + (size_t)c * B + b;
      const float v = tile[tx][ty + k];
      if constexpr (BF)
        static_cast<unsigned short*>(out)[o] = f2bf(v);
      else
        static_cast<float*>(out)[o] = v;
    }
  }
}

}  // namespace

namespace ina {

int transpose12(const float* in, void* out, int A, int B, int C, bool bf16, hipStream_t st) {
  if (A <= 0 || B <= 0 || C <= 0) return 0;
  if (A > 65535) return -1;
  const dim3 grid((C + 31) / 32, (B + 31) / 32, A);
  if (bf16)
    hipLaunchKernelGGL(transpose12_kernel<true>, grid, dim3(256), 0, st, in, out, B, C);
  else
    hipLaunchKernelGGL(transpose12_kernel<false>, grid, dim3(256), 0, st, in, out, B, C);
  INA_CHECK_LAUNCH();
  return 0;
}

int gather_pack(const float* src, const int* idx, long nb, long ntot, void* outb, float* outf, hipStream_t st,
                const float* ma) {
  if (ntot <= 0) return 0;
  long g = (ntot + 255) / 256;
  if (g > 2048) g = 2048;
  hipLaunchKernelGGL(gather_pack_kernel, dim3((unsigned)g), dim3(256), 0, st, src, idx, nb, ntot,
                     (unsigned short*)outb, outf, ma);
  INA_CHECK_LAUNCH();
  return 0;
}

int head_loss(const float* probs, const int* labels, long rows, int N, float scale, int ce, float* dz, float* out,
              float* part, int blocks, hipStream_t st) {
  if (N > HL_NMAX || rows <= 0) return -1;
  if (N == 5)
    hipLaunchKernelGGL(head_loss_kernel<5>, dim3(blocks), dim3(256), 0, st, probs, labels, rows, N, scale, ce, dz, part);
  else
    hipLaunchKernelGGL(head_loss_kernel<0>, dim3(blocks), dim3(256), 0, st, probs, labels, rows, N, scale, ce, dz, part);
  INA_CHECK_LAUNCH();
  hipLaunchKernelGGL(head_loss_finish_kernel, dim3(1), dim3(256), 0, st, part, blocks, rows, N, scale, out);
  INA_CHECK_LAUNCH();
  return 0;
}

int head_loss_part_floats() { return HL_PART; }

int slab_scatter(const SlabJobs& jobs, float* dst, float* ws, hipStream_t st) {
  const long nb1 = jobs.bbase[jobs.njobs], nb2 = jobs.fbase[jobs.njobs];
  if (nb2 <= 0) return 0;
  hipLaunchKernelGGL(slab_partial_kernel, dim3((unsigned)nb1), dim3(256), 0, st, jobs, ws);
  INA_CHECK_LAUNCH();
  hipLaunchKernelGGL(slab_finish_kernel, dim3((unsigned)nb2), dim3(256), 0, st, jobs, (const float*)ws, dst);
  INA_CHECK_LAUNCH();
  return 0;
}

}  // namespace ina
