// Induction + relation head at widths outside the fused head kernels (routing.hip / ntn.hip need
// H in {16, 40, 64}, N*Q <= 64): the paper's H = 2u = 256 with Q = 20 (N*Q = 100), the reference's
// Base default u = 100 (H = 200), BERT's H = 768.  The GEMM-shaped work (e_hat = S W_s, the NTN's
// P = C M and T = Q P^T, their backward GEMMs) runs on hipBLASLt from ops/wide.py; this file holds
// the parts that are NOT GEMMs and that ran as ~150 small PyTorch launches per step:
//
//  routing_wide_fwd : the R routing iterations (softmax over K, weighted sum, squash, agreement
//                     update) for one (episode, class) item per wave; e_hat rows staged in LDS,
//                     lane = feature column (H / 64 columns per lane), the K routing logits in lanes
//                     0..K-1.  Writes the class vectors fp32 and bf16 (the P GEMM operand).
//  routing_wide_bwd : recomputes the forward keeping every iteration's (d, |c_hat|^2) in registers and
//                     (c_hat, c) in the lane's own LDS columns, then the exact reverse through all
//                     iterations; dE_hat accumulates in LDS (each lane owns its columns: no bank
//                     conflicts, no atomics).  H <= 1024 (BERT's 768 included), K <= 64, R <= 5.
//  ntn_wide_epi_fwd : ReLU -> FC (reference W[h*N, N] over column s*N + c, or the paper's per-pair
//                     w in R^h) -> bias -> sigmoid over T[row][c*h + s], one wave per query row.
//  ntn_wide_epi_bwd : dT = [T > 0] * dV (bf16, the operand of the dQ / dP GEMMs), T <- ReLU(T) in
//                     place (the operand of the FC weight-gradient GEMM) and the upstream-scaled dz.
//
// Reference: model/layer_module.py:8-47 (NTN), :101-162 (routing), model/graph.py:57-86.  The
// fp32 oracle is models/reference.py::dynamic_routing / relation_probs.
#include "ina_common.h"
#include "ina_launch.h"

using namespace ina;

namespace {

constexpr int RW_RMAX = 5;    // routing iterations kept in registers by the backward
constexpr int RW_KMAX = 64;   // supports per class: one routing logit per lane
constexpr int EPI_NMAX = 16;  // reference head: classes (FC output columns) per row

INA_DEVICE float squash_scale(float n) { return n / (1.f + n) / sqrtf(n + 1e-9f); }
// d/dn of squash_scale (routing.hip): (n + 2eps - n^2) / (2 r^3 (1+n)^2), r = sqrt(n + eps)
INA_DEVICE float squash_scale_grad(float n) {
  const float r = sqrtf(n + 1e-9f);
  const float onep = 1.f + n;
  return (n + 2e-9f - n * n) / (2.f * r * r * r * onep * onep);
}
INA_DEVICE float bcast(float v, int k) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), k));
}

// softmax over the K routing logits held by lanes 0..K-1 (every lane of the wave active)
INA_DEVICE float lane_softmax(float b, int K, int lane) {
  const float m = wave_max(lane < K ? b : -INFINITY);
  const float x = lane < K ? __expf(b - m) : 0.f;
  return x / wave_sum(x);
}

// sm: this item's e_hat rows [K][H] in LDS.  One routing iteration's forward: d (lane k), c_hat and
// c (columns h = lane + 64 j), |c_hat|^2.  Returns through the references.
template <int HJ>
INA_DEVICE void rw_iter(const float* sm, int K, int H, int lane, float b, float& d, float (&ch)[HJ],
                        float (&c)[HJ], float& n2) {
  d = lane_softmax(b, K, lane);
#pragma unroll
  for (int j = 0; j < HJ; ++j) ch[j] = 0.f;
  for (int k = 0; k < K; ++k) {
    const float dk = bcast(d, k);
#pragma unroll
    for (int j = 0; j < HJ; ++j) {
      const int h = lane + 64 * j;
      ch[j] += dk * (h < H ? sm[k * H + h] : 0.f);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < HJ; ++j) s += ch[j] * ch[j];
  n2 = wave_sum(s);
  const float sc = squash_scale(n2);
#pragma unroll
  for (int j = 0; j < HJ; ++j) c[j] = ch[j] * sc;
}

// b_k += e_hat_k . c  (lane k)
template <int HJ>
INA_DEVICE float rw_agree(const float* sm, int K, int H, int lane, float b, const float (&c)[HJ]) {
  for (int k = 0; k < K; ++k) {
    float a = 0.f;
#pragma unroll
    for (int j = 0; j < HJ; ++j) {
      const int h = lane + 64 * j;
      a += (h < H ? sm[k * H + h] : 0.f) * c[j];
    }
    a = wave_sum(a);
    if (lane == k) b += a;
  }
  return b;
}

template <int HJ>
__global__ __launch_bounds__(64) void routing_wide_fwd_kernel(const float* __restrict__ eh, int K, int H, int R,
                                                              float* __restrict__ cls,
                                                              unsigned short* __restrict__ cls_bf) {
  extern __shared__ float sm[];
  const int lane = threadIdx.x;
  const long item = blockIdx.x;
  const float* src = eh + item * K * H;
  for (int i = lane; i < K * H; i += 64) sm[i] = src[i];
  __syncthreads();
  float b = 0.f, d, n2;
  float ch[HJ], c[HJ];
  for (int r = 0; r < R; ++r) {
    rw_iter<HJ>(sm, K, H, lane, b, d, ch, c, n2);
    if (r + 1 < R) b = rw_agree<HJ>(sm, K, H, lane, b, c);   // the last update is unused
  }
#pragma unroll
  for (int j = 0; j < HJ; ++j) {
    const int h = lane + 64 * j;
    if (h < H) {
      cls[item * H + h] = c[j];
      cls_bf[item * H + h] = f2bf(c[j]);
    }
  }
}

template <int HJ>
__global__ __launch_bounds__(64) void routing_wide_bwd_kernel(const float* __restrict__ eh,
                                                              const float* __restrict__ dcls, int K, int H, int R,
                                                              float* __restrict__ deh) {
  // LDS: e_hat [K][H] | dE_hat [K][H] | c_hat per iteration [R][H] | c per iteration [R][H]
  extern __shared__ float sm[];
  float* de = sm + K * H;
  float* chs = de + K * H;
  float* cs = chs + R * H;
  const int lane = threadIdx.x;
  const long item = blockIdx.x;
  const float* src = eh + item * K * H;
  for (int i = lane; i < K * H; i += 64) {
    sm[i] = src[i];
    de[i] = 0.f;
  }
  __syncthreads();
  // forward recompute; every iteration's state kept (c_hat, c in this lane's own LDS columns)
  float dr[RW_RMAX], nr[RW_RMAX];
  float b = 0.f;
#pragma unroll
  for (int r = 0; r < RW_RMAX; ++r) {
    if (r < R) {
      float ch[HJ], c[HJ];
      rw_iter<HJ>(sm, K, H, lane, b, dr[r], ch, c, nr[r]);
#pragma unroll
      for (int j = 0; j < HJ; ++j) {
        const int h = lane + 64 * j;
        if (h < H) {
          chs[r * H + h] = ch[j];
          cs[r * H + h] = c[j];
        }
      }
      if (r + 1 < R) b = rw_agree<HJ>(sm, K, H, lane, b, c);
    }
  }
  float gc[HJ];
#pragma unroll
  for (int j = 0; j < HJ; ++j) {
    const int h = lane + 64 * j;
    gc[j] = h < H ? dcls[item * H + h] : 0.f;
  }
  float gb = 0.f;   // lane k: dL / d b^{r+1} while iteration r is reversed
#pragma unroll
  for (int r = RW_RMAX - 1; r >= 0; --r) {
    if (r >= R) continue;
    if (r + 1 < R) {   // b^{r+1} = b^r + e_hat . c^r: c^r reaches the output only through it
#pragma unroll
      for (int j = 0; j < HJ; ++j) gc[j] = 0.f;
      for (int k = 0; k < K; ++k) {
        const float g = bcast(gb, k);
#pragma unroll
        for (int j = 0; j < HJ; ++j) {
          const int h = lane + 64 * j;
          if (h < H) {
            gc[j] += g * sm[k * H + h];
            de[k * H + h] += g * cs[r * H + h];
          }
        }
      }
    }
    // squash: c = c_hat s(n), n = |c_hat|^2
    float chv[HJ];
    float dot = 0.f;
#pragma unroll
    for (int j = 0; j < HJ; ++j) {
      const int h = lane + 64 * j;
      chv[j] = h < H ? chs[r * H + h] : 0.f;
      dot += chv[j] * gc[j];
    }
    dot = wave_sum(dot);
    const float s = squash_scale(nr[r]), sg2 = 2.f * squash_scale_grad(nr[r]) * dot;
    float dch[HJ];
#pragma unroll
    for (int j = 0; j < HJ; ++j) dch[j] = gc[j] * s + chv[j] * sg2;
    // c_hat = sum_k d_k e_hat_k
    float dd = 0.f;
    for (int k = 0; k < K; ++k) {
      const float dk = bcast(dr[r], k);
      float p = 0.f;
#pragma unroll
      for (int j = 0; j < HJ; ++j) {
        const int h = lane + 64 * j;
        if (h < H) {
          de[k * H + h] += dk * dch[j];
          p += sm[k * H + h] * dch[j];
        }
      }
      p = wave_sum(p);
      if (lane == k) dd = p;
    }
    // d = softmax(b^r)
    const float sdd = wave_sum(lane < K ? dr[r] * dd : 0.f);
    if (lane < K) gb += dr[r] * (dd - sdd);
  }
  __syncthreads();
  float* dst = deh + item * K * H;
  for (int i = lane; i < K * H; i += 64) dst[i] = de[i];
}

INA_DEVICE float sigmoid_exact(float x) { return 1.f / (1.f + expf(-x)); }

// T [rows][N*h] (column c*h + s), one wave per row, 4 rows per workgroup, grid-stride.
template <bool PAPER>
__global__ __launch_bounds__(256) void ntn_wide_epi_fwd_kernel(const float* __restrict__ T, long rows, int N, int h,
                                                               const float* __restrict__ w,
                                                               const float* __restrict__ bias,
                                                               float* __restrict__ probs) {
  const int lane = threadIdx.x & 63;
  for (long row = (long)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); row < rows; row += (long)gridDim.x * 4) {
    const float* t = T + row * N * h;
    if constexpr (PAPER) {
      for (int c = 0; c < N; ++c) {
        float a = 0.f;
        for (int s = lane; s < h; s += 64) a += fmaxf(t[c * h + s], 0.f) * w[s];
        a = wave_sum(a);
        if (lane == 0) probs[row * N + c] = sigmoid_exact(a + bias[0]);
      }
    } else {
      float acc[EPI_NMAX];
#pragma unroll
      for (int o = 0; o < EPI_NMAX; ++o) acc[o] = 0.f;
      for (int c = 0; c < N; ++c)
        for (int s = lane; s < h; s += 64) {
          const float v = fmaxf(t[c * h + s], 0.f);
          const float* wr = w + (long)(s * N + c) * N;
#pragma unroll
          for (int o = 0; o < EPI_NMAX; ++o)
            if (o < N) acc[o] += v * wr[o];
        }
#pragma unroll
      for (int o = 0; o < EPI_NMAX; ++o)
        if (o < N) {
          const float a = wave_sum(acc[o]);
          if (lane == 0) probs[row * N + o] = sigmoid_exact(a + bias[o]);
        }
    }
  }
}

// dz [rows][N]: dL/dlogit (ina.head_loss); g: optional device scalar (the upstream loss gradient).
// Writes dT [rows][N*h] bf16 = [T > 0] * dV, T <- max(T, 0), dzs = g * dz.
template <bool PAPER>
__global__ __launch_bounds__(256) void ntn_wide_epi_bwd_kernel(float* __restrict__ T, long rows, int N, int h,
                                                               const float* __restrict__ w,
                                                               const float* __restrict__ dz,
                                                               const float* __restrict__ g,
                                                               unsigned short* __restrict__ dT,
                                                               float* __restrict__ dzs) {
  const int lane = threadIdx.x & 63;
  const float gs = g != nullptr ? g[0] : 1.f;
  for (long row = (long)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); row < rows; row += (long)gridDim.x * 4) {
    float* t = T + row * N * h;
    unsigned short* dt = dT + row * N * h;
    const float* z = dz + row * N;
    for (int c = lane; c < N; c += 64) dzs[row * N + c] = z[c] * gs;
    for (int c = 0; c < N; ++c) {
      const float zc = z[c] * gs;
      for (int s = lane; s < h; s += 64) {
        const float v = t[c * h + s];
        float gv;
        if constexpr (PAPER) {
          gv = w[s] * zc;
        } else {
          const float* wr = w + (long)(s * N + c) * N;
          gv = 0.f;
          for (int o = 0; o < N; ++o) gv += wr[o] * z[o];
          gv *= gs;
        }
        dt[c * h + s] = f2bf(v > 0.f ? gv : 0.f);
        t[c * h + s] = fmaxf(v, 0.f);
      }
    }
  }
}

size_t rw_bwd_lds(int K, int H, int R) { return (size_t)(2 * K + 2 * R) * H * sizeof(float); }

template <int HJ>
int rw_fwd_launch(const float* eh, int items, int K, int H, int R, float* cls, void* cls_bf, hipStream_t st) {
  hipLaunchKernelGGL(routing_wide_fwd_kernel<HJ>, dim3(items), dim3(64), (size_t)K * H * sizeof(float), st, eh, K, H,
                     R, cls, (unsigned short*)cls_bf);
  INA_CHECK_LAUNCH();
  return 0;
}
template <int HJ>
int rw_bwd_launch(const float* eh, const float* dcls, int items, int K, int H, int R, float* deh, hipStream_t st) {
  hipLaunchKernelGGL(routing_wide_bwd_kernel<HJ>, dim3(items), dim3(64), rw_bwd_lds(K, H, R), st, eh,
                     dcls, K, H, R, deh);
  INA_CHECK_LAUNCH();
  return 0;
}

int epi_grid(long rows) {
  const long g = (rows + 3) / 4;
  return (int)(g < 8192 ? (g > 0 ? g : 1) : 8192);
}

}  // namespace

namespace ina {

bool routing_wide_supported(int K, int H, int R) {
  return K >= 1 && K <= RW_KMAX && H >= 1 && H <= 1024 && R >= 1 && R <= RW_RMAX && rw_bwd_lds(K, H, R) <= 64 * 1024;
}

int routing_wide_fwd(const float* eh, int items, int K, int H, int R, float* cls, void* cls_bf, hipStream_t st) {
  if (!routing_wide_supported(K, H, R)) return -1;
  if (items <= 0) return 0;
  if (H <= 128) return rw_fwd_launch<2>(eh, items, K, H, R, cls, cls_bf, st);
  if (H <= 256) return rw_fwd_launch<4>(eh, items, K, H, R, cls, cls_bf, st);
  if (H <= 512) return rw_fwd_launch<8>(eh, items, K, H, R, cls, cls_bf, st);
  return rw_fwd_launch<16>(eh, items, K, H, R, cls, cls_bf, st);
}

int routing_wide_bwd(const float* eh, const float* dcls, int items, int K, int H, int R, float* deh, hipStream_t st) {
  if (!routing_wide_supported(K, H, R)) return -1;
  if (items <= 0) return 0;
  if (H <= 128) return rw_bwd_launch<2>(eh, dcls, items, K, H, R, deh, st);
  if (H <= 256) return rw_bwd_launch<4>(eh, dcls, items, K, H, R, deh, st);
  if (H <= 512) return rw_bwd_launch<8>(eh, dcls, items, K, H, R, deh, st);
  return rw_bwd_launch<16>(eh, dcls, items, K, H, R, deh, st);
}

bool ntn_wide_epi_supported(int N, bool paper) { return N >= 1 && (paper || N <= EPI_NMAX); }

int ntn_wide_epi_fwd(const float* T, long rows, int N, int h, const float* w, const float* b, bool paper, float* probs,
                     hipStream_t st) {
  if (!ntn_wide_epi_supported(N, paper)) return -1;
  if (rows <= 0) return 0;
  if (paper)
    hipLaunchKernelGGL(ntn_wide_epi_fwd_kernel<true>, dim3(epi_grid(rows)), dim3(256), 0, st, T, rows, N, h, w, b,
                       probs);
  else
    hipLaunchKernelGGL(ntn_wide_epi_fwd_kernel<false>, dim3(epi_grid(rows)), dim3(256), 0, st, T, rows, N, h, w, b,
                       probs);
  INA_CHECK_LAUNCH();
  return 0;
}

int ntn_wide_epi_bwd(float* T, long rows, int N, int h, const float* w, const float* dz, const float* g, bool paper,
                     void* dT, float* dzs, hipStream_t st) {
  if (!ntn_wide_epi_supported(N, paper)) return -1;
  if (rows <= 0) return 0;
  auto* d = (unsigned short*)dT;
  if (paper)
    hipLaunchKernelGGL(ntn_wide_epi_bwd_kernel<true>, dim3(epi_grid(rows)), dim3(256), 0, st, T, rows, N, h, w, dz, g,
                       d, dzs);
  else
    hipLaunchKernelGGL(ntn_wide_epi_bwd_kernel<false>, dim3(epi_grid(rows)), dim3(256), 0, st, T, rows, N, h, w, dz,
                       g, d, dzs);
  INA_CHECK_LAUNCH();
  return 0;
}

}  // namespace ina
