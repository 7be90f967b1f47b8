// Fused dynamic-routing induction module, forward and backward (K6 of SURVEY 2.3).
//
// Reference (model/layer_module.py:101-162, model/graph.py:69-79):
//   e_hat = S @ W_s                 (shared W_s, no bias; S = support [N, K, H])
//   b = 0 [N, K]
//   repeat iters:  d = softmax_K(b);  c_hat = sum_k d_k e_hat_k;  c = squash(c_hat);
//                  b += e_hat . c
//   return c        (the last b update is unused)
//   squash(v) = v * n/(1+n) / sqrt(n + 1e-9),  n = |v|^2
//
// One wave per (episode, class) work item (classes route independently; W_s is the only shared
// operand), lane = feature column h (H <= 64).  The backward recomputes the forward keeping every
// iteration's (d, c_hat, c, n) in wave-private LDS, then runs the exact reverse-mode recurrence
// through all iterations (softmax / squash / agreement update), and accumulates dW_s = S^T dE_hat
// in registers across the work items the wave visits.
#include "ina_common.h"

using namespace ina;

namespace {

INA_DEVICE void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

INA_DEVICE float squash_scale(float n) { return n / (1.f + n) / sqrtf(n + 1e-9f); }
// d/dn of squash_scale: (n + 2eps - n^2) / (2 r^3 (1+n)^2), r = sqrt(n + eps)
INA_DEVICE float squash_scale_grad(float n) {
  const float r = sqrtf(n + 1e-9f);
  const float onep = 1.f + n;
  return (n + 2e-9f - n * n) / (2.f * r * r * r * onep * onep);
}

// per-wave LDS carve (floats), ONE class of one episode per work item:
//   sup[K*H] eh[K*H] deh[K*H] chat[R*H] cv[R*H] d[R*K] n2[R] b[K] gb[K] dd[K]
// (routing is independent across the N classes of an episode: the only shared operand is W_s, so
// the work is split per (episode, class) -- N times more waves, N times shorter serial chains)
__host__ __device__ inline size_t rt_wave_floats(int N, int K, int H, int R) {
  (void)N;
  return (size_t)3 * K * H + (size_t)2 * R * H + (size_t)R * K + R + 3 * K;
}

template <int H>
INA_DEVICE void routing_forward(const float* __restrict__ e, long sup_row0, int K, int R, const float* ws_col,
                                float* sup, float* eh, float* chat_s, float* cv_s, float* d_s, float* n2_s, float* b,
                                int lane) {
  const int h = lane;
  if (h < H)
    for (int k = 0; k < K; ++k) sup[k * H + h] = e[(sup_row0 + k) * H + h];
  wave_lds_sync();
  for (int k = 0; k < K; ++k) {
    float acc = 0.f;
#pragma unroll
    for (int a = 0; a < H; ++a) acc += sup[k * H + a] * ws_col[a];
    if (h < H) eh[k * H + h] = acc;
    if (lane == 0) b[k] = 0.f;
  }
  wave_lds_sync();
  for (int r = 0; r < R; ++r) {
    float mx = -INFINITY;
    for (int k = 0; k < K; ++k) mx = fmaxf(mx, b[k]);
    float den = 0.f;
    for (int k = 0; k < K; ++k) den += __expf(b[k] - mx);
    const float inv = 1.f / den;
    float ch = 0.f;
    for (int k = 0; k < K; ++k) {
      const float dk = __expf(b[k] - mx) * inv;
      if (lane == 0) d_s[r * K + k] = dk;
      ch += dk * (h < H ? eh[k * H + h] : 0.f);
    }
    const float n2 = wave_sum(h < H ? ch * ch : 0.f);
    const float cvh = ch * squash_scale(n2);
    if (h < H) {
      chat_s[r * H + h] = ch;
      cv_s[r * H + h] = cvh;
    }
    if (lane == 0) n2_s[r] = n2;
    if (r + 1 < R) {   // the last agreement update is unused (reference quirk)
      for (int k = 0; k < K; ++k) {
        const float ag = wave_sum(h < H ? eh[k * H + h] * cvh : 0.f);
        if (lane == 0) b[k] += ag;
      }
      wave_lds_sync();
    }
  }
}

}  // namespace

template <int H>
__global__ __launch_bounds__(64) void routing_fwd_kernel(const float* __restrict__ e, const float* __restrict__ Ws, int E,
                                                         int N, int K, int Q, int R, float* __restrict__ cls) {
  extern __shared__ __attribute__((aligned(16))) float rsm[];
  const int lane = threadIdx.x;
  float* sup = rsm;
  float* eh = sup + K * H;
  float* deh = eh + K * H;
  float* chat = deh + K * H;
  float* cv = chat + R * H;
  float* d = cv + R * H;
  float* n2 = d + R * K;
  float* b = n2 + R;
  float ws_col[H];
#pragma unroll
  for (int a = 0; a < H; ++a) ws_col[a] = lane < H ? Ws[a * H + lane] : 0.f;
  const int NK = N * K;
  for (int w = blockIdx.x; w < E * N; w += gridDim.x) {
    const int ep = w / N, c = w - ep * N;
    const long row0 = (long)ep * (NK + N * Q) + (long)c * K;
    routing_forward<H>(e, row0, K, R, ws_col, sup, eh, chat, cv, d, n2, b, lane);
    if (lane < H) cls[((long)ep * N + c) * H + lane] = cv[(R - 1) * H + lane];
    wave_lds_sync();
  }
}

// dws_slab: [gridDim.x][H*H] (row a, col h)
template <int H>
__global__ __launch_bounds__(64) void routing_bwd_kernel(const float* __restrict__ e, const float* __restrict__ Ws, int E,
                                                         int N, int K, int Q, int R, const float* __restrict__ dcls,
                                                         float* __restrict__ de, float* __restrict__ dws_slab) {
  extern __shared__ __attribute__((aligned(16))) float rsm[];
  const int lane = threadIdx.x, h = lane;
  float* sup = rsm;
  float* eh = sup + K * H;
  float* deh = eh + K * H;
  float* chat = deh + K * H;
  float* cv = chat + R * H;
  float* d = cv + R * H;
  float* n2 = d + R * K;
  float* b = n2 + R;
  float* gb = b + K;
  float* dd = gb + K;
  float* wst = dd + K;  // [H][H] W_s^T (wst[h*H + a] = W_s[a][h]): dS reads are lane-contiguous
  float ws_col[H], dws[H];
#pragma unroll
  for (int a = 0; a < H; ++a) {
    ws_col[a] = lane < H ? Ws[a * H + lane] : 0.f;
    dws[a] = 0.f;
  }
  for (int i = lane; i < H * H; i += 64) {
    const int a = i / H, hh = i - a * H;
    wst[hh * H + a] = Ws[i];
  }
  wave_lds_sync();
  const int NK = N * K;
  for (int w = blockIdx.x; w < E * N; w += gridDim.x) {
    const int ep = w / N, c = w - ep * N;
    const long row0 = (long)ep * (NK + N * Q) + (long)c * K;
    routing_forward<H>(e, row0, K, R, ws_col, sup, eh, chat, cv, d, n2, b, lane);
    for (int k = 0; k < K; ++k) {
      if (h < H) deh[k * H + h] = 0.f;
      if (lane == 0) gb[k] = 0.f;
    }
    wave_lds_sync();
    for (int r = R - 1; r >= 0; --r) {
      // gradient into c_r: from the output (last iteration) and from b_{r+1} = b_r + e_hat . c_r
      float dc = (r == R - 1 && h < H) ? dcls[((long)ep * N + c) * H + h] : 0.f;
      const float cvh = h < H ? cv[r * H + h] : 0.f;
      for (int k = 0; k < K; ++k) {
        const float g = gb[k];
        if (h < H) {
          dc += g * eh[k * H + h];
          deh[k * H + h] += g * cvh;
        }
      }
      // squash backward
      const float ch = h < H ? chat[r * H + h] : 0.f;
      const float nn = n2[r];
      const float dot = wave_sum(ch * dc);
      const float dch = squash_scale(nn) * dc + 2.f * ch * dot * squash_scale_grad(nn);
      // c_hat = sum_k d_k e_hat_k
      float sdd = 0.f;
      for (int k = 0; k < K; ++k) {
        const float ehv = h < H ? eh[k * H + h] : 0.f;
        const float ddk = wave_sum(ehv * dch);
        const float dk = d[r * K + k];
        if (h < H) deh[k * H + h] += dk * dch;
        if (lane == 0) dd[k] = ddk;
        sdd += dk * ddk;
      }
      wave_lds_sync();
      // softmax backward; gb accumulates dL/db_r (identity path from b_{r+1} already inside)
      if (lane == 0)
        for (int k = 0; k < K; ++k) gb[k] += d[r * K + k] * (dd[k] - sdd);
      wave_lds_sync();
    }
    // dS = dE_hat W_s^T  (lane = a),  dW_s[a][h] += sum_k S[k][a] dE_hat[k][h]  (lane = h)
    for (int k = 0; k < K; ++k) {
      if (lane < H) {
        float acc = 0.f;
#pragma unroll
        for (int hh = 0; hh < H; ++hh) acc += deh[k * H + hh] * wst[hh * H + lane];
        de[(row0 + k) * H + lane] = acc;
      }
      const float dv = h < H ? deh[k * H + h] : 0.f;
#pragma unroll
      for (int a = 0; a < H; ++a) dws[a] += sup[k * H + a] * dv;
    }
    wave_lds_sync();
  }
  if (lane < H) {
#pragma unroll
    for (int a = 0; a < H; ++a) dws_slab[(size_t)blockIdx.x * H * H + a * H + lane] = dws[a];
  }
}

// ------------------------------------------------------------------------------------------
// Grouped routing (the default shapes: H in {16, 40, 64}, K in {1, 2, 3, 5, 10}, R <= 4).
// The per-item kernels above run one (episode, class) item per wave with lane = feature: 24 of 64
// lanes idle at H = 40, every reduction a 64-lane one, and the routing state round-tripping LDS
// between dependent steps (issue-bound: ~230 us backward for 40960 items).  Here a wave runs FOUR
// items, one per 16-lane group; lane (g = l >> 4, j = l & 15) owns features h = j + 16 f (f < HF)
// of item g, and the whole routing state (e_hat[K][HF], b, d, c_hat, c and the backward's per-
// iteration stash) lives in registers.  Reductions over features are 16-lane DPP sums (group16_sum,
// bitwise identical in every lane of the group), the softmax over the K supports is lane-local.
//   e_hat = S W_s  and  dS = dE_hat W_s^T: lane-owned outputs, fp32 FMAs, S / dE_hat rows staged in
//     wave-private LDS (broadcast float4 reads within a group), W_s / W_s^T staged once per block;
//   dW_s = S^T dE_hat over the wave's 4K (item, support) rows: v_mfma_f32_16x16x4_f32 from the same
//     staging (register accumulators across the wave's items, deterministic block reduction, one
//     slab per block).
// Items past E*N are clamped to the last one with zeroed support rows (no output, zero dW_s).
template <int H>
struct RGShape {
  static constexpr int HF = (H + 15) / 16, HP = 16 * HF;
};
constexpr int RG_WAVES = 4, RG_RMAX = 3;   // R <= 3 (the reference default 3); other R: per-item kernels

template <int H, int K>
INA_DEVICE void rg_load_stage(const float* __restrict__ e, long row0, bool ok, float* S, int g, int j) {
  constexpr int HF = RGShape<H>::HF, HP = RGShape<H>::HP;
  float sv[K][HF];
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int f = 0; f < HF; ++f) {
      const int hh = j + 16 * f;
      const bool in = ok && hh < H;
      sv[k][f] = e[in ? (row0 + k) * H + hh : 0] * (in ? 1.f : 0.f);   // unconditional clamped loads
    }
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int f = 0; f < HF; ++f) S[(g * K + k) * HP + j + 16 * f] = sv[k][f];
}

// out[k][f] = sum_x X[g*K + k][x] * Wl[x * HP + j + 16 f]  (x < H; X rows staged with stride HP)
template <int H, int K>
INA_DEVICE void rg_rowmat(const float* X, const float* Wl, int g, int j, float (&out)[K][RGShape<H>::HF]) {
  constexpr int HF = RGShape<H>::HF, HP = RGShape<H>::HP;
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int f = 0; f < HF; ++f) out[k][f] = 0.f;
#pragma unroll 2   // (full unrolling hoisted every LDS read: 450 registers at H = 40)
  for (int x4 = 0; x4 < H; x4 += 4) {   // H % 8 == 0
    float4 xv[K];
#pragma unroll
    for (int k = 0; k < K; ++k) xv[k] = *reinterpret_cast<const float4*>(X + (g * K + k) * HP + x4);
#pragma unroll
    for (int dx = 0; dx < 4; ++dx) {
      float wv[HF];
#pragma unroll
      for (int f = 0; f < HF; ++f) wv[f] = Wl[(x4 + dx) * HP + j + 16 * f];
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const float xk = dx == 0 ? xv[k].x : dx == 1 ? xv[k].y : dx == 2 ? xv[k].z : xv[k].w;
#pragma unroll
        for (int f = 0; f < HF; ++f) out[k][f] = fmaf(xk, wv[f], out[k][f]);
      }
    }
  }
}

// forward routing iterations of one item from e_hat; STASH keeps each iteration's d, c_hat, c, n
template <int K, int HF, bool STASH>
INA_DEVICE void rg_iterate(const float (&eh)[K][HF], int R, float (&cv)[HF], float (&d_s)[RG_RMAX][K],
                           float (&ch_s)[RG_RMAX][HF], float (&cv_s)[RG_RMAX][HF], float (&n2_s)[RG_RMAX]) {
  float b[K];
#pragma unroll
  for (int k = 0; k < K; ++k) b[k] = 0.f;
#pragma unroll
  for (int r = 0; r < RG_RMAX; ++r) {
    if (r >= R) break;
    float mx = b[0];
#pragma unroll
    for (int k = 1; k < K; ++k) mx = fmaxf(mx, b[k]);
    float ex[K], den = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      ex[k] = __expf(b[k] - mx);
      den += ex[k];
    }
    const float inv = 1.f / den;
    float d[K], ch[HF];
#pragma unroll
    for (int k = 0; k < K; ++k) d[k] = ex[k] * inv;
#pragma unroll
    for (int f = 0; f < HF; ++f) {
      ch[f] = 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k) ch[f] += d[k] * eh[k][f];
    }
    float p = 0.f;
#pragma unroll
    for (int f = 0; f < HF; ++f) p += ch[f] * ch[f];
    const float n2 = group16_sum(p);
    const float sc = squash_scale(n2);
#pragma unroll
    for (int f = 0; f < HF; ++f) cv[f] = ch[f] * sc;
    if (STASH) {
#pragma unroll
      for (int k = 0; k < K; ++k) d_s[r][k] = d[k];
#pragma unroll
      for (int f = 0; f < HF; ++f) {
        ch_s[r][f] = ch[f];
        cv_s[r][f] = cv[f];
      }
      n2_s[r] = n2;
    }
    if (r + 1 < R) {   // the last agreement update is unused (reference quirk)
#pragma unroll
      for (int k = 0; k < K; ++k) {
        float a = 0.f;
#pragma unroll
        for (int f = 0; f < HF; ++f) a += eh[k][f] * cv[f];
        b[k] += group16_sum(a);
      }
    }
  }
}

template <int H, int K>
__global__ __launch_bounds__(256) void routing_g_fwd_kernel(const float* __restrict__ e, const float* __restrict__ Ws,
                                                            int E, int N, int Q, int R, float* __restrict__ cls) {
  constexpr int HF = RGShape<H>::HF, HP = RGShape<H>::HP;
  extern __shared__ __attribute__((aligned(16))) float rgs[];
  float* wsh = rgs;                                   // W_s[a][h] (h padded to HP with zeros)
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), g = lane >> 4, j = lane & 15;
  float* S = rgs + H * HP + wave * 4 * K * HP;        // this wave's [4K][HP] support rows
  for (int i = threadIdx.x; i < H * HP; i += 256) {
    const int a = i / HP, hh = i - a * HP;
    wsh[i] = hh < H ? Ws[a * H + hh] : 0.f;
  }
  __syncthreads();
  const int EN = E * N, NK = N * K;
  const int nquads = (EN + 3) / 4;
  float d_s[RG_RMAX][K], ch_s[RG_RMAX][HF], cv_s[RG_RMAX][HF], n2_s[RG_RMAX];
  for (int qd = blockIdx.x * RG_WAVES + wave; qd < nquads; qd += gridDim.x * RG_WAVES) {
    const int w = qd * 4 + g;
    const bool ok = w < EN;
    const int wc = ok ? w : EN - 1;
    const int ep = wc / N, c = wc - ep * N;
    const long row0 = (long)ep * (NK + N * Q) + (long)c * K;
    rg_load_stage<H, K>(e, row0, ok, S, g, j);
    wave_lds_sync();
    float eh[K][HF];
    rg_rowmat<H, K>(S, wsh, g, j, eh);
    float cv[HF];
    rg_iterate<K, HF, false>(eh, R, cv, d_s, ch_s, cv_s, n2_s);
#pragma unroll
    for (int f = 0; f < HF; ++f) {
      const int hh = j + 16 * f;
      if (ok && hh < H) cls[((long)ep * N + c) * H + hh] = cv[f];
    }
    wave_lds_sync();   // S is rewritten by the next quad
  }
}

// dws_slab: [gridDim.x][H][H] (row a, col h)
template <int H, int K>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void routing_g_bwd_kernel(const float* __restrict__ e, const float* __restrict__ Ws,
                                                            int E, int N, int Q, int R,
                                                            const float* __restrict__ dcls, float* __restrict__ de,
                                                            float* __restrict__ dws_slab) {
  constexpr int HF = RGShape<H>::HF, HP = RGShape<H>::HP;
  extern __shared__ __attribute__((aligned(16))) float rgs[];
  float* wsh = rgs;                 // W_s[a][h]
  float* wst = rgs + H * HP;        // W_s^T[h][a]
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), g = lane >> 4, j = lane & 15;
  float* S = rgs + 2 * H * HP + wave * 8 * K * HP;   // [4K][HP] support rows
  float* D = S + 4 * K * HP;                          // [4K][HP] dE_hat rows
  for (int i = threadIdx.x; i < H * HP; i += 256) {
    const int a = i / HP, hh = i - a * HP;
    wsh[i] = hh < H ? Ws[a * H + hh] : 0.f;
    wst[i] = hh < H ? Ws[hh * H + a] : 0.f;
  }
  __syncthreads();
  f32x4_t acc[HF][HF];
#pragma unroll
  for (int ta = 0; ta < HF; ++ta)
#pragma unroll
    for (int th = 0; th < HF; ++th) acc[ta][th] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int EN = E * N, NK = N * K;
  const int nquads = (EN + 3) / 4;
  for (int qd = blockIdx.x * RG_WAVES + wave; qd < nquads; qd += gridDim.x * RG_WAVES) {
    const int w = qd * 4 + g;
    const bool ok = w < EN;
    const int wc = ok ? w : EN - 1;
    const int ep = wc / N, c = wc - ep * N;
    const long row0 = (long)ep * (NK + N * Q) + (long)c * K;
    float dcl[HF];
#pragma unroll
    for (int f = 0; f < HF; ++f) {
      const int hh = j + 16 * f;
      const bool in = hh < H;
      dcl[f] = dcls[in ? ((long)ep * N + c) * H + hh : 0] * (in ? 1.f : 0.f);
    }
    rg_load_stage<H, K>(e, row0, ok, S, g, j);
    wave_lds_sync();
    float eh[K][HF];
    rg_rowmat<H, K>(S, wsh, g, j, eh);
    float cv[HF], d_s[RG_RMAX][K], ch_s[RG_RMAX][HF], cv_s[RG_RMAX][HF], n2_s[RG_RMAX];
    rg_iterate<K, HF, true>(eh, R, cv, d_s, ch_s, cv_s, n2_s);
    // reverse through the iterations (exact; see routing_bwd_kernel)
    float gb[K], deh[K][HF];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      gb[k] = 0.f;
#pragma unroll
      for (int f = 0; f < HF; ++f) deh[k][f] = 0.f;
    }
#pragma unroll
    for (int r = RG_RMAX - 1; r >= 0; --r) {
      if (r >= R) continue;
      float dc[HF];
#pragma unroll
      for (int f = 0; f < HF; ++f) dc[f] = r == R - 1 ? dcl[f] : 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k)
#pragma unroll
        for (int f = 0; f < HF; ++f) {
          dc[f] += gb[k] * eh[k][f];
          deh[k][f] += gb[k] * cv_s[r][f];
        }
      float p = 0.f;
#pragma unroll
      for (int f = 0; f < HF; ++f) p += ch_s[r][f] * dc[f];
      const float dot = group16_sum(p);
      const float nn = n2_s[r];
      const float s0 = squash_scale(nn), s1 = 2.f * dot * squash_scale_grad(nn);
      float dch[HF];
#pragma unroll
      for (int f = 0; f < HF; ++f) dch[f] = s0 * dc[f] + ch_s[r][f] * s1;
      float dd[K], sdd = 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        float a = 0.f;
#pragma unroll
        for (int f = 0; f < HF; ++f) a += eh[k][f] * dch[f];
        dd[k] = group16_sum(a);
#pragma unroll
        for (int f = 0; f < HF; ++f) deh[k][f] += d_s[r][k] * dch[f];
        sdd += d_s[r][k] * dd[k];
      }
#pragma unroll
      for (int k = 0; k < K; ++k) gb[k] += d_s[r][k] * (dd[k] - sdd);
    }
    // stage dE_hat (zero for clamped items: no dW_s contribution)
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
      for (int f = 0; f < HF; ++f) D[(g * K + k) * HP + j + 16 * f] = ok ? deh[k][f] : 0.f;
    wave_lds_sync();
    // dS[k][a] = sum_h dE_hat[k][h] W_s[a][h]  (lane-owned a = j + 16 f)
    float dsv[K][HF];
    rg_rowmat<H, K>(D, wst, g, j, dsv);
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
      for (int f = 0; f < HF; ++f) {
        const int a = j + 16 * f;
        if (ok && a < H) de[(row0 + k) * H + a] = dsv[k][f];
      }
    // dW_s[a][h] += sum over the wave's 4K rows of S[row][a] dE_hat[row][h]
#pragma unroll
    for (int st = 0; st < K; ++st) {
      const int row = 4 * st + g;
      float av[HF], bv[HF];
#pragma unroll
      for (int t = 0; t < HF; ++t) {
        av[t] = S[row * HP + 16 * t + j];
        bv[t] = D[row * HP + 16 * t + j];
      }
#pragma unroll
      for (int ta = 0; ta < HF; ++ta)
#pragma unroll
        for (int th = 0; th < HF; ++th) acc[ta][th] = mfma_f32(av[ta], bv[th], acc[ta][th]);
    }
    wave_lds_sync();   // S / D are rewritten by the next quad
  }
  // deterministic block reduction: waves add their tiles into LDS in wave order
  __syncthreads();
  float* red = rgs + 2 * H * HP;   // reuse the staging region (>= H*H floats: host check)
  for (int i = threadIdx.x; i < H * H; i += 256) red[i] = 0.f;
  __syncthreads();
  ordered_wave_accumulate(wave, RG_WAVES, [&] {
#pragma unroll
    for (int ta = 0; ta < HF; ++ta)
#pragma unroll
      for (int th = 0; th < HF; ++th)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int a = 16 * ta + 4 * g + r, hh = 16 * th + j;
          if (a < H && hh < H) red[a * H + hh] += acc[ta][th][r];
        }
  });
  for (int i = threadIdx.x; i < H * H; i += 256) dws_slab[(size_t)blockIdx.x * H * H + i] = red[i];
}

namespace ina {

static bool rg_supported(int K, int H, int R) {
  return (H == 16 || H == 40 || H == 64) && (K == 1 || K == 2 || K == 3 || K == 5 || K == 10) && R >= 1 &&
         R <= RG_RMAX;
}
static size_t rg_lds_bytes(int K, int H, bool bwd) {
  const int HP = 16 * ((H + 15) / 16);
  const size_t stage = (size_t)RG_WAVES * (bwd ? 8 : 4) * K * HP;
  return ((bwd ? 2 : 1) * (size_t)H * HP + (bwd && stage < (size_t)H * H ? (size_t)H * H : stage)) * 4;
}
size_t routing_lds_bytes(int N, int K, int H, int R, bool bwd) {
  if (rg_supported(K, H, R)) return rg_lds_bytes(K, H, bwd);
  size_t f = rt_wave_floats(N, K, H, R);
  if (bwd) f += (size_t)H * H;
  return f * 4;
}

template <int H>
static int rt_fwd_t(const float* e, const float* Ws, int E, int N, int K, int Q, int R, float* cls, int blocks,
                    hipStream_t st) {
  const size_t lds = routing_lds_bytes(N, K, H, R, false);
  if (lds > 64 * 1024)   // large N*K (e.g. 10-way 5-shot at H=64): opt in to the full 160 KB LDS
    (void)hipFuncSetAttribute((const void*)routing_fwd_kernel<H>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
  hipLaunchKernelGGL((routing_fwd_kernel<H>), dim3(blocks), dim3(64), lds, st, e, Ws, E, N, K, Q, R, cls);
  INA_CHECK_LAUNCH();
  return 0;
}
template <int H>
static int rt_bwd_t(const float* e, const float* Ws, int E, int N, int K, int Q, int R, const float* dcls, float* de,
                    float* slab, int blocks, hipStream_t st) {
  const size_t lds = routing_lds_bytes(N, K, H, R, true);
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute((const void*)routing_bwd_kernel<H>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
  hipLaunchKernelGGL((routing_bwd_kernel<H>), dim3(blocks), dim3(64), lds, st, e, Ws, E, N, K, Q, R, dcls, de, slab);
  INA_CHECK_LAUNCH();
  return 0;
}

int routing_bwd_default_blocks(int N, int K, int H, int R) {
  (void)N;
  return rg_supported(K, H, R) ? 1024 : 4096;
}
template <int H, int K>
static int rg_launch(bool bwd, const float* e, const float* Ws, int E, int N, int Q, int R, const float* dcls, float* de,
                     float* out, int blocks, hipStream_t st) {
  const size_t lds = rg_lds_bytes(K, H, bwd);
  if (bwd) {
    if (lds > 64 * 1024)
      (void)hipFuncSetAttribute((const void*)routing_g_bwd_kernel<H, K>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                160 * 1024);
    hipLaunchKernelGGL((routing_g_bwd_kernel<H, K>), dim3(blocks), dim3(256), lds, st, e, Ws, E, N, Q, R, dcls, de, out);
  } else {
    if (lds > 64 * 1024)
      (void)hipFuncSetAttribute((const void*)routing_g_fwd_kernel<H, K>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                160 * 1024);
    hipLaunchKernelGGL((routing_g_fwd_kernel<H, K>), dim3(blocks), dim3(256), lds, st, e, Ws, E, N, Q, R, out);
  }
  INA_CHECK_LAUNCH();
  return 0;
}
template <int H>
static int rg_k(bool bwd, const float* e, const float* Ws, int E, int N, int K, int Q, int R, const float* dcls,
                float* de, float* out, int blocks, hipStream_t st) {
  switch (K) {
    case 1: return rg_launch<H, 1>(bwd, e, Ws, E, N, Q, R, dcls, de, out, blocks, st);
    case 2: return rg_launch<H, 2>(bwd, e, Ws, E, N, Q, R, dcls, de, out, blocks, st);
    case 3: return rg_launch<H, 3>(bwd, e, Ws, E, N, Q, R, dcls, de, out, blocks, st);
    case 5: return rg_launch<H, 5>(bwd, e, Ws, E, N, Q, R, dcls, de, out, blocks, st);
    case 10: return rg_launch<H, 10>(bwd, e, Ws, E, N, Q, R, dcls, de, out, blocks, st);
  }
  return -1;
}
static int rg_dispatch(bool bwd, const float* e, const float* Ws, int E, int N, int K, int Q, int R, int H,
                       const float* dcls, float* de, float* out, int blocks, hipStream_t st) {
  switch (H) {
    case 16: return rg_k<16>(bwd, e, Ws, E, N, K, Q, R, dcls, de, out, blocks, st);
    case 40: return rg_k<40>(bwd, e, Ws, E, N, K, Q, R, dcls, de, out, blocks, st);
    case 64: return rg_k<64>(bwd, e, Ws, E, N, K, Q, R, dcls, de, out, blocks, st);
  }
  return -1;
}

int routing_fwd(const float* e, const float* Ws, int E, int N, int K, int Q, int R, int H, float* cls, int blocks,
                hipStream_t st) {
  if (rg_supported(K, H, R)) {
    const int quads = (E * N + 3) / 4;
    const int nb = (quads + RG_WAVES - 1) / RG_WAVES;
    return rg_dispatch(false, e, Ws, E, N, K, Q, R, H, nullptr, nullptr, cls, nb < 2048 ? nb : 2048, st);
  }
  switch (H) {
    case 16: return rt_fwd_t<16>(e, Ws, E, N, K, Q, R, cls, blocks, st);
    case 40: return rt_fwd_t<40>(e, Ws, E, N, K, Q, R, cls, blocks, st);
    case 64: return rt_fwd_t<64>(e, Ws, E, N, K, Q, R, cls, blocks, st);
  }
  return -1;
}
int routing_bwd(const float* e, const float* Ws, int E, int N, int K, int Q, int R, int H, const float* dcls, float* de,
                float* slab, int blocks, hipStream_t st) {
  // grouped path: exactly `blocks` blocks (the slab has one row per block; idle blocks write zeros)
  if (rg_supported(K, H, R)) return rg_dispatch(true, e, Ws, E, N, K, Q, R, H, dcls, de, slab, blocks, st);
  switch (H) {
    case 16: return rt_bwd_t<16>(e, Ws, E, N, K, Q, R, dcls, de, slab, blocks, st);
    case 40: return rt_bwd_t<40>(e, Ws, E, N, K, Q, R, dcls, de, slab, blocks, st);
    case 64: return rt_bwd_t<64>(e, Ws, E, N, K, Q, R, dcls, de, slab, blocks, st);
  }
  return -1;
}

}  // namespace ina
