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

namespace ina {

size_t routing_lds_bytes(int N, int K, int H, int R, bool bwd) {
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

int routing_fwd(const float* e, const float* Ws, int E, int N, int K, int Q, int R, int H, float* cls, int blocks,
                hipStream_t st) {
  switch (H) {
    case 16: return rt_fwd_t<16>(e, Ws, E, N, K, Q, R, cls, blocks, st);
    case 40: return rt_fwd_t<40>(e, Ws, E, N, K, Q, R, cls, blocks, st);
    case 64: return rt_fwd_t<64>(e, Ws, E, N, K, Q, R, cls, blocks, st);
  }
  return -1;
}
int routing_bwd(const float* e, const float* Ws, int E, int N, int K, int Q, int R, int H, const float* dcls, float* de,
                float* slab, int blocks, hipStream_t st) {
  switch (H) {
    case 16: return rt_bwd_t<16>(e, Ws, E, N, K, Q, R, dcls, de, slab, blocks, st);
    case 40: return rt_bwd_t<40>(e, Ws, E, N, K, Q, R, dcls, de, slab, blocks, st);
    case 64: return rt_bwd_t<64>(e, Ws, E, N, K, Q, R, dcls, de, slab, blocks, st);
  }
  return -1;
}

}  // namespace ina
