// Accumulate chains that mix MFMA shapes on gfx950: D = mfma_16x16x32(A, B, 0); D = mfma_16x16x16(a, b, D)
// back to back (SrcC = the previous MFMA's D).  hipcc (ROCm 7.2) puts no wait states between the two; this probe
// compares the chained result with the same products accumulated in separate registers and added on the VALU,
// for the four orders (32 -> 16, 16 -> 32, 32 -> 32, 16 -> 16).  Prints the max abs difference per order.
// Build: hipcc --offload-arch=gfx950 -O3 mfma_chain.hip -o mfma_chain
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

__device__ unsigned short bfbits(float x) { return (unsigned short)(__builtin_bit_cast(unsigned, x) >> 16); }

// order: 0 = 32 then 16, 1 = 16 then 32, 2 = 32 then 32, 3 = 16 then 16
template <int ORDER>
__global__ __launch_bounds__(64) void chain(const float* __restrict__ in, float* __restrict__ out) {
  const int l = threadIdx.x;
  s16x8_t a8, b8;
  s16x4_t a4, b4;
  for (int j = 0; j < 8; ++j) {
    a8[j] = (short)bfbits(in[l * 8 + j]);
    b8[j] = (short)bfbits(in[512 + l * 8 + j]);
  }
  for (int j = 0; j < 4; ++j) {
    a4[j] = (short)bfbits(in[1024 + l * 4 + j]);
    b4[j] = (short)bfbits(in[1280 + l * 4 + j]);
  }
  const bf16x8_t A8 = __builtin_bit_cast(bf16x8_t, a8), B8 = __builtin_bit_cast(bf16x8_t, b8);
  const f32x4_t z = {0.f, 0.f, 0.f, 0.f};
  f32x4_t chained, p, r;
  // the separate products first; sched_barrier keeps the chain's two MFMAs back to back
  if (ORDER == 0 || ORDER == 1) {
    p = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A8, B8, z, 0, 0, 0);
    r = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, z, 0, 0, 0);
  } else if (ORDER == 2) {
    p = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A8, B8, z, 0, 0, 0);
    r = __builtin_amdgcn_mfma_f32_16x16x32_bf16(B8, A8, z, 0, 0, 0);
  } else {
    p = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, z, 0, 0, 0);
    r = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(b4, a4, z, 0, 0, 0);
  }
  __builtin_amdgcn_sched_barrier(0);
  // the chain's operands through an empty asm: no CSE with the separate products above
  asm volatile("" : "+v"(a8), "+v"(b8), "+v"(a4), "+v"(b4));
  const bf16x8_t A8c = __builtin_bit_cast(bf16x8_t, a8), B8c = __builtin_bit_cast(bf16x8_t, b8);
  __builtin_amdgcn_sched_barrier(0);
  if (ORDER == 0) {
    chained = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A8c, B8c, z, 0, 0, 0);
    chained = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, chained, 0, 0, 0);
  } else if (ORDER == 1) {
    chained = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, z, 0, 0, 0);
    chained = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A8c, B8c, chained, 0, 0, 0);
  } else if (ORDER == 2) {
    chained = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A8c, B8c, z, 0, 0, 0);
    chained = __builtin_amdgcn_mfma_f32_16x16x32_bf16(B8c, A8c, chained, 0, 0, 0);
  } else {
    chained = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, z, 0, 0, 0);
    chained = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(b4, a4, chained, 0, 0, 0);
  }
  __builtin_amdgcn_sched_barrier(0);
  float d = 0.f;
  for (int i = 0; i < 4; ++i) d = fmaxf(d, fabsf(chained[i] - (p[i] + r[i])));
  out[l] = d;
}

template <int ORDER>
float run(const float* din, float* dout) {
  hipLaunchKernelGGL(chain<ORDER>, dim3(1), dim3(64), 0, 0, din, dout);
  float h[64];
  (void)hipMemcpy(h, dout, sizeof(h), hipMemcpyDeviceToHost);
  float m = 0.f;
  for (float v : h) m = fmaxf(m, v);
  return m;
}

int main() {
  float hin[1536];
  unsigned s = 12345u;
  for (float& v : hin) {
    s = s * 1664525u + 1013904223u;
    v = (float)((int)(s >> 9) % 2001 - 1000) / 500.f;
  }
  float *din, *dout;
  (void)hipMalloc(&din, sizeof(hin));
  (void)hipMalloc(&dout, 64 * sizeof(float));
  (void)hipMemcpy(din, hin, sizeof(hin), hipMemcpyHostToDevice);
  const char* names[4] = {"16x16x32 -> 16x16x16", "16x16x16 -> 16x16x32", "16x16x32 -> 16x16x32", "16x16x16 -> 16x16x16"};
  const float d[4] = {run<0>(din, dout), run<1>(din, dout), run<2>(din, dout), run<3>(din, dout)};
  for (int i = 0; i < 4; ++i) printf("chain %-22s max |chained - separate| = %g\n", names[i], d[i]);
  return 0;
}
