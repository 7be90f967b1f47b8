// Issue rate of v_mfma_f32_16x16x16_bf16 vs v_mfma_f32_16x16x32_bf16 on gfx950 (4 independent accumulators,
// one wave per SIMD, every CU): kernel time under rocprofv3 --kernel-trace --stats.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
constexpr int ITERS = 20000;
template <int K32>
__global__ __launch_bounds__(256) void rate(float* out, float seed) {
  f32x4_t c0 = {seed, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  const short s = (short)threadIdx.x;
  s16x4_t a4 = {s, 1, 2, 3};
  bf16x8_t a8 = __builtin_bit_cast(bf16x8_t, (short __attribute__((ext_vector_type(8)))){s, 1, 2, 3, 4, 5, 6, 7});
  for (int i = 0; i < ITERS; ++i) {
    if (K32) {
      c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, a8, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, a8, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, a8, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, a8, c3, 0, 0, 0);
    } else {
      c0 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, a4, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, a4, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, a4, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, a4, c3, 0, 0, 0);
    }
  }
  const f32x4_t c = c0 + c1 + c2 + c3;
  if (c[0] == 12345.f) out[threadIdx.x] = c[1];
}
int main() {
  float* d;
  (void)hipMalloc(&d, 4096);
  for (int r = 0; r < 3; ++r) {
    hipLaunchKernelGGL(rate<1>, dim3(256), dim3(256), 0, 0, d, 1.f);
    hipLaunchKernelGGL(rate<0>, dim3(256), dim3(256), 0, 0, d, 1.f);
  }
  (void)hipDeviceSynchronize();
  printf("done\n");
  return 0;
}
