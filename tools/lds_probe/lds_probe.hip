// LDS bank-conflict probe for the NTN image access patterns (csrc/kernels/ntn.hip): each kernel repeats ONE
// access pattern of the real kernel on a zeroed LDS image; run under
//   rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT -- ./lds_probe
// and compare conflict cycles per instruction.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef unsigned short u16x8_t __attribute__((ext_vector_type(8)));

__device__ __forceinline__ s16x4_t trr(const unsigned char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)p);
}
__device__ int mask_m(int a) { return ((a & 2) << 1) | (a & 8); }
__device__ int mask_p(int r) { return (r & 6) << 1; }

constexpr int REPS = 4096;

// 0: M-image transposed read, rows 8q + (n>>2), chunk 4mb + (n&3), XOR mask_m (all rows real)
// 1: same, lanes q >= 2 redirected to one zero address
// 2: same rows, no swizzle
// 3: P-image row read (ds_read_b128): row n, chunk pair 2q ^ mask_p(n)
// 4: P-image transposed read (16x16x16 pattern): rows 4q + (n>>2), chunk (n&3) ^ mask_p
template <int V>
__global__ __launch_bounds__(256) void probe(int* out, int sel) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[16384 + 256];
  for (int i = threadIdx.x; i < (16384 + 256) / 4; i += 256) reinterpret_cast<int*>(lds)[i] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, q = lane >> 4, n = lane & 15;
  int acc = 0;
  for (int it = 0; it < REPS; ++it) {
    const int mb = (it + sel) & 1;
    if (V <= 2) {
      const int a0 = 8 * q + (n >> 2), c8 = 4 * mb + (n & 3);
      int off = a0 * 128 + ((V == 2 ? c8 : (c8 ^ mask_m(a0))) << 3);
      if (V == 1 && q >= 2) off = 16384;
      s16x4_t v = trr(lds + off);
      acc += v[0] + v[3];
    } else if (V == 5) {   // P-image write from the stacked P^T accumulator: lane n < 10 -> image n / 5, row sl*5 + n % 5
      const int sl = it % 3, g = n / 5, c = n % 5, row = sl * 5 + c;
      if (n < 10) *reinterpret_cast<s16x4_t*>(lds + g * 2048 + row * 128 + (((4 * mb + q) ^ mask_p(row)) << 3)) = s16x4_t{1, 2, 3, (short)it};
    } else if (V == 6) {   // same, images 2048 + 128 B apart
      const int sl = it % 3, g = n / 5, c = n % 5, row = sl * 5 + c;
      if (n < 10) *reinterpret_cast<s16x4_t*>(lds + g * (2048 + 128) + row * 128 + (((4 * mb + q) ^ mask_p(row)) << 3)) = s16x4_t{1, 2, 3, (short)it};
    } else if (V == 7) {   // D write: row n, chunk 4 mb + q
      *reinterpret_cast<s16x4_t*>(lds + n * 128 + (((4 * mb + q) ^ mask_p(n)) << 3)) = s16x4_t{1, 2, 3, (short)it};
    } else if (V == 3) {
      u16x8_t v = *reinterpret_cast<const u16x8_t*>(lds + n * 128 + (((8 * mb + 2 * q) ^ mask_p(n)) << 3));
      acc += v[0] + v[7];
    } else {
      const int pr = 4 * q + (n >> 2);
      s16x4_t v = trr(lds + pr * 128 + (((4 * mb + (n & 3)) ^ mask_p(pr)) << 3));
      acc += v[0] + v[3];
    }
    asm volatile("" : "+v"(acc));
  }
  if (acc == 12345) out[0] = acc;
}

int main() {
  int* d;
  hipMalloc(&d, 4);
  for (int r = 0; r < 2; ++r) {
    hipLaunchKernelGGL(probe<0>, dim3(256), dim3(256), 0, 0, d, r);
    hipLaunchKernelGGL(probe<1>, dim3(256), dim3(256), 0, 0, d, r);
    hipLaunchKernelGGL(probe<2>, dim3(256), dim3(256), 0, 0, d, r);
    hipLaunchKernelGGL(probe<3>, dim3(256), dim3(256), 0, 0, d, r);
    hipLaunchKernelGGL(probe<4>, dim3(256), dim3(256), 0, 0, d, r);
    hipLaunchKernelGGL(probe<5>, dim3(256), dim3(256), 0, 0, d, r);
    hipLaunchKernelGGL(probe<6>, dim3(256), dim3(256), 0, 0, d, r);
    hipLaunchKernelGGL(probe<7>, dim3(256), dim3(256), 0, 0, d, r);
  }
  hipDeviceSynchronize();
  printf("done\n");
  return 0;
}
