// permlane32_swap / permlane16_swap semantics on gfx950 (the GEMM epilogue's store widening): each lane starts
// with X = 1000 + lane, Y = 2000 + lane; prints the pair each lane holds after (a) permlane32_swap(X, Y),
// (b) permlane16_swap on (a)'s results, both through the builtins.
// Build: hipcc --offload-arch=gfx950 -O3 permlane_probe.hip -o permlane_probe
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(unsigned* out) {
  const unsigned l = threadIdx.x;
  unsigned X = 1000 + l, Y = 2000 + l;
  auto r = __builtin_amdgcn_permlane32_swap(X, Y, false, false);
  out[l * 4 + 0] = r[0];
  out[l * 4 + 1] = r[1];
  auto q = __builtin_amdgcn_permlane16_swap(r[0], r[1], false, false);
  out[l * 4 + 2] = q[0];
  out[l * 4 + 3] = q[1];
}

int main() {
  unsigned* d;
  unsigned h[256];
  (void)hipMalloc(&d, sizeof(h));
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; l += 4)
    printf("lane %2d: p32 (%u, %u)  p32+p16 (%u, %u)\n", l, h[l * 4], h[l * 4 + 1], h[l * 4 + 2], h[l * 4 + 3]);
  return 0;
}
