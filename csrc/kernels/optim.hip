// Fused multi-tensor optimizers over ONE flat fp32 parameter buffer (K10 of SURVEY 2.3).
// The same flat gradient buffer is the data-parallel all-reduce bucket, so the whole update is a
// single streaming kernel.  Reference: tf.contrib.layers.optimize_loss(optimizer="Adam") with
// staircase exponential decay (model/base.py:94-99); TF1 Adam update form:
//   lr_t = lr * sqrt(1 - b2^t) / (1 - b1^t)
// t is the number of APPLIED updates: t = (host step count | device step counter) - skips, where
// skips counts the steps the NaN/Inf guard skipped.  The bias correction is computed in the kernel
// from that device count, so a skipped step does not advance Adam's t (skips only changes in
// skipped launches, which never read t: no read/write race between workgroups).
//   m = b1 m + (1 - b1) g ;  v = b2 v + (1 - b2) g^2 ;  p -= lr_t * m / (sqrt(v) + eps)
// Optional L2 (the reference's dead L2 term, opt-in): g += l2 * p where l2mask[i] != 0.
// Adagrad (the paper's optimizer, TF1 form): acc += g^2 ; p -= lr * g / sqrt(acc).
// NaN/Inf guard: nonfinite_flag_kernel sets *flag when any gradient (or the loss) is not finite; the
// optimizer kernels then leave parameters and moments untouched and count the skip on the device
// (no host synchronisation, works inside a captured hipGraph).  The flag lives in the tail of the
// flat gradient buffer, so the per-step gradient zeroing clears it.
#include "ina_common.h"

__global__ __launch_bounds__(256) void nonfinite_flag_kernel(const float* __restrict__ g, long n,
                                                             const float* __restrict__ loss, float* __restrict__ flag) {
  const long stride = (long)gridDim.x * blockDim.x;
  const long t0 = (long)blockIdx.x * blockDim.x + threadIdx.x;
  bool bad = false;
  const long n4 = n >> 2;
  const float4* g4 = reinterpret_cast<const float4*>(g);
  for (long i = t0; i < n4; i += stride) {
    const float4 x = g4[i];
    // |x| <= FLT_MAX is false for NaN and +-Inf
    bad |= !(fabsf(x.x) <= 3.402823466e38f) | !(fabsf(x.y) <= 3.402823466e38f) |
           !(fabsf(x.z) <= 3.402823466e38f) | !(fabsf(x.w) <= 3.402823466e38f);
  }
  for (long i = (n4 << 2) + t0; i < n; i += stride) bad |= !(fabsf(g[i]) <= 3.402823466e38f);
  if (loss && t0 == 0) bad |= !(fabsf(loss[0]) <= 3.402823466e38f);
  if (bad) flag[0] = 1.f;   // benign race: every writer stores the same value
}

__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, float* __restrict__ m, float* __restrict__ v,
                                                   const float* __restrict__ g, const unsigned char* __restrict__ l2mask,
                                                   long n, float lr, int t_host, float b1, float b2, float eps,
                                                   float gscale, float l2, const float* __restrict__ lr_dev,
                                                   const int* __restrict__ t_dev, const float* __restrict__ guard,
                                                   int* __restrict__ skips) {
  if (guard && guard[0] != 0.f) {   // non-finite step: no update; block 0 counts it
    if (blockIdx.x == 0 && threadIdx.x == 0) skips[0] = skips[0] + 1;
    return;
  }
  if (lr_dev) lr = lr_dev[0];   // device-resident schedule (HIP-graph replay)
  const int t = (t_dev ? t_dev[0] : t_host) - (skips ? skips[0] : 0);
  const float lr_t = (float)((double)lr * sqrt(1.0 - pow((double)b2, (double)t)) / (1.0 - pow((double)b1, (double)t)));
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float gi = g[i] * gscale;
    const float pi = p[i];
    if (l2mask && l2mask[i]) gi += l2 * pi;
    const float mi = b1 * m[i] + (1.f - b1) * gi;
    const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    p[i] = pi - lr_t * mi / (sqrtf(vi) + eps);
  }
}

__global__ __launch_bounds__(256) void adagrad_kernel(float* __restrict__ p, float* __restrict__ acc,
                                                      const float* __restrict__ g,
                                                      const unsigned char* __restrict__ l2mask, long n, float lr,
                                                      float gscale, float l2, const float* __restrict__ lr_dev,
                                                      const float* __restrict__ guard, int* __restrict__ skips) {
  if (guard && guard[0] != 0.f) {
    if (blockIdx.x == 0 && threadIdx.x == 0) skips[0] = skips[0] + 1;
    return;
  }
  if (lr_dev) lr = lr_dev[0];
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float gi = g[i] * gscale;
    const float pi = p[i];
    if (l2mask && l2mask[i]) gi += l2 * pi;
    const float a = acc[i] + gi * gi;
    acc[i] = a;
    p[i] = pi - lr * gi * rsqrtf(a);
  }
}

// Per-step control block for HIP-graph replay: a captured step cannot take new scalar kernel
// arguments, so the per-step values are computed on the device by the graph's first kernel from
// counters that live in device memory (the same formulas as the host: runtime/trainer.py
// dropout_seed, ops/sampler.py seeds, ops/optim.py lr_at + TF1 Adam bias correction).
// ctl: [0] dropout seed, [1] sampler seed, [2] global step, [3] sampler calls, [4] optimizer step calls
// lrt: [0] scheduled learning rate for the optimizer kernel (Adam corrects it from ctl[4] - skips)
__global__ void step_control_kernel(int* __restrict__ ctl, float* __restrict__ lrt, long long seedA, long long seedB,
                                    double lr0, double decay_steps, double decay_rate, int staircase, int constant,
                                    int adam, double b1, double b2) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const long long step = ctl[2], calls = ctl[3];
  const long long t = (long long)ctl[4] + 1;
  ctl[0] = (int)((seedA + step * 97LL) & 0x7FFFFFFFLL);
  ctl[1] = (int)((seedB + calls * 7919LL) & 0x7FFFFFFFLL);
  double lr = lr0;
  if (!constant) {
    const double e = staircase ? floor((double)step / decay_steps) : (double)step / decay_steps;
    lr = lr0 * pow(decay_rate, e);
  }
  (void)adam; (void)b1; (void)b2;   // bias correction: adam_kernel, from the applied-step count
  lrt[0] = (float)lr;
  ctl[2] = (int)(step + 1);
  ctl[3] = (int)(calls + 1);
  ctl[4] = (int)t;
}

// Sum `nslab` contiguous slabs of length `len` (fp32) into out (out = sum, or out += sum).
__global__ __launch_bounds__(256) void slab_reduce_kernel(const float* __restrict__ slabs, long nslab, long len,
                                                          float* __restrict__ out, int accumulate) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < len; i += stride) {
    float s = 0.f;
    for (long k = 0; k < nslab; ++k) s += slabs[k * len + i];
    out[i] = accumulate ? out[i] + s : s;
  }
}
// float4 form (len % 4 == 0, 16-byte aligned): four slabs' loads in flight per step, same summation
// order as the scalar kernel (slab 0 first) -- the split-K weight-gradient partials of the BERT GEMMs
// (16 x [o*i]) summed straight into the flat gradient span
__global__ __launch_bounds__(256) void slab_reduce4_kernel(const float4* __restrict__ slabs, long nslab, long len4,
                                                           float4* __restrict__ out, int accumulate) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < len4; i += stride) {
    float4 s = accumulate ? out[i] : float4{0.f, 0.f, 0.f, 0.f};
    float4 t = {0.f, 0.f, 0.f, 0.f};
    long k = 0;
    for (; k + 4 <= nslab; k += 4) {
      const float4 a = slabs[k * len4 + i], b = slabs[(k + 1) * len4 + i], c = slabs[(k + 2) * len4 + i],
                   d = slabs[(k + 3) * len4 + i];
      t.x += a.x; t.y += a.y; t.z += a.z; t.w += a.w;
      t.x += b.x; t.y += b.y; t.z += b.z; t.w += b.w;
      t.x += c.x; t.y += c.y; t.z += c.z; t.w += c.w;
      t.x += d.x; t.y += d.y; t.z += d.z; t.w += d.w;
    }
    for (; k < nslab; ++k) {
      const float4 a = slabs[k * len4 + i];
      t.x += a.x; t.y += a.y; t.z += a.z; t.w += a.w;
    }
    s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w;
    out[i] = s;
  }
}

namespace ina {

static int grid_for(long n) {
  long b = (n + 255) / 256;
  if (b > 2048) b = 2048;
  if (b < 1) b = 1;
  return (int)b;
}

int adam_step(float* p, float* m, float* v, const float* g, const unsigned char* l2mask, long n, float lr, int t_host,
              float b1, float b2, float eps, float gscale, float l2, const float* lr_dev, const int* t_dev,
              const float* guard, int* skips, hipStream_t st) {
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n)), dim3(256), 0, st, p, m, v, g, l2mask, n, lr, t_host, b1, b2, eps,
                     gscale, l2, lr_dev, t_dev, guard, skips);
  INA_CHECK_LAUNCH();
  return 0;
}

int adagrad_step(float* p, float* acc, const float* g, const unsigned char* l2mask, long n, float lr, float gscale,
                 float l2, const float* lr_dev, const float* guard, int* skips, hipStream_t st) {
  hipLaunchKernelGGL(adagrad_kernel, dim3(grid_for(n)), dim3(256), 0, st, p, acc, g, l2mask, n, lr, gscale, l2, lr_dev,
                     guard, skips);
  INA_CHECK_LAUNCH();
  return 0;
}

int nonfinite_flag(const float* g, long n, const float* loss, float* flag, hipStream_t st) {
  long b = (n / 4 + 255) / 256;
  b = b < 1 ? 1 : (b > 512 ? 512 : b);
  hipLaunchKernelGGL(nonfinite_flag_kernel, dim3((int)b), dim3(256), 0, st, g, n, loss, flag);
  INA_CHECK_LAUNCH();
  return 0;
}

int step_control(int* ctl, float* lrt, long long seedA, long long seedB, double lr0, double decay_steps,
                 double decay_rate, int staircase, int constant, int adam, double b1, double b2, hipStream_t st) {
  hipLaunchKernelGGL(step_control_kernel, dim3(1), dim3(64), 0, st, ctl, lrt, seedA, seedB, lr0, decay_steps, decay_rate,
                     staircase, constant, adam, b1, b2);
  INA_CHECK_LAUNCH();
  return 0;
}

int slab_reduce(const float* slabs, long nslab, long len, float* out, int accumulate, hipStream_t st) {
  if (len % 4 == 0 && ((uintptr_t)slabs & 15) == 0 && ((uintptr_t)out & 15) == 0) {
    hipLaunchKernelGGL(slab_reduce4_kernel, dim3(grid_for(len / 4)), dim3(256), 0, st, (const float4*)slabs, nslab,
                       len / 4, (float4*)out, accumulate);
    INA_CHECK_LAUNCH();
    return 0;
  }
  hipLaunchKernelGGL(slab_reduce_kernel, dim3(grid_for(len)), dim3(256), 0, st, slabs, nslab, len, out, accumulate);
  INA_CHECK_LAUNCH();
  return 0;
}

}  // namespace ina
