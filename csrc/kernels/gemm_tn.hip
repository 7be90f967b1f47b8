// Reduction ("wgrad") GEMM over a long K, both operands K-major rows, fp32 split slabs:
//
//     slab[s][i][j] = sum_{k in split s} A[k][i] B[k][j]      A [K][lda] bf16 (i < MI <= 64), B [K][ldb] bf16
//
// The headline use is the NTN's dM = C^T dP (reference model/layer_module.py:16-37 through autodiff): K = E N
// class rows (40,960 at 8192 episodes), MI = H = 40, NJ = h H = 4,000 -- a 40 x 4,000 output streamed from a
// 328 MB dP.  The step glue sums the split slabs in a fixed order (deterministic) while scattering them into
// the flat gradient.
//
// Workgroup: 8 waves, tile 64 (i) x 256 (j) x 64 (k) per K-step; wave w owns columns 32 w .. 32 w + 31 and all
// i tiles (16x16x32 bf16 MFMA, fp32 accumulation).  Both operands are staged by LDS-DMA (inline asm, double
// buffered, one barrier per K-step) as K-major images and read TRANSPOSED with ds_read_b64_tr_b16: A^T[i][k]
// and B[k][j] fragments come straight out of the row-major [k][.] images.  16-byte chunks of image row k are
// XOR-swizzled (A: 128-B rows, chunk ^ 2 ((k >> 1 & 1) | (k >> 3 & 1) << 1); B: 512-B rows,
// chunk ^ 2 ((k & 3) | (k >> 3 & 1) << 2)) so the transposed reads (rows 8q + 0..3, 8q + 8..11 of a lane
// group) are bank-conflict free; the swizzle is applied to the DMA SOURCE address (LDS-DMA writes lane-linearly).
// A's columns i >= MI stage from a zero buffer; B's columns past NJ stage from a clamped address and are
// never stored.  K must be a multiple of 64 (callers pad the operand rows with zeros).
#include "ina_common.h"
#include "ina_launch.h"

using namespace ina;

namespace {

constexpr int TK = 64, TJ = 256, TI = 64, TN_THREADS = 512;
constexpr int A_IMG = TK * TI * 2;            // 8 KiB
constexpr int B_IMG = TK * TJ * 2;            // 32 KiB
constexpr int TN_BUF = A_IMG + B_IMG;
constexpr int TN_LDS = 2 * TN_BUF;            // 80 KiB: two workgroups per CU

INA_DEVICE int fa(int k) { return 2 * (((k >> 1) & 1) | (((k >> 3) & 1) << 1)); }
INA_DEVICE int fb(int k) { return 2 * ((k & 3) | (((k >> 3) & 1) << 2)); }
INA_DEVICE s16x4_t trr(uint32_t a) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)(uintptr_t)a);
}
INA_DEVICE u16x8_t cat8(const s16x4_t& lo, const s16x4_t& hi) {
  return u16x8_t{(unsigned short)lo[0], (unsigned short)lo[1], (unsigned short)lo[2], (unsigned short)lo[3],
                 (unsigned short)hi[0], (unsigned short)hi[1], (unsigned short)hi[2], (unsigned short)hi[3]};
}

struct TnArgs {
  const unsigned short* A;
  const unsigned short* B;
  const unsigned short* zero;   // >= 16 B of zeros
  float* slab;
  int K, MI, NJ, lda, ldb, ksteps;   // ksteps: K-steps per split
};

template <int MIT>
__global__ __launch_bounds__(TN_THREADS, 2) void gemm_tn_slab_kernel(TnArgs g) {
  extern __shared__ __attribute__((aligned(16))) unsigned char tn_lds[];
  const int lane = threadIdx.x & 63, q = lane >> 4, n = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int j0 = blockIdx.x * TJ, split = blockIdx.y;
  const int kb0 = split * g.ksteps;
  const int nks = min(g.ksteps, g.K / TK - kb0);
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_addr(tn_lds));
  // DMA geometry.  A: wave w fills image rows 8 w .. 8 w + 7 (lane: row l >> 3, 16-B chunk l & 7);
  // B: wave w fills rows 8 w .. 8 w + 7, four 1-KiB pieces of two rows (lane: row l >> 5, chunk l & 31)
  const int ar = 8 * wave + (lane >> 3), ap = lane & 7, alog = ap ^ fa(ar);
  const bool a_ok = 8 * alog < g.MI;
  const unsigned char* asrc = a_ok ? reinterpret_cast<const unsigned char*>(g.A) + ((long)ar * g.lda + 8 * alog) * 2
                                   : reinterpret_cast<const unsigned char*>(g.zero);
  const long astep = a_ok ? (long)TK * g.lda * 2 : 0;
  const unsigned char* bsrc[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const int br = 8 * wave + 2 * d + (lane >> 5), bp = lane & 31, blog = bp ^ fb(br);
    int j = j0 + 8 * blog;
    if (j > g.NJ - 8) j = g.NJ - 8;   // columns past NJ: any valid bytes (never stored)
    bsrc[d] = reinterpret_cast<const unsigned char*>(g.B) + ((long)br * g.ldb + j) * 2;
  }
  const long bstep = (long)TK * g.ldb * 2;
  auto stage = [&](int buf, int ks) {   // K-step ks (absolute) -> buffer buf
    const uint32_t base = lds0 + buf * TN_BUF;
    glds16_asm(asrc + (long)ks * astep, base + wave * 1024);
#pragma unroll
    for (int d = 0; d < 4; ++d) glds16_asm(bsrc[d] + (long)ks * bstep, base + A_IMG + (4 * wave + d) * 1024);
  };
  f32x4_t acc[MIT][2];
#pragma unroll
  for (int it = 0; it < MIT; ++it) acc[it][0] = acc[it][1] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  if (nks > 0) stage(0, kb0);
  for (int s = 0; s < nks; ++s) {
    const int buf = s & 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();   // K-step s landed for every wave; everyone is done with buffer buf ^ 1
    if (s + 1 < nks) stage(buf ^ 1, kb0 + s + 1);
    const uint32_t abase = lds0 + buf * TN_BUF, bbase = abase + A_IMG;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int r0 = 32 * kk + 8 * q + (n >> 2), r1 = r0 + 4;
      u16x8_t bf[2];
#pragma unroll
      for (int jt = 0; jt < 2; ++jt) {
        const int P = 4 * (2 * wave + jt) + (n & 3);   // logical 8-B piece of the row: j = 4 P
        const int c = P >> 1, h = (P & 1) * 8;
        bf[jt] = cat8(trr(bbase + r0 * 512 + ((c ^ fb(r0)) << 4) + h), trr(bbase + r1 * 512 + ((c ^ fb(r1)) << 4) + h));
      }
#pragma unroll
      for (int it = 0; it < MIT; ++it) {
        const int P = 4 * it + (n & 3);
        const int c = P >> 1, h = (P & 1) * 8;
        const u16x8_t af = cat8(trr(abase + r0 * 128 + ((c ^ fa(r0)) << 4) + h), trr(abase + r1 * 128 + ((c ^ fa(r1)) << 4) + h));
#pragma unroll
        for (int jt = 0; jt < 2; ++jt) acc[it][jt] = mfma_bf16(af, bf[jt], acc[it][jt]);
      }
    }
  }
  float* out = g.slab + (long)split * g.MI * g.NJ;
#pragma unroll
  for (int it = 0; it < MIT; ++it)
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) {
      const int j = j0 + 32 * wave + 16 * jt + n;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 16 * it + 4 * q + r;
        if (i < g.MI && j < g.NJ) out[(long)i * g.NJ + j] = acc[it][jt][r];
      }
    }
}

template <int MIT>
int launch_tn(const TnArgs& a, int splits, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute((const void*)gemm_tn_slab_kernel<MIT>, hipFuncAttributeMaxDynamicSharedMemorySize, TN_LDS) !=
        hipSuccess)
      return 2;
    attr = true;
  }
  hipLaunchKernelGGL(gemm_tn_slab_kernel<MIT>, dim3((a.NJ + TJ - 1) / TJ, splits), dim3(TN_THREADS), TN_LDS, st, a);
  INA_CHECK_LAUNCH();
  return 0;
}

}  // namespace

namespace ina {

int gemm_tn_splits(int K, int MI, int NJ) {
  const int ksteps = K / TK, jt = (NJ + TJ - 1) / TJ;
  int s = (512 + jt - 1) / jt;   // ~512 workgroups (two per CU)
  if (s > ksteps) s = ksteps;
  return s > 0 ? s : 1;
}

int gemm_tn_slab(const void* A, int lda, const void* B, int ldb, int K, int MI, int NJ, const void* zero, float* slab,
                 int splits, hipStream_t st) {
  if (K <= 0 || K % TK != 0 || MI <= 0 || MI > TI || MI % 8 != 0 || NJ < 8 || NJ % 8 != 0) return 1;
  if (lda < MI || ldb < NJ || lda % 8 != 0 || ldb % 8 != 0 || splits <= 0) return 1;
  const int ksteps_total = K / TK;
  TnArgs a{(const unsigned short*)A, (const unsigned short*)B, (const unsigned short*)zero, slab, K, MI, NJ, lda, ldb,
           (ksteps_total + splits - 1) / splits};
  const int MIT = (MI + 15) / 16;
  if (MIT == 1) return launch_tn<1>(a, splits, st);
  if (MIT == 2) return launch_tn<2>(a, splits, st);
  if (MIT == 3) return launch_tn<3>(a, splits, st);
  return launch_tn<4>(a, splits, st);
}

}  // namespace ina
