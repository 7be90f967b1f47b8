// Length-sorted row plan of the ragged record path (ops/encoder.py::ragged_plan) as a stable counting
// sort: sequence lengths are small integers (0..L, L <= 64), so a histogram + scan + ordered scatter
// replaces torch.argsort(stable=True) -- rocprim's merge sort took ~9 merge passes + partitions
// (~130 us per step at 409,600 rows) plus ~8 index / clamp / cast launches around it.
//
//   ragged_hist    : per 1024-row block, the row count of every length bin (ballot + popcount per bin:
//                    no atomics, deterministic) -> counts[bin][block]
//   ragged_scan    : one workgroup, exclusive scan of counts in (bin, block) order -> offsets
//   ragged_scatter : row r of block B with length b goes to offsets[b][B] + (rows of b in earlier waves
//                    of B) + (rows of b in earlier lanes of its wave): exactly the stable argsort.
//                    Writes perm, inst_sorted, slen and, for the last row of every 16-row tile, the
//                    tile's longest length tlen = max(1, slen[16 t + 15]).
#include "ina_common.h"
#include "ina_launch.h"

using namespace ina;

namespace {

constexpr int RS_ROWS = 1024;   // rows per block (16 waves x 64)
constexpr int RS_BINS = 72;     // lengths 0..71

INA_DEVICE uint64_t lanemask_lt(int lane) { return lane == 0 ? 0ull : (~0ull >> (64 - lane)); }

// the row's length bin (clamped into [0, nbins - 1]: a corrupt length can never index past the LDS
// tables or the offsets), -1 past the last row
INA_DEVICE int row_len(const int* __restrict__ inst, const int* __restrict__ lengths, long r, long S, int nbins) {
  if (r >= S) return -1;
  const int v = lengths[inst[r]];
  return v < 0 ? 0 : (v >= nbins ? nbins - 1 : v);
}

__global__ __launch_bounds__(RS_ROWS) void ragged_hist_kernel(const int* __restrict__ inst,
                                                              const int* __restrict__ lengths, long S, int nbins,
                                                              int* __restrict__ counts) {
  __shared__ int wc[16][RS_BINS];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long r = (long)blockIdx.x * RS_ROWS + threadIdx.x;
  const int b = row_len(inst, lengths, r, S, nbins);
  for (int k = 0; k < nbins; ++k) {
    const uint64_t m = __ballot(b == k);
    if (lane == 0) wc[wave][k] = __popcll(m);
  }
  __syncthreads();
  for (int k = threadIdx.x; k < nbins; k += RS_ROWS) {
    int s = 0;
    for (int w = 0; w < 16; ++w) s += wc[w][k];
    counts[(long)k * gridDim.x + blockIdx.x] = s;
  }
}

// exclusive scan of n ints in one 1024-thread workgroup.  n <= 16 * 1024 (the default shapes): the counts
// go through LDS with coalesced loads / stores (thread-contiguous chunks read straight from global memory
// touched a different cache line per lane and instruction: ~13 us for 60 KB), each thread scans its
// contiguous chunk of <= 16 from LDS, and the block scan is a wave-shuffle scan plus the 16 wave totals.
// Larger n: the same with the chunks read from global memory.
constexpr int SC_REG = 16;
__global__ __launch_bounds__(1024) void ragged_scan_kernel(const int* __restrict__ counts, long n,
                                                           int* __restrict__ offsets) {
  __shared__ int buf[SC_REG * 1024];
  __shared__ int part[16];
  const long chunk = (n + 1023) / 1024;
  const long beg = threadIdx.x * chunk, end = beg + chunk < n ? beg + chunk : n;
  const bool lds = chunk <= SC_REG;   // uniform
  int v[SC_REG];
  int s = 0;
  if (lds) {
    for (long i = threadIdx.x; i < n; i += 1024) buf[i] = counts[i];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < SC_REG; ++j) {
      v[j] = (beg + j < end) ? buf[beg + j] : 0;
      s += v[j];
    }
  } else {
    for (long i = beg; i < end; ++i) s += counts[i];
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int inc = s;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int x = __shfl_up(inc, d, 64);
    if (lane >= d) inc += x;
  }
  if (lane == 63) part[wave] = inc;
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int w = 0; w < 16; ++w) {
      const int t = part[w];
      part[w] = acc;
      acc += t;
    }
  }
  __syncthreads();
  int run = part[wave] + inc - s;   // exclusive prefix of this thread's chunk
  if (lds) {
#pragma unroll
    for (int j = 0; j < SC_REG; ++j) {
      if (beg + j < end) buf[beg + j] = run;
      run += v[j];
    }
    __syncthreads();
    for (long i = threadIdx.x; i < n; i += 1024) offsets[i] = buf[i];
  } else {
    for (long i = beg; i < end; ++i) {
      offsets[i] = run;
      run += counts[i];
    }
  }
}

__global__ __launch_bounds__(RS_ROWS) void ragged_scatter_kernel(const int* __restrict__ inst,
                                                                 const int* __restrict__ lengths, long S,
                                                                 int nbins, const int* __restrict__ offsets,
                                                                 int* __restrict__ perm, int* __restrict__ inst_s,
                                                                 int* __restrict__ slen, int* __restrict__ tlen) {
  __shared__ int wc[16][RS_BINS];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long r = (long)blockIdx.x * RS_ROWS + threadIdx.x;
  const int b = row_len(inst, lengths, r, S, nbins);
  int rank = 0;
  for (int k = 0; k < nbins; ++k) {
    const uint64_t m = __ballot(b == k);
    if (lane == 0) wc[wave][k] = __popcll(m);
    if (b == k) rank = __popcll(m & lanemask_lt(lane));
  }
  __syncthreads();
  if (r < S) {
    int before = 0;
    for (int w = 0; w < wave; ++w) before += wc[w][b];
    const long pos = offsets[(long)b * gridDim.x + blockIdx.x] + before + rank;
    perm[pos] = (int)r;
    inst_s[pos] = inst[r];
    slen[pos] = b;
    if ((pos & 15) == 15 || pos == S - 1) tlen[pos >> 4] = b > 1 ? b : 1;
  }
}

}  // namespace

namespace ina {

int ragged_blocks(long S) { return (int)((S + RS_ROWS - 1) / RS_ROWS); }
int ragged_max_len() { return RS_BINS - 1; }

// ws: >= 2 * nbins * ragged_blocks(S) ints
int ragged_sort(const int* inst, const int* lengths, long S, int L, int* ws, int* perm, int* inst_s, int* slen,
                int* tlen, hipStream_t st) {
  if (L < 0 || L > RS_BINS - 1) return -1;
  if (S <= 0) return 0;
  const int nb = ragged_blocks(S), nbins = L + 1;
  int* counts = ws;
  int* offsets = ws + (long)nbins * nb;
  hipLaunchKernelGGL(ragged_hist_kernel, dim3(nb), dim3(RS_ROWS), 0, st, inst, lengths, S, nbins, counts);
  hipLaunchKernelGGL(ragged_scan_kernel, dim3(1), dim3(1024), 0, st, counts, (long)nbins * nb, offsets);
  hipLaunchKernelGGL(ragged_scatter_kernel, dim3(nb), dim3(RS_ROWS), 0, st, inst, lengths, S, nbins, offsets, perm,
                     inst_s, slen, tlen);
  INA_CHECK_LAUNCH();
  return 0;
}

}  // namespace ina
