// Device-resident episode sampler (replaces the reference's per-step host sampling + H2D copy,
// util/data_loader.py:259-309, SURVEY 3.1 hot loop #1).
//
// Contract (identical to data/sampler.py::EpisodeSampler.sample_indices):
//   * N distinct relations out of R; K+Q distinct instances per relation from its scope;
//   * row layout per episode: support class-major [N*K], then queries [N*Q] randomly permuted;
//   * query label = class index in sampled order; with probability nota_rate a query is
//     replaced by an instance of a relation outside the episode and labelled N (FewRel 2.0).
// Randomness: counter-based hash of (seed, episode, draw) -> independent of launch geometry,
// reproducible, and rank-disjoint when the caller folds the DP rank into the seed.
#include "ina_common.h"

using namespace ina;

namespace {

struct Rng {
  uint32_t key, ctr;
  INA_DEVICE uint32_t next() {
    ctr += 1;
    return hash_u32(hash_u32(key ^ (ctr * 0x9E3779B9u)) + ctr);
  }
  INA_DEVICE uint32_t below(uint32_t n) { return (uint32_t)(((unsigned long long)next() * n) >> 32); }
  INA_DEVICE float uniform() { return (next() >> 8) * (1.0f / 16777216.0f); }
};

constexpr int MAXN = 32;    // ways
constexpr int MAXKQ = 64;   // K + Q per class
constexpr int MAXNQ = 512;  // N * Q

}  // namespace

__global__ __launch_bounds__(64) void sample_episodes_kernel(const int* __restrict__ scopes, int R, int E, int N, int K,
                                                             int Q, uint32_t seed, float nota_rate,
                                                             int* __restrict__ idx_out, int* __restrict__ lab_out,
                                                             const int* __restrict__ seed_dev) {
  if (seed_dev) seed = (uint32_t)seed_dev[0];   // device-resident seed (HIP-graph replay)
  const int ep = blockIdx.x * blockDim.x + threadIdx.x;
  if (ep >= E) return;
  Rng rng{hash_u32(seed * 0x85EBCA77u + 0x27D4EB2Fu) ^ hash_u32((uint32_t)ep + 0x165667B1u), 0u};
  int cls[MAXN];
  for (int i = 0; i < N; ++i) {
    int c;
    bool dup;
    do {
      c = (int)rng.below((uint32_t)R);
      dup = false;
      for (int j = 0; j < i; ++j) dup |= (cls[j] == c);
    } while (dup);
    cls[i] = c;
  }
  const int rowlen = N * K + N * Q;
  int* row = idx_out + (long)ep * rowlen;
  int* lab = lab_out + (long)ep * N * Q;
  int qidx[MAXNQ], qlab[MAXNQ];
  for (int i = 0; i < N; ++i) {
    const int b = scopes[2 * cls[i]], e = scopes[2 * cls[i] + 1];
    const int span = e - b;
    int pick[MAXKQ];
    for (int j = 0; j < K + Q; ++j) {
      int x;
      bool dup;
      do {
        x = (int)rng.below((uint32_t)span);
        dup = false;
        for (int t = 0; t < j; ++t) dup |= (pick[t] == x);
      } while (dup);
      pick[j] = x;
    }
    for (int j = 0; j < K; ++j) row[i * K + j] = b + pick[j];
    for (int j = 0; j < Q; ++j) {
      qidx[i * Q + j] = b + pick[K + j];
      qlab[i * Q + j] = i;
    }
  }
  if (nota_rate > 0.f && R > N) {
    for (int qq = 0; qq < N * Q; ++qq) {
      if (rng.uniform() < nota_rate) {
        int c;
        bool in;
        do {
          c = (int)rng.below((uint32_t)R);
          in = false;
          for (int j = 0; j < N; ++j) in |= (cls[j] == c);
        } while (in);
        const int b = scopes[2 * c], e = scopes[2 * c + 1];
        qidx[qq] = b + (int)rng.below((uint32_t)(e - b));
        qlab[qq] = N;
      }
    }
  }
  // Fisher-Yates permutation of the queries
  for (int i = N * Q - 1; i > 0; --i) {
    const int j = (int)rng.below((uint32_t)(i + 1));
    const int ti = qidx[i], tl = qlab[i];
    qidx[i] = qidx[j];
    qlab[i] = qlab[j];
    qidx[j] = ti;
    qlab[j] = tl;
  }
  for (int i = 0; i < N * Q; ++i) {
    row[N * K + i] = qidx[i];
    lab[i] = qlab[i];
  }
}

namespace ina {

bool sampler_supported(int N, int K, int Q) { return N <= MAXN && K + Q <= MAXKQ && N * Q <= MAXNQ; }

int sample_episodes(const int* scopes, int R, int E, int N, int K, int Q, uint32_t seed, float nota_rate, int* idx,
                    int* lab, const int* seed_dev, hipStream_t st) {
  hipLaunchKernelGGL(sample_episodes_kernel, dim3((E + 63) / 64), dim3(64), 0, st, scopes, R, E, N, K, Q, seed,
                     nota_rate, idx, lab, seed_dev);
  INA_CHECK_LAUNCH();
  return 0;
}

}  // namespace ina
