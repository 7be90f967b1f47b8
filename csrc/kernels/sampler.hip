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
// Every rejection loop ends after MAX_ROUNDS (an exit each wave reaches); one that runs out sets the
// caller's device flag `fail` (the host checks it at log points, ops/sampler.py).
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
constexpr int MAXKQ = 64;   // K + Q per class (one lane per draw)
constexpr int MAXNQ = 512;  // N * Q
constexpr int SW = 4;       // episodes (waves) per workgroup
constexpr int MAX_ROUNDS = 256;   // rejection rounds: an exit every wave reaches (host checks spans >= K + Q)

INA_DEVICE uint32_t stream_key(uint32_t ekey, uint32_t id) { return hash_u32(ekey ^ ((id + 1u) * 0x632BE5ABu)); }

INA_DEVICE void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

}  // namespace

// One wave per episode (the first version ran one THREAD per episode: 32 waves for 2048 episodes and
// the pick / query arrays in scratch).  Lanes work in parallel wherever the draws are independent:
//   classes  : lane i holds class i; a wave-uniform rejection loop (ballot duplicate test);
//   instances: per class, lane j draws pick j from its own counter stream; lanes that collide with a
//              lower lane redraw (ballot) -- K + Q distinct instances in a few rounds;
//   NOTA     : per query, lane-parallel;
//   query permutation: random 32-bit key per query, rank = #smaller keys (ties by index) -> scatter.
__global__ __launch_bounds__(256) void sample_episodes_kernel(const int* __restrict__ scopes, int R, int E, int N, int K,
                                                              int Q, uint32_t seed, float nota_rate,
                                                              int* __restrict__ idx_out, int* __restrict__ lab_out,
                                                              const int* __restrict__ seed_dev, int* __restrict__ fail) {
  __shared__ int s_q[SW][MAXNQ];
  __shared__ int s_l[SW][MAXNQ];
  __shared__ uint32_t s_key[SW][MAXNQ];
  __shared__ int s_x[SW][64];
  if (seed_dev) seed = (uint32_t)seed_dev[0];   // device-resident seed (HIP-graph replay)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int ep = blockIdx.x * SW + w;
  if (ep >= E) return;   // wave-level synchronisation only below
  const uint32_t ekey = hash_u32(seed * 0x85EBCA77u + 0x27D4EB2Fu) ^ hash_u32((uint32_t)ep + 0x165667B1u);
  const int NQ = N * Q, KQ = K + Q;
  const int rowlen = N * K + NQ;
  int* row = idx_out + (long)ep * rowlen;
  int* lab = lab_out + (long)ep * NQ;
  // ---- N distinct classes (every lane runs the same stream: wave-uniform control flow)
  Rng rc{ekey, 0u};
  int my_cls = -1;
  bool exhausted = false;   // a rejection loop ran out of rounds: the episode may hold duplicates
  for (int i = 0; i < N; ++i) {
    int c = 0;
    int round = 0;
    for (; round < MAX_ROUNDS; ++round) {
      c = (int)rc.below((uint32_t)R);
      if (__ballot(lane < i && my_cls == c) == 0) break;
    }
    exhausted |= round == MAX_ROUNDS;
    if (lane == i) my_cls = c;
  }
  // ---- K + Q distinct instances of each class (the N classes' scopes loaded at once: one latency)
  int my_b = 0, my_e = 0;
  if (lane < N) {
    my_b = scopes[2 * my_cls];
    my_e = scopes[2 * my_cls + 1];
  }
  for (int i = 0; i < N; ++i) {
    const int b = __shfl(my_b, i, 64), span = __shfl(my_e, i, 64) - b;
    Rng ri{stream_key(ekey, (uint32_t)(i * 64 + lane)), 0u};
    int x = 0;
    bool need = lane < KQ;
    int round = 0;
    for (; round < MAX_ROUNDS; ++round) {
      if (need) x = (int)ri.below((uint32_t)span);
      s_x[w][lane] = x;
      wave_lds_sync();
      bool dup = false;
      if (lane < KQ)
        for (int k = 0; k < lane; ++k) dup |= (s_x[w][k] == x);
      wave_lds_sync();
      need = dup;
      if (__ballot(need) == 0) break;
    }
    exhausted |= round == MAX_ROUNDS;
    if (lane < K) row[i * K + lane] = b + x;
    else if (lane < KQ) {
      s_q[w][i * Q + lane - K] = b + x;
      s_l[w][i * Q + lane - K] = i;
    }
  }
  wave_lds_sync();
  // ---- NOTA queries: an instance of a relation outside the episode, label N
  if (nota_rate > 0.f && R > N) {
    for (int qq = lane; qq < NQ; qq += 64) {
      Rng rn{stream_key(ekey, (uint32_t)(MAXN * 64 + qq)), 0u};
      if (rn.uniform() < nota_rate) {
        int c = 0;
        int round = 0;
        for (; round < MAX_ROUNDS; ++round) {
          c = (int)rn.below((uint32_t)R);
          bool in = false;
          for (int j = 0; j < N; ++j) in |= (__shfl(my_cls, j, 64) == c);
          if (!in) break;
        }
        if (round == MAX_ROUNDS && fail) fail[0] = 1;   // (lane-divergent: a vector store)
        const int b = scopes[2 * c], e = scopes[2 * c + 1];
        s_q[w][qq] = b + (int)rn.below((uint32_t)(e - b));
        s_l[w][qq] = N;
      }
    }
  }
  if (exhausted && fail && lane == 0) fail[0] = 1;   // every writer stores the same value
  // ---- uniform random permutation of the queries: rank by random keys (ties broken by index)
  for (int qq = lane; qq < NQ; qq += 64) {
    Rng rk{stream_key(ekey, (uint32_t)(2 * MAXN * 64 + qq)), 0u};
    s_key[w][qq] = rk.next();
  }
  wave_lds_sync();
  for (int qq = lane; qq < NQ; qq += 64) {
    const uint32_t kq = s_key[w][qq];
    int rank = 0;
    for (int k = 0; k < NQ; ++k) {
      const uint32_t kk = s_key[w][k];
      rank += (kk < kq || (kk == kq && k < qq)) ? 1 : 0;
    }
    row[N * K + rank] = s_q[w][qq];
    lab[rank] = s_l[w][qq];
  }
}

namespace ina {

bool sampler_supported(int N, int K, int Q) { return N <= MAXN && N <= 64 && K + Q <= MAXKQ && N * Q <= MAXNQ; }

int sample_episodes(const int* scopes, int R, int E, int N, int K, int Q, uint32_t seed, float nota_rate, int* idx,
                    int* lab, const int* seed_dev, int* fail, hipStream_t st) {
  hipLaunchKernelGGL(sample_episodes_kernel, dim3((E + SW - 1) / SW), dim3(256), 0, st, scopes, R, E, N, K, Q, seed,
                     nota_rate, idx, lab, seed_dev, fail);
  INA_CHECK_LAUNCH();
  return 0;
}

}  // namespace ina
