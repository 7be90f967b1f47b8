// Host-side launcher interface shared by csrc/kernels/*.hip and csrc/bindings.cpp.
// ONE definition of every argument struct (an ODR mismatch between translation units silently
// shifts field offsets, i.e. garbage device pointers).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace ina {
struct LstmArgs {
  const int* inst;
  int S;
  const int* word;
  const int* pos1;
  const int* pos2;
  int L;
  const float* wemb;
  int E;
  const float* p1emb;
  const float* p2emb;
  int PD;
  const void* apack;
  const void* a2pack;
  const float* bias;
  void* hraw;
  void* cst;        // bf16 mode: fp16 cell states; fp32 mode: fp32
  const void* dH;   // bf16 mode: bf16; fp32 mode: fp32
  float* dw_slab;
  float* dpos_slab;
  float* dwemb;
  int bwd_blocks;
  void* hdrop;
  uint32_t seed, thr;
  float inv_kp;
  int drop;
};
int lstm_fwd(const LstmArgs& a, int U, int NX, bool bf16, hipStream_t st);
int lstm_bwd(const LstmArgs& a, int U, int NX, bool bf16, hipStream_t st);
bool lstm_supported(int U, int NX);
size_t lstm_bwd_lds_bytes(int U, int NX, bool bf16, int L, int PD);

struct AttnArgs {
  const void* hraw;
  const int* inst;
  const int* mask;
  int S, L;
  const void* w1pack;
  const void* w1tpack;
  const float* b1;
  const float* w2;
  float* e;
  float* alphas;
  const float* de;
  void* dHraw;      // bf16 mode: bf16; fp32 mode: fp32
  float* slab;
  int blocks;
};
int attn_fwd(const AttnArgs& a, int U, int NT, bool bf16, hipStream_t st);
int attn_bwd(const AttnArgs& a, int U, int NT, bool bf16, hipStream_t st);

int routing_fwd(const float* e, const float* Ws, int E, int N, int K, int Q, int R, int H, float* cls, int blocks,
                hipStream_t st);
int routing_bwd(const float* e, const float* Ws, int E, int N, int K, int Q, int R, int H, const float* dcls, float* de,
                float* slab, int blocks, hipStream_t st);
size_t routing_lds_bytes(int N, int K, int H, int R, bool bwd);

struct NtnArgs {
  const float* cls;
  const float* e;
  int E, N, K, Q, H, h;
  const void* mpack;
  const void* m2pack;
  const void* wpack;
  const void* wtpack;
  const float* wvec;
  const float* bias;
  float* probs;
  const float* dz;
  float* dcls;
  float* de;
  void* dp_out;
  float* dw_slab;
  int blocks;
  int paper;
};
int ntn_fwd(const NtnArgs& a, hipStream_t st);
int ntn_bwd(const NtnArgs& a, hipStream_t st);

int adam_step(float* p, float* m, float* v, const float* g, const unsigned char* l2mask, long n, float lr_t, float b1,
              float b2, float eps, float gscale, float l2, hipStream_t st);
int adagrad_step(float* p, float* acc, const float* g, const unsigned char* l2mask, long n, float lr, float gscale,
                 float l2, hipStream_t st);
int slab_reduce(const float* slabs, long nslab, long len, float* out, int accumulate, hipStream_t st);
bool sampler_supported(int N, int K, int Q);
int sample_episodes(const int* scopes, int R, int E, int N, int K, int Q, uint32_t seed, float nota_rate, int* idx,
                    int* lab, hipStream_t st);
}  // namespace ina
