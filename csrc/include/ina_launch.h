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
  unsigned char* dmask;  // [tiles][2][L][64] dropout keep bits (bit m = unit 4m+q), written by fwd, read by bwd
  const int* seed_dev;   // optional device-resident dropout seed (overrides seed; HIP-graph replay)
  void* dxp;             // bf16 bwd: pos-feature gradients [2 dir][tiles][L][2PD + 1 (trash row)][16] (reduced by pos_grad)
  void* xg;              // bf16: x_gather output [tiles][L][64 lanes][NX] (input of lstm_fwd / lstm_bwd)
  const unsigned short* posb;   // bf16: x_gather position ids [tiles][L][16] = pos1 | pos2 << 8
  const void* wrows;     // optional bf16 [NI * L][8]: word rows per token, zero padded (x_gather DIRECT)
  uint32_t seed, thr;
  float inv_kp;
  int drop;
  int dh_lane;           // bwd: dH in the step-record lane layout [tiles][2][L][U/4][64] (else [S][L][2U])
  // ragged tiles (bf16 record path; rows sorted by length on the host, ops/encoder.py): tlen[tile] = the
  // tile's longest valid length.  The forward direction and the attention stop there (padding outputs are
  // masked: exact); the backward direction runs all L steps (parity) or, with slen (the sorted rows'
  // lengths; lstm_skip_padding), starts at tlen - 1 and resets each row's state past its own length
  const int* tlen;
  const int* slen;
  const int* perm;   // x_gather: record row s is original row perm[s] (dropout hash counter)
  int wblank;        // bwd with a trained word table: the padding (BLANK) row id, summed in registers (-1: none)
  // direct x (bf16 record path, NX == 4, shifted position ids, wrows given): lstm_fwd / lstm_bwd read each
  // token's word features straight from wrows (q-interleaved rows [f0 f4 f1 f5 f2 f6 f3 f7], one dword per
  // lane-step) and its position features from block-resident LDS tables at o_s + t; x_gather then writes
  // only posb / dmask (no xg record).  wbytes = wrows' size in bytes (buffer range: rows past it read 0)
  int xd;
  uint32_t wbytes;
  void* xdtab;   // direct x: the position tables (x_gather writes them, the recurrences copy them into LDS)
};
// bf16 mode: gather every token's x features once into a.xg / a.posb, and (a.drop) the dropout keep
// bits into a.dmask (lstm.hip x_gather_kernel); must run before lstm_fwd in bf16 mode
int x_gather(const LstmArgs& a, int U, int NX, hipStream_t st);
int lstm_fwd(const LstmArgs& a, int U, int NX, bool bf16, hipStream_t st);
// bf16: the h slots of lstm_fwd's step records [tiles][2][L][2][U/4][64] -> natural rows
// [16 * tiles][L][2U], with the dropout keep bits [tiles][2][L][64] applied when dmask is non-null
int h_natural(const void* rec, const unsigned char* dmask, float inv_kp, int S, int L, int U, void* hnat,
              hipStream_t st);
int lstm_bwd_resident_blocks(int U, int NX, bool bf16, int L, int PD);
int lstm_bwd(const LstmArgs& a, int U, int NX, bool bf16, hipStream_t st);
// bf16 mode: reduce a.dxp into slab [blocks][2 tables][2L][PD] (needs 2L <= 128, 2PD <= 16)
int pos_grad(const LstmArgs& a, int blocks, float* slab, hipStream_t st);
// bf16 mode, position ids pos[s][t] = o_s + t (checked by the caller): the same reduction as a
// per-sequence one-hot GEMM (gpart: pos_shift_workspace_floats floats) -> out [2 tables][2L][PD]
size_t pos_shift_workspace_floats(int S, int L, int PD, int* nchunk, int* kps);
int pos_grad_shift(const LstmArgs& a, float* gpart, float* out, hipStream_t st);
bool lstm_supported(int U, int NX);
size_t lstm_bwd_lds_bytes(int U, int NX, bool bf16, int L, int PD, bool direct_x = false);
// direct-x position tables in LDS: [4 lane groups q][2 tables][2L rows][4 slots] bf16
inline size_t xd_table_bytes(int L) { return (size_t)4 * 2 * 2 * L * 4 * 2; }

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
  const int* tlen;  // rec_attn: per-tile step count (ragged tiles; nullptr = L)
  const int* perm;  // rec_attn: row s of the (length-sorted) records is row perm[s] of e / alphas / de
};
int attn_fwd(const AttnArgs& a, int U, int NT, bool bf16, hipStream_t st);
int attn_bwd(const AttnArgs& a, int U, int NT, bool bf16, hipStream_t st);
int attn_bwd_resident_blocks(int U, int NT, bool bf16);
// bf16, attention straight from lstm_fwd's step records (+ keep bits), rec_attn.hip:
//   fwd: a.w1pack = w1r pack -> a.e, a.alphas
//   bwd: a.w1pack / a.w1tpack = w1r / w1rt packs, a.de, a.e (forward output), a.alphas -> a.dHraw (bf16 [tiles][2][L][U/4][64]),
//        a.slab [a.blocks][H2*H2 + 2*H2]
int rec_attn_fwd(const void* rec, const unsigned char* dmask, float inv_kp, const AttnArgs& a, int U, hipStream_t st);
int rec_attn_bwd(const void* rec, const unsigned char* dmask, float inv_kp, const AttnArgs& a, int U, hipStream_t st);
int rec_attn_bwd_resident_blocks(int U);

int routing_fwd(const float* e, const float* Ws, int E, int N, int K, int Q, int R, int H, float* cls, int blocks,
                hipStream_t st);
int routing_bwd(const float* e, const float* Ws, int E, int N, int K, int Q, int R, int H, const float* dcls, float* de,
                float* slab, int blocks, hipStream_t st);
size_t routing_lds_bytes(int N, int K, int H, int R, bool bwd);
int routing_bwd_default_blocks(int N, int K, int H, int R);

// Neural tensor layer (ntn.hip).  The weights come as ONE per-step "tile pack" (ops/packing.py::pack_ntn_tiles):
// slice tile t (SG = ntn_slices_per_tile(N) slices, rows (slice, class) of the MFMA tiles) = SG swizzled bf16
// images of M[:, :, s] [16 MTH rows a][64 cols b] + the 16x16x16 fragments W [(s,c)][c'] and Wt [c'][(s,c)]
// of the relation FC (reference head: w[s N + c][c']; paper head: w[s] on the diagonal c == c').
struct NtnArgs {
  const float* cls;      // [E][N][H] class vectors
  const float* e;        // [E * (N K + N Q)][H] sentence vectors (query rows used)
  int E, N, K, Q, H, h;
  const void* tiles;     // [ntile][tpb bytes] tile pack
  int G;                 // episodes stacked per wave (class rows (g, c) of the P / dC tiles), ntn_episodes_per_wave
  int SG, ntile, tpb;    // slices per tile, tiles, bytes per tile
  int paper;
  const float* bias;
  float* probs;          // fwd: [E][NQ][N]
  const float* dz;       // bwd: dL/dlogit [E][NQ][N]
  const float* gscale;   // bwd: optional device scalar multiplying dz (upstream loss gradient)
  float* dcls;           // bwd: [E][N][H]
  float* de;             // bwd: query rows of [E * (N K + N Q)][H]
  void* dp_out;          // bwd: bf16 dP [Kp][h H] (Kp = E N padded to 64; operand of the dM GEMM), + trash tail
  float* dw_slab;        // bwd: [ngroups][ntile][SG N][N] (reference) / [ngroups][ntile][SG] (paper)
  void* cls_bf;          // bwd: bf16 copy of cls [Kp][H] (the dM GEMM's other operand)
  int blocks;
  // slice split (small E, ntn_split): grid.y workgroup rows over the tiles; partials in part (fwd: logits
  // [split][E][NQ][N]; bwd: dC [split][E][N][H]) and part2 (bwd: dQ [split][E][NQ][H])
  int split;
  float* part;
  float* part2;
};
int ntn_slices_per_tile(int N);
int ntn_episodes_per_wave(int N, int Q);
int ntn_split(int E, int N, int Q, int h);
int ntn_groups(int E, int N, int Q);   // workgroup groups of episodes (rows of the dw slab)
int ntn_fwd(const NtnArgs& a, hipStream_t st);

// step glue (glue.hip)
constexpr int SLAB_MAX_JOBS = 8;
struct SlabJobs {   // passed by value as a kernel argument (no per-step host->device copies)
  const float* src[SLAB_MAX_JOBS];    // slab [nblk][n] fp32
  const int* map[SLAB_MAX_JOBS];      // [n] destination index (-1 = skip)
  const float* scale[SLAB_MAX_JOBS];  // optional device scalar multiplier
  long n[SLAB_MAX_JOBS];
  int nblk[SLAB_MAX_JOBS];
  int nch[SLAB_MAX_JOBS];             // row chunks of the job (partial sums)
  long wsbase[SLAB_MAX_JOBS];         // job's partials in the workspace: [nch][n]
  int vec[SLAB_MAX_JOBS];             // partial launch in float4 columns (n % 4 == 0, 16-byte aligned rows)
  long bbase[SLAB_MAX_JOBS + 1];      // prefix sums of ceil(n/cw) * nch, cw = 256 (vec) or 64 (partial workgroups)
  long fbase[SLAB_MAX_JOBS + 1];      // prefix sums of ceil(n/256) (finish-launch workgroups, a thread per column)
  int njobs;
};
// out[a][c][b] = in[a][b][c] for in [A][B][C] fp32; out fp32 or bf16 (glue.hip)
int transpose12(const float* in, void* out, int A, int B, int C, bool bf16, hipStream_t st);
int gather_pack(const float* src, const int* idx, long nb, long ntot, void* outb, float* outf, hipStream_t st,
                const float* ma = nullptr);
int head_loss(const float* probs, const int* labels, long rows, int N, float scale, int ce, float* dz, float* out,
              float* part, int blocks, hipStream_t st);
int head_loss_part_floats();
int slab_scatter(const SlabJobs& jobs, float* dst, float* ws, hipStream_t st);
int ntn_bwd(const NtnArgs& a, hipStream_t st);

int adam_step(float* p, float* m, float* v, const float* g, const unsigned char* l2mask, long n, float lr, int t_host,
              float b1, float b2, float eps, float gscale, float l2, const float* lr_dev, const int* t_dev,
              const float* guard, int* skips, hipStream_t st);
int adagrad_step(float* p, float* acc, const float* g, const unsigned char* l2mask, long n, float lr, float gscale,
                 float l2, const float* lr_dev, const float* guard, int* skips, hipStream_t st);
int nonfinite_flag(const float* g, long n, const float* loss, float* flag, hipStream_t st);
int step_control(int* ctl, float* lrt, long long seedA, long long seedB, double lr0, double decay_steps,
                 double decay_rate, int staircase, int constant, int adam, double b1, double b2, hipStream_t st);
int slab_reduce(const float* slabs, long nslab, long len, float* out, int accumulate, hipStream_t st);
bool sampler_supported(int N, int K, int Q);
int sample_episodes(const int* scopes, int R, int E, int N, int K, int Q, uint32_t seed, float nota_rate, int* idx,
                    int* lab, const int* seed_dev, int* fail, hipStream_t st);

// ---------------------------------------------------------------- wide BiLSTM cell (lstm_wide.hip)
struct LstmWideArgs {
  int S, L, U;
  const float* gx;    // [2][S][L][4U] fp32
  const float* gh;    // [2][S][4U]
  float* c;           // [2][S][U]
  void* hcur;         // [2][S][U] bf16
  void* hall;         // [2][S][L][U] bf16
  float* call;        // [2][S][L][U]
  void* acts;         // [2][S][L][4U] bf16
  void* hout;         // [S][L][2U] bf16
  const void* dH;     // [S][L][2U] bf16
  const float* dhrec; // [2][S][U]
  float* dcrec;       // [2][S][U]
  void* dG;           // [2][S][L][4U] bf16
  void* dGcur;        // [2][S][4U] bf16
  uint32_t salt0, salt1, thr;
  float inv_kp;
  int drop;
};
int lstm_wide_fwd_step(const LstmWideArgs& a, int tau, hipStream_t st);
int lstm_wide_bwd_step(const LstmWideArgs& a, int tau, hipStream_t st);
// persistent wide BiLSTM (whole recurrence in one launch per pass; U in {64, 100, 128}, lstm_wide.hip):
// gate columns permuted to c = 4u + g (u < UP = U padded to 32), ops/packing.py::pack_lstm_wide
struct WideSeqArgs {
  int S, L, U;
  const void* gx;         // [S*L][2][G4] bf16: x W_x (pre-scaled, row s*L + t, both directions)
  const float* bx;        // [2][G4] fp32: pre-scaled biases (forget gate +1)
  const void* apk;        // [2][NW][4][KS][64] x 8 bf16 forward W_h fragments (pre-scaled)
  const void* a2pk;       // [2][NW][KS2][64] x 8 bf16 backward W_h fragments
  void* hprev;            // bf16 each step's recurrent input h_{t-1} (dW_h GEMM operand): direction d, row s L + t at
                          // hprev + d hdo + (s L + t) hld ([2][S][L][UP]: hld = UP, hdo = S L UP; or columns of
                          // the x rows [S L][DP + 2 UP]: hld = DP + 2 UP, hdo = UP)
  int hld;
  long hdo;
  void* acts;             // i, j, f, o activations, bf16, tile-major (lstm_wide.hip WideStash)
  void* cst;              // cell states, fp16, tile-major (lstm_wide.hip WideStash)
  void* hout;             // [S][L][2U] bf16: DropoutWrapper output (attention input)
  const void* dH;         // [S][L][2U] bf16: gradient w.r.t. hout
  void* dG;               // [S*L][2][G4] bf16: pre-activation gate gradients (both directions)
  const void* wpk;        // [2][KS2][64] x 8 bf16 W_pos^T fragments (backward dX_pos; with dxp)
  float* dxp;             // [2][S*L][np] fp32: dX_pos = dG W_pos^T per direction (nullptr: not computed)
  int np;                 // position columns (2 PD <= 16)
  uint32_t salt0, salt1, thr;
  float inv_kp;
  int drop;
  int stash;              // forward: write hprev / acts / cst (training)
};
bool lstm_wide_seq_supported(int U);
int wide_x_gather(const int* inst, int S, int L, const int* word, const int* pos1, const int* pos2, const void* wemb,
                  bool wemb_bf16, int E, const float* p1emb, const float* p2emb, int PD, int DP, void* xb, int ldx,
                  hipStream_t st);
int wide_pos_grad(const float* dxp, const int* inst, const int* pos1, const int* pos2, int S, int L, int PD, int P2,
                  int chunks, int planes, float* part, hipStream_t st);
int lstm_wide_seq_fwd(const WideSeqArgs& a, hipStream_t st);
int lstm_wide_seq_bwd(const WideSeqArgs& a, hipStream_t st);

// self-attention pooling over the wide BiLSTM outputs, H = 2u in {128, 200, 256} (attn_wide.hip)
struct WideAttnArgs {
  int S, L, H, SB;        // SB sequences per workgroup
  const void* hin;        // [S][L][H] bf16 (the BiLSTM output)
  const int* inst;        // [S] dataset rows of the sequences
  const int* mask;        // [rows][L] int32, > 0 = real token
  const void* w1t;        // [HP/16][HP/32][64] x 8 bf16: A fragments of W1^T (row j, k = input feature)
  const void* w1;         // [HP/16][HP/32][64] x 8 bf16: A fragments of W1 (row k, k-dim j)
  const float* b1;        // [HP]
  const float* w2;        // [HP]
  float* e;               // forward: [S][H] pooled output
  float* alpha;           // forward out / backward in: [S][L]
  const float* de;        // backward: [S][H]
  void* dH;               // backward: [S][L][H] bf16
  void* dZ;               // backward: [S*L][H] bf16 (pre-activation gradient, the dW1 GEMM operand)
  float* part;            // backward: [grid][2][HP] (dw2, db1) partial sums, one row per workgroup
};
int wide_attn_hp(int H);                        // padded H (0: unsupported)
int wide_attn_sb(int L);                        // sequences per block
size_t wide_attn_smem(int H, int L, bool bwd);  // dynamic LDS bytes
int wide_attn_grid(int H, int L, int S, bool bwd);   // persistent grid (resident workgroups); < 0 on error
int wide_attn_fwd(const WideAttnArgs& a, int grid, hipStream_t st);
int wide_attn_bwd(const WideAttnArgs& a, int grid, hipStream_t st);   // part: [grid][2][HP]

// stable counting sort of rows by valid length (ragged.hip); ws >= 2 * (L + 1) * ragged_blocks(S) ints
int ragged_blocks(long S);
int ragged_max_len();
int ragged_sort(const int* inst, const int* lengths, long S, int L, int* ws, int* perm, int* inst_s, int* slen,
                int* tlen, hipStream_t st);

// wide induction / relation head (head_wide.hip): routing iterations over e_hat [items][K][H] fp32
// (items = episodes * N), NTN ReLU / FC / sigmoid epilogue over T [rows][N*h] (column c*h + s)
bool routing_wide_supported(int K, int H, int R);
int routing_wide_fwd(const float* eh, int items, int K, int H, int R, float* cls, void* cls_bf, hipStream_t st);
int routing_wide_bwd(const float* eh, const float* dcls, int items, int K, int H, int R, float* deh, hipStream_t st);
bool ntn_wide_epi_supported(int N, bool paper);
int ntn_wide_epi_fwd(const float* T, long rows, int N, int h, const float* w, const float* b, bool paper, float* probs,
                     hipStream_t st);
int ntn_wide_epi_bwd(float* T, long rows, int N, int h, const float* w, const float* dz, const float* g, bool paper,
                     void* dT, float* dzs, hipStream_t st);

// ---------------------------------------------------------------- BERT (csrc/kernels/bert.hip)
struct BertLnArgs {          // y = LN(res + dropout(a)); HD = 256 * {1..4}
  const void* a;
  const void* res;
  const float* gamma;
  const float* beta;
  void* y;
  float* stats;              // [T, 2] mean, rstd
  const void* dy;
  void* dres;
  void* da;
  float* slab;               // [blocks, 2, HD]
  int T, HD, blocks;
  uint32_t salt, thr;
  float inv_kp;
  int drop;
};
int ln_res_fwd(const BertLnArgs& a, hipStream_t st);
int ln_res_bwd(const BertLnArgs& a, hipStream_t st);

struct BertEmbArgs {         // y = dropout(LN(word[ids[inst[s], t]] + pos[t] + type[0]))
  const int* inst;
  const int* ids;            // [NI, L]
  int S, L, HD, blocks;
  const float* wemb;
  const float* pemb;
  const float* temb;
  const float* gamma;
  const float* beta;
  void* y;
  float* stats;
  const void* dy;
  float* dx;                 // [S*L, HD] fp32
  float* slab;
  uint32_t salt, thr;
  float inv_kp;
  int drop;
};
int embed_ln_fwd(const BertEmbArgs& a, hipStream_t st);
int embed_ln_bwd(const BertEmbArgs& a, hipStream_t st);

int bias_gelu_fwd(const void* x, const float* b, void* y, long T, int I, hipStream_t st);
// gemm.hip: C = A B^T (bf16, A [M][K] / B [N][K] K-contiguous), epi 0 plain (+bias), 1 bias+GELU with the
// pre-activation in aux, 2 C * GELU'(aux) with column-sum slab [2 ceil(M/256)][N].  N % 8 == 0, K % 64 == 0.
// reduction GEMM slab[s][i][j] = sum_{k in split s} A[k][i] B[k][j] (gemm_tn.hip): K % 64 == 0, MI <= 64, MI % 8 == 0
int gemm_tn_splits(int K, int MI, int NJ);
int gemm_tn_slab(const void* A, int lda, const void* B, int ldb, int K, int MI, int NJ, const void* zero, float* slab,
                 int splits, hipStream_t st);
int gemm_bf16_nt(const void* A, int lda, const void* B, int ldb, int M, int N, int K, const float* bias, void* out,
                 int ldo, void* aux, int ldx, float* slab, int epi, hipStream_t st);
// gemm.hip, every layout: layout 0 NT (A [M][K], B [N][K]), 1 NN (A [M][K], B [K][N]), 2 TN (A [K][M], B [K][N]);
// epi 0 plain (+bias), 1 bias+GELU (aux), 2 C * GELU'(aux) + column-sum slab, 4 C + out (residual, in place),
// 5 fp32 split-K slabs out[split][M][ldo] (TN only).  N % 8 == 0; K-major A needs M % 8 == 0; direct operands
// K % 64 == 0; zero: >= 16 zero bytes (K-major rows past K).
int gemm_bf16(int layout, const void* A, int lda, const void* B, int ldb, int M, int N, int K, const float* bias,
              void* out, int ldo, void* aux, int ldx, float* slab, const void* zero, int epi, int splits, hipStream_t st);
int gemm_wgrad_splits(int M, int N, int K);
int bias_gelu_bwd(const void* dy, const void* x, const float* b, void* dx, float* slab, int T, int I, int blocks,
                  hipStream_t st);

struct BertMhaArgs {         // fused attention, head dim 64, L <= 128
  const void* qkv;           // [S*L, 3*nh*64] bf16
  const int* inst;
  const int* mask;           // [NI, L] int32 key mask
  int S, L, nh;
  void* ctx;                 // [S*L, nh*64] bf16
  float* lse;                // [S, nh, LP]
  const void* dctx;
  void* dqkv;
  float* bsum;               // bwd, optional: [S*nh][3][64] per-block column sums of dQ | dK | dV
  uint32_t salt, thr;
  float inv_kp;
  int drop;
};
int mha_lp(int L);
int mha_fwd(const BertMhaArgs& a, hipStream_t st);
int mha_bwd(const BertMhaArgs& a, hipStream_t st);
}  // namespace ina
