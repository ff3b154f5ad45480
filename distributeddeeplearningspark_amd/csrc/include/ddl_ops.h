// Launchers of the non-GEMM kernels (normalisation, pooling, losses, optimizers,
// data movement).  All tensors are NHWC / row-major, bf16 activations, fp32 statistics,
// fp32 master weights.  Every launcher returns a hipError_t as int.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ddl {

// Dropout rate -> threshold byte (the rate is quantised to 1/256, as uint8-threshold dropout does: p = 0.1
// keeps 230 / 256) and the scale of the kept values, the inverse of the quantised keep rate
// (ddl_common.h:drop_keep, ops/transformer.py:drop_thresh / drop_scale).
inline uint32_t drop_t8(double p) {
  if (!(p > 0.0)) return 0u;
  const double t = p * 256.0 + 0.5;
  return t < 1.0 ? 1u : (t >= 255.0 ? 255u : (uint32_t)t);
}
inline float drop_scale8(uint32_t t8) { return t8 ? (float)(256.0 / (256.0 - (double)t8)) : 1.f; }

constexpr int kBnShards = 32;     // == kStatShards: sharded atomic sums of the fused GEMM-epilogue statistics
constexpr int kMaxPartials = 512;  // partial rows of a column-reduction sweep

// ---------------- batch norm (x: [M, C] bf16, C % 8 == 0) ----------------
// Per-channel sums live in a workspace ws[S][2][C] (S partial rows, summed by the finalize):
//   * fused conv-epilogue statistics: S = kBnShards, zeroed, accumulated with atomics;
//   * bn_stats / bn_bwd_reduce sweeps: S = bn_partial_rows(M, C), every row written (no zeroing).
int bn_partial_rows(long M, int C);
int splitk_finalize(float* ws, void* y, const float* bias, float* stats, long M, int C, int relu, int splits,
                    long slab_stride, hipStream_t s, long brows = 0,
                    long zbias = 0);  // splits > 0: ws = `splits` slabs slab_stride floats apart
int bn_stats(const void* x, float* ws, long M, int C, hipStream_t s);
// ws -> mean/invstd (saved for backward), scale/shift for apply, running stats update
int bn_finalize(const float* ws, int S, long M, int C, const float* gamma, const float* beta, float eps,
                float momentum, float* running_mean, float* running_var, float* save_mean, float* save_invstd,
                float* scale, float* shift, hipStream_t s);
// y = relu?(x*scale[c] + shift[c] + resid)
// mask (optional): one byte per 8 channels, bit i = (pre-ReLU output > 0), the mode-3 backward mask
int bn_apply(const void* x, const float* scale, const float* shift, const void* resid, void* y, void* mask, long M,
             int C, int relu, hipStream_t s, const float* res_scale = nullptr, const float* res_shift = nullptr);
// backward pass 1: dy' = dy * relu-mask ; ws[shard][0][c] += sum dy', ws[shard][1][c] += sum dy'*(x-mean)
// mask mode: 0 none, 1 (y > 0) from the forward output, 2 (x*scale+shift > 0) recomputed from x
int bn_bwd_reduce(const void* dy, const void* x, const void* y, const float* scale, const float* shift,
                  const float* mean, float* ws, long M, int C, int mode, hipStream_t s);
// pass 2: grads of gamma/beta (+=) and per-channel dx = A*dy' + B*x + K coefficients
int bn_bwd_finalize(const float* ws, int S, long M, int C, const float* gamma, const float* mean, const float* invstd,
                    float* dgamma, float* dbeta, float* coef, hipStream_t s);
// pass 3: dx = A*dy' + B*x + K;  optionally dres = dy' (masked gradient of the residual branch)
// x2 / mean2 / ws2 (optional): the same sweep writes the backward partial sums of a second BN fed by dy'
// (ws2 [bn_partial_rows(M, C)][2][C]: sum dy', sum dy' * (x2 - mean2)) — see bn.hip
int bn_bwd_dx(const void* dy, const void* x, const void* y, const float* scale, const float* shift,
              const float* coef, void* dx, void* dres, long M, int C, int mode, hipStream_t s,
              const void* x2 = nullptr, const float* mean2 = nullptr, float* ws2 = nullptr);

// ResNet stem: BN backward through the fused 3x3 / 2 / pad-1 max pool (pooled gradient dy + argmax bytes, the
// BN output gradient recomputed per pixel, never stored): dx == nullptr -> reduce partials into ws
// [S][2][C] (one row per workgroup); else dx = A d' + B x + K (coef) — bn.hip
bool pool3s2_bn_bwd_ok(int N, int H, int W, int C, int Ho, int Wo, int k = 3);  // k: 3 = 3x3/2/p1, 2 = 2x2/2
int pool3s2_bn_bwd(const void* dy, const uint8_t* am, const void* x, const float* scale, const float* shift,
                   const float* mean, const float* coef, float* ws, int S, void* dx, int N, int H, int W, int C, int Ho,
                   int Wo, hipStream_t s, int k = 3);

// ---------------- pooling (NHWC) ----------------
int maxpool_fwd(const void* x, void* y, uint8_t* argmax, int N, int H, int W, int C, int Ho, int Wo, int kh, int kw,
                int sh, int sw, int ph, int pw, hipStream_t s, const float* scale = nullptr, const float* shift = nullptr);
int maxpool_bwd(const void* dy, const uint8_t* argmax, void* dx, int N, int H, int W, int C, int Ho, int Wo, int kh,
                int kw, int sh, int sw, int ph, int pw, hipStream_t s);
int avgpool_global_fwd(const void* x, void* y, int N, int HW, int C, hipStream_t s);
int avgpool_global_bwd(const void* dy, void* dx, int N, int HW, int C, hipStream_t s);

// ---------------- losses ----------------
// logits [B, K] (bf16 or fp32), target: class index (int64) OR probability rows (fp32 [B,K]).
// loss_rows[b] = CE; dlogits = (softmax - target) * grad_scale  (same dtype as logits)
int softmax_xent(const void* logits, int logits_bf16, const int64_t* labels, const float* target_probs,
                 float* loss_rows, void* dlogits, int B, int K, long ld, float grad_scale, float label_smoothing,
                 int ignore_index, hipStream_t s, const float* grad_scale_dev = nullptr, float* loss_out = nullptr,
                 float out_scale = 1.f, int zrows = 0);
int label_count_inv(const int64_t* labels, long n, int ignore_index, float* inv, hipStream_t s);
int rows_sum_scaled(const float* rows, long n, float scale, const float* dev, float* out, hipStream_t s);
int scale_bf16_dev(void* x, long n, const float* s_dev, hipStream_t s);
// loss[0] = mean((pred - target)^2); grad = 2 (pred - target) / n  (fp32, one launch)
int mse_fwd_bwd(const float* pred, const float* target, long n, float* loss, float* grad, hipStream_t s);
// Keras CE on probabilities: loss_rows[b] = -sum y log clip(p), dp = -scale * y / p inside the clip range
int prob_xent(const float* p, const int64_t* labels, const float* target, float* loss_rows, float* dp, int B, int K,
              float eps, float scale, int ignore_index, hipStream_t s);

// ---------------- elementwise ----------------
int cast_f32_bf16(const float* x, void* y, long n, hipStream_t s);
int cast_bf16_f32(const void* x, float* y, long n, hipStream_t s);
int sum_rows_bf16(const void* x, void* y, int R, long n, hipStream_t s);
int relu_bwd(const void* dy, const void* y, void* dx, long n, hipStream_t s);
int add_bf16(const void* a, const void* b, void* y, long n, hipStream_t s);
// db[n] (+)= sum_m dy[m][n]; deterministic mode: det_ws (bias_grad_rows(M) x N floats) holds per-workgroup
// partial rows summed in order by colsum_partials (without it: one workgroup per column block)
// zcount > 1: replica-batched, dy = zcount stacked [M][N] blocks, db of block z at db + z * zdb
int bias_grad(const void* dy, float* db, long M, int N, int accumulate, hipStream_t s, float* det_ws = nullptr,
              const void* relu_y = nullptr, void* relu_dx = nullptr, int zcount = 1, long zdb = 0);
// zero-padded [R][Kp] copy of a row-strided [R][K] bf16 view
int pad_cols_bf16(const void* x, long ldx, void* out, long R, int K, int Kp, hipStream_t s);
constexpr int kMaxZeroRanges = 8;
struct ZeroRanges {                    // buffers zeroed by one launch: p[k] (16-B aligned), pre[k + 1] - pre[k]
  void* p[kMaxZeroRanges];             // 16-B vectors followed by tail_words[k] (< 4) 4-B words
  long pre[kMaxZeroRanges + 1];
  int tail_words[kMaxZeroRanges];
  int count;
};
int zero_ranges(const ZeroRanges& r, hipStream_t s);
int gather_bf16(const void* src, const int* idx, void* out, long n, hipStream_t s);
int scatter_add_f32(const float* src, const int* idx, float* dst, long n, hipStream_t s);
int bias_grad_rows(long M);
// c = beta * c + sum over split-K partial slabs ws[splits][M][N] (split order, one writer per element)
int slab_reduce(const float* ws, int splits, float* c, long M, int N, long ldc, float beta, hipStream_t s);
// y[C][R] = x[R][C]^T (bf16; R, C, ldx multiples of 8)
int transpose_bf16(const void* x, void* y, int R, int C, long ldx, hipStream_t s);
int im2col(const void* x, void* col, int n, int hi, int wi, int c, int ho, int wo, int sh, int sw, int ntaps,
           const int* dh, const int* dw, int kpad, hipStream_t s);
// stem space-to-depth: [N][H][W][C<=4] -> [N][Ho][Wo][16] (block 2, zero padding `pad`)
int s2d_pad(const void* x, void* y, int N, int H, int W, int C, int Ho, int Wo, int pad, hipStream_t s);
// ingest: uint8 NHWC images -> bf16 normalised, channel-padded NHWC (cpad >= c)
int normalize_u8(const uint8_t* x, void* y, long npix, int c, int cpad, const float* mean, const float* invstd,
                 hipStream_t s);

// ---------------- optimizers over flat fp32 buffers (multi-tensor via the flat arena) ----------------
// every kernel optionally writes the bf16 compute copy of the updated parameters (w16 != nullptr)
int sgd_step(float* w, const float* g, float* mom, void* w16, long n, float lr, float momentum, float dampening,
             float wd, int nesterov, float gscale, hipStream_t s);
int adam_step(float* w, const float* g, float* m, float* v, void* w16, long n, float lr, float b1, float b2,
              float eps, float wd, int adamw, float bc1, float bc2, float gscale, float* tstep,
              hipStream_t s, unsigned* tick_ctr = nullptr);
int step_tick(float* t, hipStream_t s);
int adagrad_step(float* w, const float* g, float* acc, void* w16, long n, float lr, float eps, float wd, float gscale,
                 hipStream_t s);
int rmsprop_step(float* w, const float* g, float* acc, void* w16, long n, float lr, float rho, float eps, float wd,
                 float gscale, hipStream_t s);
// sum of squares of a flat fp32 buffer into out[0] (for grad-norm clipping / checksums); out must be zeroed
int sumsq_f32(const float* x, long n, float* out, hipStream_t s);

// ---------------- transformer ops (BERT) ----------------
// Fused multi-head attention, head dim 64, S % 128 == 0 (kernels/attention.hip).
struct AttnParams {
  const uint16_t* qkv; long ld;   // [B*S][ld] bf16, head h of q/k/v at q_off/k_off/v_off + 64h
  int q_off, k_off, v_off;
  uint16_t* o; long ldo;          // [B*S][ldo] context, head h at 64h (forward output, backward input)
  float* lse;                     // [B][H][S] base-2 log-sum-exp of the scaled scores
  const int* lens;                // [B] valid keys per sequence (nullable)
  int B, H, S;
  float scale, scale_log2;        // softmax scale, scale * log2(e)
  uint32_t drop_t8;               // attention-probability dropout: keep iff hash byte >= t8 (0 = off)
  float drop_scale;
  unsigned long long drop_seed;
  // backward only
  const uint16_t* dout; long lddo;  // dO
  float* dvec;                      // [B][H][S] scratch: rowsum(dO * O)
  uint16_t* dqkv; long lddqkv;      // gradient of the qkv buffer (same column layout)
  int xcd_remap;                    // set by the launchers (DDL_ATTN_XCD): blocks of one (b, h) share an XCD
};
int attn_fwd(const AttnParams& p, hipStream_t s);
int attn_bwd(const AttnParams& p, hipStream_t s);

// LayerNorm over rows of x [M][H] bf16 (H % 8 == 0, H <= 4096); gamma/beta fp32; saves mean/rstd.
// optional output dropout (drop_p > 0; element index row*H + n) — BERT embedding dropout
int layernorm_fwd(const void* x, const float* gamma, const float* beta, void* y, float* mean, float* rstd, long M,
                  int H, float eps, float drop_p, unsigned long long seed, hipStream_t s);
// dx = LN'(dy); dx_drop = dx * dropout-mask(seed, m*H+n) * 1/(1-p) (the gradient entering the
// dropout of the residual branch, nullable); per-wave partial rows ws[P][2][H] of dgamma/dbeta
int ln_partial_rows(long M);
// partial rows [P][parts][H] that layernorm_bwd writes (its ws and colsum size)
int ln_bwd_rows(long M, int H);
// in_drop_p/in_seed: dy is first masked by the forward's output dropout
// parts = 2: ws[P][2][H] = (dgamma, dbeta); parts = 3: ws[P][3][H] = (dbias, dgamma, dbeta) where
// dbias = column sums of dx_drop, the bias gradient of the GEMM whose dropped output fed the residual sum
int layernorm_bwd(const void* dy, const void* x, const float* mean, const float* rstd, const float* gamma, void* dx,
                  void* dx_drop, float drop_p, unsigned long long seed, float* ws, int P, long M, int H,
                  float in_drop_p, unsigned long long in_seed, int parts, hipStream_t s);
// word-embedding gradient from tokens sorted by id (no atomics); position gradient (sum over batch)
int embed_word_grad(const int64_t* sorted_ids, const int64_t* perm, const void* ds, float* gword, long T, int H,
                    hipStream_t s);
int embed_word_grad_atomic(const int64_t* ids, const void* ds, float* gword, long T, int H, long V, hipStream_t s);
int embed_pos_grad(const void* ds, float* gpos, int B, int S, int H, hipStream_t s);
// out[n] (+)= sum_p ws[p][n]
int colsum_partials(const float* ws, int P, int N, float* out, int accumulate, hipStream_t s, long ld = 0);
// out[t] = word[ids[t]] + pos[t % S] + type[types[t]]  (bf16 tables, types nullable -> row 0)
// BERT MLM head rows (layernorm.hip): out[b P + i] = h[b S + pos[b][i]] (bf16 [B S][H] -> [B P][H]) and its
// backward dh[b S + q] = sum_{i : pos[b][i] == q} dout[b P + i] (every row of dh written, zeros elsewhere)
int mlm_gather(const void* h, const int64_t* pos, void* out, int B, int S, int P, int H, hipStream_t s);
int mlm_scatter(const void* dout, const int64_t* pos, void* dh, int B, int S, int P, int H, hipStream_t s);
int embed_fwd(const int64_t* ids, const int64_t* types, const void* word, const void* pos, const void* type,
              void* out, long T, int S, int H, hipStream_t s);
// gword[ids[t]] += ds[t] (fp32 atomics), gpos[t % S] += ds[t]; per-wave partial rows of the
// token-type gradient wsT[P][ntypes][H] (ntypes <= 2)
int embed_bwd(const int64_t* ids, const int64_t* types, const void* ds, float* gword, float* gpos, float* wsT, int P,
              int ntypes, long T, int S, int H, hipStream_t s);

// ---------------- persistent recurrent cells (Keras GRU reset_after=False / LSTM, fp32) ----------------
// xw: [B][T][G*H] input projections (incl. bias) or nullptr: then the fast path (H = 64/128,
// I <= 8) computes x W + b in-kernel from x [B][T][I], W [I][G*H], b (nullable);
// hs/cs: [B][T+1][H]; gates: [B][T][G*H] post-activation
// Replica-batched recurrent step (parallel/replica_batch.py): R co-located dist-keras workers whose models
// are RNN(H) -> Dense(K) with an MSE loss step as ONE launch per phase.  Replica r owns global batch
// rows [r B, (r+1) B) of every activation buffer; parameters, gradients, optimizer state and the resident
// shard are its own (pointer tables).  The replicas step in lockstep on one device step counter; shards may
// be ragged (the reference's repartition(num_workers) shards differ by a row, ddl_nyiso_aztk.py:193): replica r
// fetches mini-batch ctr % nbr[r] and is live while ctr < steps[r] — past that it neither records, ticks nor
// updates its parameters (the per-replica path's exhausted worker), while the others keep stepping.
constexpr int kMaxRnnRep = 16;
struct RnnRep {
  const float* x[kMaxRnnRep];  // resident input shard [nb B][T][I]
  const float* y[kMaxRnnRep];  // resident target shard [nb B][K]
  const float* W[kMaxRnnRep];  // [I][GH]
  const float* U[kMaxRnnRep];  // [H][GH]
  const float* b[kMaxRnnRep];  // [GH] or null
  const float* Wd[kMaxRnnRep]; // Dense kernel [K][H]
  const float* bd[kMaxRnnRep]; // Dense bias [K] or null
  float* gW[kMaxRnnRep];
  float* gU[kMaxRnnRep];
  float* gb[kMaxRnnRep];
  float* gWd[kMaxRnnRep];
  float* gbd[kMaxRnnRep];
  float* hist[kMaxRnnRep];     // per-replica loss history [>= steps[r]]
  int nbr[kMaxRnnRep];         // mini-batches per epoch of replica r's shard
  int steps[kMaxRnnRep];       // steps replica r takes in total (live while ctr < steps[r])
  int* ctr;                    // device step counter (batch index = ctr % nbr[r], history slot = ctr)
  int* live;                   // [R] live flags of the current step (written by the head kernel)
  int B, K;
};
struct OptRep {
  float* w[kMaxRnnRep];
  const float* g[kMaxRnnRep];
  float* s1[kMaxRnnRep];       // adagrad accumulator / adam m / sgd momentum (or null)
  float* s2[kMaxRnnRep];       // adam v
  float* t[kMaxRnnRep];        // adam device step counters
};
// one training step of the R replicas: rnn forward, Dense + MSE forward / backward (+ loss record, Adam
// step tick), rnn backward, recurrent parameter gradients, optimizer (+ step counter advance); buffers:
// hs / cs / gates / dgates [R B][T(+1)][..], h_last / dh [R B][H].  opt: 0 sgd, 1 adagrad, 2 adam (mode bits
// of adam_step in amode).
int rnn_replica_step(int cell, const RnnRep& rp, int R, int T, int H, int I, float* hs, float* cs, float* gates,
                     float* hlast, float* dh, float* dgates, const OptRep& op, long n, int opt, float lr, float p1,
                     float p2, float eps, float wd, int amode, hipStream_t s);
bool rnn_replica_ok(int cell, int H, int I, int K, int B);

bool rnn_fast_path(int H);
bool rnn_fuses_input(int H, int I);
// the register-resident kernels apply for this (cell, H, activations)
bool rnn_reg_path(int cell, int H, int act, int ract);
// cell 0 = GRU, 1 = LSTM, 2 = SimpleRNN; act / ract = ActCode of the activation / recurrent activation
// (the register-resident fast path serves tanh + hard_sigmoid GRU/LSTM, the generic kernels the rest)
int rnn_fwd(int cell, const float* xw, const float* x, const float* W, const float* b, int I, const float* U,
            float* hs, float* cs, float* gates, float* y, int B, int T, int H, int rs, int act, int ract,
            hipStream_t s);
// gU/gW/gb (fp32, nullable gb) += parameter gradients from dgates (one launch, atomics)
int rnn_param_grad(int cell, const float* dg, const float* hs, const float* gates, const float* x, float* gU,
                   float* gW, float* gb, int B, int T, int H, int I, hipStream_t s);
// UT = U^T [G*H][H] (generic path only); dgates [B][T][G*H] = gradients of the gate pre-activations
bool rnn_bwd_uses_ut(int H);
int rnn_bwd(int cell, const float* dy, const float* U, const float* UT, const float* hs, const float* cs,
            const float* gates, float* dgates, int B, int T, int H, int rs, int act, int ract, hipStream_t s);

// ---------------- Keras layer element-wise ops (kernels/layer_ops.hip) ----------------
// activation codes shared by the standalone Activation layer and the recurrent cells
enum ActCode : int {
  ACT_C_LINEAR = 0, ACT_C_RELU = 1, ACT_C_TANH = 2, ACT_C_SIGMOID = 3, ACT_C_HARD_SIGMOID = 4,
  ACT_C_ELU = 5, ACT_C_SELU = 6, ACT_C_SOFTPLUS = 7, ACT_C_GELU = 8,
};
// y = f(x); dx = dy * f'(.) from ref = y (ref = x for GELU).  bf16 != 0: bf16 storage, else fp32
int act_fwd(const void* x, void* y, long n, int code, int bf16, hipStream_t s);
int act_bwd(const void* dy, const void* ref, void* dx, long n, int code, int bf16, hipStream_t s);
// softmax over the last axis of [R][N]; dx = y * (dy - <dy, y>)
int softmax_rows_fwd(const void* x, void* y, long R, int N, int bf16, hipStream_t s);
int softmax_rows_bwd(const void* dy, const void* y, void* dx, long R, int N, int bf16, hipStream_t s);
// y = keep(i) ? x * scale : 0 with keep(i) = drop_keep(seed, i, thresh), thresh = drop_t8(p) (also the backward)
int dropout_apply(const void* x, void* y, long n, unsigned long long seed, uint32_t thresh, float scale, int bf16,
                  hipStream_t s, const float* dstep = nullptr);
// NHWC average pooling, padding excluded from the divisor
int avgpool2d_fwd(const void* x, void* y, int N, int H, int W, int C, int Ho, int Wo, int kh, int kw, int sh, int sw,
                  int ph, int pw, int bf16, hipStream_t s);
int avgpool2d_bwd(const void* dy, void* dx, int N, int H, int W, int C, int Ho, int Wo, int kh, int kw, int sh, int sw,
                  int ph, int pw, int bf16, hipStream_t s);
// Keras Embedding: out[t] = table[ids[t]] (bad[0] |= 1 on an out-of-range id, row zeroed);
// backward gw[ids[t]] += dy[t] (fp32 atomics)
int embedding_gather(const int64_t* ids, const void* table, void* out, long n, int D, long V, int* bad, int bf16,
                     hipStream_t s);
int embedding_scatter(const int64_t* ids, const void* dy, float* gw, long n, int D, long V, int bf16, hipStream_t s);
// conv data-gradient filter layouts: out[ci][t][co] = w[co][taps.t[t]][ci] (bf16, nt <= 64 taps)
constexpr int kMaxFilterTaps = 64;
struct FilterTaps { int16_t t[kMaxFilterTaps]; };
// one job of taps_batch: dst[ci][t][co] = src[co][taps[t]][ci], t < nt (blk0: its first block in the grid)
struct TapsJob {
  const uint16_t* src;
  uint16_t* dst;
  int Co, T, Ci, nt, blk0, pad_;
  int16_t taps[kMaxFilterTaps];
};
int taps_batch(const TapsJob* jobs, int njobs, int blocks, hipStream_t s);
int taps_job_blocks(int Co, int Ci, int nt, int T);
int filter_taps_transpose(const void* w, void* out, int Co, int T, int Ci, const FilterTaps& taps, int nt,
                          hipStream_t s, int zcount = 1, long zw = 0, long zo = 0);
// y[C][R] = x[R][C] (fp32)
int transpose_f32(const float* x, float* y, int R, int C, hipStream_t s);
// db[n] += sum_m dy[m][n] (fp32, dense rows of N)
int colsum_f32(const float* dy, float* db, long M, int N, hipStream_t s);
// fp32 MFMA GEMM (kernels/gemm_f32.hip): C = alpha * A B + beta * C (+ bias[n]) (relu);
// A(m,k) = a[m*sam + k*sak], B(k,n) = b[k*sbk + n*sbn]
int gemm_f32(const float* a, long sam, long sak, const float* b, long sbk, long sbn, float* c, long ldc, int M, int N,
             int K, float alpha, float beta, const float* bias, int relu, hipStream_t s);

// ---------------- device ETL (dist-keras column transformers, fp64) ----------------
int etl_minmax(const double* x, double* y, long n, double o_min, double scale, double n_min, hipStream_t s);
int etl_one_hot(const int64_t* labels, double* y, long n, int K, int* bad, hipStream_t s);
int etl_argmax(const double* x, long rows, int K, long ld, int64_t* out, hipStream_t s);


// dist-keras commit rounds (optim.hip): X = scale (W - center) [, W -= X]; center += sum_j X_j [, W = center]
constexpr int kMaxCommitPeers = 16;
struct CommitPtrs { const float* p[kMaxCommitPeers]; };
int commit_delta(float* W, const float* center, float* X, void* w16, long n, float scale, int elastic, hipStream_t s);
int commit_apply(const CommitPtrs& xs, int nx, float* center, float* W, void* w16, long n, hipStream_t s);

// Deterministic-reduction mode (DDL_DETERMINISTIC=1, ops/determinism.py): every launcher that would add
// partial sums with fp32 atomics from several workgroups instead reduces in a fixed order (one writer per
// output element, partial rows summed by index).  Process-wide switch, set from Python.
void set_deterministic(int on);
int deterministic();
// word-embedding gradient, deterministic: tokens sorted by id (stable), ONE writer per run of equal ids
// (the wave whose chunk holds the run's first position walks the whole run in order)
int embed_word_grad_det(const int64_t* sorted_ids, const int64_t* perm, const void* ds, float* gword, long T, int H,
                        long V, float* part, hipStream_t s);  // part: embed_word_grad_det_ws(T, H) floats
long embed_word_grad_det_ws(long T, int H);

// in-process replica groups (replica.hip): one commit kernel over R replicas' arenas, and the device-side
// mini-batch fetch / loss record of a graph-replayed replica step
constexpr int kMaxReplicas = 16;
struct ReplicaPtrs {
  float* w[kMaxReplicas];
  void* w16[kMaxReplicas];
  float scale[kMaxReplicas];
};
int commit_replicas(const ReplicaPtrs& rp, int nr, float* center, float* sum, long n, int elastic, int mode,
                    hipStream_t s);
constexpr int kMaxBatchCopies = 32;  // 2 per replica of a batched group (parallel/replica_seq.py)
struct BatchCopy {
  const void* src[kMaxBatchCopies];
  void* dst[kMaxBatchCopies];
  long bytes[kMaxBatchCopies];   // bytes of ONE mini-batch of copy q
  long nbatch[kMaxBatchCopies];  // mini-batches per epoch of copy q's shard (ragged shards differ)
};
int batch_fetch(const BatchCopy& bc, int ncopy, const int* ctr, hipStream_t s);
// steps (nullable, int32 [nrep]): replica r records only while ctr < steps[r]; ts (nullable, fp32 [nrep]): the
// live replicas' Adam step counters advance by one (after the stacked optimizer below has read them)
int step_record(const float* loss, float* hist, int cap, int* ctr, hipStream_t s, int nrep = 1,
                const int* steps = nullptr, float* ts = nullptr);
// Optimizer sweep over R stacked replica arenas [R][n] (parallel/replica_seq.py): replica r is live while
// *ctr < steps[r] (ragged shards), a dead replica keeps its parameters and state; gradients are zeroed either
// way.  opt 0: SGD (+ momentum mu, s1), 2: Adam (s1 = m, s2 = v, t = ts[r] + 1, amode bit0 AdamW, bit1 Keras
// epsilon).  w16 (nullable): bf16 compute copy [R][n].
int opt_stack_step(int opt, float* w, float* g, float* s1, float* s2, void* w16, long n, int R, const int* ctr,
                   const int* steps, const float* ts, float lr, float mu, float b1, float b2, float eps, float wd,
                   int amode, hipStream_t s);

}  // namespace ddl
