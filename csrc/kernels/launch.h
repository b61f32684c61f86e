// Host-side launch interface of the fed_tgan_amd HIP kernels (raw pointers + hipStream_t).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fedtgan {

enum Epilogue : int { EPI_NONE = 0, EPI_LRELU_DROPOUT = 1, EPI_MASK = 2, EPI_RELU = 3, EPI_BN_EVAL_RELU = 4 };

struct RngArgs;

// Batched clients (fed_tgan_amd/models/batched.py): K federated clients' training steps in ONE launch
// per kernel.  Every buffer a kernel touches lives in one device arena, client c's copy exactly `stride`
// bytes after client c-1's (identical layouts), so client c = blockIdx.z (the GEMM folds it with its
// split-K index) offsets every pointer by c * stride and its Philox seed by c * seed_step.  k = 1 (the
// default) is the plain single-client launch.  The host context is per thread (set by the bindings
// around a batched engine's launches); in a batched launch every pointer must lie in client 0's slab
// [base, base + stride), which the launchers verify (check_slab).
struct ClientBatch {
  int k;
  int64_t stride;
  uint64_t seed_step;
  const char* base;
  int xcd;     // 1: place each client's workgroups on its own XCD(s) (common.h xcd_client_map)
};
extern int g_xcd_clients;   // set_tuning("xcd_clients"): the ClientBatch::xcd of new batched contexts
ClientBatch& client_batch();
// host: throws std::runtime_error when a batched launch is handed a pointer outside client 0's slab
void check_slab(const void* p, const char* what);
// host: throws when the launch has no batched form
void require_unbatched(const char* what);
template <class... P>
inline void check_slabs(const char* what, P... ps) {
  (check_slab((const void*)ps, what), ...);
}

struct GemmArgs {
  const float* a;
  const float* b;
  float* c;
  const float* bias;
  float* ms;   // EPI_MASK: read; EPI_LRELU_DROPOUT: written (slope * keep / (1 - p))
  // EPI_LRELU_DROPOUT on D's last hidden layer (nullable): also write the backward seed of that
  // layer, head_a[m, n] = head_coef[m] * head_v[n] * (slope * keep / (1 - p))  (the D head's
  // A_{L-1} = coef * v * MS_{L-1}, which needs no reduction)
  const float* head_coef;
  const float* head_v;
  float* head_a;
  int ldha;
  float* ws;   // split-K partial slabs [splitk][M][N]
  int M, N, K;
  int lda, ldb, ldc, ldms;
  int ta, tb;
  float alpha, beta;
  int epi;
  float slope, p_drop;
  // EPI_BN_EVAL_RELU: out = relu((v - rm) * rsqrt(rv + eps) * gamma + beta)
  const float* bn_gamma;
  const float* bn_beta;
  const float* bn_rm;
  const float* bn_rv;
  float bn_eps;
  uint64_t seed;
  const uint64_t* rng_ctr;
  uint32_t rng_stream;
  int splitk, kchunk;
  int vec;     // 1: both operands may be read with 16-B loads (see gemm.hip Chunk::load)
  int tile;    // output tile edge: 64 (default) or 32 (4x the workgroups, for short-K GEMMs)
  int f32;     // 1: exact-fp32 MFMA (v_mfma_f32_16x16x4_f32); 0: bf16 operands, fp32 accumulate
  int xcd_remap;   // XCD-contiguous tile order (set by launch_gemm): 1 N-fastest, 2 M-fastest
  int wt;          // 1: write-through (sc1) output stores (set by launch_gemm)
  // One-hot conditional block (nullable): the K columns of op(A) are only the DENSE part of the
  // input; its trailing one-hot block (the conditional vector c, exactly one 1 per row at
  // oh_off[oh_col[m]] + oh_opt[m]) is applied as a gather of one weight column per row in the
  // epilogue: v += oh_w[n * oh_ld + oh_off[oh_col[m]] + oh_opt[m]]   (op(B) = B^T row-major weight)
  const float* oh_w;
  int oh_ld;
  int oh_trans;   // 1: oh_w is the transposed block [C, N] (coalesced gathers: lanes of a row read
                  //    consecutive n) -- v += oh_w[(oh_off[oh_col[m]] + oh_opt[m]) * oh_ld + n]
  const int* oh_col;
  const int* oh_opt;
  const int* oh_off;
  // BatchNorm partial statistics (nullable; 32/64 tiles, no split-K, plain C = A B^T + bias): every
  // tile writes, per output column and batch (rows [0, bn_rpg) / [bn_rpg, M)), its row count, mean
  // and sum of squared deviations: bn_part[((m_tile * 2 + batch) * 3 + {0,1,2}) * N + n]
  float* bn_part;
  int bn_rpg;
  int oh_c;       // width of the one-hot block (checked build: gather index bound)
  // Split-K reduced inside the GEMM launch (nullable): one arrival counter per output tile, zero
  // between launches.  Every K-slice workgroup publishes its slab write-through and takes a ticket;
  // the one that completes a tile sums the tile's slabs and applies the epilogue (no
  // gemm_splitk_epilogue launch).  red_inl is set by the launcher where the shape allows it.
  unsigned* tile_cnt;
  int red_inl;
  // bf16 storage (generation): bin = 1 -> both operands are bf16 rows (a16 [M, K] / b16 [N, K], k
  // contiguous, 16-B aligned, ld % 8 == 0), staged into LDS without conversion; c16 (nullable) ->
  // the epilogue writes bf16 (no split-K, no beta).  The values are the ones the fp32 path rounds
  // to bf16 at staging, so a bf16 activation buffer gives bit-identical products.
  const uint16_t* a16;
  const uint16_t* b16;
  uint16_t* c16;
  int bin;
  // Adam applied in the epilogue (gemm_adam_kernel only; nullable): the output is a weight gradient
  // inside an optimizer's flat gradient buffer; adam_p / adam_m / adam_v point at the same offset of
  // the parameter / moment buffers, so output (m, n) updates element m * ldc + n of each.  The
  // gradient itself is still written to c.
  float* adam_p;
  float* adam_m;
  float* adam_v;
  const float* adam_step;
  float adam_lr, adam_b1, adam_b2, adam_eps, adam_wd;
  int adam_grad;   // gemm_shortk_kernel<ADAM>: also store the gradient (gemm_adam_kernel always does)
  // chained GEMM (host-side pointer, nullable; chain_epilogue_kernel): once this GEMM's output C [M, N]
  // is final, the tail C2 = epi2(C B2^T + bias2) (the tail's own GemmArgs: op(A2) = this C, row-local,
  // K2 = N <= 1024) is computed in this GEMM's reduction launch, as fp32 dot products
  const struct GemmArgs* chain;
  // batched clients (ClientBatch; set by the launchers): nclient = grid.z / splitk
  int64_t cstride;
  uint64_t seed_step;
  int nclient;
  int xcd_cl;   // ClientBatch::xcd
  int chain_co;   // chained tail (chain_epilogue_kernel): lane-contiguous weight rows + wave sums (g_chain_coalesced)
  // chained tail with a head seed (head_a = A1) only, nullable: the backward link A0 = (A1 W1) . MS0 formed in the
  // same launch (gemm_achain_next): each (row group, 64-column slab) workgroup stores its slab's partial product
  // A1[:, slab] W1[slab, :] into ach_ws [slabs, M, K] write-through and takes a ticket on ach_cnt[row group] (zero
  // between launches); the row group's last workgroup sums the slabs in order and applies the head's mask MS0
  float* ach_out;
  float* ach_ws;
  unsigned* ach_cnt;
  int ld_ach;
};

void launch_gemm(GemmArgs g, hipStream_t stream);
// checked build: the OR of the check bits raised since the last call in each kernel TU (cleared)
unsigned check_status_gemm();
unsigned check_status_ctgan_ops();
unsigned check_status_vgm();
// two independent GEMMs in one launch where the pair is instantiated, else two launches
void launch_gemm_pair(GemmArgs g1, GemmArgs g2, hipStream_t stream);
extern int g_gemm_pairs;
extern int g_gemm_pair_max_wg;

struct SampleArgs {
  int B, E, C, Dd, n_col, maxw, n_rows;
  float* h;            // generator input rows: z at h[r*ldh + zc], cond at h[r*ldh + cc]
  int ldh, zc, cc;
  // generation into a bf16 activation buffer (nullable): z as bf16 at h16[r*ldh16 + zc16]; h and
  // the one-hot block are then not written (the GEMMs gather the condition from col / opt)
  uint16_t* h16;
  int ldh16, zc16;
  float* xf;           // fake block of the D input (cond copy at xf[r*ldx + Dd]); nullable
  float* xr;           // real block [data row | cond of the permuted fake row]; nullable
  int ldx;
  const float* cdf;    // [n_col, maxw]
  const int* cond_off;
  const int* cond_w;
  const int64_t* row_off;   // [n_col, maxw]
  const int64_t* row_cnt;   // [n_col, maxw]
  const int64_t* rows;      // CSR row lists
  int64_t n_entries;        // length of `rows` (checked build: CSR pick bound)
  const float* data;        // encoded training matrix [n_rows, Dd]
  int* col;
  int* opt;
  int n_real;               // rows [0, n_real) also draw a real row into xr (xr has n_real rows)
  float* step_bump;         // optimizer step counter bumped by this launch (nullable)
  float* step_bump2;        // a second one (both phases of a step drawn by one launch; nullable)
  float* metrics;           // zeroed by this launch when zero_metrics
  int zero_metrics;
  uint64_t seed;
  const uint64_t* rng_ctr;
  uint32_t rng_stream;
  // draws > 1: the batches of `draws` consecutive training steps in ONE launch (blockIdx.y = draw k, keyed on
  // RNG step *rng_ctr + k, its outputs at the pointers above + k x draw_*).  step_bump / step_bump2 then point at
  // [draws] per-step counter arrays whose last entry is the canonical counter: entry q becomes last + q + 1 (the
  // value the q-th per-step launch would have bumped it to), and metrics at [draws, 4] zeroed.
  int draws;
  int64_t draw_h, draw_x, draw_col;
  ClientBatch cb;           // set by launch_sample
};

void launch_sample(const SampleArgs& a, hipStream_t stream);

struct SpanTables {
  const int* start;
  const int* width;
  const int* kind;      // 0 tanh, 1 softmax
  const int* cond_idx;  // softmax span -> conditional column index (or -1)
  // host-packed copy of every table the activation kernels stage in LDS, in LDS order:
  // [elem_span | SOFTMAX bit (D) | kind (S) | start (S) | width (S) | cond_idx (S)], zero-padded to a
  // multiple of 4 ints (one 16-B-load copy per workgroup instead of per-table loops)
  const int* packed;
  int n_span;
  int dim;              // data_dim (sum of widths)
};
inline int span_packed_len(int dim, int n_span) { return (dim + 4 * n_span + 3) & ~3; }

size_t activation_smem_bytes(const SpanTables& sp);   // dynamic LDS of the activation kernels

// optional slerp(real, fake) fused onto the activation of the fake rows (real == nullptr: off)
struct SlerpFuse {
  const float* real;   // [rows, ld] real rows
  float* out;          // [rows, ld] interpolates
  int ld, cols;        // cols = data_dim + n_opt (the fake row continues past the activation)
  int rows;            // only activation rows r < rows are interpolated
  uint32_t stream;
};
void launch_activate(const float* logits, int ldl, float* out, int ldo, int rows, SpanTables sp, float tau,
                     uint64_t seed, const uint64_t* ctr, uint32_t stream_id, SlerpFuse sl, hipStream_t stream);

void launch_act_bwd_ce(const float* dact, int ldd, const float* act, int lda, const float* logits, int ldl, SpanTables sp,
                       const int* col, const int* opt, float* dlogits, int ldg, int rows, float tau, float* loss,
                       int loss_per_row, hipStream_t stream);

void launch_slerp(const float* real, const float* fake, float* out, int rows, int cols, int ld, uint64_t seed,
                  const uint64_t* ctr, uint32_t stream_id, hipStream_t stream);

// ws (nullable, >= rows * ceil(cols / 8192) floats): rows wider than 8,192 run as a chunk-split partial-sum
// launch + a scale launch (g_gp_split) instead of one workgroup per row
void launch_gp_scale(const float* g, int ldg, float* out, int ldo, int rows, int cols, float lam, float* loss,
                     int loss_per_row, float* ws, int64_t ws_n, hipStream_t stream);
extern int g_gp_split;
extern int g_chain_coalesced;   // set_tuning("chain_coalesced")
extern int g_chain_pre;         // set_tuning("chain_pre")
extern int g_chain_rows;        // set_tuning("chain_rows")
extern int g_gp_threads;   // register-resident gp_scale workgroup size (set_tuning("gp_threads"))
extern int g_bn_threads;   // BN workgroup size (set_tuning("bn_threads"))
extern int g_act_rowreg_narrow;   // narrow rows on the register-resident row kernels (set_tuning("act_rowreg_narrow"))

// Weight gradient of a one-hot conditional input block (generator layers, input-major weights): row k of the
// block's gradient is the sum of the upstream-gradient rows whose condition index is k (rows in batch order, so
// the result is deterministic); every other row stays zero.  zero != 0 clears the rows the batch touched (after
// the optimizer has read them), restoring the all-zero block for the next step.
struct OnehotWJob {
  const float* dy;   // [B, n] upstream gradient rows
  float* w;          // row k of the block's gradient at w + k * ldw
  int ldy, ldw, n;
};
struct OnehotWBatch {
  OnehotWJob jobs[4];
  int n_jobs, B;
  const int* col;        // [B] conditioned column
  const int* opt;        // [B] its option
  const int* cond_off;   // [n_col] first block row of each column
};
void launch_onehot_wgrad(const OnehotWBatch& bt, int zero, hipStream_t stream);

void launch_d_head(const float* d, int ldd, const float* ms, int ldms, const float* v, const float* e,
                   const float* coef, const float* wloss, float* y, float* a, int lda, int rows, int cols, float* loss,
                   hipStream_t stream);

// out[c] = sum_r w[r] a[r, c] (w nullable = 1; out nullable); with dot_v, additionally
// *dot_out += sum_c dot_v[c] * (sum_r u[r] a[r, c]) + dot_e[0] * sum_r u[r], u = dot_w (or w
// when dot_w is null): the WGAN loss sum_r u[r] (d_r . v + e) of the D head, folded into the
// bias-gradient launch.  With dot_w, one job gives the head's weight gradient (weights w) and
// the loss (weights dot_w) from one pass over the rows.
struct ColsumJob {
  const float* a;
  int lda, rows, cols;
  float* out;
  const float* w;
  const float* dot_v;
  const float* dot_e;
  float* dot_out;
  const float* dot_w;
};
void launch_colsum(const ColsumJob* jobs, int n_jobs, hipStream_t stream);

// Adam over a flat buffer with up to 8 column-sum jobs folded into the same launch; a job whose
// output lies in the gradient buffer owns [own_lo, own_hi) (elements, 4-aligned) and the Adam
// update of those elements is applied from the freshly reduced sums.
constexpr int ACS_COLS = 16, ACS_GROUPS = 64;
struct AdamColsum {
  ColsumJob jobs[8];
  int n_jobs;
  int vec[8];         // rows 16-B aligned and padded to >= ceil4(cols): float4 loads
  int blk_start[9];   // filled by the launcher
  int64_t own_lo[8], own_hi[8];
  int dot_self[8];    // dot_v is this job's own output's parameters: use the pre-update values
  int64_t skip_lo, skip_hi;   // elements updated by a fused GEMM's Adam epilogue (gemm_adam_kernel)
  int64_t skip2_lo, skip2_hi; // and by a short-K weight gradient that applied Adam ahead of this launch
                              // (launch_gemm_shortk_adam); both ranges 4-aligned, disjoint, skip_lo <= skip2_lo
};
// C = A^T B by gemm_shortk_kernel with Adam applied to the outputs in its epilogue (g.adam_* set as for
// gemm_adam_kernel; the gradient itself is stored only with g.adam_grad); false: shape not taken
bool launch_gemm_shortk_adam(GemmArgs g, hipStream_t stream);
void launch_adam_colsum(float* p, const float* g, float* m, float* v, const float* step, int64_t n, float lr, float b1,
                        float b2, float eps, float wd, uint64_t* rng_ctr_bump, const AdamColsum& cs,
                        hipStream_t stream);
// a weight-gradient GEMM (g.adam_* set, unsplit) and the Adam + column-sum launch of the same
// optimizer (its flat range [cs.skip_lo, cs.skip_hi) left to the GEMM) in ONE launch; returns false
// (nothing launched) where that GEMM shape is not instantiated
bool launch_gemm_adam(GemmArgs g, float* p, const float* gr, float* m, float* v, const float* step, int64_t n,
                      float lr, float b1, float b2, float eps, float wd, uint64_t* rng_ctr_bump, const AdamColsum& cs,
                      hipStream_t stream);

extern int g_gemm_xcd_remap;   // GEMM XCD-contiguous tile order: 0 off, 1 long-K tiles, 2 always
extern int g_gemm_xcd_nmajor;  // let a GEMM take the M-fastest XCD tile order when it touches fewer bytes
extern int g_adam_store;       // Adam p/m/v store policy: 0 plain, 2 nt, 16 sc1 write-through
extern int g_adam_max_blocks;  // Adam grid cap (grid-stride beyond it)
extern int64_t g_adam_u_min;   // Adam launches over >= this many float4 (x clients) load ADAM_U float4 per thread
extern int g_gemm_store_wt;   // GEMM outputs / split-K slabs: plain (0) or write-through sc1 (1)
extern int g_gemm_shortk;          // 1: C = A^T B with K <= 160, M <= 256 and wide N by gemm_shortk_kernel
extern int g_gemm_shortk_min_n;    // narrowest N that takes it
extern int g_gemm_shortk_store;    // its output stores: 0 plain, 1 non-temporal, 2 write-through (sc1)
extern int g_gemm_splitk_inlaunch;   // split-K reduced inside the GEMM launch where a tile counter is given (1)
extern int g_act_row_mode;   // activation kernels on rows wider than 512: one workgroup per row (1) or per 1-4 rows
extern int g_decode_rows;   // generation decode: one wave per row (1) or one thread per (row, column) (0)
extern int g_bn_cols;   // BatchNorm kernels: columns per workgroup (4 / 8 / 16); set_tuning("bn_cols")
void launch_bn_relu_train(const float* a, int lda, const float* gamma, const float* beta, float* out, int ldo,
                          float* nhat, int ldn, float* mean, float* invstd, float* rm, float* rv, int rows, int cols,
                          int groups, float momentum, float eps, hipStream_t stream);

// Linear -> BatchNorm(train) -> ReLU in one launch by column ownership (kernels/bn_fused.hip): a
// workgroup owns 16 output columns of one batch.  x [groups * rpg, K] (unit column stride),
// W(n, k) = w[n * w_sn + k * w_sk]; the optional one-hot block adds oh_w[n * oh_sn + j * oh_sc] with
// j = oh_off[oh_col[r]] + oh_opt[r]; stat [groups][2][N] and cnt [ceil(N / 16)] (zero between launches)
// carry the batch statistics to the running-stat update when groups == 2.
struct ColOwnArgs {
  const float* x;
  int ldx;
  const float* w;
  int64_t w_sn, w_sk;
  const float* bias;
  const float* oh_w;
  int64_t oh_sn, oh_sc;
  const int* oh_col;
  const int* oh_opt;
  const int* oh_off;
  const float* gamma;
  const float* beta;
  float* out;
  int ldo;
  float* nhat;
  int ldn;
  float* mean;
  float* invstd;
  float* rm;
  float* rv;
  float* stat;
  unsigned* cnt;
  int rpg, groups, K, N;
  float momentum, eps;
  int64_t cstride;   // set by the launcher (batched clients)
  int dbg;           // phase-cost probe (set_tuning("colown_dbg")): 1 no GEMM, 2 no staging, 4 no stores
};
extern int g_colown_dbg;
size_t colown_smem_bytes(int K, int rpg);
void launch_linear_bn_relu_colown(ColOwnArgs g, bool vec, hipStream_t stream);

// BatchNorm(train) + ReLU from the GEMM's per-tile partial statistics (kernels/ctgan_ops.hip)
void launch_bn_relu_apply(const float* a, int lda, const float* part, int n_tiles, const float* gamma,
                          const float* beta, float* out, int ldo, float* nhat, int ldn, float* mean, float* invstd,
                          float* rm, float* rv, int rows, int cols, int groups, float momentum, float eps,
                          hipStream_t stream);
void launch_bn_relu_bwd(const float* dr, int lddr, const float* r, int ldr, const float* nhat, int ldn,
                        const float* gamma, const float* invstd, float* da, int ldda, float* dgamma, float* dbeta,
                        float* dbias, int rows, int cols, hipStream_t stream);
// operands of one BatchNorm(train) + ReLU backward (bn_bwd.h)
struct BnBwdArgs {
  const float* dr;
  int lddr;
  const float* r;
  int ldr;
  const float* nhat;
  int ldn;
  const float* gamma;
  const float* invstd;
  float* da;
  int ldda;
  float* dgamma;
  float* dbeta;
  float* dbias;   // nullable
  int rows, cols;
};
// the BN backward's column workgroups and an INDEPENDENT weight-gradient GEMM (op(A) = A^T, bf16 MFMA, 32/64
// tile) in ONE launch (horizontal fusion: the 32-64 narrow, latency-bound BN workgroups no longer run alone on the
// chip).  Returns false (nothing launched) where that combination is not instantiated.
bool launch_gemm_bnbwd(GemmArgs g, const BnBwdArgs& b, hipStream_t stream);
extern int g_bnb_first;   // gemm_bnbwd_kernel: BN workgroups before (1) or after (0) the GEMM tiles
extern int g_bnb_cols;    // gemm_bnbwd_kernel: columns per BN workgroup (4 or 8)

void launch_adam(float* p, const float* g, float* m, float* v, const float* step, int64_t n, float lr, float b1,
                 float b2, float eps, float wd, uint64_t* rng_ctr_bump, hipStream_t stream);

struct DecodeArgs {
  const float* logits;
  int ldl, rows, n_cols;
  const int* kind;      // per output column: 0 continuous, 1 categorical
  const int* start;     // span start (continuous: the tanh unit; modes follow)
  const int* width;     // #valid modes / #categories
  const int* cont;      // continuous column index into mu/sd
  const int* code_off;  // categorical: offset into codes
  const double* codes;
  int n_codes;          // length of `codes` (checked build)
  const double* mu;     // [n_cont, K]
  const double* sd;
  int K;
  double* out;          // [rows, n_cols]
  uint64_t seed;
  const uint64_t* rng_ctr;
  uint32_t rng_stream;
  int dim;              // logits per row
  const int* ecol;      // [dim] element -> output column whose argmax it enters (-1: none, e.g. alpha)
  // [n_quads][2] (nullable): every run of up to 4 logits of one column that share a Philox word:
  // {column | count << 24, offset-in-span << 16 | position}
  const int* quads;
  int n_quads;
};
void launch_sample_decode(const DecodeArgs& a, hipStream_t stream);

void launch_rng_bump(uint64_t* ctr, hipStream_t stream);

struct GenWeightJob {
  const float* w;   // fp32 weight, element (n, k) at w[n * ldw + k * skw] (skw = 1: [N, K] rows; ldw = 1: input-major storage)
  int N, ldw, skw, kd, C;
  uint16_t* w16;    // [N, ld16] bf16: columns [0, kd)
  int ld16;
  float* wt;        // [C, N] fp32: columns [kd, kd + C) transposed
};
struct GenWeightPrep {
  GenWeightJob jobs[4];
  int n_jobs;
};
void launch_gen_weight_prep(const GenWeightPrep& a, hipStream_t stream);

// VGM encode (kernels/vgm.hip): one thread per (row, column) cell of the label-encoded table
struct VgmEncodeArgs {
  const double* x;      // label codes / continuous values: x[r * ldx + j * ldc] (row- or column-major)
  int ldx, n_rows, n_cols;
  int64_t ldc;
  float* out;           // [n_rows, ldo] encoded matrix (zero-filled by the caller)
  int ldo;
  int* opt;             // [n_rows, n_span] option index per conditional span
  int n_span;
  const int* col_kind;  // 0 continuous, 1 categorical
  const int* col_pos;   // output column of the alpha / first one-hot slot
  const int* col_aux;   // continuous: bank row; categorical: LUT offset
  const int* col_span;  // conditional span of the column's one-hot
  const int* col_lut_n; // categorical: LUT length (codes are clamped into it)
  const float* consts;  // [n_cont, 10] constant part of the weighted log prob
  const float* means;   // [n_cont, 10]
  const float* prec;    // [n_cont, 10] precision Cholesky (1 / sigma)
  const float* stds;    // [n_cont, 10]
  const int* vrank;     // [n_cont, 10] position among the valid modes, -1 if invalid
  const int* lut;       // categorical code -> option position
  uint64_t seed;
  uint32_t stream;
};
void launch_vgm_encode(const VgmEncodeArgs& a, hipStream_t stream);

// init_ops.hip: the federator's pooled GMM sample (segment s = (column, client, component) covers pool elements
// [seg_off[s], seg_off[s + 1]); element e = mean[s] + sd[s] * N(0, 1) keyed on (seed, e))
struct PoolSampleArgs {
  double* pool;
  const int64_t* seg_off;   // [nseg + 1]
  const double* mean;       // [nseg]
  const double* sd;         // [nseg]
  int nseg;
  int64_t n;
  uint64_t seed;
};
void launch_pool_sample(const PoolSampleArgs& a, hipStream_t stream);
// init_ops.hip: rows of a contiguous fp64 x [rows, n] centred in place; shift[row] = the row's mean
void launch_row_center(double* x, double* shift, int rows, int64_t n, hipStream_t stream);
// init_ops.hip: CSR real-row lists of an option matrix opt [n, n_col] (row-major, ldo): rows[s * n + ...] holds,
// for every span s and option o < width[s], the rows with that option in ascending order starting at offset[s, o];
// count[s, o] their number (offset / count 0 on padding slots o >= width[s]).  part: [n_col, chunks, maxw] scratch.
struct CsrArgs {
  const int* opt;
  int ldo;
  const int* width;
  int n, n_col, maxw, chunk, chunks;
  int* part;
  int64_t* count;
  int64_t* offset;
  int64_t* rows;
};
void launch_csr_rows(const CsrArgs& a, hipStream_t stream);

// Batched 1-D DP-GMM fit passes (kernels/vgm_fit.hip)
struct VgmFitArgs {
  const double* x;       // [n_cols, ldx] centred column data (row r valid for r < n_rows[col])
  int ldx, n_cols, max_rows, rows_per_block;
  const int* n_rows;     // [n_cols]
  const double* consts;  // [n_cols, 10] E-step: constant part of the weighted log prob
  const double* means;   // [n_cols, 10] E-step: posterior means; k-means: centres
  const double* prec;    // [n_cols, 10] E-step: precision Cholesky
  double* partial;       // [n_cols, chunks, 31] (E-step) or [n_cols, chunks, 30] (k-means)
};
void launch_vgm_estep(const VgmFitArgs& a, hipStream_t stream);
void launch_kmeans_step(const VgmFitArgs& a, hipStream_t stream);

// The whole fit of every column, one workgroup per column (kernels/vgm_fit.hip)
struct VgmFitAllArgs {
  const double* x;            // [n_cols, ldx] centred column data
  int ldx, n_cols;
  const int* n_rows;          // [n_cols]
  const double* init_centers; // [n_cols, 10] k-means centres to start from, or null (k-means++ + Lloyd)
  uint64_t seed;
  double wprior, tol, reg_covar;
  int max_iter, km_iter;
  double* out;                // [n_cols, 6, 10]: stick a, stick b, beta, means, dof, covariances
  int* info;                  // [n_cols, 2]: EM iterations, converged (-1: a cluster barrier timed out)
  double* lower_bound;        // [n_cols]
  // Split fit (split = G > 1 workgroups per column): every workgroup of a column seeds, runs Lloyd and the
  // M-steps on the whole column as before, but each E-step pass covers 1/G of the rows and the G partial records
  // meet through xpart [n_cols, 2, G, 32] (double-buffered by iteration) behind an arrival counter per column
  // (sync [n_cols * 32], zeroed by the caller).  split <= 1: one workgroup per column.
  int split;
  double* xpart;
  unsigned* sync;
};
// workgroups per column for a fit of n_cols columns of <= max_rows rows (set_tuning("vgm_split"): 0 = auto,
// 1 = one workgroup per column, n = n, capped by what the device holds at once)
int vgm_fit_split(int n_cols, int max_rows);
extern int g_vgm_split;
void launch_vgm_fit(const VgmFitAllArgs& a, hipStream_t stream);

}  // namespace fedtgan
