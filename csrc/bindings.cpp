// torch.ops.fedtgan.* — PyTorch bindings of the gfx950 kernels and the native host code.
// Every op validates shapes/strides on the host before launching (a wrong shape must never
// reach a kernel) and launches on the current HIP stream so hipGraph capture works.
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <cstring>
#include <utility>
#include <string>
#include <vector>

#include "comm/rccl_comm.h"
#include "host/csv_writer.h"
#include "kernels/launch.h"

using at::Tensor;
using c10::optional;

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check_f32_2d(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == at::kFloat, name, " must be float32");
  TORCH_CHECK(t.dim() == 2, name, " must be 2-D");
  TORCH_CHECK(t.size(1) <= 1 || t.stride(1) == 1, name, " must have unit column stride");
}

int ld_of(const Tensor& t) { return (int)(t.size(0) <= 1 ? std::max<int64_t>(t.size(1), 1) : t.stride(0)); }

// May a GEMM operand be read with 16-B loads?  Base 16-B aligned, ld % 4 == 0, and every row's
// contiguous extent rounded up to a multiple of 4 fits in ld and -- for the last row -- inside
// the tensor's storage (reads past the logical edge hit padding or the next row, which staging
// zeroes; never memory outside the storage).
bool vec_ok(const Tensor& t) {
  const int64_t ld = ld_of(t);
  const int64_t ext4 = (t.size(1) + 3) / 4 * 4;
  if (reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 != 0 || ld % 4 != 0 || ext4 > ld) return false;
  const int64_t storage = (int64_t)(t.storage().nbytes() / sizeof(float));
  return t.storage_offset() + (t.size(0) - 1) * ld + ext4 <= storage;
}

// bf16 GEMM operand (GemmArgs::bin): k-contiguous rows, 16-B aligned base, ld % 8 == 0, and every
// row's extent rounded up to 8 inside the storage (the kernel's 16-B loads are clamped to that).
void check_bf16_operand(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && t.dim() == 2, name, " must be a 2-D bf16 GPU tensor");
  TORCH_CHECK(t.size(1) <= 1 || t.stride(1) == 1, name, " must have unit column stride");
  const int64_t ld = ld_of(t);
  const int64_t ext8 = (t.size(1) + 7) / 8 * 8;
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0 && ld % 8 == 0 && ext8 <= ld, name,
              ": bf16 operands need a 16-B aligned base and a leading dimension divisible by 8 covering the row");
  const int64_t storage = (int64_t)(t.storage().nbytes() / 2);
  TORCH_CHECK(t.storage_offset() + (t.size(0) - 1) * ld + ext8 <= storage, name, ": rows padded to 8 must fit the storage");
}

uint16_t* hp(const Tensor& t) { return reinterpret_cast<uint16_t*>(t.data_ptr()); }

float* fp(const Tensor& t) { return t.data_ptr<float>(); }
const float* cfp(const Tensor& t) { return t.data_ptr<float>(); }
template <typename T>
T* optp(const optional<Tensor>& t) {
  return (t.has_value() && t->defined()) ? t->data_ptr<T>() : nullptr;
}
const uint64_t* ctr_ptr(const optional<Tensor>& t) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->scalar_type() == at::kLong && t->numel() >= 1 && t->is_cuda(), "rng_ctr must be a cuda int64 tensor");
  return reinterpret_cast<const uint64_t*>(t->data_ptr<int64_t>());
}

// pairing state of gemm(..., group): a GEMM held for launch_gemm_pair (group 1 / 2) or for the next
// adam_cs launch (group 3)
thread_local fedtgan::GemmArgs held{};
thread_local bool has_held = false;
thread_local hipStream_t held_stream = nullptr;
struct AdamHeld {
  fedtgan::GemmArgs g;
  hipStream_t stream;
  float* c;
  int64_t M, N, ldc;
  bool active;
};
thread_local AdamHeld g_adam_held{};
// a short-K weight gradient held for the next adam_cs launch (gemm(..., group=6)): launched just before it, with
// Adam in its own epilogue (launch_gemm_shortk_adam), its range cut out of the optimizer launch
thread_local AdamHeld g_adam_pre{};
// a chain tail (gemm(..., group=4)) waiting for its head (gemm(..., chain=True)); the head's launch copies
// the tail's arguments by value when it enqueues the reduction kernel
struct ChainTail {
  fedtgan::GemmArgs g;
  const void* a;
  int64_t M, K;
  bool active;
};
thread_local ChainTail g_chain_tail{};
thread_local fedtgan::GemmArgs g_chain_args{};

// The fused A-chain for the NEXT chain tail held by this thread (gemm_achain_next, launch.h GemmArgs::ach_*)
struct AchPending {
  Tensor out, ws, cnt;
  bool active;
};
thread_local AchPending g_ach{};

// drop every GEMM held by this thread (pairing, chain tail, Adam fusion) without launching it: called at
// the start of every step and when a step raises between a hold and its consumer, so a stale held GEMM
// (whose operand pointers may since have been freed) can never be launched or block the next step.
// Returns the number of holds that were dropped.
void pool_sample(const Tensor& pool, const Tensor& seg_off, const Tensor& mean, const Tensor& sd, int64_t seed) {
  TORCH_CHECK(pool.is_cuda() && pool.scalar_type() == at::kDouble && pool.is_contiguous(), "pool_sample: pool");
  TORCH_CHECK(seg_off.is_cuda() && seg_off.scalar_type() == at::kLong && seg_off.is_contiguous() && seg_off.numel() >= 2,
              "pool_sample: seg_off");
  const int64_t nseg = seg_off.numel() - 1;
  TORCH_CHECK(mean.is_cuda() && sd.is_cuda() && mean.scalar_type() == at::kDouble && sd.scalar_type() == at::kDouble &&
                  mean.is_contiguous() && sd.is_contiguous() && mean.numel() == nseg && sd.numel() == nseg,
              "pool_sample: mean / sd [nseg] fp64");
  fedtgan::PoolSampleArgs a{pool.data_ptr<double>(), seg_off.data_ptr<int64_t>(), mean.data_ptr<double>(),
                            sd.data_ptr<double>(), (int)nseg, pool.numel(), (uint64_t)seed};
  fedtgan::launch_pool_sample(a, cur_stream());
}

void row_center(const Tensor& x, const Tensor& shift) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kDouble && x.dim() == 2 && x.is_contiguous(), "row_center: x");
  TORCH_CHECK(shift.is_cuda() && shift.scalar_type() == at::kDouble && shift.numel() == x.size(0) && shift.is_contiguous(),
              "row_center: shift [rows] fp64");
  fedtgan::launch_row_center(x.data_ptr<double>(), shift.data_ptr<double>(), (int)x.size(0), x.size(1), cur_stream());
}

void csr_rows(const Tensor& opt, const Tensor& width, int64_t maxw, const Tensor& part, const Tensor& count,
              const Tensor& offset, const Tensor& rows, int64_t chunk) {
  TORCH_CHECK(opt.is_cuda() && opt.scalar_type() == at::kInt && opt.dim() == 2 && opt.stride(1) == 1, "csr_rows: opt");
  const int64_t n = opt.size(0), n_col = opt.size(1);
  const int64_t chunks = (n + chunk - 1) / std::max<int64_t>(chunk, 1);
  TORCH_CHECK(chunk > 0 && maxw > 0, "csr_rows: chunk / maxw");
  TORCH_CHECK(width.is_cuda() && width.scalar_type() == at::kInt && width.numel() == n_col, "csr_rows: width");
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kInt && part.is_contiguous() && part.numel() >= n_col * chunks * maxw,
              "csr_rows: part scratch [n_col, chunks, maxw] int32");
  for (const Tensor* t : {&count, &offset})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kLong && t->is_contiguous() && t->numel() == n_col * maxw,
                "csr_rows: count / offset [n_col, maxw] int64");
  TORCH_CHECK(rows.is_cuda() && rows.scalar_type() == at::kLong && rows.is_contiguous() && rows.numel() == n * n_col,
              "csr_rows: rows [n_col * n] int64");
  fedtgan::CsrArgs a{opt.data_ptr<int>(), (int)opt.stride(0), width.data_ptr<int>(), (int)n, (int)n_col, (int)maxw,
                     (int)chunk, (int)chunks, part.data_ptr<int>(), count.data_ptr<int64_t>(), offset.data_ptr<int64_t>(),
                     rows.data_ptr<int64_t>()};
  fedtgan::launch_csr_rows(a, cur_stream());
}

// hipDeviceSynchronize + hipDeviceReset of the current device: the process' HIP queues, events and memory are
// torn down NOW, while every component attached to the runtime (e.g. rocprofv3's tool library) is still live,
// instead of by libamdhip64's exit-time destructor (bench.py --device-reset-at-exit; profiles/exit_r6.txt).
// Nothing may touch the device afterwards; returns the hipError_t of the reset.
int64_t device_reset() {
  (void)hipDeviceSynchronize();
  return (int64_t)hipDeviceReset();
}

int64_t reset_held() {
  const int64_t n = (has_held ? 1 : 0) + (g_adam_held.active ? 1 : 0) + (g_adam_pre.active ? 1 : 0) +
                    (g_chain_tail.active ? 1 : 0) +
                    (g_ach.active ? 1 : 0);
  g_ach = AchPending{};
  has_held = false;
  held_stream = nullptr;
  g_adam_held.active = false;
  g_adam_pre.active = false;
  g_chain_tail.active = false;
  return n;
}

// Batched clients (kernels/launch.h ClientBatch): the calling thread's launches from here on run K clients at
// once -- client c's buffers `stride` bytes after client c-1's (one arena, identical layouts), its Philox seed
// seed + c * seed_step; base = client 0's slab start (every pointer of a batched launch is checked to lie in
// [base, base + stride)).  k = 1 restores plain launches.  Returns the previous k.
int64_t set_client_batch(int64_t k, int64_t stride, int64_t seed_step, int64_t base) {
  TORCH_CHECK(k >= 1 && k <= 65535, "set_client_batch: k");
  TORCH_CHECK(k == 1 || (stride > 0 && stride % 256 == 0 && base != 0),
              "set_client_batch: a batched context needs a 256-B aligned slab stride and a base");
  fedtgan::ClientBatch& cb = fedtgan::client_batch();
  const int64_t prev = cb.k;
  cb.k = (int)k;
  cb.stride = k > 1 ? stride : 0;
  cb.seed_step = k > 1 ? (uint64_t)seed_step : 0;
  cb.base = k > 1 ? reinterpret_cast<const char*>(base) : nullptr;
  cb.xcd = k > 1 ? fedtgan::g_xcd_clients : 0;
  return prev;
}

// The next chain tail (gemm(..., group=4) with a head seed head_a = A1 [M, N1], weights W1 [N1, K1]) also forms
// out [M, K1] = (A1 W1) . MS0 in the chain launch, MS0 = the chain head's mask; ws = fp32 scratch of at least
// ceil(N1 / 64) * M * K1 elements, cnt = int32 counters, at least one per head row, all zero (kept zero by the kernel).
void gemm_achain_next(const Tensor& out, const Tensor& ws, const Tensor& cnt) {
  TORCH_CHECK(!g_ach.active, "gemm_achain_next: already pending");
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kFloat && out.dim() == 2 && out.stride(1) == 1,
              "gemm_achain_next: out fp32 [M, K] rows");
  TORCH_CHECK(ws.is_cuda() && ws.scalar_type() == at::kFloat && ws.is_contiguous(), "gemm_achain_next: ws fp32");
  TORCH_CHECK(cnt.is_cuda() && cnt.scalar_type() == at::kInt && cnt.is_contiguous(), "gemm_achain_next: cnt int32");
  TORCH_CHECK(fedtgan::client_batch().k == 1, "gemm_achain_next: one client");
  g_ach = AchPending{out, ws, cnt, true};
}

void gemm(const Tensor& a, const Tensor& b, const Tensor& c, bool ta, bool tb, double alpha, double beta,
          const optional<Tensor>& bias, int64_t epi, const optional<Tensor>& ms, double slope, double p_drop,
          const optional<Tensor>& ws, int64_t splitk, int64_t seed, const optional<Tensor>& rng_ctr, int64_t stream,
          const optional<Tensor>& bn_gamma, const optional<Tensor>& bn_beta, const optional<Tensor>& bn_rm,
          const optional<Tensor>& bn_rv, double bn_eps, bool f32, const optional<Tensor>& head_coef,
          const optional<Tensor>& head_v, const optional<Tensor>& head_a, int64_t tile, int64_t group,
          const optional<Tensor>& oh_w, const optional<Tensor>& oh_col, const optional<Tensor>& oh_opt,
          const optional<Tensor>& oh_off, bool oh_trans, const optional<Tensor>& bn_part, int64_t bn_rpg,
          const optional<Tensor>& tile_cnt, bool chain) {
  const bool bin = a.scalar_type() == at::kBFloat16;
  const bool cbf = c.scalar_type() == at::kBFloat16;
  // op(A) = A^T (weight gradients): the kernels' A^T instantiations carry no epilogue code
  TORCH_CHECK(!ta || epi == fedtgan::EPI_NONE, "gemm: op(A) = A^T takes the plain epilogue only (bias / alpha / beta)");
  if (bin) {
    TORCH_CHECK(!ta && tb && !f32, "gemm: bf16 operands need C = A B^T on the bf16 MFMA path");
    check_bf16_operand(a, "a");
    check_bf16_operand(b, "b");
  } else {
    check_f32_2d(a, "a");
    check_f32_2d(b, "b");
  }
  if (cbf) {
    TORCH_CHECK(c.is_cuda() && c.dim() == 2 && (c.size(1) <= 1 || c.stride(1) == 1), "gemm: c");
    TORCH_CHECK(beta == 0.0 && (epi == fedtgan::EPI_NONE || epi == fedtgan::EPI_RELU || epi == fedtgan::EPI_BN_EVAL_RELU) &&
                    !(head_a.has_value() && head_a->defined()) && !(bn_part.has_value() && bn_part->defined()) &&
                    group == 0,
                "gemm: a bf16 output takes beta = 0 and the NONE / RELU / BN_EVAL_RELU epilogues, unpaired");
  } else {
    check_f32_2d(c, "c");
  }
  const int64_t M = ta ? a.size(1) : a.size(0);
  const int64_t K = ta ? a.size(0) : a.size(1);
  const int64_t Kb = tb ? b.size(1) : b.size(0);
  const int64_t N = tb ? b.size(0) : b.size(1);
  TORCH_CHECK(K == Kb, "gemm: inner dims differ (", K, " vs ", Kb, ")");
  TORCH_CHECK(c.size(0) == M && c.size(1) == N, "gemm: c is ", c.sizes(), " expected [", M, ", ", N, "]");
  if (bias.has_value() && bias->defined()) TORCH_CHECK(bias->numel() == N && bias->is_contiguous(), "gemm: bias");
  fedtgan::GemmArgs g{};
  if (bin) {
    g.a16 = hp(a);
    g.b16 = hp(b);
    g.bin = 1;
  } else {
    g.a = cfp(a);
    g.b = cfp(b);
  }
  if (cbf) g.c16 = hp(c);
  else g.c = fp(c);
  g.bias = optp<float>(bias);
  g.M = (int)M; g.N = (int)N; g.K = (int)K;
  g.lda = ld_of(a); g.ldb = ld_of(b); g.ldc = ld_of(c);
  g.ta = ta; g.tb = tb;
  g.alpha = (float)alpha; g.beta = (float)beta;
  g.epi = (int)epi;
  g.slope = (float)slope; g.p_drop = (float)p_drop;
  if (epi == fedtgan::EPI_MASK || epi == fedtgan::EPI_LRELU_DROPOUT) {
    TORCH_CHECK(ms.has_value() && ms->defined(), "gemm: epilogue needs ms");
    check_f32_2d(*ms, "ms");
    TORCH_CHECK(ms->size(0) == M && ms->size(1) == N, "gemm: ms shape");
    g.ms = fp(*ms);
    g.ldms = ld_of(*ms);
  }
  if (epi == fedtgan::EPI_BN_EVAL_RELU) {
    TORCH_CHECK(bn_gamma.has_value() && bn_beta.has_value() && bn_rm.has_value() && bn_rv.has_value(), "gemm: bn");
    g.bn_gamma = optp<float>(bn_gamma); g.bn_beta = optp<float>(bn_beta);
    g.bn_rm = optp<float>(bn_rm); g.bn_rv = optp<float>(bn_rv);
    g.bn_eps = (float)bn_eps;
  }
  g.splitk = (int)std::max<int64_t>(splitk, 1);
  if (g.splitk > 1) {
    TORCH_CHECK(ws.has_value() && ws->defined() && ws->scalar_type() == at::kFloat, "gemm: split-K needs ws");
    // the launcher rounds K slices up to whole bursts, so the effective split count never exceeds splitk
    TORCH_CHECK(ws->numel() >= (int64_t)g.splitk * M * N, "gemm: workspace too small");
    g.ws = fp(*ws);
  }
  g.seed = (uint64_t)seed;
  g.rng_ctr = ctr_ptr(rng_ctr);
  g.rng_stream = (uint32_t)stream;
  g.f32 = f32 ? 1 : 0;
  TORCH_CHECK(tile == 32 || tile == 64 || tile == 128, "gemm: tile must be 32, 64 or 128");
  g.vec = bin ? 1 : ((vec_ok(a) && vec_ok(b)) ? 1 : 0);
  g.tile = (int)tile;
  if (head_a.has_value() && head_a->defined()) {
    TORCH_CHECK(epi == fedtgan::EPI_LRELU_DROPOUT, "gemm: the head seed needs the LeakyReLU+dropout epilogue");
    check_f32_2d(*head_a, "head_a");
    TORCH_CHECK(head_a->size(0) == M && head_a->size(1) == N, "gemm: head_a shape");
    TORCH_CHECK(head_coef.has_value() && head_coef->numel() == M && head_coef->is_contiguous() && head_v.has_value() &&
                    head_v->numel() == N && head_v->is_contiguous(), "gemm: head coef [M] / v [N]");
    g.head_a = fp(*head_a);
    g.ldha = ld_of(*head_a);
    g.head_coef = cfp(*head_coef);
    g.head_v = cfp(*head_v);
  }
  if (oh_w.has_value() && oh_w->defined()) {
    TORCH_CHECK(!ta, "gemm: the one-hot block needs row-major A (its rows carry the conditions)");
    TORCH_CHECK(alpha == 1.0, "gemm: the one-hot block needs alpha = 1 (it is folded into the accumulators)");
    check_f32_2d(*oh_w, "oh_w");
    TORCH_CHECK(oh_trans ? oh_w->size(1) == N : oh_w->size(0) == N, "gemm: oh_w must be [N, C] (or [C, N] transposed)");
    g.oh_trans = oh_trans ? 1 : 0;
    g.oh_c = (int)(oh_trans ? oh_w->size(0) : oh_w->size(1));
    TORCH_CHECK(oh_col.has_value() && oh_opt.has_value() && oh_off.has_value(), "gemm: one-hot needs col / opt / off");
    for (const auto* t : {&*oh_col, &*oh_opt, &*oh_off})
      TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kInt && t->is_contiguous(), "gemm: one-hot int32 tables");
    TORCH_CHECK(oh_col->numel() >= M && oh_opt->numel() >= M, "gemm: one-hot col / opt need M entries");
    g.oh_w = cfp(*oh_w);
    g.oh_ld = ld_of(*oh_w);
    g.oh_col = oh_col->data_ptr<int>();
    g.oh_opt = oh_opt->data_ptr<int>();
    g.oh_off = oh_off->data_ptr<int>();
  }
  if (bn_part.has_value() && bn_part->defined()) {
    TORCH_CHECK(!ta && !bin && !cbf && epi == fedtgan::EPI_NONE && alpha == 1.0 && beta == 0.0 && g.splitk == 1 &&
                    (tile == 32 || tile == 64) && group == 0 && g.vec,
                "gemm: BN partials need a plain unsplit C = A op(B) + bias on 32/64 tiles with 16-B operands");
    const int64_t tiles = (M + tile - 1) / tile;
    TORCH_CHECK(bn_part->is_cuda() && bn_part->scalar_type() == at::kFloat && bn_part->is_contiguous() &&
                    bn_part->numel() >= tiles * 6 * N, "gemm: bn_part must hold [m_tiles, 2, 3, N] floats");
    TORCH_CHECK(bn_rpg >= 1 && bn_rpg <= M, "gemm: bn_rpg");
    g.bn_part = fp(*bn_part);
    g.bn_rpg = (int)bn_rpg;
  }
  if (tile_cnt.has_value() && tile_cnt->defined() && g.splitk > 1) {
    // one arrival counter per output tile, all zero (the reducing workgroup re-zeroes its tile's)
    const int64_t tiles = ((M + tile - 1) / tile) * ((N + tile - 1) / tile);
    TORCH_CHECK(tile_cnt->is_cuda() && tile_cnt->scalar_type() == at::kInt && tile_cnt->is_contiguous() &&
                    tile_cnt->numel() >= tiles, "gemm: tile_cnt must hold one int32 per output tile");
    g.tile_cnt = reinterpret_cast<unsigned*>(tile_cnt->data_ptr<int>());
  }
  if (group == 4) {
    // the tail of a chain (held for the next gemm(..., chain=True), whose output is this GEMM's A): its
    // own epilogue, computed row by row in the head's reduction launch (chain_epilogue_kernel)
    TORCH_CHECK(!g_chain_tail.active, "gemm: a chain tail is already held");
    TORCH_CHECK(!ta && tb && !bin && !cbf && !g.oh_w && !g.bn_part && beta == 0.0 && K <= 1024 && K % 16 == 0 &&
                    ld_of(b) % 4 == 0 &&
                    (reinterpret_cast<uintptr_t>(b.data_ptr()) & 15) == 0,
                "gemm: a chain tail is C = A B^T with fp32 16-B aligned B rows (ld % 4 == 0), K <= 1024, K % 16 == 0, "
                "no one-hot block / BN partials");
    g.splitk = 1;
    if (g_ach.active) {
      AchPending q = g_ach;
      g_ach = AchPending{};
      TORCH_CHECK(g.head_a && epi == fedtgan::EPI_LRELU_DROPOUT, "gemm: the fused A-chain needs a tail with a head seed");
      TORCH_CHECK(q.out.size(0) == M && q.out.size(1) == K && q.ws.numel() >= ((N + 63) / 64) * M * K && q.cnt.numel() >= M,
                  "gemm: fused A-chain out [M, K] / ws [ceil(N / 64), M, K] / cnt [M]");
      g.ach_out = q.out.data_ptr<float>();
      g.ld_ach = (int)q.out.stride(0);
      g.ach_ws = q.ws.data_ptr<float>();
      g.ach_cnt = reinterpret_cast<unsigned*>(q.cnt.data_ptr<int>());
    }
    g_chain_tail = ChainTail{g, a.data_ptr(), (int64_t)M, (int64_t)K, true};
    return;
  }
  TORCH_CHECK(!g_ach.active, "gemm: gemm_achain_next is pending but this GEMM is no chain tail");
  if (chain) {
    TORCH_CHECK(g_chain_tail.active && group != 1, "gemm: chain=True needs a tail held with group=4 (and no group 1)");
    const ChainTail& t = g_chain_tail;
    TORCH_CHECK(t.a == c.data_ptr() && t.M == M && t.K == N && !cbf,
                "gemm: the chain tail's A must be this GEMM's fp32 output (same rows, K = N)");
    g_chain_args = t.g;
    g_chain_tail.active = false;
    g.chain = &g_chain_args;
  } else {
    TORCH_CHECK(!g_chain_tail.active || group == 1, "gemm: a chain tail is held; the next unpaired GEMM must be its head");
  }
  // group 1: hold this GEMM; group 2: launch it together with the held one (launch_gemm_pair: the two
  // must be independent -- neither reads what the other writes); group 3: hold it for the next
  // adam_cs launch on this stream (a weight gradient inside that optimizer's gradient buffer: the
  // two become one launch, gemm_adam_kernel); group 0: launch now
  const hipStream_t hs = cur_stream();
  if (group == 6 || group == 7) {
    // group 7: the same, with the gradient itself stored too (GemmArgs::adam_grad)
    TORCH_CHECK(!g_adam_pre.active, "gemm: a short-K GEMM is already held for the Adam launch");
    g.adam_grad = group == 7 ? 1 : 0;
    TORCH_CHECK(ta && !tb && epi == fedtgan::EPI_NONE && alpha == 1.0 && beta == 0.0 && !g.bias && !g.oh_w && !g.head_a &&
                    !g.bn_part && !cbf && !bin && !chain && fedtgan::client_batch().k == 1,
                "gemm: group 6 holds a plain C = A^T B weight gradient of one client (short-K Adam)");
    g_adam_pre = AdamHeld{g, hs, c.data_ptr<float>(), (int64_t)M, (int64_t)N, (int64_t)g.ldc, true};
    return;
  }
  if (group == 3) {
    TORCH_CHECK(!g_adam_held.active, "gemm: a GEMM is already held for the Adam launch");
    TORCH_CHECK(epi == fedtgan::EPI_NONE && beta == 0.0 && !g.bias && !g.oh_w && !g.head_a && !g.bn_part && !cbf && !bin,
                "gemm: a GEMM fused with Adam takes a plain epilogue (no bias / beta / one-hot / head / BN partials)");
    g_adam_held = AdamHeld{g, hs, c.data_ptr<float>(), (int64_t)M, (int64_t)N, (int64_t)g.ldc, true};
    return;
  }
  if (group == 1) {
    TORCH_CHECK(!has_held, "gemm: a GEMM is already held for pairing");
    held = g;
    has_held = true;
    held_stream = hs;
    return;
  }
  if (group == 2) {
    TORCH_CHECK(has_held && held_stream == hs, "gemm: group 2 needs a held GEMM on the same stream");
    TORCH_CHECK(!(held.splitk > 1 && g.splitk > 1 && held.ws == g.ws), "gemm: paired split-K GEMMs share a workspace");
    TORCH_CHECK(!(held.tile_cnt && g.tile_cnt && held.tile_cnt == g.tile_cnt), "gemm: paired GEMMs share tile counters");
    has_held = false;
    fedtgan::launch_gemm_pair(held, g, hs);
    return;
  }
  TORCH_CHECK(!has_held, "gemm: a held GEMM was never paired");
  fedtgan::launch_gemm(g, hs);
}

void sample(const Tensor& h, int64_t zc, int64_t cc, int64_t E, const optional<Tensor>& xf, const optional<Tensor>& xr,
            int64_t Dd, const Tensor& cdf, const Tensor& cond_off, const Tensor& cond_w, const optional<Tensor>& row_off,
            const optional<Tensor>& row_cnt, const optional<Tensor>& rows, const optional<Tensor>& data,
            const optional<Tensor>& col, const optional<Tensor>& opt, const optional<Tensor>& step_bump,
            const optional<Tensor>& step_bump2, const optional<Tensor>& metrics, bool zero_metrics, int64_t seed,
            const Tensor& rng_ctr, int64_t stream, int64_t draws, int64_t draw_h, int64_t draw_x, int64_t draw_col) {
  fedtgan::SampleArgs a{};
  const bool h16 = h.scalar_type() == at::kBFloat16;
  a.B = (int)h.size(0);
  a.E = (int)E;
  a.Dd = (int)Dd;
  a.n_col = (int)cond_w.numel();
  a.maxw = cdf.dim() == 2 ? (int)cdf.size(1) : 0;
  TORCH_CHECK(cond_off.scalar_type() == at::kInt && cond_w.scalar_type() == at::kInt, "sample: int32 tables");
  TORCH_CHECK(cdf.is_contiguous() && cdf.scalar_type() == at::kFloat, "sample: cdf");
  if (h16) {
    // generation into a bf16 activation buffer: only z is written (the condition goes to col / opt)
    TORCH_CHECK(h.is_cuda() && h.dim() == 2 && (h.size(1) <= 1 || h.stride(1) == 1), "sample: h");
    TORCH_CHECK(zc >= 0 && zc + E <= h.size(1), "sample: z columns");
    TORCH_CHECK(!(xf.has_value() && xf->defined()) && !(xr.has_value() && xr->defined()),
                "sample: a bf16 h takes no D-input blocks");
    TORCH_CHECK(a.n_col == 0 || (col.has_value() && opt.has_value()), "sample: a bf16 h needs col / opt outputs");
    a.h16 = hp(h); a.ldh16 = ld_of(h); a.zc16 = (int)zc;
  } else {
    check_f32_2d(h, "h");
    a.C = (int)(h.size(1) - cc);
    TORCH_CHECK(zc + E <= h.size(1) && cc <= h.size(1), "sample: column ranges");
    a.h = fp(h); a.ldh = ld_of(h); a.zc = (int)zc; a.cc = (int)cc;
  }
  a.ldx = 0;
  if (xf.has_value() && xf->defined()) {
    check_f32_2d(*xf, "xf");
    TORCH_CHECK(xf->size(0) == a.B && xf->size(1) == Dd + a.C, "sample: xf shape");
    a.xf = fp(*xf); a.ldx = ld_of(*xf);
  }
  if (xr.has_value() && xr->defined()) {
    check_f32_2d(*xr, "xr");
    // the real block may cover only the leading rows (a D-phase batch drawn together with a G-phase one)
    TORCH_CHECK(xr->size(0) >= 1 && xr->size(0) <= a.B && xr->size(1) == Dd + a.C, "sample: xr shape");
    a.n_real = (int)xr->size(0);
    TORCH_CHECK(row_off.has_value() && row_cnt.has_value() && rows.has_value() && data.has_value(), "sample: tables");
    TORCH_CHECK(data->size(1) == Dd && data->is_contiguous(), "sample: data");
    a.xr = fp(*xr);
    if (a.ldx == 0) a.ldx = ld_of(*xr);
    TORCH_CHECK(ld_of(*xr) == a.ldx, "sample: xf/xr strides differ");
    a.row_off = optp<int64_t>(row_off); a.row_cnt = optp<int64_t>(row_cnt); a.rows = optp<int64_t>(rows);
    a.n_entries = rows->numel();
    a.data = data->data_ptr<float>();
    a.n_rows = (int)data->size(0);
  }
  a.cdf = cfp(cdf);
  a.cond_off = cond_off.data_ptr<int>();
  a.cond_w = cond_w.data_ptr<int>();
  for (const auto* t : {&col, &opt})
    if (t->has_value() && (*t)->defined())
      TORCH_CHECK((*t)->is_cuda() && (*t)->scalar_type() == at::kInt && (*t)->is_contiguous() && (*t)->numel() >= a.B,
                  "sample: col / opt must be int32 with one entry per row");
  a.col = optp<int>(col);
  a.opt = optp<int>(opt);
  a.step_bump = optp<float>(step_bump);
  a.step_bump2 = optp<float>(step_bump2);
  a.metrics = optp<float>(metrics);
  a.zero_metrics = zero_metrics ? 1 : 0;
  a.seed = (uint64_t)seed;
  a.rng_ctr = ctr_ptr(rng_ctr);
  a.rng_stream = (uint32_t)stream;
  a.draws = (int)std::max<int64_t>(draws, 1);
  if (a.draws > 1) {
    // every draw's buffers must lie inside their tensors' storage: draw k writes at the same views + k x stride
    TORCH_CHECK(!h16 && draw_h > 0 && draw_col > 0 && (draw_x > 0 || !(xf.has_value() && xf->defined())),
                "sample: multi-step draws need fp32 h and positive strides");
    auto fits = [&](const Tensor& t, int64_t stride, const char* what) {
      const int64_t span = (t.size(0) - 1) * t.stride(0) + (t.dim() > 1 ? t.size(1) : 1);
      const int64_t last = t.storage_offset() + (a.draws - 1) * stride + span;
      TORCH_CHECK(last * (int64_t)t.element_size() <= (int64_t)t.storage().nbytes(), "sample: draw ", a.draws - 1,
                  " of ", what, " runs past its storage");
    };
    fits(h, draw_h, "h");
    if (xf.has_value() && xf->defined()) fits(*xf, draw_x, "xf");
    if (xr.has_value() && xr->defined()) fits(*xr, draw_x, "xr");
    for (const auto* t : {&col, &opt})
      if (t->has_value() && (*t)->defined()) fits(**t, draw_col, "col / opt");
    for (const auto* t : {&step_bump, &step_bump2})
      if (t->has_value() && (*t)->defined())
        TORCH_CHECK((*t)->numel() >= a.draws && (*t)->is_contiguous(), "sample: per-step counters need [draws]");
    if (metrics.has_value() && metrics->defined())
      TORCH_CHECK(metrics->numel() >= 4 * a.draws && metrics->is_contiguous(), "sample: metrics need [draws, 4]");
    a.draw_h = draw_h;
    a.draw_x = draw_x;
    a.draw_col = draw_col;
  }
  fedtgan::launch_sample(a, cur_stream());
}

fedtgan::SpanTables spans_of(const Tensor& start, const Tensor& width, const Tensor& kind, const Tensor& cidx,
                             const Tensor& packed, int64_t dim) {
  TORCH_CHECK(start.scalar_type() == at::kInt && width.scalar_type() == at::kInt && kind.scalar_type() == at::kInt &&
                  cidx.scalar_type() == at::kInt && packed.scalar_type() == at::kInt,
              "span tables must be int32");
  TORCH_CHECK(start.numel() == width.numel() && start.numel() == kind.numel() && start.numel() == cidx.numel(),
              "span tables: sizes");
  const int S = (int)start.numel();
  TORCH_CHECK(packed.is_contiguous() && packed.numel() == fedtgan::span_packed_len((int)dim, S) &&
                  reinterpret_cast<uintptr_t>(packed.data_ptr()) % 16 == 0,
              "span tables: packed table must hold [elem | kind | start | width | cidx] padded to 4 ints");
  fedtgan::SpanTables sp{start.data_ptr<int>(), width.data_ptr<int>(), kind.data_ptr<int>(), cidx.data_ptr<int>(),
                         packed.data_ptr<int>(), S, (int)dim};
  TORCH_CHECK(fedtgan::activation_smem_bytes(sp) <= 160 * 1024, "activation: row image exceeds the 160 KiB LDS");
  return sp;
}

void activate(const Tensor& logits, const Tensor& out, const Tensor& start, const Tensor& width, const Tensor& kind,
              const Tensor& cidx, const Tensor& elem, double tau, int64_t seed, const Tensor& rng_ctr, int64_t stream,
              const optional<Tensor>& slerp_real, const optional<Tensor>& slerp_out, int64_t slerp_cols,
              int64_t slerp_stream) {
  check_f32_2d(logits, "logits");
  check_f32_2d(out, "out");
  TORCH_CHECK(out.size(0) == logits.size(0) && out.size(1) >= logits.size(1), "activate: shapes");
  fedtgan::SlerpFuse sl{};
  if (slerp_real.has_value() && slerp_real->defined()) {
    TORCH_CHECK(slerp_out.has_value() && slerp_out->defined(), "activate: slerp needs an output");
    check_f32_2d(*slerp_real, "slerp real");
    check_f32_2d(*slerp_out, "slerp out");
    TORCH_CHECK(ld_of(*slerp_real) == ld_of(*slerp_out) && ld_of(*slerp_real) == ld_of(out), "activate: slerp strides");
    TORCH_CHECK(slerp_real->size(0) >= 1 && slerp_real->size(0) <= out.size(0) &&
                    slerp_out->size(0) == slerp_real->size(0) &&
                    slerp_real->size(1) == slerp_cols && slerp_out->size(1) == slerp_cols &&
                    slerp_cols >= logits.size(1) && slerp_cols <= ld_of(out), "activate: slerp shapes");
    sl.real = cfp(*slerp_real);
    sl.out = fp(*slerp_out);
    sl.ld = ld_of(out);
    sl.cols = (int)slerp_cols;
    sl.rows = (int)slerp_real->size(0);
    sl.stream = (uint32_t)slerp_stream;
  }
  fedtgan::launch_activate(cfp(logits), ld_of(logits), fp(out), ld_of(out), (int)logits.size(0),
                           spans_of(start, width, kind, cidx, elem, logits.size(1)), (float)tau, (uint64_t)seed, ctr_ptr(rng_ctr),
                           (uint32_t)stream, sl, cur_stream());
}

void act_bwd_ce(const Tensor& dact, const Tensor& act, const Tensor& logits, const Tensor& start, const Tensor& width,
                const Tensor& kind, const Tensor& cidx, const Tensor& elem, const Tensor& col, const Tensor& opt,
                const Tensor& dlogits, const Tensor& loss, double tau) {
  check_f32_2d(dact, "dact");
  check_f32_2d(act, "act");
  check_f32_2d(logits, "logits");
  check_f32_2d(dlogits, "dlogits");
  const int64_t rows = logits.size(0);
  TORCH_CHECK(dact.size(0) == rows && act.size(0) == rows && dlogits.size(0) == rows && col.numel() >= rows,
              "act_bwd_ce: rows");
  // loss with one entry per row: per-row terms (summed later), else accumulated into loss[0]
  const bool per_row = rows > 1 && loss.numel() == rows;
  TORCH_CHECK(per_row || loss.numel() >= 1, "act_bwd_ce: loss");
  fedtgan::launch_act_bwd_ce(cfp(dact), ld_of(dact), cfp(act), ld_of(act), cfp(logits), ld_of(logits),
                             spans_of(start, width, kind, cidx, elem, logits.size(1)), col.data_ptr<int>(), opt.data_ptr<int>(), fp(dlogits),
                             ld_of(dlogits), (int)rows, (float)tau, fp(loss), per_row ? 1 : 0, cur_stream());
}

void slerp(const Tensor& real, const Tensor& fake, const Tensor& out, int64_t seed, const Tensor& rng_ctr,
           int64_t stream) {
  check_f32_2d(real, "real");
  check_f32_2d(fake, "fake");
  check_f32_2d(out, "out");
  TORCH_CHECK(real.sizes() == fake.sizes() && real.sizes() == out.sizes(), "slerp: shapes");
  TORCH_CHECK(ld_of(real) == ld_of(fake) && ld_of(real) == ld_of(out), "slerp: strides");
  fedtgan::launch_slerp(cfp(real), cfp(fake), fp(out), (int)real.size(0), (int)real.size(1), ld_of(real),
                        (uint64_t)seed, ctr_ptr(rng_ctr), (uint32_t)stream, cur_stream());
}

void gp_scale(const Tensor& g, const Tensor& out, double lam, const Tensor& loss, const optional<Tensor>& ws) {
  check_f32_2d(g, "g");
  check_f32_2d(out, "out");
  TORCH_CHECK(g.sizes() == out.sizes(), "gp_scale: shapes");
  const bool per_row = g.size(0) > 1 && loss.numel() == g.size(0);   // per-pack terms, summed later
  float* wsp = nullptr;
  int64_t wsn = 0;
  if (ws.has_value()) {
    TORCH_CHECK(ws->is_cuda() && ws->scalar_type() == at::kFloat && ws->is_contiguous(), "gp_scale: float32 workspace");
    wsp = fp(*ws);
    wsn = ws->numel();
  }
  fedtgan::launch_gp_scale(cfp(g), ld_of(g), fp(out), ld_of(out), (int)g.size(0), (int)g.size(1), (float)lam,
                           fp(loss), per_row ? 1 : 0, wsp, wsn, cur_stream());
}

void onehot_wgrad(const std::vector<Tensor>& dy, const std::vector<Tensor>& w, const Tensor& col, const Tensor& opt,
                  const Tensor& cond_off, int64_t zero) {
  TORCH_CHECK(dy.size() == w.size() && !dy.empty() && dy.size() <= 4, "onehot_wgrad: 1-4 (dy, w) jobs");
  TORCH_CHECK(col.scalar_type() == at::kInt && opt.scalar_type() == at::kInt && cond_off.scalar_type() == at::kInt &&
                  col.is_contiguous() && opt.is_contiguous() && cond_off.is_contiguous(),
              "onehot_wgrad: int32 contiguous col / opt / cond_off");
  fedtgan::OnehotWBatch bt{};
  bt.n_jobs = (int)dy.size();
  bt.B = (int)dy[0].size(0);
  TORCH_CHECK(col.numel() >= bt.B && opt.numel() >= bt.B, "onehot_wgrad: col / opt rows");
  for (size_t j = 0; j < dy.size(); ++j) {
    check_f32_2d(dy[j], "dy");
    check_f32_2d(w[j], "w");
    TORCH_CHECK(dy[j].size(0) == bt.B && dy[j].size(1) == w[j].size(1), "onehot_wgrad: shapes");
    bt.jobs[j] = fedtgan::OnehotWJob{cfp(dy[j]), fp(w[j]), (int)ld_of(dy[j]), (int)ld_of(w[j]), (int)w[j].size(1)};
  }
  bt.col = col.data_ptr<int>();
  bt.opt = opt.data_ptr<int>();
  bt.cond_off = cond_off.data_ptr<int>();
  fedtgan::launch_onehot_wgrad(bt, (int)zero, cur_stream());
}

void d_head(const Tensor& d, const Tensor& ms, const Tensor& v, const Tensor& e, const Tensor& coef,
            const Tensor& wloss, const Tensor& y, const Tensor& a, const Tensor& loss) {
  check_f32_2d(d, "d");
  check_f32_2d(ms, "ms");
  check_f32_2d(a, "a");
  const int64_t rows = d.size(0), cols = d.size(1);
  TORCH_CHECK(ms.sizes() == d.sizes() && a.sizes() == d.sizes() && v.numel() == cols && coef.numel() >= rows &&
                  wloss.numel() >= rows && y.numel() >= rows,
              "d_head: shapes");
  fedtgan::launch_d_head(cfp(d), ld_of(d), cfp(ms), ld_of(ms), cfp(v), cfp(e), cfp(coef), cfp(wloss), fp(y), fp(a),
                         ld_of(a), (int)rows, (int)cols, fp(loss), cur_stream());
}

std::vector<fedtgan::ColsumJob> colsum_jobs(at::TensorList srcs, const c10::List<optional<Tensor>>& outs,
                                            const c10::List<optional<Tensor>>& w,
                                            const c10::List<optional<Tensor>>& dot_v,
                                            const c10::List<optional<Tensor>>& dot_e,
                                            const c10::List<optional<Tensor>>& dot_out,
                                            const c10::List<optional<Tensor>>& dot_w) {
  const size_t n = srcs.size();
  TORCH_CHECK(n <= 8 && outs.size() == n && w.size() == n && dot_v.size() == n && dot_e.size() == n &&
                  dot_out.size() == n && dot_w.size() == n, "colsum_ex: up to 8 jobs, one entry per job in every list");
  std::vector<fedtgan::ColsumJob> jobs;
  for (size_t i = 0; i < n; ++i) {
    check_f32_2d(srcs[i], "colsum src");
    const int64_t rows = srcs[i].size(0), cols = srcs[i].size(1);
    fedtgan::ColsumJob j{cfp(srcs[i]), ld_of(srcs[i]), (int)rows, (int)cols, nullptr, nullptr, nullptr, nullptr, nullptr,
                         nullptr};
    const optional<Tensor> o = outs[i], wi = w[i], dv = dot_v[i], de = dot_e[i], dout = dot_out[i];
    if (o.has_value() && o->defined()) {
      TORCH_CHECK(o->numel() == cols && o->is_contiguous(), "colsum_ex: out");
      j.out = fp(*o);
    }
    if (wi.has_value() && wi->defined()) {
      TORCH_CHECK(wi->numel() == rows && wi->is_contiguous(), "colsum_ex: row weights");
      j.w = cfp(*wi);
    }
    if (dv.has_value() && dv->defined()) {
      TORCH_CHECK(dv->numel() == cols && dv->is_contiguous() && dout.has_value() && dout->defined(), "colsum_ex: dot");
      j.dot_v = cfp(*dv);
      j.dot_out = fp(*dout);
      if (de.has_value() && de->defined()) j.dot_e = cfp(*de);
      const optional<Tensor> dw = dot_w[i];
      if (dw.has_value() && dw->defined()) {
        TORCH_CHECK(dw->numel() == rows && dw->is_contiguous(), "colsum_ex: dot row weights");
        j.dot_w = cfp(*dw);
      }
    }
    jobs.push_back(j);
  }
  return jobs;
}

void colsum_ex(at::TensorList srcs, const c10::List<optional<Tensor>>& outs, const c10::List<optional<Tensor>>& w,
               const c10::List<optional<Tensor>>& dot_v, const c10::List<optional<Tensor>>& dot_e,
               const c10::List<optional<Tensor>>& dot_out, const c10::List<optional<Tensor>>& dot_w) {
  const auto jobs = colsum_jobs(srcs, outs, w, dot_v, dot_e, dot_out, dot_w);
  fedtgan::launch_colsum(jobs.data(), (int)jobs.size(), cur_stream());
}

void colsum(at::TensorList srcs, at::TensorList outs) {
  TORCH_CHECK(srcs.size() == outs.size() && srcs.size() <= 8, "colsum: up to 8 jobs");
  std::vector<fedtgan::ColsumJob> jobs;
  for (size_t i = 0; i < srcs.size(); ++i) {
    check_f32_2d(srcs[i], "colsum src");
    TORCH_CHECK(outs[i].numel() == srcs[i].size(1) && outs[i].is_contiguous(), "colsum: out");
    jobs.push_back({cfp(srcs[i]), ld_of(srcs[i]), (int)srcs[i].size(0), (int)srcs[i].size(1), fp(outs[i]), nullptr,
                    nullptr, nullptr, nullptr});
  }
  fedtgan::launch_colsum(jobs.data(), (int)jobs.size(), cur_stream());
}

void bn_relu_train(const Tensor& a, const Tensor& gamma, const Tensor& beta, const Tensor& out, const Tensor& nhat,
                   const Tensor& mean, const Tensor& invstd, const Tensor& rm, const Tensor& rv, double momentum,
                   double eps, int64_t groups) {
  check_f32_2d(a, "a");
  check_f32_2d(out, "out");
  check_f32_2d(nhat, "nhat");
  TORCH_CHECK(a.size(0) >= 1, "bn_relu_train: empty batch");
  TORCH_CHECK(groups == 1 || groups == 2, "bn_relu_train: 1 or 2 batches");
  TORCH_CHECK(a.size(0) % groups == 0 && a.size(0) / groups >= 1, "bn_relu_train: rows must split evenly");
  TORCH_CHECK(out.sizes() == a.sizes() && nhat.sizes() == a.sizes() && gamma.numel() == a.size(1), "bn: shapes");
  TORCH_CHECK(mean.is_contiguous() && invstd.is_contiguous() && mean.numel() == groups * a.size(1) &&
                  invstd.numel() == groups * a.size(1), "bn_relu_train: mean/invstd must be contiguous [groups, cols]");
  fedtgan::launch_bn_relu_train(cfp(a), ld_of(a), cfp(gamma), cfp(beta), fp(out), ld_of(out), fp(nhat), ld_of(nhat),
                                fp(mean), fp(invstd), fp(rm), fp(rv), (int)a.size(0), (int)a.size(1), (int)groups,
                                (float)momentum, (float)eps, cur_stream());
}

void bn_relu_apply(const Tensor& a, const Tensor& part, int64_t n_tiles, const Tensor& gamma, const Tensor& beta,
                   const Tensor& out, const Tensor& nhat, const Tensor& mean, const Tensor& invstd, const Tensor& rm,
                   const Tensor& rv, double momentum, double eps, int64_t groups) {
  check_f32_2d(a, "a");
  check_f32_2d(out, "out");
  check_f32_2d(nhat, "nhat");
  const int64_t rows = a.size(0), cols = a.size(1);
  TORCH_CHECK(groups == 1 || groups == 2, "bn_relu_apply: 1 or 2 batches");
  TORCH_CHECK(rows >= 1 && rows % groups == 0, "bn_relu_apply: rows must split evenly");
  TORCH_CHECK(out.sizes() == a.sizes() && nhat.sizes() == a.sizes() && gamma.numel() == cols && beta.numel() == cols &&
                  rm.numel() == cols && rv.numel() == cols, "bn_relu_apply: shapes");
  TORCH_CHECK(mean.is_contiguous() && invstd.is_contiguous() && mean.numel() == groups * cols &&
                  invstd.numel() == groups * cols, "bn_relu_apply: mean/invstd must be contiguous [groups, cols]");
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.is_contiguous() &&
                  part.numel() >= n_tiles * 6 * cols && n_tiles >= 1 && n_tiles <= 64,
              "bn_relu_apply: partials [n_tiles <= 64, 2, 3, cols]");
  fedtgan::launch_bn_relu_apply(cfp(a), ld_of(a), cfp(part), (int)n_tiles, cfp(gamma), cfp(beta), fp(out), ld_of(out),
                                fp(nhat), ld_of(nhat), fp(mean), fp(invstd), fp(rm), fp(rv), (int)rows, (int)cols,
                                (int)groups, (float)momentum, (float)eps, cur_stream());
}

// Linear -> BatchNorm(train) -> ReLU, one launch (kernels/bn_fused.hip).  x: the dense input columns
// [groups * rpg, K]; W: [N, K] (any strides); one-hot block as for gemm (oh_w [N, C], or [C, N] with
// oh_trans); stat: >= groups * 2 * N floats; cnt: >= ceil(N / 16) zeroed int32 counters.
void linear_bn_relu_colown(const Tensor& x, const Tensor& w, const optional<Tensor>& bias, const Tensor& gamma,
                           const Tensor& beta, const Tensor& out, const Tensor& nhat, const Tensor& mean,
                           const Tensor& invstd, const Tensor& rm, const Tensor& rv, double momentum, double eps,
                           int64_t groups, const optional<Tensor>& oh_w, const optional<Tensor>& oh_col,
                           const optional<Tensor>& oh_opt, const optional<Tensor>& oh_off, bool oh_trans,
                           const Tensor& stat, const Tensor& cnt) {
  check_f32_2d(x, "x");
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kFloat && w.dim() == 2, "colown: w must be a 2-D fp32 GPU tensor");
  check_f32_2d(out, "out");
  check_f32_2d(nhat, "nhat");
  const int64_t rows = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(groups == 1 || groups == 2, "colown: 1 or 2 batches");
  TORCH_CHECK(rows >= 2 && rows % groups == 0, "colown: rows must split evenly");
  TORCH_CHECK(K >= 1 && w.size(1) == K, "colown: w is ", w.sizes(), ", x has K = ", K);
  TORCH_CHECK(out.size(0) == rows && out.size(1) == N && nhat.size(0) == rows && nhat.size(1) == N, "colown: out / nhat");
  TORCH_CHECK(gamma.numel() == N && beta.numel() == N && rm.numel() == N && rv.numel() == N && gamma.is_contiguous() &&
                  beta.is_contiguous() && rm.is_contiguous() && rv.is_contiguous(), "colown: BN vectors");
  TORCH_CHECK(mean.is_contiguous() && invstd.is_contiguous() && mean.numel() == groups * N &&
                  invstd.numel() == groups * N, "colown: mean/invstd must be contiguous [groups, cols]");
  const int64_t rpg = rows / groups;
  TORCH_CHECK(fedtgan::colown_smem_bytes((int)K, (int)rpg) <= 64 * 1024, "colown: batch x K too large for LDS");
  TORCH_CHECK(stat.is_cuda() && stat.scalar_type() == at::kFloat && stat.is_contiguous() && stat.numel() >= groups * 2 * N,
              "colown: stat");
  TORCH_CHECK(cnt.is_cuda() && cnt.scalar_type() == at::kInt && cnt.is_contiguous() && cnt.numel() >= (N + 15) / 16,
              "colown: cnt");
  if (bias.has_value() && bias->defined()) TORCH_CHECK(bias->numel() == N && bias->is_contiguous(), "colown: bias");
  fedtgan::ColOwnArgs g{};
  g.x = cfp(x);
  g.ldx = (int)ld_of(x);
  g.w = w.data_ptr<float>();
  g.w_sn = w.stride(0);
  g.w_sk = w.stride(1);
  g.bias = optp<float>(bias);
  if (oh_w.has_value() && oh_w->defined()) {
    TORCH_CHECK(oh_col.has_value() && oh_opt.has_value() && oh_off.has_value(), "colown: one-hot needs col/opt/off");
    TORCH_CHECK(oh_col->numel() == rows && oh_opt->numel() == rows && oh_col->scalar_type() == at::kInt &&
                    oh_opt->scalar_type() == at::kInt && oh_off->scalar_type() == at::kInt, "colown: one-hot indices");
    TORCH_CHECK(oh_w->scalar_type() == at::kFloat && oh_w->dim() == 2 && oh_w->size(oh_trans ? 1 : 0) == N,
                "colown: one-hot block");
    g.oh_w = oh_w->data_ptr<float>();
    g.oh_sn = oh_trans ? oh_w->stride(1) : oh_w->stride(0);
    g.oh_sc = oh_trans ? oh_w->stride(0) : oh_w->stride(1);
    g.oh_col = oh_col->data_ptr<int>();
    g.oh_opt = oh_opt->data_ptr<int>();
    g.oh_off = oh_off->data_ptr<int>();
  }
  g.gamma = cfp(gamma);
  g.beta = cfp(beta);
  g.out = fp(out);
  g.ldo = (int)ld_of(out);
  g.nhat = fp(nhat);
  g.ldn = (int)ld_of(nhat);
  g.mean = fp(mean);
  g.invstd = fp(invstd);
  g.rm = fp(rm);
  g.rv = fp(rv);
  g.stat = fp(stat);
  g.cnt = reinterpret_cast<unsigned*>(cnt.data_ptr<int>());
  g.rpg = (int)rpg;
  g.groups = (int)groups;
  g.K = (int)K;
  g.N = (int)N;
  g.momentum = (float)momentum;
  g.eps = (float)eps;
  const bool vec = (reinterpret_cast<uintptr_t>(x.data_ptr()) & 15) == 0 && g.ldx % 4 == 0;
  fedtgan::launch_linear_bn_relu_colown(g, vec, cur_stream());
}

void bn_relu_bwd(const Tensor& dr, const Tensor& r, const Tensor& nhat, const Tensor& gamma, const Tensor& invstd,
                 const Tensor& da, const Tensor& dgamma, const Tensor& dbeta, const optional<Tensor>& dbias,
                 bool paired) {
  check_f32_2d(dr, "dr");
  check_f32_2d(r, "r");
  check_f32_2d(nhat, "nhat");
  check_f32_2d(da, "da");
  TORCH_CHECK(dr.size(0) >= 1, "bn_relu_bwd: empty batch");
  TORCH_CHECK(r.sizes() == dr.sizes() && nhat.sizes() == dr.sizes() && da.sizes() == dr.sizes(), "bn bwd: shapes");
  TORCH_CHECK(gamma.numel() >= dr.size(1) && invstd.numel() >= dr.size(1) && dgamma.numel() >= dr.size(1) &&
                  dbeta.numel() >= dr.size(1) && (!(dbias.has_value() && dbias->defined()) || dbias->numel() >= dr.size(1)),
              "bn bwd: per-column vectors");
  if (paired) {
    // the GEMM held with group=1 (an independent weight gradient) runs in the same launch (gemm_bnbwd_kernel)
    const hipStream_t hs = cur_stream();
    TORCH_CHECK(has_held && held_stream == hs, "bn_relu_bwd(paired=True) needs a GEMM held with group=1 on this stream");
    has_held = false;
    const fedtgan::BnBwdArgs b{cfp(dr), ld_of(dr), cfp(r), ld_of(r), cfp(nhat), ld_of(nhat), cfp(gamma), cfp(invstd),
                               fp(da), ld_of(da), fp(dgamma), fp(dbeta), optp<float>(dbias), (int)dr.size(0),
                               (int)dr.size(1)};
    if (fedtgan::launch_gemm_bnbwd(held, b, hs)) return;
    fedtgan::launch_gemm(held, hs);     // (a shape the fused launch does not take: two launches)
  }
  fedtgan::launch_bn_relu_bwd(cfp(dr), ld_of(dr), cfp(r), ld_of(r), cfp(nhat), ld_of(nhat), cfp(gamma), cfp(invstd),
                              fp(da), ld_of(da), fp(dgamma), fp(dbeta), optp<float>(dbias), (int)dr.size(0),
                              (int)dr.size(1), cur_stream());
}

void adam(const Tensor& p, const Tensor& g, const Tensor& m, const Tensor& v, const Tensor& step, double lr, double b1,
          double b2, double eps, double wd, const optional<Tensor>& rng_bump) {
  TORCH_CHECK(!g_adam_held.active && !g_adam_pre.active,
              "adam: a GEMM held for the Adam launch needs adam_cs (the column-sum form)");
  TORCH_CHECK(p.is_contiguous() && g.is_contiguous() && m.is_contiguous() && v.is_contiguous(), "adam: contiguous");
  TORCH_CHECK(p.numel() == g.numel() && p.numel() == m.numel() && p.numel() == v.numel(), "adam: sizes");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(p.data_ptr()) & 15) == 0 && (reinterpret_cast<uintptr_t>(g.data_ptr()) & 15) == 0,
              "adam: buffers must be 16-byte aligned");
  uint64_t* bump = nullptr;
  if (rng_bump.has_value() && rng_bump->defined()) bump = reinterpret_cast<uint64_t*>(rng_bump->data_ptr<int64_t>());
  fedtgan::launch_adam(fp(p), cfp(g), fp(m), fp(v), cfp(step), p.numel(), (float)lr, (float)b1, (float)b2, (float)eps,
                       (float)wd, bump, cur_stream());
}

// adam + colsum_ex jobs in one launch.  A job whose output lies in g owns ceil4(cols) elements
// there (16-B aligned start; the flat layout pads every tensor to 4 floats) and gets its Adam
// update from the reduced sums; outputs elsewhere (metrics) are just written.
void adam_cs(const Tensor& p, const Tensor& g, const Tensor& m, const Tensor& v, const Tensor& step, double lr,
             double b1, double b2, double eps, double wd, const optional<Tensor>& rng_bump, at::TensorList srcs,
             const c10::List<optional<Tensor>>& outs, const c10::List<optional<Tensor>>& w,
             const c10::List<optional<Tensor>>& dot_v, const c10::List<optional<Tensor>>& dot_e,
             const c10::List<optional<Tensor>>& dot_out, const c10::List<optional<Tensor>>& dot_w) {
  TORCH_CHECK(p.is_contiguous() && g.is_contiguous() && m.is_contiguous() && v.is_contiguous(), "adam_cs: contiguous");
  TORCH_CHECK(p.numel() == g.numel() && p.numel() == m.numel() && p.numel() == v.numel(), "adam_cs: sizes");
  TORCH_CHECK(p.numel() % 4 == 0, "adam_cs: buffer length must be a multiple of 4");
  for (const Tensor* t : {&p, &g, &m, &v})
    TORCH_CHECK((reinterpret_cast<uintptr_t>(t->data_ptr()) & 15) == 0, "adam_cs: buffers must be 16-byte aligned");
  const auto jobs = colsum_jobs(srcs, outs, w, dot_v, dot_e, dot_out, dot_w);
  fedtgan::AdamColsum cs{};
  cs.n_jobs = (int)jobs.size();
  const float* g0 = cfp(g);
  const int64_t n = g.numel();
  for (int k = 0; k < cs.n_jobs; ++k) {
    cs.jobs[k] = jobs[k];
    cs.own_lo[k] = cs.own_hi[k] = 0;
    const int c4 = (jobs[k].cols + 3) / 4 * 4;
    cs.vec[k] = (reinterpret_cast<uintptr_t>(jobs[k].a) & 15) == 0 && jobs[k].lda % 4 == 0 &&
                (jobs[k].rows <= 1 || jobs[k].lda >= c4) &&
                srcs[k].storage().nbytes() >= (size_t)((char*)jobs[k].a - (char*)srcs[k].storage().data()) +
                    ((size_t)(jobs[k].rows - 1) * jobs[k].lda + c4) * sizeof(float);
    const float* o = jobs[k].out;
    if (o && o >= g0 && o < g0 + n) {
      const int64_t off = o - g0, len = ((int64_t)jobs[k].cols + 3) / 4 * 4;
      TORCH_CHECK(off % 4 == 0 && off + len <= n, "adam_cs: a job output inside the gradient buffer must start "
                  "4-aligned and own ceil4(cols) elements");
      for (int q = 0; q < k; ++q)
        TORCH_CHECK(off >= cs.own_hi[q] || off + len <= cs.own_lo[q], "adam_cs: overlapping job outputs");
      cs.own_lo[k] = off;
      cs.own_hi[k] = off + len;
    }
    // a dot over parameters this launch updates must be this job's own (read pre-update by
    // the updating lane); any other overlap with p would race with the update
    const float* p0 = cfp(p);
    const float* dv = jobs[k].dot_v;
    cs.dot_self[k] = dv && cs.own_hi[k] > cs.own_lo[k] && dv == p0 + cs.own_lo[k];
    TORCH_CHECK(!dv || cs.dot_self[k] || dv + jobs[k].cols <= p0 || dv >= p0 + n,
                "adam_cs: a dot over parameters updated by this launch must belong to the same job");
  }
  uint64_t* bump = nullptr;
  if (rng_bump.has_value() && rng_bump->defined()) bump = reinterpret_cast<uint64_t*>(rng_bump->data_ptr<int64_t>());
  const hipStream_t hs = cur_stream();
  if (g_adam_pre.active) {
    // the held short-K weight gradient applies Adam to its own block now (it reads only A, B and the step
    // counter, and writes only its block of p / m / v: independent of this launch's other elements)
    AdamHeld h = g_adam_pre;
    g_adam_pre.active = false;
    TORCH_CHECK(h.stream == hs, "adam_cs: the short-K GEMM held for it was issued on another stream");
    const int64_t off = h.c - g0;
    TORCH_CHECK(h.c >= g0 && off % 4 == 0 && h.ldc % 4 == 0 && off + h.M * h.ldc <= n,
                "adam_cs: the held short-K GEMM's output must be a 4-aligned block inside the gradient buffer");
    for (int k = 0; k < cs.n_jobs; ++k)
      TORCH_CHECK(off >= cs.own_hi[k] || off + h.M * h.ldc <= cs.own_lo[k], "adam_cs: the short-K GEMM overlaps a job");
    fedtgan::GemmArgs q = h.g;
    q.adam_p = fp(p) + off;
    q.adam_m = fp(m) + off;
    q.adam_v = fp(v) + off;
    q.adam_step = cfp(step);
    q.adam_lr = (float)lr;
    q.adam_b1 = (float)b1;
    q.adam_b2 = (float)b2;
    q.adam_eps = (float)eps;
    q.adam_wd = (float)wd;
    if (fedtgan::launch_gemm_shortk_adam(q, hs)) {
      cs.skip2_lo = off;
      cs.skip2_hi = off + h.M * h.ldc;
    } else {
      fedtgan::launch_gemm(h.g, hs);     // (a shape the short-K kernel does not take: the plain GEMM, Adam below)
    }
  }
  if (g_adam_held.active) {
    // the held weight-gradient GEMM (gemm(..., group=3)) writes rows [0, M) x [0, N) at stride ldc of a
    // block inside g: Adam over that whole block is left to the GEMM's tiles (elements of the block
    // outside M x N -- padding -- keep their values, as their gradient is zero)
    AdamHeld h = g_adam_held;
    g_adam_held.active = false;
    TORCH_CHECK(h.stream == hs, "adam_cs: the GEMM held for it was issued on another stream");
    const int64_t off = h.c - g0, len = (h.M - 1) * h.ldc + h.N;
    TORCH_CHECK(h.c >= g0 && off % 4 == 0 && h.ldc % 4 == 0 && off + (h.M * h.ldc) <= n && len > 0,
                "adam_cs: the held GEMM's output must be a 4-aligned block inside the gradient buffer");
    for (int k = 0; k < cs.n_jobs; ++k)
      TORCH_CHECK(off >= cs.own_hi[k] || off + h.M * h.ldc <= cs.own_lo[k], "adam_cs: the held GEMM overlaps a job output");
    TORCH_CHECK(cs.skip2_hi <= off || off + h.M * h.ldc <= cs.skip2_lo, "adam_cs: the two held GEMMs overlap");
    cs.skip_lo = off;
    cs.skip_hi = off + h.M * h.ldc;
    if (cs.skip2_hi > cs.skip2_lo && cs.skip2_lo < cs.skip_lo) {   // (adam_cs_body: the lower range first)
      std::swap(cs.skip_lo, cs.skip2_lo);
      std::swap(cs.skip_hi, cs.skip2_hi);
    }
    if (fedtgan::launch_gemm_adam(h.g, fp(p), cfp(g), fp(m), fp(v), cfp(step), n, (float)lr, (float)b1, (float)b2,
                                  (float)eps, (float)wd, bump, cs, hs))
      return;
    // shape not instantiated: the GEMM, then the plain launch (keeping the short-K range cut out, if any)
    if (cs.skip_lo == off) cs.skip_lo = cs.skip_hi = 0;
    else cs.skip2_lo = cs.skip2_hi = 0;
    if (cs.skip_hi <= cs.skip_lo && cs.skip2_hi > cs.skip2_lo) {
      std::swap(cs.skip_lo, cs.skip2_lo);
      std::swap(cs.skip_hi, cs.skip2_hi);
    }
    fedtgan::launch_gemm(h.g, hs);
  }
  fedtgan::launch_adam_colsum(fp(p), cfp(g), fp(m), fp(v), cfp(step), p.numel(), (float)lr, (float)b1, (float)b2,
                              (float)eps, (float)wd, bump, cs, hs);
}

void sample_decode(const Tensor& logits, const Tensor& out, const Tensor& kind, const Tensor& start,
                   const Tensor& width, const Tensor& cont, const Tensor& code_off, const Tensor& codes,
                   const Tensor& mu, const Tensor& sd, int64_t seed, const Tensor& rng_ctr, int64_t stream,
                   const optional<Tensor>& ecol, const optional<Tensor>& quads) {
  check_f32_2d(logits, "logits");
  TORCH_CHECK(out.scalar_type() == at::kDouble && out.is_contiguous() && out.dim() == 2, "decode: out f64");
  TORCH_CHECK(out.size(0) == logits.size(0) && out.size(1) == kind.numel(), "decode: shapes");
  TORCH_CHECK(mu.scalar_type() == at::kDouble && sd.scalar_type() == at::kDouble && codes.scalar_type() == at::kDouble,
              "decode: f64 tables");
  fedtgan::DecodeArgs a{};
  a.logits = cfp(logits);
  a.ldl = ld_of(logits);
  a.rows = (int)logits.size(0);
  a.n_cols = (int)kind.numel();
  a.kind = kind.data_ptr<int>();
  a.start = start.data_ptr<int>();
  a.width = width.data_ptr<int>();
  a.cont = cont.data_ptr<int>();
  a.code_off = code_off.data_ptr<int>();
  a.codes = codes.data_ptr<double>();
  a.n_codes = (int)codes.numel();
  a.mu = mu.data_ptr<double>();
  a.sd = sd.data_ptr<double>();
  a.K = mu.dim() == 2 ? (int)mu.size(1) : 1;
  a.out = out.data_ptr<double>();
  a.seed = (uint64_t)seed;
  a.rng_ctr = ctr_ptr(rng_ctr);
  a.rng_stream = (uint32_t)stream;
  a.dim = (int)logits.size(1);
  if (ecol.has_value() && ecol->defined()) {
    TORCH_CHECK(ecol->scalar_type() == at::kInt && ecol->is_contiguous() && ecol->numel() == logits.size(1),
                "decode: ecol must be int32 [data_dim]");
    // the row kernel keeps one 8-byte maximum per output column and wave in LDS
    if (a.n_cols * 4 * 8 <= 64 * 1024) a.ecol = ecol->data_ptr<int>();
  }
  if (quads.has_value() && quads->defined()) {
    TORCH_CHECK(quads->scalar_type() == at::kInt && quads->is_contiguous() && quads->dim() == 2 && quads->size(1) == 2,
                "decode: quads must be int32 [n, 2]");
    TORCH_CHECK(logits.size(1) < 65536, "decode: quads address positions below 65536");
    // every entry: a column, 1-4 logits inside the row and inside that column's span (host-built)
    a.quads = quads->data_ptr<int>();
    a.n_quads = (int)quads->size(0);
  }
  fedtgan::launch_sample_decode(a, cur_stream());
}

void gen_weight_prep(const std::vector<Tensor>& w, std::vector<int64_t> kd, const std::vector<Tensor>& w16,
                     const std::vector<Tensor>& wt) {
  const size_t n = w.size();
  TORCH_CHECK(n >= 1 && n <= 4 && kd.size() == n && w16.size() == n && wt.size() == n, "gen_weight_prep: 1-4 jobs");
  fedtgan::GenWeightPrep a{};
  a.n_jobs = (int)n;
  for (size_t j = 0; j < n; ++j) {
    // the weight as stored: [N, K] rows (unit k stride) or input-major (EngineConfig.g_wt: unit n stride)
    TORCH_CHECK(w[j].is_cuda() && w[j].scalar_type() == at::kFloat && w[j].dim() == 2 &&
                    (w[j].stride(1) == 1 || w[j].stride(0) == 1), "gen_weight_prep w: 2-D fp32, one unit stride");
    const int64_t N = w[j].size(0), K = w[j].size(1);
    TORCH_CHECK(kd[j] >= 0 && kd[j] <= K, "gen_weight_prep: kd");
    TORCH_CHECK(w16[j].is_cuda() && w16[j].scalar_type() == at::kBFloat16 && w16[j].dim() == 2 && w16[j].size(0) == N &&
                    w16[j].size(1) >= kd[j] && w16[j].stride(1) == 1, "gen_weight_prep: w16 [N, >= kd] bf16");
    check_f32_2d(wt[j], "gen_weight_prep wt");
    TORCH_CHECK(wt[j].is_contiguous() && wt[j].size(0) == K - kd[j] && wt[j].size(1) == N, "gen_weight_prep: wt [C, N]");
    const bool kmaj = w[j].stride(1) == 1;
    a.jobs[j] = fedtgan::GenWeightJob{cfp(w[j]), (int)N, kmaj ? ld_of(w[j]) : 1, kmaj ? 1 : (int)w[j].stride(1),
                                      (int)kd[j], (int)(K - kd[j]), hp(w16[j]),
                                      (int)w16[j].stride(0), fp(wt[j])};
  }
  fedtgan::launch_gen_weight_prep(a, cur_stream());
}

void rng_bump(const Tensor& ctr) {
  TORCH_CHECK(ctr.scalar_type() == at::kLong && ctr.is_cuda(), "rng_bump: cuda int64");
  fedtgan::launch_rng_bump(reinterpret_cast<uint64_t*>(ctr.data_ptr<int64_t>()), cur_stream());
}

// ----------------------------------------------------------------------------- native RCCL plane (csrc/comm)
void rccl_load_op(const std::string& path) { fedtgan::comm::rccl_load(path); }

Tensor rccl_unique_id_op() {
  const std::vector<uint8_t> v = fedtgan::comm::rccl_unique_id();
  Tensor t = at::empty({(int64_t)v.size()}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(t.data_ptr(), v.data(), v.size());
  return t;
}

int64_t rccl_init_op(const Tensor& id, int64_t rank, int64_t nranks) {
  TORCH_CHECK(id.device().is_cpu() && id.scalar_type() == at::kByte && id.numel() == 128 && id.is_contiguous(),
              "rccl_init: id must be the 128-byte CPU uint8 tensor of rccl_unique_id()");
  return fedtgan::comm::rccl_init(id.data_ptr<uint8_t>(), (int)rank, (int)nranks);
}

// in place on the current HIP stream (capturable); premul: this rank's weight, folded into the collective
void rccl_all_reduce_op(int64_t comm, const Tensor& x, double premul) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat && x.is_contiguous(),
              "rccl_all_reduce: x must be a contiguous fp32 device tensor");
  fedtgan::comm::rccl_all_reduce_f32(comm, x.data_ptr<float>(), (size_t)x.numel(), (float)premul, cur_stream());
}

void rccl_destroy_op(int64_t comm) { fedtgan::comm::rccl_destroy(comm); }

void write_csv(const std::string& path, const Tensor& values, std::vector<std::string> names, std::vector<int64_t> kinds,
               std::vector<std::string> vocab_flat, std::vector<int64_t> vocab_offsets, int64_t threads,
               std::vector<int64_t> src, std::vector<int64_t> date_desc, std::vector<int64_t> date_lut,
               const optional<Tensor>& aux) {
  // output column j: kinds[j], names[j], vocabulary vocab_flat[vocab_offsets[j], vocab_offsets[j + 1]), source
  // column src[j] of values (default j).  Date columns (kind 3) take their description from date_desc, in
  // output order: [mode, n_parts, (src, elem, lut_off, lut_len) x n_parts], code -> value tables in date_lut.
  TORCH_CHECK(!values.is_cuda() && values.scalar_type() == at::kDouble && values.is_contiguous() && values.dim() == 2,
              "write_csv: values must be a contiguous CPU float64 matrix");
  const int64_t cols = values.size(1);
  const int64_t n_out = (int64_t)kinds.size();
  const bool has_aux = aux.has_value() && aux->defined();
  if (has_aux)
    TORCH_CHECK(!aux->is_cuda() && aux->scalar_type() == at::kDouble && aux->is_contiguous() && aux->dim() == 2 &&
                    aux->size(0) == values.size(0), "write_csv: aux must be a contiguous CPU float64 [rows, n] matrix");
  const int64_t aux_cols = has_aux ? aux->size(1) : 0;
  TORCH_CHECK((int64_t)names.size() == n_out && (int64_t)vocab_offsets.size() == n_out + 1 &&
                  (src.empty() ? n_out == cols : (int64_t)src.size() == n_out),
              "write_csv: descriptors");
  std::vector<fedtgan::CsvColumn> out((size_t)n_out);
  size_t dp = 0;
  for (int64_t j = 0; j < n_out; ++j) {
    auto& c = out[(size_t)j];
    c.kind = (int)kinds[(size_t)j];
    TORCH_CHECK(c.kind >= fedtgan::CSV_FLOAT && c.kind <= fedtgan::CSV_DATE, "write_csv: kind");
    c.src = (int)(src.empty() ? j : src[(size_t)j]);
    TORCH_CHECK(vocab_offsets[(size_t)j] <= vocab_offsets[(size_t)j + 1] &&
                    vocab_offsets[(size_t)j + 1] <= (int64_t)vocab_flat.size(), "write_csv: vocab offsets");
    c.vocab.assign(vocab_flat.begin() + vocab_offsets[(size_t)j], vocab_flat.begin() + vocab_offsets[(size_t)j + 1]);
    if (c.kind != fedtgan::CSV_DATE) {
      TORCH_CHECK(c.src >= 0 && c.src < cols + aux_cols, "write_csv: source column out of range");
      continue;
    }
    TORCH_CHECK(dp + 2 <= date_desc.size(), "write_csv: date_desc too short");
    c.date_mode = (int)date_desc[dp++];
    const int64_t np = date_desc[dp++];
    TORCH_CHECK(np >= 1 && np <= 6 && dp + 4 * (size_t)np <= date_desc.size(), "write_csv: date parts");
    for (int64_t q = 0; q < np; ++q) {
      fedtgan::CsvDatePart part;
      part.src = (int)date_desc[dp++];
      part.elem = (int)date_desc[dp++];
      const int64_t off = date_desc[dp++], len = date_desc[dp++];
      TORCH_CHECK(part.src >= 0 && part.src < cols && part.elem >= 0 && part.elem <= 5 && off >= 0 && len >= 0 &&
                      off + len <= (int64_t)date_lut.size(), "write_csv: date part descriptor");
      part.lut.assign(date_lut.begin() + off, date_lut.begin() + off + len);
      c.parts.push_back(std::move(part));
    }
  }
  TORCH_CHECK(dp == date_desc.size(), "write_csv: unused date_desc entries");
  fedtgan::write_csv_columns(path, values.data_ptr<double>(), values.size(0), cols, names, out, (int)threads,
                             has_aux ? aux->data_ptr<double>() : nullptr, aux_cols);
}

void vgm_encode(const Tensor& x, const Tensor& out, const Tensor& opt, const Tensor& col_kind, const Tensor& col_pos,
                const Tensor& col_aux, const Tensor& col_span, const Tensor& col_lut_n, const Tensor& consts, const Tensor& means,
                const Tensor& prec, const Tensor& stds, const Tensor& vrank, const Tensor& lut, int64_t seed,
                int64_t stream) {
  // row-major, or column-major (a table uploaded as its [cols, rows] transpose: no device transposing copy)
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kDouble && x.dim() == 2 &&
                  (x.stride(1) == 1 || x.stride(0) == 1 || x.size(0) <= 1 || x.size(1) <= 1), "vgm_encode: x");
  check_f32_2d(out, "out");
  TORCH_CHECK(opt.is_cuda() && opt.scalar_type() == at::kInt && opt.is_contiguous() && opt.size(0) == x.size(0),
              "vgm_encode: opt");
  const int64_t n_cols = x.size(1);
  for (const Tensor* t : {&col_kind, &col_pos, &col_aux, &col_span, &col_lut_n})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kInt && t->numel() == n_cols && t->is_contiguous(),
                "vgm_encode: column tables");
  for (const Tensor* t : {&consts, &means, &prec, &stds})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous() && t->numel() == vrank.numel(),
                "vgm_encode: bank tables");
  TORCH_CHECK(vrank.scalar_type() == at::kInt && lut.scalar_type() == at::kInt && lut.is_contiguous(), "vgm_encode");
  fedtgan::VgmEncodeArgs a{};
  a.x = x.data_ptr<double>();
  a.ldx = (int)x.stride(0);
  a.ldc = x.stride(1);
  a.n_rows = (int)x.size(0);
  a.n_cols = (int)n_cols;
  a.out = fp(out);
  a.ldo = ld_of(out);
  a.opt = opt.data_ptr<int>();
  a.n_span = (int)opt.size(1);
  a.col_kind = col_kind.data_ptr<int>();
  a.col_pos = col_pos.data_ptr<int>();
  a.col_aux = col_aux.data_ptr<int>();
  a.col_span = col_span.data_ptr<int>();
  a.col_lut_n = col_lut_n.data_ptr<int>();
  a.consts = consts.data_ptr<float>();
  a.means = means.data_ptr<float>();
  a.prec = prec.data_ptr<float>();
  a.stds = stds.data_ptr<float>();
  a.vrank = vrank.data_ptr<int>();
  a.lut = lut.data_ptr<int>();
  a.seed = (uint64_t)seed;
  a.stream = (uint32_t)stream;
  fedtgan::launch_vgm_encode(a, cur_stream());
}

fedtgan::VgmFitArgs fit_args(const Tensor& x, const Tensor& n_rows, const Tensor& means, const Tensor& partial,
                             int64_t rows_per_block, int64_t nv) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kDouble && x.dim() == 2 && x.stride(1) == 1, "vgm fit: x");
  TORCH_CHECK(n_rows.is_cuda() && n_rows.scalar_type() == at::kInt && n_rows.numel() == x.size(0), "vgm fit: n_rows");
  TORCH_CHECK(means.scalar_type() == at::kDouble && means.is_contiguous() && means.numel() == x.size(0) * 10,
              "vgm fit: [n_cols, 10] tables");
  TORCH_CHECK(rows_per_block > 0, "vgm fit: rows_per_block");
  const int64_t chunks = (x.size(1) + rows_per_block - 1) / rows_per_block;
  TORCH_CHECK(partial.scalar_type() == at::kDouble && partial.is_contiguous() &&
                  partial.numel() == x.size(0) * chunks * nv, "vgm fit: partial must be [n_cols, chunks, ", nv, "]");
  fedtgan::VgmFitArgs a{};
  a.x = x.data_ptr<double>();
  a.ldx = (int)x.stride(0);
  a.n_cols = (int)x.size(0);
  a.max_rows = (int)x.size(1);
  a.rows_per_block = (int)rows_per_block;
  a.n_rows = n_rows.data_ptr<int>();
  a.means = means.data_ptr<double>();
  a.partial = partial.data_ptr<double>();
  return a;
}

void vgm_estep(const Tensor& x, const Tensor& n_rows, const Tensor& consts, const Tensor& means, const Tensor& prec,
               const Tensor& partial, int64_t rows_per_block) {
  auto a = fit_args(x, n_rows, means, partial, rows_per_block, 31);
  TORCH_CHECK(consts.scalar_type() == at::kDouble && consts.is_contiguous() && consts.numel() == means.numel() &&
                  prec.scalar_type() == at::kDouble && prec.is_contiguous() && prec.numel() == means.numel(),
              "vgm_estep: tables");
  a.consts = consts.data_ptr<double>();
  a.prec = prec.data_ptr<double>();
  fedtgan::launch_vgm_estep(a, cur_stream());
}

void kmeans_step(const Tensor& x, const Tensor& n_rows, const Tensor& centers, const Tensor& partial,
                 int64_t rows_per_block) {
  auto a = fit_args(x, n_rows, centers, partial, rows_per_block, 30);
  fedtgan::launch_kmeans_step(a, cur_stream());
}

void vgm_fit(const Tensor& x, const Tensor& n_rows, const c10::optional<Tensor>& init_centers, int64_t seed,
             double wprior, double tol, double reg_covar, int64_t max_iter, int64_t km_iter, const Tensor& out,
             const Tensor& info, const Tensor& lower_bound) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kDouble && x.dim() == 2 && x.stride(1) == 1, "vgm_fit: x");
  const int64_t nc = x.size(0);
  TORCH_CHECK(n_rows.is_cuda() && n_rows.scalar_type() == at::kInt && n_rows.is_contiguous() && n_rows.numel() == nc,
              "vgm_fit: n_rows");
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kDouble && out.is_contiguous() && out.numel() == nc * 60,
              "vgm_fit: out must be [n_cols, 6, 10] fp64");
  TORCH_CHECK(info.is_cuda() && info.scalar_type() == at::kInt && info.is_contiguous() && info.numel() == nc * 2,
              "vgm_fit: info");
  TORCH_CHECK(lower_bound.is_cuda() && lower_bound.scalar_type() == at::kDouble && lower_bound.numel() == nc,
              "vgm_fit: lower_bound");
  fedtgan::VgmFitAllArgs a{};
  a.x = x.data_ptr<double>();
  a.ldx = (int)x.stride(0);
  a.n_cols = (int)nc;
  a.n_rows = n_rows.data_ptr<int>();
  if (init_centers.has_value()) {
    TORCH_CHECK(init_centers->is_cuda() && init_centers->scalar_type() == at::kDouble &&
                    init_centers->is_contiguous() && init_centers->numel() == nc * 10,
                "vgm_fit: init_centers must be [n_cols, 10] fp64");
    a.init_centers = init_centers->data_ptr<double>();
  }
  a.seed = (uint64_t)seed;
  a.wprior = wprior;
  a.tol = tol;
  a.reg_covar = reg_covar;
  a.max_iter = (int)max_iter;
  a.km_iter = (int)km_iter;
  a.out = out.data_ptr<double>();
  a.info = info.data_ptr<int>();
  a.lower_bound = lower_bound.data_ptr<double>();
  // split fit: a cluster of workgroups per column (the record buffer and the zeroed arrival counters live
  // until the launch has run: stream-ordered caching-allocator blocks)
  a.split = fedtgan::vgm_fit_split((int)nc, (int)x.size(1));
  Tensor xpart, sync;
  if (a.split > 1) {
    xpart = at::empty({nc * 2 * a.split * 32}, x.options());
    sync = at::zeros({nc * 32}, x.options().dtype(at::kInt));
    a.xpart = xpart.data_ptr<double>();
    a.sync = reinterpret_cast<unsigned*>(sync.data_ptr<int>());
  }
  fedtgan::launch_vgm_fit(a, cur_stream());
}

// checked build: the check bits raised by every kernel since the last call (cleared); synchronises
int64_t check_status() {
  (void)hipDeviceSynchronize();
  return (int64_t)(fedtgan::check_status_gemm() | fedtgan::check_status_ctgan_ops() | fedtgan::check_status_vgm());
}

#ifdef FEDTGAN_CHECKED
bool is_checked() { return true; }
#else
bool is_checked() { return false; }
#endif

std::string py_float(double x) { return fedtgan::format_py_float(x); }

// kernel variant knobs for measured sweeps (tools/microbench.py); returns the previous value
int64_t set_tuning(const std::string& key, int64_t value) {
  if (key == "colown_dbg") {   // phase-cost probe of linear_bn_relu_colown (results are wrong while set)
    TORCH_CHECK(value >= 0 && value <= 7, "colown_dbg: bit mask 0..7");
    const int64_t prev = fedtgan::g_colown_dbg;
    fedtgan::g_colown_dbg = (int)value;
    return prev;
  }
  if (key == "bn_cols") {
    TORCH_CHECK(value == 4 || value == 8 || value == 16, "bn_cols must be 4, 8 or 16");
    const int64_t prev = fedtgan::g_bn_cols;
    fedtgan::g_bn_cols = (int)value;
    return prev;
  }
  if (key == "decode_rows") {
    TORCH_CHECK(value >= 0 && value <= 2, "decode_rows: 0 per cell, 1 per row, 2 per row over Philox quads");
    const int prev = fedtgan::g_decode_rows;
    fedtgan::g_decode_rows = (int)value;
    return prev;
  }
  if (key == "chain_pre") {   // chained tail weights prefetched: 0 never, 1 grids of <= 512 workgroups, 2 always
    TORCH_CHECK(value >= 0 && value <= 2, "chain_pre: 0, 1 or 2");
    const int prev = fedtgan::g_chain_pre;
    fedtgan::g_chain_pre = (int)value;
    return prev;
  }
  if (key == "chain_rows") {  // head rows per chain workgroup when the one-row grid is too large to prefetch
    TORCH_CHECK(value == 1 || value == 2, "chain_rows: 1 or 2");
    const int prev = fedtgan::g_chain_rows;
    fedtgan::g_chain_rows = (int)value;
    return prev;
  }
  if (key == "chain_coalesced") {   // chained tail GEMM: lane-contiguous weight rows + wave sums (1)
    const int prev = fedtgan::g_chain_coalesced;
    fedtgan::g_chain_coalesced = value ? 1 : 0;
    return prev;
  }
  if (key == "gp_threads") {
    TORCH_CHECK(value == 256 || value == 1024, "gp_threads: 256 or 1024");
    const int prev = fedtgan::g_gp_threads;
    fedtgan::g_gp_threads = (int)value;
    return prev;
  }
  if (key == "bn_threads") {
    TORCH_CHECK(value == 512 || value == 1024, "bn_threads: 512 or 1024");
    const int prev = fedtgan::g_bn_threads;
    fedtgan::g_bn_threads = (int)value;
    return prev;
  }
  if (key == "act_rowreg_narrow") {   // rows <= 512 wide: per-wave kernels (0), row kernels 2-4 waves (1), a block per wave (2)
    TORCH_CHECK(value >= 0 && value <= 2, "act_rowreg_narrow: 0, 1 or 2");
    const int prev = fedtgan::g_act_rowreg_narrow;
    fedtgan::g_act_rowreg_narrow = (int)value;
    return prev;
  }
  if (key == "gp_split") {   // gradient-penalty scale of rows wider than 8,192: chunk-split (1) or one workgroup per row (0)
    const int prev = fedtgan::g_gp_split;
    fedtgan::g_gp_split = value ? 1 : 0;
    return prev;
  }
  if (key == "act_row_mode") {
    TORCH_CHECK(value >= 0 && value <= 2, "act_row_mode: 0 per-wave, 1 row (LDS image), 2 row (registers; forward)");
    const int prev = fedtgan::g_act_row_mode;
    fedtgan::g_act_row_mode = (int)value;
    return prev;
  }
  if (key == "xcd_clients") {   // batched launches: each client on its own XCD(s) (1) or round-robin (0)
    TORCH_CHECK(value == 0 || value == 1, "xcd_clients: 0 or 1");
    const int64_t prev = fedtgan::g_xcd_clients;
    fedtgan::g_xcd_clients = (int)value;
    return prev;
  }
  if (key == "adam_store") {
    TORCH_CHECK(value == 0 || value == 2 || value == 16, "adam_store: 0 plain, 2 nt, 16 sc1");
    const int64_t prev = fedtgan::g_adam_store;
    fedtgan::g_adam_store = (int)value;
    return prev;
  }
  if (key == "adam_u_min") {   // float4 count (x clients) from which the Adam loop loads ADAM_U float4 per thread
    TORCH_CHECK(value >= 0, "adam_u_min: >= 0");
    const int64_t prev = fedtgan::g_adam_u_min;
    fedtgan::g_adam_u_min = value;
    return prev;
  }
  if (key == "bnb_first") {   // gemm_bnbwd_kernel: BN workgroups first (1) or last (0)
    const int64_t prev = fedtgan::g_bnb_first;
    fedtgan::g_bnb_first = value ? 1 : 0;
    return prev;
  }
  if (key == "bnb_cols") {    // gemm_bnbwd_kernel: columns per BN workgroup, 4 or 8
    TORCH_CHECK(value == 4 || value == 8, "bnb_cols: 4 or 8");
    const int64_t prev = fedtgan::g_bnb_cols;
    fedtgan::g_bnb_cols = (int)value;
    return prev;
  }
  if (key == "vgm_split") {   // workgroups per column of the whole-fit VGM kernel: 0 auto, 1 one, n n
    TORCH_CHECK(value >= 0 && value <= 64, "vgm_split: 0..64");
    const int64_t prev = fedtgan::g_vgm_split;
    fedtgan::g_vgm_split = (int)value;
    return prev;
  }
  if (key == "vgm_split_of") {   // read-only probe: the split a fit of `value` columns x 40000 rows would use
    return fedtgan::vgm_fit_split((int)value, 40000);
  }
  if (key == "adam_max_blocks") {
    TORCH_CHECK(value >= 1 && value <= 65535, "adam_max_blocks: 1..65535");
    const int64_t prev = fedtgan::g_adam_max_blocks;
    fedtgan::g_adam_max_blocks = (int)value;
    return prev;
  }
  if (key == "gemm_store_wt") {
    const int64_t prev = fedtgan::g_gemm_store_wt;
    fedtgan::g_gemm_store_wt = value ? 1 : 0;
    return prev;
  }
  if (key == "gemm_shortk") {
    const int64_t prev = fedtgan::g_gemm_shortk;
    fedtgan::g_gemm_shortk = value ? 1 : 0;
    return prev;
  }
  if (key == "gemm_shortk_store") {
    TORCH_CHECK(value >= 0 && value <= 2, "gemm_shortk_store: 0 plain, 1 non-temporal, 2 write-through");
    const int64_t prev = fedtgan::g_gemm_shortk_store;
    fedtgan::g_gemm_shortk_store = (int)value;
    return prev;
  }
  if (key == "gemm_shortk_min_n") {
    TORCH_CHECK(value >= 4, "gemm_shortk_min_n: >= 4");
    const int64_t prev = fedtgan::g_gemm_shortk_min_n;
    fedtgan::g_gemm_shortk_min_n = (int)value;
    return prev;
  }
  if (key == "gemm_splitk_inlaunch") {
    const int64_t prev = fedtgan::g_gemm_splitk_inlaunch;
    fedtgan::g_gemm_splitk_inlaunch = value ? 1 : 0;
    return prev;
  }
  if (key == "gemm_pairs") {
    const int64_t prev = fedtgan::g_gemm_pairs;
    fedtgan::g_gemm_pairs = value ? 1 : 0;
    return prev;
  }
  if (key == "gemm_pair_max_wg") {   // pairs with more workgroups than this launch as two GEMMs (0: no limit)
    TORCH_CHECK(value >= 0, "gemm_pair_max_wg: >= 0");
    const int64_t prev = fedtgan::g_gemm_pair_max_wg;
    fedtgan::g_gemm_pair_max_wg = (int)value;
    return prev;
  }
  if (key == "gemm_xcd_nmajor") {
    const int64_t prev = fedtgan::g_gemm_xcd_nmajor;
    fedtgan::g_gemm_xcd_nmajor = value ? 1 : 0;
    return prev;
  }
  if (key == "gemm_xcd_remap") {
    const int64_t prev = fedtgan::g_gemm_xcd_remap;
    TORCH_CHECK(value >= 0 && value <= 2, "gemm_xcd_remap: 0 off, 1 long-K tiles, 2 always");
    fedtgan::g_gemm_xcd_remap = (int)value;
    return prev;
  }
  TORCH_CHECK(false, "unknown tuning key ", key);
}

}  // namespace

TORCH_LIBRARY(fedtgan, m) {
  m.def("gen_weight_prep(Tensor[] w, int[] kd, Tensor(a!)[] w16, Tensor(b!)[] wt) -> ()");
  m.def(
      "gemm(Tensor a, Tensor b, Tensor(a!) c, bool ta, bool tb, float alpha, float beta, Tensor? bias, int epi, "
      "Tensor(b!)? ms, float slope, float p_drop, Tensor(d!)? ws, int splitk, int seed, Tensor? rng_ctr, int stream, "
      "Tensor? bn_gamma, Tensor? bn_beta, Tensor? bn_rm, Tensor? bn_rv, float bn_eps, bool f32, Tensor? head_coef, "
      "Tensor? head_v, Tensor(e!)? head_a, int tile, int group=0, Tensor? oh_w=None, Tensor? oh_col=None, "
      "Tensor? oh_opt=None, Tensor? oh_off=None, bool oh_trans=False, Tensor(f!)? bn_part=None, int bn_rpg=0, "
      "Tensor(g!)? tile_cnt=None, bool chain=False) -> ()");
  m.def(
      "sample(Tensor(a!) h, int zc, int cc, int E, Tensor(b!)? xf, Tensor(c!)? xr, int Dd, Tensor cdf, Tensor cond_off, "
      "Tensor cond_w, Tensor? row_off, Tensor? row_cnt, Tensor? rows, Tensor? data, Tensor(d!)? col, Tensor(e!)? opt, "
      "Tensor(f!)? step_bump, Tensor(h!)? step_bump2, Tensor(g!)? metrics, bool zero_metrics, int seed, Tensor rng_ctr, "
      "int stream, int draws=1, int draw_h=0, int draw_x=0, int draw_col=0) -> ()");
  m.def(
      "activate(Tensor logits, Tensor(a!) out, Tensor start, Tensor width, Tensor kind, Tensor cidx, Tensor elem, "
      "float tau, int seed, Tensor rng_ctr, int stream, Tensor? slerp_real, Tensor(b!)? slerp_out, int slerp_cols, "
      "int slerp_stream) -> ()");
  m.def(
      "act_bwd_ce(Tensor dact, Tensor act, Tensor logits, Tensor start, Tensor width, Tensor kind, Tensor cidx, "
      "Tensor elem, Tensor col, Tensor opt, Tensor(a!) dlogits, Tensor(b!) loss, float tau) -> ()");
  m.def("slerp(Tensor real, Tensor fake, Tensor(a!) out, int seed, Tensor rng_ctr, int stream) -> ()");
  m.def("gp_scale(Tensor g, Tensor(a!) out, float lam, Tensor(b!) loss, Tensor(c!)? ws=None) -> ()");
  m.def("onehot_wgrad(Tensor[] dy, Tensor(a!)[] w, Tensor col, Tensor opt, Tensor cond_off, int zero) -> ()");
  m.def(
      "d_head(Tensor d, Tensor ms, Tensor v, Tensor e, Tensor coef, Tensor wloss, Tensor(a!) y, Tensor(b!) a, "
      "Tensor(c!) loss) -> ()");
  m.def("colsum(Tensor[] srcs, Tensor(a!)[] outs) -> ()");
  m.def(
      "colsum_ex(Tensor[] srcs, Tensor?[] outs, Tensor?[] w, Tensor?[] dot_v, Tensor?[] dot_e, Tensor?[] dot_out, "
      "Tensor?[] dot_w) -> ()");
  m.def(
      "linear_bn_relu_colown(Tensor x, Tensor w, Tensor? bias, Tensor gamma, Tensor beta, Tensor(a!) out, "
      "Tensor(b!) nhat, Tensor(c!) mean, Tensor(d!) invstd, Tensor(e!) rm, Tensor(f!) rv, float momentum, float eps, "
      "int groups, Tensor? oh_w, Tensor? oh_col, Tensor? oh_opt, Tensor? oh_off, bool oh_trans, Tensor(g!) stat, "
      "Tensor(h!) cnt) -> ()");
  m.def(
      "bn_relu_train(Tensor a, Tensor gamma, Tensor beta, Tensor(a!) out, Tensor(b!) nhat, Tensor(c!) mean, "
      "Tensor(d!) invstd, Tensor(e!) rm, Tensor(f!) rv, float momentum, float eps, int groups) -> ()");
  m.def(
      "bn_relu_apply(Tensor a, Tensor part, int n_tiles, Tensor gamma, Tensor beta, Tensor(a!) out, Tensor(b!) nhat, "
      "Tensor(c!) mean, Tensor(d!) invstd, Tensor(e!) rm, Tensor(f!) rv, float momentum, float eps, int groups) -> ()");
  m.def(
      "bn_relu_bwd(Tensor dr, Tensor r, Tensor nhat, Tensor gamma, Tensor invstd, Tensor(a!) da, Tensor(b!) dgamma, "
      "Tensor(c!) dbeta, Tensor(d!)? dbias, bool paired=False) -> ()");
  m.def(
      "adam(Tensor(a!) p, Tensor g, Tensor(b!) m, Tensor(c!) v, Tensor step, float lr, float b1, float b2, float eps, "
      "float wd, Tensor(d!)? rng_bump) -> ()");
  m.def(
      "adam_cs(Tensor(a!) p, Tensor(e!) g, Tensor(b!) m, Tensor(c!) v, Tensor step, float lr, float b1, float b2, "
      "float eps, float wd, Tensor(d!)? rng_bump, Tensor[] srcs, Tensor?[] outs, Tensor?[] w, Tensor?[] dot_v, "
      "Tensor?[] dot_e, Tensor?[] dot_out, Tensor?[] dot_w) -> ()");
  m.def(
      "sample_decode(Tensor logits, Tensor(a!) out, Tensor kind, Tensor start, Tensor width, Tensor cont, "
      "Tensor code_off, Tensor codes, Tensor mu, Tensor sd, int seed, Tensor rng_ctr, int stream, "
      "Tensor? ecol=None, Tensor? quads=None) -> ()");
  m.def("rng_bump(Tensor(a!) ctr) -> ()");
  m.def(
      "vgm_estep(Tensor x, Tensor n_rows, Tensor consts, Tensor means, Tensor prec, Tensor(a!) partial, "
      "int rows_per_block) -> ()");
  m.def("kmeans_step(Tensor x, Tensor n_rows, Tensor centers, Tensor(a!) partial, int rows_per_block) -> ()");
  m.def(
      "vgm_fit(Tensor x, Tensor n_rows, Tensor? init_centers, int seed, float wprior, float tol, float reg_covar, "
      "int max_iter, int km_iter, Tensor(a!) out, Tensor(b!) info, Tensor(c!) lower_bound) -> ()");
  m.def(
      "vgm_encode(Tensor x, Tensor(a!) out, Tensor(b!) opt, Tensor col_kind, Tensor col_pos, Tensor col_aux, "
      "Tensor col_span, Tensor col_lut_n, Tensor consts, Tensor means, Tensor prec, Tensor stds, Tensor vrank, Tensor lut, int seed, "
      "int stream) -> ()");
  m.def(
      "write_csv(str path, Tensor values, str[] names, int[] kinds, str[] vocab_flat, int[] vocab_offsets, "
      "int threads, int[] src=[], int[] date_desc=[], int[] date_lut=[], Tensor? aux=None) -> ()");
  m.def("py_float(float x) -> str", &py_float);
  m.def("rccl_load(str path) -> ()", &rccl_load_op);
  m.def("rccl_unique_id() -> Tensor", &rccl_unique_id_op);
  m.def("rccl_init(Tensor id, int rank, int nranks) -> int", &rccl_init_op);
  m.def("rccl_all_reduce(int comm, Tensor(a!) x, float premul) -> ()", &rccl_all_reduce_op);
  m.def("rccl_destroy(int comm) -> ()", &rccl_destroy_op);
  m.def("set_tuning(str key, int value) -> int", &set_tuning);
  m.def("reset_held() -> int", &reset_held);
  m.def("device_reset() -> int", &device_reset);
  m.def("pool_sample(Tensor(a!) pool, Tensor seg_off, Tensor mean, Tensor sd, int seed) -> ()");
  m.def("row_center(Tensor(a!) x, Tensor(b!) shift) -> ()");
  m.def("csr_rows(Tensor opt, Tensor width, int maxw, Tensor(a!) part, Tensor(b!) count, Tensor(c!) offset, "
        "Tensor(d!) rows, int chunk) -> ()");
  m.def("gemm_achain_next(Tensor out, Tensor ws, Tensor cnt) -> ()", &gemm_achain_next);
  m.def("set_client_batch(int k, int stride, int seed_step, int base) -> int", &set_client_batch);
  m.def("check_status() -> int", &check_status);
  m.def("is_checked() -> bool", &is_checked);
}

TORCH_LIBRARY_IMPL(fedtgan, CUDA, m) {
  m.impl("gemm", &gemm);
  m.impl("gen_weight_prep", &gen_weight_prep);
  m.impl("sample", &sample);
  m.impl("activate", &activate);
  m.impl("act_bwd_ce", &act_bwd_ce);
  m.impl("slerp", &slerp);
  m.impl("gp_scale", &gp_scale);
  m.impl("onehot_wgrad", &onehot_wgrad);
  m.impl("d_head", &d_head);
  m.impl("colsum", &colsum);
  m.impl("colsum_ex", &colsum_ex);
  m.impl("bn_relu_train", &bn_relu_train);
  m.impl("bn_relu_bwd", &bn_relu_bwd);
  m.impl("bn_relu_apply", &bn_relu_apply);
  m.impl("linear_bn_relu_colown", &linear_bn_relu_colown);
  m.impl("adam", &adam);
  m.impl("adam_cs", &adam_cs);
  m.impl("sample_decode", &sample_decode);
  m.impl("rng_bump", &rng_bump);
  m.impl("vgm_encode", &vgm_encode);
  m.impl("vgm_estep", &vgm_estep);
  m.impl("kmeans_step", &kmeans_step);
  m.impl("vgm_fit", &vgm_fit);
  m.impl("pool_sample", &pool_sample);
  m.impl("row_center", &row_center);
  m.impl("csr_rows", &csr_rows);
}

TORCH_LIBRARY_IMPL(fedtgan, CPU, m) { m.impl("write_csv", &write_csv); }
