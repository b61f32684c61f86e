// Fused CTGAN step kernels for gfx950 (everything in the WGAN-GP step that is not a GEMM).
//
//  sample_kernel       conditional vector + noise + (optional) permutation + real-row gather
//                      in ONE launch (`Cond.sample` + `Sampler.sample` + H2D copies of the
//                      reference, `Server/dtds/synthesizers/ctgan.py:147-161, 221-228`)
//  activate_kernel     tanh / Gumbel-softmax(tau) per output span (`ctgan.py:67-82`)
//  act_bwd_ce_kernel   activation backward + fused conditional cross-entropy (`ctgan.py:174-194`)
//  slerp_kernel        spherical interpolation for the gradient penalty (`ctgan.py:231-237`)
//  gp_scale_kernel     pack-wise gradient norm, penalty value and d(pen)/d(grad)
//  d_head_kernel       D output unit + WGAN loss + backward seed of the last hidden layer
//  colsum_kernel       batched bias gradients
//  bn_relu_*           BatchNorm1d (train) + ReLU forward / backward (`ctgan.py:33-44`)
//  adam_kernel         torch.optim.Adam (L2 decay on the gradient) over a flat buffer
//  sample_decode       generation: Gumbel-argmax + tanh + VGM / label decode to fp64
//
// Randomness: Philox streams (common.h) indexed by (seed, stream id, device step counter,
// element); the step counter is bumped by the generator's Adam launch (last of a step).
#include <algorithm>
#include <stdexcept>
#include <string>

#include "common.h"
#include "launch.h"
#include "adam_cs.h"

namespace fedtgan {

// ---------------------------------------------------------------------------- batched clients (launch.h)
int g_xcd_clients = 1;
ClientBatch& client_batch() {
  static thread_local ClientBatch cb{1, 0, 0, nullptr, 0};
  return cb;
}

void check_slab(const void* p, const char* what) {
  const ClientBatch& cb = client_batch();
  if (cb.k <= 1 || p == nullptr) return;
  const char* c = static_cast<const char*>(p);
  if (c < cb.base || c >= cb.base + cb.stride)
    throw std::runtime_error(std::string("batched launch: ") + what +
                             " is not in client 0's arena slab (every buffer of a batched step must be)");
}

void require_unbatched(const char* what) {
  if (client_batch().k > 1) throw std::runtime_error(std::string(what) + " has no batched-clients form");
}


#if FT_CHECKED
__device__ unsigned g_check_ops = 0u;
unsigned check_status_ctgan_ops() {
  unsigned v = 0u, z = 0u;
  (void)hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_check_ops), sizeof(v));
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_check_ops), &z, sizeof(z));
  return v;
}
#else
unsigned check_status_ctgan_ops() { return 0u; }
#endif

// ============================================================================ sampling
// One wave per batch row.  The option of the sampled conditional column is found with a
// lane-parallel inverse-CDF search (each lane tests one CDF entry, a ballot picks the first
// hit) -- one memory round trip instead of a serial scan over the span.  A D-phase row needs two
// such draws (its own condition and the one of the permuted fake row its real row serves); their
// first CDF chunks are requested together, and the noise is generated while they are in flight.
constexpr int SAMPLE_THREADS = 256;
constexpr int SAMPLE_ROWS = SAMPLE_THREADS / 64;   // rows per workgroup (one per wave)

struct CondDraw {
  int col, w;
  float u;
  const float* cdf;
};

__device__ __forceinline__ CondDraw cond_draw_begin(const SampleArgs& a, uint64_t step, int b) {
  RngArgs rng{a.seed, a.rng_ctr, a.rng_stream};
  const uint4 r = rng4(rng, step, (uint64_t)b);
  CondDraw d;
  d.col = min((int)(u01(r.x) * a.n_col), a.n_col - 1);
  d.u = u01(r.y);
  d.cdf = a.cdf + (size_t)d.col * a.maxw;
  d.w = a.cond_w[d.col];
  return d;
}

// first chunk already loaded (cv0 = cdf[lane]); rare wider spans continue chunk by chunk
__device__ __forceinline__ int cond_draw_finish(const SampleArgs& a, const CondDraw& d, float cv0, int lane) {
  unsigned long long hit = __ballot(lane < d.w && cv0 > d.u);
  if (hit) return min(__ffsll((long long)hit) - 1, d.w - 1);
  for (int base = 64; base < d.w; base += 64) {
    const int i = base + lane;
    const float cv = d.cdf[min(i, a.maxw - 1)];
    hit = __ballot(i < d.w && cv > d.u);
    if (hit) return min(base + __ffsll((long long)hit) - 1, d.w - 1);
  }
  return d.w - 1;
}

// Keyed pseudo-random permutation of [0, n): a 4-round Feistel network on the smallest even
// number of bits covering n, with cycle walking.  Every thread evaluates perm(b) on its own --
// no sort, no LDS, no barrier -- and a fresh key per step gives a fresh permutation.
__device__ __forceinline__ uint32_t feistel_perm(uint32_t x, uint32_t n, uint4 key) {
  int bits = 2;
  while ((1u << bits) < n) bits += 2;
  const int h = bits / 2;
  const uint32_t mask = (1u << h) - 1u;
  const uint32_t ks[4] = {key.x, key.y, key.z, key.w};
  do {
    uint32_t L = x >> h, R = x & mask;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      uint32_t f = (R ^ ks[r]) * 0x9E3779B1u;
      f ^= f >> 15;
      f *= 0x85EBCA77u;
      f ^= f >> 13;
      const uint32_t nl = R;
      R = L ^ (f & mask);
      L = nl;
    }
    x = (L << h) | R;
  } while (x >= n);
  return x;
}

// p[0, C) = one-hot(hot) written by one wave: scalar stores up to the first 16-B boundary, then 16-B stores
// (the wide table's condition blocks are 6,762 floats per row, three of them per D-phase row: a plain
// per-float loop was 3 x 106 store instructions per wave)
__device__ __forceinline__ void onehot_row(float* __restrict__ p, int C, int hot, int lane) {
  if (C < 1024) {   // (narrow blocks: the plain loop measured 0.6 us faster per sampler launch on Intrusion's 303)
    for (int i = lane; i < C; i += 64) p[i] = i == hot ? 1.f : 0.f;
    return;
  }
  const int head = min((int)(((16u - (uint32_t)(reinterpret_cast<uintptr_t>(p) & 15u)) & 15u) >> 2), C);
  if (lane < head) p[lane] = lane == hot ? 1.f : 0.f;
  const int n4 = (C - head) >> 2;
  float4* q = reinterpret_cast<float4*>(p + head);
  for (int k = lane; k < n4; k += 64) {
    const int i0 = head + 4 * k;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (hot >= i0 && hot < i0 + 4) {
      v.x = hot == i0 ? 1.f : 0.f;
      v.y = hot == i0 + 1 ? 1.f : 0.f;
      v.z = hot == i0 + 2 ? 1.f : 0.f;
      v.w = hot == i0 + 3 ? 1.f : 0.f;
    }
    q[k] = v;
  }
  for (int i = head + 4 * n4 + lane; i < C; i += 64) p[i] = i == hot ? 1.f : 0.f;
}

template <bool BT_ = false, bool MULTI = false>
__global__ __launch_bounds__(SAMPLE_THREADS) void sample_kernel(SampleArgs a) {
  const BIdx bi_ = batch_bidx<BT_>(a.cb.xcd);
  if (bi_.z) {   // batched clients: this client's buffers and seed
    const int64_t o = (int64_t)bi_.z * a.cb.stride;
    a.h = cptr(a.h, o);
    a.h16 = cptr(a.h16, o);
    a.xf = cptr(a.xf, o);
    a.xr = cptr(a.xr, o);
    a.cdf = cptr(a.cdf, o);
    a.cond_off = cptr(a.cond_off, o);
    a.cond_w = cptr(a.cond_w, o);
    a.row_off = cptr(a.row_off, o);
    a.row_cnt = cptr(a.row_cnt, o);
    a.rows = cptr(a.rows, o);
    a.data = cptr(a.data, o);
    a.col = cptr(a.col, o);
    a.opt = cptr(a.opt, o);
    a.step_bump = cptr(a.step_bump, o);
    a.step_bump2 = cptr(a.step_bump2, o);
    a.metrics = cptr(a.metrics, o);
    a.rng_ctr = cptr(a.rng_ctr, o);
    a.seed += (uint64_t)bi_.z * a.cb.seed_step;
  }
  uint64_t step = a.rng_ctr ? *a.rng_ctr : 0ull;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if constexpr (MULTI) {
    // draw k of a multi-step launch: step k's RNG key and buffers; ONE thread writes every step's counters
    // (reading the canonical last entry before overwriting it) and zeroes every step's metrics
    const int k = (int)blockIdx.y;
    step += (uint64_t)k;
    a.h += (size_t)k * a.draw_h;
    if (a.xf) a.xf += (size_t)k * a.draw_x;
    if (a.xr) a.xr += (size_t)k * a.draw_x;
    if (a.col) a.col += (size_t)k * a.draw_col;
    if (a.opt) a.opt += (size_t)k * a.draw_col;
    if (bi_.x == 0 && k == 0 && tid == 0) {
      const int D = a.draws;
      if (a.step_bump) {
        const float b = a.step_bump[D - 1];
        for (int q = 0; q < D; ++q) a.step_bump[q] = b + (float)(q + 1);
      }
      if (a.step_bump2) {
        const float b = a.step_bump2[D - 1];
        for (int q = 0; q < D; ++q) a.step_bump2[q] = b + (float)(q + 1);
      }
      if (a.zero_metrics && a.metrics)
        for (int q = 0; q < 4 * D; ++q) a.metrics[q] = 0.f;
    }
  } else if (bi_.x == 0 && tid == 0) {
    if (a.step_bump) a.step_bump[0] += 1.0f;
    if (a.step_bump2) a.step_bump2[0] += 1.0f;
    if (a.zero_metrics && a.metrics) {
      a.metrics[0] = 0.f; a.metrics[1] = 0.f; a.metrics[2] = 0.f; a.metrics[3] = 0.f;
    }
  }
  const int b = bi_.x * SAMPLE_ROWS + wv;
  if (b >= a.B) return;
  // rows [0, n_real) get a real row (the D phase); the rest only noise + condition (the G phase
  // of the same step when both batches are drawn by one launch)
  const int n_real = (a.xr != nullptr && a.n_col > 0) ? a.n_real : 0;
  const bool real = b < n_real;
  // (1) both condition draws: RNG + column tables, then the first CDF chunk of each
  CondDraw own{}, per{};
  float cv_own = 0.f, cv_per = 0.f;
  int p = 0;
  if (a.n_col > 0) {
    own = cond_draw_begin(a, step, b);
    if (real) {
      RngArgs rk{a.seed, a.rng_ctr, a.rng_stream + 1u};
      p = (int)feistel_perm((uint32_t)b, (uint32_t)n_real, rng4(rk, step, 0ull));
      per = cond_draw_begin(a, step, p);     // the condition of fake row perm[b]
    }
    cv_own = own.cdf[min(lane, a.maxw - 1)];
    if (real) cv_per = per.cdf[min(lane, a.maxw - 1)];
  }
  // (2) the noise while the CDF chunks are in flight
  RngArgs rz{a.seed, a.rng_ctr, a.rng_stream + 2u};
  if (a.h16) {
    // bf16 generation buffer: the same draws, rounded as the GEMM's staging would round them
    uint16_t* hrow16 = a.h16 + (size_t)b * a.ldh16 + a.zc16;
    for (int i = lane; i < (a.E + 1) / 2; i += 64) {
      const uint4 r = rng4(rz, step, (uint64_t)b * a.E + i);
      const float2 z = box_muller(r.x, r.y);
      if (2 * i + 1 < a.E && ((a.zc16 | a.ldh16) & 1) == 0) {
        *reinterpret_cast<uint32_t*>(hrow16 + 2 * i) = pack_bf16x2(z.x, z.y);
      } else {
        hrow16[2 * i] = f2bf(z.x);
        if (2 * i + 1 < a.E) hrow16[2 * i + 1] = f2bf(z.y);
      }
    }
    int col = 0, opt = 0;
    if (a.n_col > 0) {
      col = own.col;
      opt = cond_draw_finish(a, own, cv_own, lane);
    }
    if (lane == 0 && a.col) { a.col[b] = col; a.opt[b] = opt; }
    return;
  }
  float* hrow = a.h + (size_t)b * a.ldh;
  for (int i = lane; i < (a.E + 1) / 2; i += 64) {
    const uint4 r = rng4(rz, step, (uint64_t)b * a.E + i);
    const float2 z = box_muller(r.x, r.y);
    hrow[a.zc + 2 * i] = z.x;
    if (2 * i + 1 < a.E) hrow[a.zc + 2 * i + 1] = z.y;
  }
  // (3) options, one-hot conditions
  int col = 0, opt = 0;
  if (a.n_col > 0) {
    col = own.col;
    opt = cond_draw_finish(a, own, cv_own, lane);
  }
  const int hot = a.n_col > 0 ? a.cond_off[col] + opt : -1;
  float* xf = a.xf ? a.xf + (size_t)b * a.ldx + a.Dd : nullptr;
  onehot_row(hrow + a.cc, a.C, hot, lane);
  if (xf) onehot_row(xf, a.C, hot, lane);
  if (lane == 0 && a.col) { a.col[b] = col; a.opt[b] = opt; }
  if (!real) return;
  // (4) real row for the permuted condition: count -> CSR entry -> row copy
  const int pc = per.col, po = cond_draw_finish(a, per, cv_per, lane);
#if FT_CHECKED
  FT_CHECK(&g_check_ops, pc >= 0 && pc < a.n_col && po >= 0 && po < a.maxw, CHK_COND);
#endif
  const size_t cell = (size_t)pc * a.maxw + po;
  const int64_t cnt = a.row_cnt[cell];
  const int64_t off = a.row_off[cell];
  RngArgs rp{a.seed, a.rng_ctr, a.rng_stream + 3u};
  const uint4 r4 = rng4(rp, step, (uint64_t)b);
  int64_t pick = (int64_t)(u01d(r4.x, r4.y) * (double)(cnt > 0 ? cnt : 1));
  if (pick >= cnt) pick = cnt > 0 ? cnt - 1 : 0;
#if FT_CHECKED
  FT_CHECK(&g_check_ops, off >= 0 && off + pick < a.n_entries, CHK_CSR_PICK);
  int64_t row = a.rows[min(max(off + pick, (int64_t)0), a.n_entries - 1)];
  FT_CHECK(&g_check_ops, row >= 0 && row < a.n_rows, CHK_DATA_ROW);
  row = min(max(row, (int64_t)0), (int64_t)a.n_rows - 1);
#else
  const int64_t row = a.rows[off + pick];
#endif
  const float* src = a.data + (size_t)row * a.Dd;
  float* dst = a.xr + (size_t)b * a.ldx;
  // the row copy: CP loads in flight per lane before their stores (a plain strided loop waits one memory
  // round trip per 64 columns -- the compiler cannot move a load of `src` above a store to `dst`); the
  // one-hot block is stored while the first loads are in flight
  constexpr int CP = 8;
  float v[CP];
#pragma unroll
  for (int u = 0; u < CP; ++u) v[u] = src[min(lane + 64 * u, a.Dd - 1)];
  const int phot = a.cond_off[pc] + po;
  onehot_row(dst + a.Dd, a.C, phot, lane);
  for (int i0 = 0; i0 < a.Dd; i0 += 64 * CP) {
    float nx[CP];
    const int n0 = i0 + 64 * CP;
#pragma unroll
    for (int u = 0; u < CP; ++u) nx[u] = n0 < a.Dd ? src[min(n0 + lane + 64 * u, a.Dd - 1)] : 0.f;
#pragma unroll
    for (int u = 0; u < CP; ++u)
      if (i0 + lane + 64 * u < a.Dd) dst[i0 + lane + 64 * u] = v[u];
#pragma unroll
    for (int u = 0; u < CP; ++u) v[u] = nx[u];
  }
}

void launch_sample(const SampleArgs& a0, hipStream_t stream) {
  SampleArgs a = a0;
  a.cb = client_batch();
  if (a.cb.k > 1) {
    for (const void* p : {(const void*)a.h, (const void*)a.h16, (const void*)a.xf, (const void*)a.xr, (const void*)a.cdf,
                          (const void*)a.cond_off, (const void*)a.cond_w, (const void*)a.row_off, (const void*)a.row_cnt,
                          (const void*)a.rows, (const void*)a.data, (const void*)a.col, (const void*)a.opt,
                          (const void*)a.step_bump, (const void*)a.step_bump2, (const void*)a.metrics,
                          (const void*)a.rng_ctr})
      check_slab(p, "sample operand");
  }
  const int blocks = (a.B + SAMPLE_ROWS - 1) / SAMPLE_ROWS;
  if (a.draws > 1) {
    if (a.cb.k > 1 || a.h16) throw std::runtime_error("sample: multi-step draws are for one client's fp32 training batches");
    hipLaunchKernelGGL((sample_kernel<false, true>), dim3(blocks, a.draws, 1), dim3(SAMPLE_THREADS), 0, stream, a);
    return;
  }
  hipLaunchKernelGGL((client_batch().xcd ? sample_kernel<true> : sample_kernel<false>), dim3(blocks, 1, a.cb.k), dim3(SAMPLE_THREADS), 0, stream, a);
}

// ============================================================================ activation
// One wave per row; the span tables are staged in LDS once per workgroup (one memory round
// trip), so the per-element work never chases a global pointer.
//   element-parallel: Gumbel-perturbed logits (or tanh) into an LDS row image
//   span-parallel   : one lane per softmax span reduces (max, sum) from LDS
//   element-parallel: normalise and store
// slerp weights of the reference's `slerp` (`Server/dtds/synthesizers/ctgan.py:231-237`), linear
// fallback when the angle degenerates; shared by the fused activation and the standalone kernel
__device__ __forceinline__ void slerp_weights(float saa, float sbb, float sab, float alpha, float& wa, float& wb) {
  float cosw = sab / (sqrtf(saa) * sqrtf(sbb));
  cosw = fminf(1.f, fmaxf(-1.f, cosw));
  const float om = acosf(cosw);
  const float so = sinf(om);
  if (so < 1e-6f) {
    wa = 1.f - alpha;
    wb = alpha;
  } else {
    wa = sinf((1.f - alpha) * om) / so;
    wb = sinf(alpha * om) / so;
  }
}

int g_act_row_mode = 2;   // wide rows: one 512-thread workgroup per row, register-resident (2) or LDS row image (1)
constexpr int ACT_WAVES = 4;   // rows (waves) per workgroup when the LDS image allows it
constexpr int ACT_PF = 8;      // logits prefetched per lane (rows up to 512 wide)
constexpr int ACT_PFS = 12;    // slerp real-row values prefetched per lane (rows up to 768 wide)
constexpr size_t LDS_BYTES = 160 * 1024;
constexpr int EI_SOFTMAX = 1 << 30;   // einfo bit: the element belongs to a softmax span

struct ActSmem {
  int* einfo;   // [D]  element -> span index | EI_SOFTMAX
  int* kind;    // [S]
  int* start;   // [S]
  int* width;   // [S]
  int* cidx;    // [S]
  float* rows;  // [waves][D + 2S]: row image, then per-span statistics
};

__device__ __forceinline__ ActSmem act_stage_tables(const SpanTables& sp, float* smem) {
  const int D = sp.dim, S = sp.n_span;
  ActSmem t;
  t.einfo = reinterpret_cast<int*>(smem);
  t.kind = t.einfo + D;
  t.start = t.kind + S;
  t.width = t.start + S;
  t.cidx = t.width + S;
  const int n4 = ((D + 4 * S + 3) & ~3) / 4;   // span_packed_len (launch.h) / 4
  t.rows = smem + 4 * n4;
  // one contiguous 16-B copy, ACT_STAGE loads in flight per thread before the first LDS store
  constexpr int ACT_STAGE = 8;
  const int4* src = reinterpret_cast<const int4*>(sp.packed);
  int4* dst = reinterpret_cast<int4*>(smem);
  for (int i0 = threadIdx.x; i0 < n4; i0 += ACT_STAGE * blockDim.x) {
    int4 v[ACT_STAGE];
#pragma unroll
    for (int u = 0; u < ACT_STAGE; ++u) v[u] = src[min(i0 + u * (int)blockDim.x, n4 - 1)];
#pragma unroll
    for (int u = 0; u < ACT_STAGE; ++u)
      if (i0 + u * (int)blockDim.x < n4) dst[i0 + u * blockDim.x] = v[u];
  }
  __syncthreads();
  return t;
}

// batched clients: a client's copy of the span tables / the fused slerp's buffers
__device__ __forceinline__ void client_off(SpanTables& sp, int64_t o) {
  sp.start = cptr(sp.start, o);
  sp.width = cptr(sp.width, o);
  sp.kind = cptr(sp.kind, o);
  sp.cond_idx = cptr(sp.cond_idx, o);
  sp.packed = cptr(sp.packed, o);
}
__device__ __forceinline__ void client_off(SlerpFuse& sl, int64_t o) {
  sl.real = cptr(sl.real, o);
  sl.out = cptr(sl.out, o);
}
static void check_slab(const SpanTables& sp) {
  check_slabs("span tables", sp.start, sp.width, sp.kind, sp.cond_idx, sp.packed);
}

// order-preserving float <-> uint map (for ds_max_u32 on floats); 0 is below every float
__device__ __forceinline__ uint32_t f2ord(float f) {
  const uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float ord2f(uint32_t u) {
  return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Segmented softmax without serial per-span loops: every lane folds its own elements into the
// span's LDS statistics with ds_max_u32 / ds_add_f32 (per-wave statistics block), so the cost
// no longer scales with the widest span.  Gumbel noise: one Philox call feeds 4 elements of a
// lane (index (row, k/4, lane)).
template <bool BT_ = false>
__global__ __launch_bounds__(ACT_WAVES * 64) void activate_kernel(const float* __restrict__ logits, int ldl,
                                                                  float* __restrict__ out, int ldo, int rows,
                                                                  SpanTables sp, float inv_tau, uint64_t seed,
                                                                  const uint64_t* ctr, uint32_t stream_id,
                                                                  SlerpFuse sl, ClientBatch cb) {
  const BIdx bi_ = batch_bidx<BT_>(cb.xcd);
  extern __shared__ float act_smem[];
  if (bi_.z) {
    const int64_t co = (int64_t)bi_.z * cb.stride;
    logits = cptr(logits, co);
    out = cptr(out, co);
    ctr = cptr(ctr, co);
    client_off(sp, co);
    client_off(sl, co);
    seed += (uint64_t)bi_.z * cb.seed_step;
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r = bi_.x * (int)(blockDim.x >> 6) + wv;
  const int rc = min(r, rows - 1);
  const int D = sp.dim, S = sp.n_span;
  const float* x = logits + (size_t)rc * ldl;
  // the row's logits (and the slerp's real row) are requested before the span tables are staged,
  // so the three global round trips overlap (rows up to ACT_PF*64 wide stay in registers)
  const bool pre = D <= ACT_PF * 64;
  float xr[ACT_PF];
#pragma unroll
  for (int k = 0; k < ACT_PF; ++k) xr[k] = pre ? x[min(lane + 64 * k, D - 1)] : 0.f;
  const bool pre_s = sl.real != nullptr && sl.cols <= ACT_PFS * 64;
  const float* a_row = sl.real ? sl.real + (size_t)min(rc, sl.rows - 1) * sl.ld : nullptr;
  float ar[ACT_PFS], fc[ACT_PFS];
  const float* f_row = out + (size_t)rc * ldo;   // the fake row's condition columns (j >= D) are in place
#pragma unroll
  for (int k = 0; k < ACT_PFS; ++k) {
    const int j = min(lane + 64 * k, sl.cols - 1);
    ar[k] = pre_s ? a_row[j] : 0.f;
    fc[k] = (pre_s && sl.cols > D) ? f_row[max(j, D)] : 0.f;   // (j <= cols - 1 already)
  }
  const ActSmem t = act_stage_tables(sp, act_smem);
  if (r >= rows) return;
  float* v = t.rows + (size_t)wv * (D + 2 * S);
  uint32_t* smax = reinterpret_cast<uint32_t*>(v + D);
  float* ssum = v + D + S;
  float* y = out + (size_t)r * ldo;
  const uint64_t step = ctr ? *ctr : 0ull;
  RngArgs rng{seed, ctr, stream_id};
  const uint64_t base = (uint64_t)r << 20;
  for (int s2 = lane; s2 < S; s2 += 64) { smax[s2] = 0u; ssum[s2] = 0.f; }
  wave_lds_sync();
  uint4 u4 = make_uint4(0u, 0u, 0u, 0u);
  auto act_elem = [&](int j, int k, float xv) {
    if ((k & 3) == 0) u4 = rng4(rng, step, base + (uint64_t)(k >> 2) * 64u + (uint64_t)lane);
    const uint32_t u = (k & 3) == 0 ? u4.x : (k & 3) == 1 ? u4.y : (k & 3) == 2 ? u4.z : u4.w;
    const int info = t.einfo[j];
    if (!(info & EI_SOFTMAX)) {
      const float th = tanhf(xv);
      y[j] = th;
      v[j] = th;    // (read back by the fused slerp; tanh elements have no softmax input)
    } else {
      const float g = (xv + gumbel(u)) * inv_tau;
      v[j] = g;
      atomicMax(&smax[info & (EI_SOFTMAX - 1)], f2ord(g));
    }
  };
  if (pre) {
#pragma unroll
    for (int k = 0; k < ACT_PF; ++k)
      if (lane + 64 * k < D) act_elem(lane + 64 * k, k, xr[k]);
  } else {
    // wide rows: chunks of ACT_PF * 64 columns, each chunk's loads issued together (a plain
    // strided loop waits one memory round trip per 64 columns)
    for (int c0 = 0; c0 < D; c0 += ACT_PF * 64) {
      float xc[ACT_PF];
#pragma unroll
      for (int k = 0; k < ACT_PF; ++k) xc[k] = x[min(c0 + lane + 64 * k, D - 1)];
#pragma unroll
      for (int k = 0; k < ACT_PF; ++k)
        if (c0 + lane + 64 * k < D) act_elem(c0 + lane + 64 * k, (c0 >> 6) + k, xc[k]);
    }
  }
  wave_lds_sync();
  for (int j = lane; j < D; j += 64) {
    const int info = t.einfo[j];
    if (info & EI_SOFTMAX) {
      const int s2 = info & (EI_SOFTMAX - 1);
      const float e = __expf(v[j] - ord2f(smax[s2]));
      v[j] = e;
      atomicAdd(&ssum[s2], e);
    }
  }
  wave_lds_sync();
  for (int j = lane; j < D; j += 64) {
    const int info = t.einfo[j];
    if (info & EI_SOFTMAX) {
      const float o = v[j] / ssum[info & (EI_SOFTMAX - 1)];
      y[j] = o;
      v[j] = o;     // each lane re-reads only its own elements below
    }
  }
  if (sl.real == nullptr || r >= sl.rows) return;
  // fused slerp(real_r, fake_r) of the gradient penalty (one launch less per step): the fake row
  // is this row's activation (LDS, j < D) followed by its conditional columns (global)
  const float* a = a_row;
  float saa = 0.f, sbb = 0.f, sab = 0.f;
  if (pre_s) {
#pragma unroll
    for (int k = 0; k < ACT_PFS; ++k) {
      const int j = lane + 64 * k;
      if (j < sl.cols) {
        const float ra = ar[k], fb = j < D ? v[j] : fc[k];
        saa += ra * ra;
        sbb += fb * fb;
        sab += ra * fb;
      }
    }
  } else {
    for (int j = lane; j < sl.cols; j += 64) {
      const float ra = a[j], fb = j < D ? v[j] : y[j];
      saa += ra * ra;
      sbb += fb * fb;
      sab += ra * fb;
    }
  }
  saa = wave_sum(saa);
  sbb = wave_sum(sbb);
  sab = wave_sum(sab);
  RngArgs srng{seed, ctr, sl.stream};
  const float alpha = u01(rng4(srng, step, (uint64_t)r).x);
  float wa, wb;
  slerp_weights(saa, sbb, sab, alpha, wa, wb);
  float* o = sl.out + (size_t)r * sl.ld;
  if (pre_s) {
#pragma unroll
    for (int k = 0; k < ACT_PFS; ++k) {
      const int j = lane + 64 * k;
      if (j < sl.cols) o[j] = wa * ar[k] + wb * (j < D ? v[j] : fc[k]);
    }
  } else {
    for (int j = lane; j < sl.cols; j += 64) o[j] = wa * a[j] + wb * (j < D ? v[j] : y[j]);
  }
}

// ---- wide rows (data_dim > ACT_PF * 64): one 512-thread workgroup per row.  The span tables
// are staged once per row instead of once per 1-2 rows, 8 waves share the row's span statistics
// (the same LDS atomics, workgroup barriers instead of wave syncs), and the grid has one
// workgroup per row.  Wave w takes groups of 4 consecutive 64-column blocks (4w, 4w+1, ..),
// striding by 32 blocks, so every element draws the same Philox word as in the narrow kernel
// (counter (row, block / 4, lane), component block % 4): the two kernels are interchangeable.
constexpr int ROW_WAVES = 8;

template <int NW = ROW_WAVES>
__device__ __forceinline__ float3 block_sum3(float a, float b, float c, float* sh) {
  a = wave_sum(a);
  b = wave_sum(b);
  c = wave_sum(c);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) {
    sh[3 * wv] = a;
    sh[3 * wv + 1] = b;
    sh[3 * wv + 2] = c;
  }
  __syncthreads();
  float3 r = make_float3(0.f, 0.f, 0.f);
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    r.x += sh[3 * w];
    r.y += sh[3 * w + 1];
    r.z += sh[3 * w + 2];
  }
  return r;
}

template <bool BT_ = false>
__global__ __launch_bounds__(ROW_WAVES * 64) void activate_row_kernel(const float* __restrict__ logits, int ldl,
                                                                      float* __restrict__ out, int ldo, int rows,
                                                                      SpanTables sp, float inv_tau, uint64_t seed,
                                                                      const uint64_t* ctr, uint32_t stream_id,
                                                                      SlerpFuse sl, ClientBatch cb) {
  const BIdx bi_ = batch_bidx<BT_>(cb.xcd);
  // LDS holds only the row image and the span statistics; the element -> span map (the first D
  // words of the packed table, shared by every row and L2-resident) is read next to the logits
  extern __shared__ float act_smem[];
  if (bi_.z) {
    const int64_t co = (int64_t)bi_.z * cb.stride;
    logits = cptr(logits, co);
    out = cptr(out, co);
    ctr = cptr(ctr, co);
    client_off(sp, co);
    client_off(sl, co);
    seed += (uint64_t)bi_.z * cb.seed_step;
  }
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int r = bi_.x;
  const int D = sp.dim, S = sp.n_span;
  const float* x = logits + (size_t)r * ldl;
  const int* einfo = sp.packed;
  float* v = act_smem;
  uint32_t* smax = reinterpret_cast<uint32_t*>(v + D);
  float* ssum = v + D + S;
  float* red = v + D + 2 * S;   // [ROW_WAVES * 3] slerp partial sums
  float* y = out + (size_t)r * ldo;
  const uint64_t step = ctr ? *ctr : 0ull;
  RngArgs rng{seed, ctr, stream_id};
  const uint64_t base = (uint64_t)r << 20;
  for (int s2 = tid; s2 < S; s2 += blockDim.x) {
    smax[s2] = 0u;
    ssum[s2] = 0.f;
  }
  __syncthreads();
  const int NB = (D + 63) / 64;
  for (int g0 = 4 * wv; g0 < NB; g0 += 4 * ROW_WAVES) {
    float xc[4];
    int ic[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = min((g0 + q) * 64 + lane, D - 1);
      xc[q] = x[j];
      ic[q] = einfo[j];
    }
    const uint4 u4 = rng4(rng, step, base + (uint64_t)(g0 >> 2) * 64u + (uint64_t)lane);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = (g0 + q) * 64 + lane;
      if (j >= D) break;
      const uint32_t u = q == 0 ? u4.x : q == 1 ? u4.y : q == 2 ? u4.z : u4.w;
      if (!(ic[q] & EI_SOFTMAX)) {
        const float th = tanhf(xc[q]);
        y[j] = th;
        v[j] = th;
      } else {
        const float gv = (xc[q] + gumbel(u)) * inv_tau;
        v[j] = gv;
        atomicMax(&smax[ic[q] & (EI_SOFTMAX - 1)], f2ord(gv));
      }
    }
  }
  __syncthreads();
  for (int j = tid; j < D; j += blockDim.x) {
    const int info = einfo[j];
    if (info & EI_SOFTMAX) {
      const int s2 = info & (EI_SOFTMAX - 1);
      const float e = __expf(v[j] - ord2f(smax[s2]));
      v[j] = e;
      atomicAdd(&ssum[s2], e);
    }
  }
  __syncthreads();
  for (int j = tid; j < D; j += blockDim.x) {
    const int info = einfo[j];
    if (info & EI_SOFTMAX) {
      const float o = v[j] / ssum[info & (EI_SOFTMAX - 1)];
      y[j] = o;
      v[j] = o;
    }
  }
  if (sl.real == nullptr || r >= sl.rows) return;   // (uniform over the workgroup)
  __syncthreads();   // every element of the row image (tanh and softmax) is final
  const float* a = sl.real + (size_t)r * sl.ld;
  float saa = 0.f, sbb = 0.f, sab = 0.f;
  for (int j = tid; j < sl.cols; j += blockDim.x) {
    const float ra = a[j], fb = j < D ? v[j] : y[j];
    saa += ra * ra;
    sbb += fb * fb;
    sab += ra * fb;
  }
  const float3 tot = block_sum3(saa, sbb, sab, red);
  RngArgs srng{seed, ctr, sl.stream};
  const float alpha = u01(rng4(srng, step, (uint64_t)r).x);
  float wa, wb;
  slerp_weights(tot.x, tot.y, tot.z, alpha, wa, wb);
  float* o = sl.out + (size_t)r * sl.ld;
  for (int j = tid; j < sl.cols; j += blockDim.x) o[j] = wa * a[j] + wb * (j < D ? v[j] : y[j]);
}

// ---- wide rows, register-resident (act_row_mode 2): the same element -> (wave, lane, Philox word) map as
// activate_row_kernel, but every element a lane owns (GPW groups of 4 blocks) stays in its registers, and the
// span map and the slerp's real row are requested with the logits in ONE burst.  The per-span max / sum are
// span-parallel: the perturbed logits go to an LDS row image and each thread folds whole spans of it (spans are
// contiguous column ranges).  Per-element LDS atomics (the LDS-image kernel above) serialise the lanes of a wave
// that hit one span: on the wide table (7,018 columns, spans ~17 wide) the LDS pipe was busy ~40 us per CU per
// launch (rocprofv3 SQ_LDS_IDX_ACTIVE, profiles/wide_pmc_r4.txt).
template <int GPW, int NW = ROW_WAVES, bool BT_ = false>
__global__ __launch_bounds__(NW * 64) void activate_rowreg_kernel(const float* __restrict__ logits, int ldl,
                                                                         float* __restrict__ out, int ldo, int rows,
                                                                         SpanTables sp, float inv_tau, uint64_t seed,
                                                                         const uint64_t* ctr, uint32_t stream_id,
                                                                         SlerpFuse sl, ClientBatch cb) {
  const BIdx bi_ = batch_bidx<BT_>(cb.xcd);
  extern __shared__ float act_smem[];
  if (bi_.z) {
    const int64_t co = (int64_t)bi_.z * cb.stride;
    logits = cptr(logits, co);
    out = cptr(out, co);
    ctr = cptr(ctr, co);
    client_off(sp, co);
    client_off(sl, co);
    seed += (uint64_t)bi_.z * cb.seed_step;
  }
  constexpr int NTH = NW * 64;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int r = bi_.x;
  const int D = sp.dim, S = sp.n_span;
  const float* x = logits + (size_t)r * ldl;
  const int* einfo = sp.packed;
  const int* kind = einfo + D;
  const int* start = kind + S;
  const int* width = start + S;
  float* vs = act_smem;          // [D] perturbed logits (softmax elements)
  float* smax = vs + D;          // [S] span max, then 1 / span sum
  float* ssum = smax + S;        // [S]
  float* red = ssum + S;         // [ROW_WAVES * 3] slerp partial sums
  float* y = out + (size_t)r * ldo;
  const bool do_sl = sl.real != nullptr && r < sl.rows;   // (uniform over the workgroup)
  const float* a = do_sl ? sl.real + (size_t)r * sl.ld : x;
  float xv[GPW][4], ar[GPW][4];
  int ic[GPW][4];
#pragma unroll
  for (int g = 0; g < GPW; ++g)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = min((4 * (wv + NW * g) + q) * 64 + lane, D - 1);
      xv[g][q] = x[j];
      ic[g][q] = einfo[j];
      ar[g][q] = a[j];
    }
  const uint64_t step = ctr ? *ctr : 0ull;
  RngArgs rng{seed, ctr, stream_id};
  const uint64_t base = (uint64_t)r << 20;
#pragma unroll
  for (int g = 0; g < GPW; ++g) {
    const int gi = wv + NW * g;
    if (4 * gi * 64 >= D) break;   // (uniform over the wave)
    const uint4 u4 = rng4(rng, step, base + (uint64_t)gi * 64u + (uint64_t)lane);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = (4 * gi + q) * 64 + lane;
      if (j >= D) break;
      const uint32_t u = q == 0 ? u4.x : q == 1 ? u4.y : q == 2 ? u4.z : u4.w;
      if (!(ic[g][q] & EI_SOFTMAX)) {
        const float th = tanhf(xv[g][q]);
        y[j] = th;
        xv[g][q] = th;
      } else {
        const float gv = (xv[g][q] + gumbel(u)) * inv_tau;
        xv[g][q] = gv;
        vs[j] = gv;
      }
    }
  }
  __syncthreads();
  // span-parallel statistics: max, then sum of exp(v - max); spans of one thread are independent loops
  for (int s2 = tid; s2 < S; s2 += NTH) {
    if (kind[s2] == 0) continue;
    const int st = start[s2], w = width[s2];
    const float* v = vs + st;
    float m = -INFINITY;
    int i = 0;
    for (; i + 4 <= w; i += 4) m = fmaxf(fmaxf(m, fmaxf(v[i], v[i + 1])), fmaxf(v[i + 2], v[i + 3]));
    for (; i < w; ++i) m = fmaxf(m, v[i]);
    float e0 = 0.f, e1 = 0.f;
    i = 0;
    for (; i + 2 <= w; i += 2) {
      e0 += __expf(v[i] - m);
      e1 += __expf(v[i + 1] - m);
    }
    if (i < w) e0 += __expf(v[i] - m);
    smax[s2] = m;
    ssum[s2] = 1.f / (e0 + e1);
  }
  __syncthreads();
#pragma unroll
  for (int g = 0; g < GPW; ++g)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = (4 * (wv + NW * g) + q) * 64 + lane;
      if (j < D && (ic[g][q] & EI_SOFTMAX)) {
        const int s2 = ic[g][q] & (EI_SOFTMAX - 1);
        const float o = __expf(xv[g][q] - smax[s2]) * ssum[s2];
        y[j] = o;
        xv[g][q] = o;
      }
    }
  if (!do_sl) return;
  // fused slerp(real_r, fake_r): the fake row is this row's activation (registers, j < D) followed by its
  // condition columns (global, written by the sampler)
  float saa = 0.f, sbb = 0.f, sab = 0.f;
#pragma unroll
  for (int g = 0; g < GPW; ++g)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = (4 * (wv + NW * g) + q) * 64 + lane;
      if (j < D) {
        saa += ar[g][q] * ar[g][q];
        sbb += xv[g][q] * xv[g][q];
        sab += ar[g][q] * xv[g][q];
      }
    }
  constexpr int TU = 4;   // tail loads in flight per thread
  for (int j0 = D; j0 < sl.cols; j0 += TU * NTH) {
    float ra[TU], fb[TU];
#pragma unroll
    for (int u = 0; u < TU; ++u) {
      const int j = min(j0 + u * NTH + tid, sl.cols - 1);
      ra[u] = a[j];
      fb[u] = y[j];
    }
#pragma unroll
    for (int u = 0; u < TU; ++u)
      if (j0 + u * NTH + tid < sl.cols) {
        saa += ra[u] * ra[u];
        sbb += fb[u] * fb[u];
        sab += ra[u] * fb[u];
      }
  }
  const float3 tot = block_sum3<NW>(saa, sbb, sab, red);
  RngArgs srng{seed, ctr, sl.stream};
  const float alpha = u01(rng4(srng, step, (uint64_t)r).x);
  float wa, wb;
  slerp_weights(tot.x, tot.y, tot.z, alpha, wa, wb);
  float* o = sl.out + (size_t)r * sl.ld;
#pragma unroll
  for (int g = 0; g < GPW; ++g)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = (4 * (wv + NW * g) + q) * 64 + lane;
      if (j < D) o[j] = wa * ar[g][q] + wb * xv[g][q];
    }
  for (int j0 = D; j0 < sl.cols; j0 += TU * NTH) {
    float ra[TU], fb[TU];
#pragma unroll
    for (int u = 0; u < TU; ++u) {
      const int j = min(j0 + u * NTH + tid, sl.cols - 1);
      ra[u] = a[j];
      fb[u] = y[j];
    }
#pragma unroll
    for (int u = 0; u < TU; ++u) {
      const int j = j0 + u * NTH + tid;
      if (j < sl.cols) o[j] = wa * ra[u] + wb * fb[u];
    }
  }
}

// ---- narrow rows (<= 64 NW columns), one 64-column block per wave (act_rowreg_narrow 2): the same Philox words
// as every other activation kernel -- block b uses component b % 4 of the call for group b / 4, so the waves of
// a group each evaluate that call (4x the RNG arithmetic of activate_rowreg_kernel) -- in exchange for one
// element per lane: the per-wave dependent chain (load, Philox, Gumbel, softmax, slerp) is a quarter as long.
template <int NW, bool BT_ = false>
__global__ __launch_bounds__(NW * 64) void activate_rowblk_kernel(const float* __restrict__ logits, int ldl,
                                                                  float* __restrict__ out, int ldo, int rows,
                                                                  SpanTables sp, float inv_tau, uint64_t seed,
                                                                  const uint64_t* ctr, uint32_t stream_id,
                                                                  SlerpFuse sl, ClientBatch cb) {
  const BIdx bi_ = batch_bidx<BT_>(cb.xcd);
  extern __shared__ float act_smem[];
  if (bi_.z) {
    const int64_t co = (int64_t)bi_.z * cb.stride;
    logits = cptr(logits, co);
    out = cptr(out, co);
    ctr = cptr(ctr, co);
    client_off(sp, co);
    client_off(sl, co);
    seed += (uint64_t)bi_.z * cb.seed_step;
  }
  constexpr int NTH = NW * 64;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int r = bi_.x;
  const int D = sp.dim, S = sp.n_span;
  const float* x = logits + (size_t)r * ldl;
  const int* einfo = sp.packed;
  const int* kind = einfo + D;
  const int* start = kind + S;
  const int* width = start + S;
  float* vs = act_smem;          // [D] perturbed logits (softmax elements)
  float* smax = vs + D;          // [S]
  float* ssum = smax + S;        // [S] 1 / span sum
  float* red = ssum + S;         // [NW * 3]
  float* y = out + (size_t)r * ldo;
  const bool do_sl = sl.real != nullptr && r < sl.rows;
  const float* a = do_sl ? sl.real + (size_t)r * sl.ld : x;
  const int j = wv * 64 + lane;          // this lane's element (block wv)
  const bool in = j < D;
  const int jc = min(j, D - 1);
  float xv = x[jc];
  const int ic = einfo[jc];
  const float ar = a[jc];
  const uint64_t step = ctr ? *ctr : 0ull;
  if (in) {
    RngArgs rng{seed, ctr, stream_id};
    const uint4 u4 = rng4(rng, step, ((uint64_t)r << 20) + (uint64_t)(wv >> 2) * 64u + (uint64_t)lane);
    const int q = wv & 3;
    const uint32_t u = q == 0 ? u4.x : q == 1 ? u4.y : q == 2 ? u4.z : u4.w;
    if (!(ic & EI_SOFTMAX)) {
      xv = tanhf(xv);
      y[j] = xv;
    } else {
      xv = (xv + gumbel(u)) * inv_tau;
      vs[j] = xv;
    }
  }
  __syncthreads();
  for (int s2 = tid; s2 < S; s2 += NTH) {
    if (kind[s2] == 0) continue;
    const int st = start[s2], w = width[s2];
    const float* v = vs + st;
    float m = -INFINITY;
    int i = 0;
    for (; i + 4 <= w; i += 4) m = fmaxf(fmaxf(m, fmaxf(v[i], v[i + 1])), fmaxf(v[i + 2], v[i + 3]));
    for (; i < w; ++i) m = fmaxf(m, v[i]);
    float e0 = 0.f, e1 = 0.f;
    i = 0;
    for (; i + 2 <= w; i += 2) {
      e0 += __expf(v[i] - m);
      e1 += __expf(v[i + 1] - m);
    }
    if (i < w) e0 += __expf(v[i] - m);
    smax[s2] = m;
    ssum[s2] = 1.f / (e0 + e1);
  }
  __syncthreads();
  if (in && (ic & EI_SOFTMAX)) {
    const int s2 = ic & (EI_SOFTMAX - 1);
    xv = __expf(xv - smax[s2]) * ssum[s2];
    y[j] = xv;
  }
  if (!do_sl) return;
  float saa = 0.f, sbb = 0.f, sab = 0.f;
  if (in) {
    saa = ar * ar;
    sbb = xv * xv;
    sab = ar * xv;
  }
  constexpr int TU = 2;
  float ra[TU], fb[TU];
#pragma unroll
  for (int u = 0; u < TU; ++u) {     // the condition columns (j >= D) of the real and fake rows
    const int jt = min(D + u * NTH + tid, sl.cols - 1);
    ra[u] = a[jt];
    fb[u] = y[jt];
  }
#pragma unroll
  for (int u = 0; u < TU; ++u)
    if (D + u * NTH + tid < sl.cols) {
      saa += ra[u] * ra[u];
      sbb += fb[u] * fb[u];
      sab += ra[u] * fb[u];
    }
  for (int jt = D + TU * NTH + tid; jt < sl.cols; jt += NTH) {   // (rare: condition blocks wider than TU * NTH)
    const float ra2 = a[jt], fb2 = y[jt];
    saa += ra2 * ra2;
    sbb += fb2 * fb2;
    sab += ra2 * fb2;
  }
  const float3 tot = block_sum3<NW>(saa, sbb, sab, red);
  RngArgs srng{seed, ctr, sl.stream};
  const float alpha = u01(rng4(srng, step, (uint64_t)r).x);
  float wa, wb;
  slerp_weights(tot.x, tot.y, tot.z, alpha, wa, wb);
  float* o = sl.out + (size_t)r * sl.ld;
  if (in) o[j] = wa * ar + wb * xv;
#pragma unroll
  for (int u = 0; u < TU; ++u) {
    const int jt = D + u * NTH + tid;
    if (jt < sl.cols) o[jt] = wa * ra[u] + wb * fb[u];
  }
  for (int jt = D + TU * NTH + tid; jt < sl.cols; jt += NTH) o[jt] = wa * a[jt] + wb * y[jt];
}

template <bool BT_ = false>
__global__ __launch_bounds__(ROW_WAVES * 64) void act_bwd_ce_row_kernel(const float* __restrict__ dact, int ldd,
                                                                        const float* __restrict__ act, int lda,
                                                                        const float* __restrict__ logits, int ldl,
                                                                        SpanTables sp, const int* __restrict__ col,
                                                                        const int* __restrict__ opt,
                                                                        float* __restrict__ dl, int ldg, int rows,
                                                                        float inv_tau, float* loss, int loss_per_row,
                                                                        ClientBatch cb) {
  const BIdx bi_ = batch_bidx<BT_>(cb.xcd);
  extern __shared__ float act_smem[];
  if (bi_.z) {
    const int64_t co = (int64_t)bi_.z * cb.stride;
    dact = cptr(dact, co);
    act = cptr(act, co);
    logits = cptr(logits, co);
    col = cptr(col, co);
    opt = cptr(opt, co);
    dl = cptr(dl, co);
    loss = cptr(loss, co);
    client_off(sp, co);
  }
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int r = bi_.x;
  const int D = sp.dim, S = sp.n_span;
  const float* g = dact + (size_t)r * ldd;
  const float* y = act + (size_t)r * lda;
  const float* x = logits + (size_t)r * ldl;
  const int cr = col[r];
  const int orow = opt[r];
  const ActSmem t = act_stage_tables(sp, act_smem);
  float* xs = t.rows;                                       // [D] the row's logits
  float* stat = xs + D;                                     // [S] per-span sum of g*y
  int* cspan = reinterpret_cast<int*>(stat + S);            // the conditioned span
  float* lse_sh = stat + S + 1;
  float* d = dl + (size_t)r * ldg;
  for (int s2 = tid; s2 < S; s2 += blockDim.x) stat[s2] = 0.f;
  if (tid == 0) *cspan = -1;
  __syncthreads();
  for (int s2 = tid; s2 < S; s2 += blockDim.x)
    if (t.kind[s2] != 0 && t.cidx[s2] == cr) *cspan = s2;   // exactly one span matches
  constexpr int U = 4;   // loads in flight per thread
  for (int c0 = 0; c0 < D; c0 += U * ROW_WAVES * 64) {
    float gc[U], yc[U], xc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = min(c0 + u * ROW_WAVES * 64 + tid, D - 1);
      gc[u] = g[j];
      yc[u] = y[j];
      xc[u] = x[j];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = c0 + u * ROW_WAVES * 64 + tid;
      if (j < D) {
        const int info = t.einfo[j];
        xs[j] = xc[u];
        if (info & EI_SOFTMAX) atomicAdd(&stat[info & (EI_SOFTMAX - 1)], gc[u] * yc[u]);
      }
    }
  }
  __syncthreads();
  const int cs = *cspan;
  int cst = 0, cw = 0;
  if (cs >= 0) {
    cst = t.start[cs];
    cw = t.width[cs];
  }
  if (wv == 0) {   // log-sum-exp over the conditioned span (one wave)
    float lse = 0.f;
    if (cs >= 0) {
      float m = -INFINITY;
      for (int i = lane; i < cw; i += 64) m = fmaxf(m, xs[cst + i]);
      m = wave_max(m);
      float sm = 0.f;
      for (int i = lane; i < cw; i += 64) sm += __expf(xs[cst + i] - m);
      sm = wave_sum(sm);
      lse = m + __logf(sm);
      if (lane == 0) {
        const float term = (lse - xs[cst + min(orow, cw - 1)]) / (float)rows;
        if (loss_per_row) loss[r] = term; else atomicAdd(loss, term);
      }
    } else if (lane == 0 && loss_per_row) {
      loss[r] = 0.f;
    }
    if (lane == 0) *lse_sh = lse;
  }
  __syncthreads();
  const float lse = *lse_sh;
  const int ot = cst + min(orow, max(cw - 1, 0));
  const float invB = 1.f / (float)rows;
  for (int c0 = 0; c0 < D; c0 += U * ROW_WAVES * 64) {
    float gc[U], yc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = min(c0 + u * ROW_WAVES * 64 + tid, D - 1);
      gc[u] = g[j];
      yc[u] = y[j];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = c0 + u * ROW_WAVES * 64 + tid;
      if (j < D) {
        const int info = t.einfo[j];
        float vv;
        if (!(info & EI_SOFTMAX)) {
          vv = gc[u] * (1.f - yc[u] * yc[u]);
        } else {
          vv = yc[u] * (gc[u] - stat[info & (EI_SOFTMAX - 1)]) * inv_tau;
          if (j >= cst && j < cst + cw) vv += (__expf(xs[j] - lse) - (j == ot ? 1.f : 0.f)) * invB;
        }
        d[j] = vv;
      }
    }
  }
}

// ---- register-resident backward (act_row_mode 2): a thread keeps its E elements (j = tid + 512 e) of the
// upstream gradient, the activation and the span map in registers from ONE burst of loads; the conditioned
// span's logits are read straight from global memory by one wave (a few dozen values, L2-resident).  The LDS
// kernel above stages the whole span table (D + 4S words, 44 KB on the wide table) per row and reads g / y twice.
template <int E, int NW = ROW_WAVES, bool BT_ = false>
__global__ __launch_bounds__(NW * 64) void act_bwd_ce_rowreg_kernel(const float* __restrict__ dact, int ldd,
                                                                           const float* __restrict__ act, int lda,
                                                                           const float* __restrict__ logits, int ldl,
                                                                           SpanTables sp, const int* __restrict__ col,
                                                                           const int* __restrict__ opt,
                                                                           float* __restrict__ dl, int ldg, int rows,
                                                                           float inv_tau, float* loss, int loss_per_row,
                                                                           ClientBatch cb) {
  const BIdx bi_ = batch_bidx<BT_>(cb.xcd);
  extern __shared__ float act_smem[];
  if (bi_.z) {
    const int64_t co = (int64_t)bi_.z * cb.stride;
    dact = cptr(dact, co);
    act = cptr(act, co);
    logits = cptr(logits, co);
    col = cptr(col, co);
    opt = cptr(opt, co);
    dl = cptr(dl, co);
    loss = cptr(loss, co);
    client_off(sp, co);
  }
  constexpr int NTH = NW * 64;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int r = bi_.x;
  const int D = sp.dim, S = sp.n_span;
  const float* g = dact + (size_t)r * ldd;
  const float* y = act + (size_t)r * lda;
  const float* x = logits + (size_t)r * ldl;
  const int* einfo = sp.packed;
  const int* kind = einfo + D;
  const int* start = kind + S;
  const int* width = start + S;
  const int* cidx = width + S;
  float gc[E], yc[E];
  int ic[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int j = min(tid + NTH * e, D - 1);
    gc[e] = g[j];
    yc[e] = y[j];
    ic[e] = einfo[j];
  }
  const int cr = col[r];
  const int orow = opt[r];
  float* gy = act_smem;                                     // [D] g*y of the softmax elements
  float* stat = gy + D;                                     // [S] per-span sum of g*y
  int* cspan = reinterpret_cast<int*>(stat + S);            // the conditioned span
  float* lse_sh = stat + S + 1;
  if (tid == 0) *cspan = -1;
#pragma unroll
  for (int e = 0; e < E; ++e)
    if (tid + NTH * e < D && (ic[e] & EI_SOFTMAX)) gy[tid + NTH * e] = gc[e] * yc[e];
  __syncthreads();
  // span-parallel sums (no per-element LDS atomics, see activate_rowreg_kernel)
  for (int s2 = tid; s2 < S; s2 += NTH) {
    if (kind[s2] == 0) continue;
    if (cidx[s2] == cr) *cspan = s2;                        // exactly one span matches
    const float* v = gy + start[s2];
    const int w = width[s2];
    float t0 = 0.f, t1 = 0.f;
    int i = 0;
    for (; i + 2 <= w; i += 2) {
      t0 += v[i];
      t1 += v[i + 1];
    }
    if (i < w) t0 += v[i];
    stat[s2] = t0 + t1;
  }
  __syncthreads();
  const int cs = *cspan;
  int cst = 0, cw = 0;
  if (cs >= 0) {
    cst = start[cs];
    cw = width[cs];
  }
  if (wv == 0) {   // log-sum-exp over the conditioned span (one wave, logits from L2)
    float lse = 0.f;
    if (cs >= 0) {
      float m = -INFINITY;
      for (int i = lane; i < cw; i += 64) m = fmaxf(m, x[cst + i]);
      m = wave_max(m);
      float sm = 0.f;
      for (int i = lane; i < cw; i += 64) sm += __expf(x[cst + i] - m);
      sm = wave_sum(sm);
      lse = m + __logf(sm);
      if (lane == 0) {
        const float term = (lse - x[cst + min(orow, cw - 1)]) / (float)rows;
        if (loss_per_row) loss[r] = term; else atomicAdd(loss, term);
      }
    } else if (lane == 0 && loss_per_row) {
      loss[r] = 0.f;
    }
    if (lane == 0) *lse_sh = lse;
  }
  __syncthreads();
  const float lse = *lse_sh;
  const int ot = cst + min(orow, max(cw - 1, 0));
  const float invB = 1.f / (float)rows;
  float* d = dl + (size_t)r * ldg;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int j = tid + NTH * e;
    if (j < D) {
      float vv;
      if (!(ic[e] & EI_SOFTMAX)) {
        vv = gc[e] * (1.f - yc[e] * yc[e]);
      } else {
        vv = yc[e] * (gc[e] - stat[ic[e] & (EI_SOFTMAX - 1)]) * inv_tau;
        if (j >= cst && j < cst + cw) vv += (__expf(x[j] - lse) - (j == ot ? 1.f : 0.f)) * invB;
      }
      d[j] = vv;
    }
  }
}

// LDS of the row kernels: tables + one row image [D + 2S] + ROW_WAVES * 3 reduction slots
static size_t act_row_smem_bytes(const SpanTables& sp) {
  return (size_t)span_packed_len(sp.dim, sp.n_span) * sizeof(int) +
         (size_t)(sp.dim + 2 * sp.n_span + 3 * ROW_WAVES) * sizeof(float);
}
static size_t act_row_fwd_smem_bytes(const SpanTables& sp) {   // activate_row_kernel: no staged tables
  return (size_t)(sp.dim + 2 * sp.n_span + 3 * ROW_WAVES) * sizeof(float);
}
static bool act_row_mode(const SpanTables& sp) { return sp.dim > ACT_PF * 64 && g_act_row_mode; }
// the register-resident row kernels: wide rows in act_row_mode 2, and -- g_act_rowreg_narrow -- narrow ones too
// (a row then gets 2-4 waves instead of the per-wave kernels' one; same Philox words, so the same draws)
int g_act_rowreg_narrow = 2;   // measured (profiles/knobs_step_r4.txt): 1: step 204.7 -> 201.0 us; 2: 200.7 -> 199.7 us, bench 16.62 -> 16.51 ms
static bool act_rowreg(const SpanTables& sp) {
  return g_act_row_mode == 2 && (sp.dim > ACT_PF * 64 || g_act_rowreg_narrow);
}

static size_t act_smem_bytes(const SpanTables& sp, int waves) {
  return (size_t)span_packed_len(sp.dim, sp.n_span) * sizeof(int) +
         (size_t)waves * (sp.dim + 2 * sp.n_span) * sizeof(float);
}

// wide tables (hundreds of columns, thousands of spans) get fewer rows per workgroup so the
// tables + row images still fit the 160 KiB LDS
static int act_waves(const SpanTables& sp) {
  for (int w = ACT_WAVES; w > 1; w /= 2)
    if (act_smem_bytes(sp, w) <= LDS_BYTES) return w;
  return 1;
}

template <typename K>
static void allow_big_lds(K kernel, size_t bytes) {
  if (bytes > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)bytes);
}

void launch_activate(const float* logits, int ldl, float* out, int ldo, int rows, SpanTables sp, float tau,
                     uint64_t seed, const uint64_t* ctr, uint32_t stream_id, SlerpFuse sl, hipStream_t stream) {
  if (rows == 0) return;
  const ClientBatch cb = client_batch();
  if (cb.k > 1) {
    check_slabs("activate operand", logits, out, ctr, sl.real, sl.out);
    check_slab(sp);
  }
  if (g_act_row_mode == 2 && g_act_rowreg_narrow == 2 && sp.dim <= ROW_WAVES * 64) {
    const int nb = (sp.dim + 63) / 64;
    const size_t lds = (size_t)(sp.dim + 2 * sp.n_span + 3 * ROW_WAVES) * sizeof(float);
    const dim3 grid(rows, 1, cb.k);
    const bool xcd = cb.xcd != 0;
    if (nb <= 4) {
      hipLaunchKernelGGL((xcd ? activate_rowblk_kernel<4, true> : activate_rowblk_kernel<4, false>), grid, dim3(256), lds,
                         stream, logits, ldl, out, ldo, rows, sp, 1.f / tau, seed, ctr, stream_id, sl, cb);
    } else {
      hipLaunchKernelGGL((xcd ? activate_rowblk_kernel<ROW_WAVES, true> : activate_rowblk_kernel<ROW_WAVES, false>), grid,
                         dim3(ROW_WAVES * 64), lds, stream, logits, ldl, out, ldo, rows, sp, 1.f / tau, seed, ctr,
                         stream_id, sl, cb);
    }
    return;
  }
  if (act_rowreg(sp)) {
    // register-resident row kernel: NW waves per row, GPW groups of 4 x 64 columns per wave
    const int ng = ((sp.dim + 63) / 64 + 3) / 4;
    const int nw = ng <= 2 ? 2 : (ng <= 4 ? 4 : ROW_WAVES), gpw = (ng + nw - 1) / nw;
    const size_t lds = (size_t)(sp.dim + 2 * sp.n_span + 3 * ROW_WAVES) * sizeof(float);
    const dim3 grid(rows, 1, cb.k), block(nw * 64);
    const bool xcd = cb.xcd != 0;
#define FEDTGAN_ACT_REG(G, W)                                                                                       \
  do {                                                                                                             \
    allow_big_lds(activate_rowreg_kernel<G, W, false>, lds);                                                       \
    allow_big_lds(activate_rowreg_kernel<G, W, true>, lds);                                                        \
    hipLaunchKernelGGL((xcd ? activate_rowreg_kernel<G, W, true> : activate_rowreg_kernel<G, W, false>), grid, block, \
                       lds, stream, logits, ldl, out, ldo, rows, sp, 1.f / tau, seed, ctr, stream_id, sl, cb);     \
    return;                                                                                                        \
  } while (0)
    if (nw == 2 && gpw <= 1) FEDTGAN_ACT_REG(1, 2);
    if (nw == 4 && gpw <= 1) FEDTGAN_ACT_REG(1, 4);
    if (nw == ROW_WAVES && gpw <= 2) FEDTGAN_ACT_REG(2, ROW_WAVES);
    if (nw == ROW_WAVES && gpw <= 4) FEDTGAN_ACT_REG(4, ROW_WAVES);
    if (nw == ROW_WAVES && gpw <= 8) FEDTGAN_ACT_REG(8, ROW_WAVES);
#undef FEDTGAN_ACT_REG
    // (wider rows: the LDS-image row kernel)
  }
  if (act_row_mode(sp)) {
    const size_t lds = act_row_fwd_smem_bytes(sp);
    allow_big_lds(activate_row_kernel<false>, lds);
    allow_big_lds(activate_row_kernel<true>, lds);
    hipLaunchKernelGGL((client_batch().xcd ? activate_row_kernel<true> : activate_row_kernel<false>), dim3(rows, 1, cb.k), dim3(ROW_WAVES * 64), lds, stream, logits, ldl, out,
                       ldo, rows, sp, 1.f / tau, seed, ctr, stream_id, sl, cb);
    return;
  }
  const int nw = act_waves(sp);
  const size_t lds = act_smem_bytes(sp, nw);
  allow_big_lds(activate_kernel<false>, lds);
    allow_big_lds(activate_kernel<true>, lds);
  hipLaunchKernelGGL((client_batch().xcd ? activate_kernel<true> : activate_kernel<false>), dim3((rows + nw - 1) / nw, 1, cb.k), dim3(nw * 64), lds, stream, logits, ldl, out,
                     ldo, rows, sp, 1.f / tau, seed, ctr, stream_id, sl, cb);
}

// backward of the activation + fused conditional cross-entropy, one wave per row; the per-span
// sums of g*y are LDS ds_add_f32 folds (no serial per-span loops)
template <bool BT_ = false>
__global__ __launch_bounds__(ACT_WAVES * 64) void act_bwd_ce_kernel(const float* __restrict__ dact, int ldd,
                                                                    const float* __restrict__ act, int lda,
                                                                    const float* __restrict__ logits, int ldl,
                                                                    SpanTables sp, const int* __restrict__ col,
                                                                    const int* __restrict__ opt, float* __restrict__ dl,
                                                                    int ldg, int rows, float inv_tau, float* loss,
                                                                    int loss_per_row, ClientBatch cb) {
  const BIdx bi_ = batch_bidx<BT_>(cb.xcd);
  extern __shared__ float act_smem[];
  if (bi_.z) {
    const int64_t co = (int64_t)bi_.z * cb.stride;
    dact = cptr(dact, co);
    act = cptr(act, co);
    logits = cptr(logits, co);
    col = cptr(col, co);
    opt = cptr(opt, co);
    dl = cptr(dl, co);
    loss = cptr(loss, co);
    client_off(sp, co);
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r = bi_.x * (int)(blockDim.x >> 6) + wv;
  const int rc = min(r, rows - 1);
  const int D = sp.dim, S = sp.n_span;
  const float* g = dact + (size_t)rc * ldd;
  const float* y = act + (size_t)rc * lda;
  const float* x = logits + (size_t)rc * ldl;
  // the row's gradients, activations and logits (and its conditional column) are requested
  // before the span tables are staged: one overlapped round trip instead of three
  const bool pre = D <= ACT_PF * 64;
  float gr[ACT_PF], yr[ACT_PF], xr[ACT_PF];
#pragma unroll
  for (int k = 0; k < ACT_PF; ++k) {
    const int j = min(lane + 64 * k, D - 1);
    gr[k] = pre ? g[j] : 0.f;
    yr[k] = pre ? y[j] : 0.f;
    xr[k] = pre ? x[j] : 0.f;
  }
  const int cr = col[rc];
  const int orow = opt[rc];
  const ActSmem t = act_stage_tables(sp, act_smem);
  if (r >= rows) return;
  float* xs = t.rows + (size_t)wv * (D + 2 * S);         // [D] the row's logits (for the CE's LSE)
  float* stat = xs + D;                                  // [S] per-span sum of g*y
  float* d = dl + (size_t)r * ldg;
  for (int s2 = lane; s2 < S; s2 += 64) stat[s2] = 0.f;
  // the conditioned span of this row (exactly one lane finds it)
  int ce_span = -1;
  for (int s2 = lane; s2 < S; s2 += 64)
    if (t.kind[s2] != 0 && t.cidx[s2] == cr) ce_span = s2;
  wave_lds_sync();
  auto fold = [&](int j, float gj, float yj, float xj) {
    const int info = t.einfo[j];
    xs[j] = xj;
    if (info & EI_SOFTMAX) atomicAdd(&stat[info & (EI_SOFTMAX - 1)], gj * yj);
  };
  if (pre) {
#pragma unroll
    for (int k = 0; k < ACT_PF; ++k)
      if (lane + 64 * k < D) fold(lane + 64 * k, gr[k], yr[k], xr[k]);
  } else {
    for (int c0 = 0; c0 < D; c0 += ACT_PF * 64) {   // chunked: one round trip per 512 columns
      float gc[ACT_PF], yc[ACT_PF], xc[ACT_PF];
#pragma unroll
      for (int k = 0; k < ACT_PF; ++k) {
        const int j = min(c0 + lane + 64 * k, D - 1);
        gc[k] = g[j];
        yc[k] = y[j];
        xc[k] = x[j];
      }
#pragma unroll
      for (int k = 0; k < ACT_PF; ++k)
        if (c0 + lane + 64 * k < D) fold(c0 + lane + 64 * k, gc[k], yc[k], xc[k]);
    }
  }
  wave_lds_sync();
  // wave-parallel log-sum-exp over the conditioned span
  const unsigned long long who = __ballot(ce_span >= 0);
  int cst = 0, cw = 0;
  float lse = 0.f;
  if (who) {
    const int src = __ffsll((long long)who) - 1;
    const int cs = __shfl(ce_span, src, 64);
    cst = t.start[cs];
    cw = t.width[cs];
    float m = -INFINITY;
    for (int i = lane; i < cw; i += 64) m = fmaxf(m, xs[cst + i]);
    m = wave_max(m);
    float sm = 0.f;
    for (int i = lane; i < cw; i += 64) sm += __expf(xs[cst + i] - m);
    sm = wave_sum(sm);
    lse = m + __logf(sm);
    const int o = min(orow, cw - 1);
    if (lane == 0) {
      const float term = (lse - xs[cst + o]) / (float)rows;
      // per-row terms are summed by a later column-sum launch: hundreds of same-address device
      // atomics serialise at the memory-side atomic unit
      if (loss_per_row) loss[r] = term; else atomicAdd(loss, term);
    }
  } else if (lane == 0 && loss_per_row) {
    loss[r] = 0.f;
  }
  wave_lds_sync();
  const int ot = cst + min(orow, max(cw - 1, 0));
  const float invB = 1.f / (float)rows;
  auto grad_elem = [&](int j, float gj, float yj, float xj) {
    const int info = t.einfo[j];
    float v;
    if (!(info & EI_SOFTMAX)) {
      v = gj * (1.f - yj * yj);
    } else {
      v = yj * (gj - stat[info & (EI_SOFTMAX - 1)]) * inv_tau;
      if (j >= cst && j < cst + cw) v += (__expf(xj - lse) - (j == ot ? 1.f : 0.f)) * invB;
    }
    d[j] = v;
  };
  if (pre) {
#pragma unroll
    for (int k = 0; k < ACT_PF; ++k)
      if (lane + 64 * k < D) grad_elem(lane + 64 * k, gr[k], yr[k], xr[k]);
  } else {
    for (int c0 = 0; c0 < D; c0 += ACT_PF * 64) {
      float gc[ACT_PF], yc[ACT_PF];
#pragma unroll
      for (int k = 0; k < ACT_PF; ++k) {
        const int j = min(c0 + lane + 64 * k, D - 1);
        gc[k] = g[j];
        yc[k] = y[j];
      }
#pragma unroll
      for (int k = 0; k < ACT_PF; ++k) {
        const int j = c0 + lane + 64 * k;
        if (j < D) grad_elem(j, gc[k], yc[k], xs[j]);    // logits from the LDS copy
      }
    }
  }
}

void launch_act_bwd_ce(const float* dact, int ldd, const float* act, int lda, const float* logits, int ldl, SpanTables sp,
                       const int* col, const int* opt, float* dlogits, int ldg, int rows, float tau, float* loss,
                       int loss_per_row, hipStream_t stream) {
  if (rows == 0) return;
  const ClientBatch cb = client_batch();
  if (cb.k > 1) {
    check_slabs("act_bwd_ce operand", dact, act, logits, col, opt, dlogits, loss);
    check_slab(sp);
  }
  if (act_rowreg(sp)) {
    const int ng = ((sp.dim + 63) / 64 + 3) / 4;
    const int nw = (g_act_rowreg_narrow == 2 || ng > 4) ? ROW_WAVES : (ng <= 2 ? 2 : 4);
    const int ept = (sp.dim + nw * 64 - 1) / (nw * 64);   // elements per thread
    const size_t lds = (size_t)(sp.dim + sp.n_span + 2) * sizeof(float);
    const dim3 grid(rows, 1, cb.k), block(nw * 64);
    const bool xcd = cb.xcd != 0;
#define FEDTGAN_BWD_REG(E, W)                                                                                          \
  do {                                                                                                                \
    allow_big_lds(act_bwd_ce_rowreg_kernel<E, W, false>, lds);                                                        \
    allow_big_lds(act_bwd_ce_rowreg_kernel<E, W, true>, lds);                                                         \
    hipLaunchKernelGGL((xcd ? act_bwd_ce_rowreg_kernel<E, W, true> : act_bwd_ce_rowreg_kernel<E, W, false>), grid, block, \
                       lds, stream, dact, ldd, act, lda, logits, ldl, sp, col, opt, dlogits, ldg, rows, 1.f / tau, loss, \
                       loss_per_row, cb);                                                                             \
    return;                                                                                                           \
  } while (0)
    if (nw == 2 && ept <= 4) FEDTGAN_BWD_REG(4, 2);
    if (nw == 4 && ept <= 4) FEDTGAN_BWD_REG(4, 4);
    if (nw == ROW_WAVES && ept <= 1) FEDTGAN_BWD_REG(1, ROW_WAVES);
    if (nw == ROW_WAVES && ept <= 8) FEDTGAN_BWD_REG(8, ROW_WAVES);
    if (nw == ROW_WAVES && ept <= 16) FEDTGAN_BWD_REG(16, ROW_WAVES);
    if (nw == ROW_WAVES && ept <= 32) FEDTGAN_BWD_REG(32, ROW_WAVES);
#undef FEDTGAN_BWD_REG
  }
  if (act_row_mode(sp)) {
    const size_t lds = act_row_smem_bytes(sp);
    allow_big_lds(act_bwd_ce_row_kernel<false>, lds);
    allow_big_lds(act_bwd_ce_row_kernel<true>, lds);
    hipLaunchKernelGGL((client_batch().xcd ? act_bwd_ce_row_kernel<true> : act_bwd_ce_row_kernel<false>), dim3(rows, 1, cb.k), dim3(ROW_WAVES * 64), lds, stream, dact, ldd, act,
                       lda, logits, ldl, sp, col, opt, dlogits, ldg, rows, 1.f / tau, loss, loss_per_row, cb);
    return;
  }
  const int nw = act_waves(sp);
  const size_t lds = act_smem_bytes(sp, nw);
  allow_big_lds(act_bwd_ce_kernel<false>, lds);
    allow_big_lds(act_bwd_ce_kernel<true>, lds);
  hipLaunchKernelGGL((client_batch().xcd ? act_bwd_ce_kernel<true> : act_bwd_ce_kernel<false>), dim3((rows + nw - 1) / nw, 1, cb.k), dim3(nw * 64), lds, stream, dact, ldd, act,
                     lda, logits, ldl, sp, col, opt, dlogits, ldg, rows, 1.f / tau, loss, loss_per_row, cb);
}

size_t activation_smem_bytes(const SpanTables& sp) {
  return act_row_mode(sp) ? act_row_smem_bytes(sp) : act_smem_bytes(sp, act_waves(sp));
}

// ============================================================================ gradient penalty pieces
// one wave per row
template <bool BT_ = false>
__global__ __launch_bounds__(256) void slerp_kernel(const float* __restrict__ real, const float* __restrict__ fake,
                                                    float* __restrict__ out, int rows, int cols, int ld, uint64_t seed,
                                                    const uint64_t* ctr, uint32_t stream_id, ClientBatch cb) {
  const BIdx bi_ = batch_bidx<BT_>(cb.xcd);
  if (bi_.z) {
    const int64_t co = (int64_t)bi_.z * cb.stride;
    real = cptr(real, co);
    fake = cptr(fake, co);
    out = cptr(out, co);
    ctr = cptr(ctr, co);
    seed += (uint64_t)bi_.z * cb.seed_step;
  }
  const int lane = threadIdx.x & 63;
  const int r = bi_.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (r >= rows) return;
  const float* a = real + (size_t)r * ld;
  const float* b = fake + (size_t)r * ld;
  float saa = 0.f, sbb = 0.f, sab = 0.f;
  for (int i = lane; i < cols; i += 64) {
    const float x = a[i], y = b[i];
    saa += x * x; sbb += y * y; sab += x * y;
  }
  saa = wave_sum(saa); sbb = wave_sum(sbb); sab = wave_sum(sab);
  const uint64_t step = ctr ? *ctr : 0ull;
  RngArgs rng{seed, ctr, stream_id};
  const float alpha = u01(rng4(rng, step, (uint64_t)r).x);
  float wa, wb;
  slerp_weights(saa, sbb, sab, alpha, wa, wb);
  float* o = out + (size_t)r * ld;
  for (int i = lane; i < cols; i += 64) o[i] = wa * a[i] + wb * b[i];
}

void launch_slerp(const float* real, const float* fake, float* out, int rows, int cols, int ld, uint64_t seed,
                  const uint64_t* ctr, uint32_t stream_id, hipStream_t stream) {
  if (rows == 0) return;
  const ClientBatch cb = client_batch();
  if (cb.k > 1) check_slabs("slerp operand", real, fake, out, ctr);
  hipLaunchKernelGGL((client_batch().xcd ? slerp_kernel<true> : slerp_kernel<false>), dim3((rows + 3) / 4, 1, cb.k), dim3(256), 0, stream, real, fake, out, rows, cols, ld,
                     seed, ctr, stream_id, cb);
}

// one workgroup per packed row.  The vector variant keeps the whole row in registers (up to
// GP_V4 float4 per thread, loaded in one burst), so the row is read once: norm, then scale.
typedef __attribute__((ext_vector_type(4))) float f32x4;
constexpr int GP_V4 = 8;    // rows up to 8 * 256 * 4 = 8192 wide stay in registers
int g_gp_split = 1;          // wider rows: chunk-split two-launch path when given a workspace (set_tuning("gp_split"))
int g_gp_threads = 256;      // workgroup size of the register-resident gp_scale (256, or 1024 for rows <= 8192; A/B knob)

__device__ __forceinline__ void gp_finish(int r, float s, int rows, float lam, float* loss, int loss_per_row,
                                          float* sh, float& coef) {
  s = block_sum(s, sh);
  const float n = sqrtf(s);
  coef = lam * 2.f * (n - 1.f) / (fmaxf(n, 1e-30f) * (float)rows);
  if (threadIdx.x == 0) {
    const float term = lam * (n - 1.f) * (n - 1.f) / (float)rows;
    if (loss_per_row) loss[r] = term; else atomicAdd(loss, term);
  }
}

template <bool BT_ = false, int NTH = 256, int V = GP_V4>
__global__ __launch_bounds__(NTH) void gp_scale_v4_kernel(const float* __restrict__ g, int ldg, float* __restrict__ out,
                                                          int ldo, int rows, int cols, float lam, float* loss,
                                                          int loss_per_row, ClientBatch cb) {
  const BIdx bi_ = batch_bidx<BT_>(cb.xcd);
  if (bi_.z) {
    const int64_t co = (int64_t)bi_.z * cb.stride;
    g = cptr(g, co);
    out = cptr(out, co);
    loss = cptr(loss, co);
  }
  __shared__ float sh[NTH / 64];
  const int r = bi_.x;
  const f32x4* x = reinterpret_cast<const f32x4*>(g + (size_t)r * ldg);
  const int n4 = cols / 4;
  f32x4 v[V];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < V; ++i) v[i] = x[min((int)threadIdx.x + NTH * i, n4 - 1)];
#pragma unroll
  for (int i = 0; i < V; ++i)
    if ((int)threadIdx.x + NTH * i < n4) s += v[i][0] * v[i][0] + v[i][1] * v[i][1] + v[i][2] * v[i][2] + v[i][3] * v[i][3];
  float coef;
  gp_finish(r, s, rows, lam, loss, loss_per_row, sh, coef);
  f32x4* o = reinterpret_cast<f32x4*>(out + (size_t)r * ldo);
#pragma unroll
  for (int i = 0; i < V; ++i)
    if ((int)threadIdx.x + NTH * i < n4) o[threadIdx.x + NTH * i] = v[i] * coef;
}

template <bool BT_ = false>
__global__ __launch_bounds__(256) void gp_scale_kernel(const float* __restrict__ g, int ldg, float* __restrict__ out,
                                                       int ldo, int rows, int cols, float lam, float* loss,
                                                       int loss_per_row, ClientBatch cb) {
  const BIdx bi_ = batch_bidx<BT_>(cb.xcd);
  if (bi_.z) {
    const int64_t co = (int64_t)bi_.z * cb.stride;
    g = cptr(g, co);
    out = cptr(out, co);
    loss = cptr(loss, co);
  }
  __shared__ float sh[8];
  const int r = bi_.x;
  const float* x = g + (size_t)r * ldg;
  float s0 = 0.f, s1 = 0.f;
  int i = threadIdx.x;
  for (; i + (int)blockDim.x < cols; i += 2 * blockDim.x) {
    const float u = x[i], w = x[i + blockDim.x];
    s0 += u * u;
    s1 += w * w;
  }
  if (i < cols) s0 += x[i] * x[i];
  float coef;
  gp_finish(r, s0 + s1, rows, lam, loss, loss_per_row, sh, coef);
  float* o = out + (size_t)r * ldo;
  for (int i = threadIdx.x; i < cols; i += blockDim.x) o[i] = coef * x[i];
}

// rows wider than the register-resident variant: two passes over the row in chunks of
// GP_V4 float4 per thread, each chunk's loads issued together
template <bool BT_ = false>
__global__ __launch_bounds__(256) void gp_scale_v4_wide_kernel(const float* __restrict__ g, int ldg,
                                                               float* __restrict__ out, int ldo, int rows, int cols,
                                                               float lam, float* loss, int loss_per_row, ClientBatch cb) {
  const BIdx bi_ = batch_bidx<BT_>(cb.xcd);
  if (bi_.z) {
    const int64_t co = (int64_t)bi_.z * cb.stride;
    g = cptr(g, co);
    out = cptr(out, co);
    loss = cptr(loss, co);
  }
  __shared__ float sh[8];
  const int r = bi_.x;
  const f32x4* x = reinterpret_cast<const f32x4*>(g + (size_t)r * ldg);
  const int n4 = cols / 4;
  float s = 0.f;
  for (int c0 = 0; c0 < n4; c0 += GP_V4 * 256) {
    f32x4 v[GP_V4];
#pragma unroll
    for (int i = 0; i < GP_V4; ++i) v[i] = x[min(c0 + (int)threadIdx.x + 256 * i, n4 - 1)];
#pragma unroll
    for (int i = 0; i < GP_V4; ++i)
      if (c0 + (int)threadIdx.x + 256 * i < n4)
        s += v[i][0] * v[i][0] + v[i][1] * v[i][1] + v[i][2] * v[i][2] + v[i][3] * v[i][3];
  }
  float coef;
  gp_finish(r, s, rows, lam, loss, loss_per_row, sh, coef);
  f32x4* o = reinterpret_cast<f32x4*>(out + (size_t)r * ldo);
  for (int c0 = 0; c0 < n4; c0 += GP_V4 * 256) {
    f32x4 v[GP_V4];
#pragma unroll
    for (int i = 0; i < GP_V4; ++i) v[i] = x[min(c0 + (int)threadIdx.x + 256 * i, n4 - 1)];
#pragma unroll
    for (int i = 0; i < GP_V4; ++i)
      if (c0 + (int)threadIdx.x + 256 * i < n4) o[c0 + threadIdx.x + 256 * i] = v[i] * coef;
  }
}

// rows wider than the register-resident variant, split over chunks of GP_V4 * 256 float4 (the wide table's 50
// packed rows of 137,800: 17 chunks each -> 850 workgroups instead of 50): partial sums of squares per chunk into a
// workspace, then every chunk's workgroup sums its row's partials in chunk order (deterministic) and scales.
constexpr int GP_CH4 = GP_V4 * 256;   // float4 per chunk

template <bool BT_ = false>
__global__ __launch_bounds__(256) void gp_partial_kernel(const float* __restrict__ g, int ldg, int cols,
                                                         float* __restrict__ part, ClientBatch cb) {
  const BIdx bi_ = batch_bidx<BT_>(cb.xcd);
  if (bi_.z) {
    const int64_t co = (int64_t)bi_.z * cb.stride;
    g = cptr(g, co);
    part = cptr(part, co);
  }
  __shared__ float sh[8];
  const int c = bi_.x, r = bi_.y, nch = gridDim.x;
  const f32x4* x = reinterpret_cast<const f32x4*>(g + (size_t)r * ldg);
  const int n4 = cols / 4, c0 = c * GP_CH4;
  f32x4 v[GP_V4];
#pragma unroll
  for (int i = 0; i < GP_V4; ++i) v[i] = x[min(c0 + (int)threadIdx.x + 256 * i, n4 - 1)];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < GP_V4; ++i)
    if (c0 + (int)threadIdx.x + 256 * i < n4) s += v[i][0] * v[i][0] + v[i][1] * v[i][1] + v[i][2] * v[i][2] + v[i][3] * v[i][3];
  s = block_sum(s, sh);
  if (threadIdx.x == 0) part[(size_t)r * nch + c] = s;
}

template <bool BT_ = false>
__global__ __launch_bounds__(256) void gp_apply_kernel(const float* __restrict__ g, int ldg, float* __restrict__ out,
                                                       int ldo, int rows, int cols, float lam, float* loss,
                                                       int loss_per_row, const float* __restrict__ part, ClientBatch cb) {
  const BIdx bi_ = batch_bidx<BT_>(cb.xcd);
  if (bi_.z) {
    const int64_t co = (int64_t)bi_.z * cb.stride;
    g = cptr(g, co);
    out = cptr(out, co);
    loss = cptr(loss, co);
    part = cptr(part, co);
  }
  const int c = bi_.x, r = bi_.y, nch = gridDim.x;
  const f32x4* x = reinterpret_cast<const f32x4*>(g + (size_t)r * ldg);
  const int n4 = cols / 4, c0 = c * GP_CH4;
  f32x4 v[GP_V4];
#pragma unroll
  for (int i = 0; i < GP_V4; ++i) v[i] = x[min(c0 + (int)threadIdx.x + 256 * i, n4 - 1)];
  float s = 0.f;
  for (int k = 0; k < nch; ++k) s += part[(size_t)r * nch + k];   // (uniform: every thread, chunk order)
  const float nrm = sqrtf(s);
  const float coef = lam * 2.f * (nrm - 1.f) / (fmaxf(nrm, 1e-30f) * (float)rows);
  if (c == 0 && threadIdx.x == 0) {
    const float term = lam * (nrm - 1.f) * (nrm - 1.f) / (float)rows;
    if (loss_per_row) loss[r] = term; else atomicAdd(loss, term);
  }
  f32x4* o = reinterpret_cast<f32x4*>(out + (size_t)r * ldo);
#pragma unroll
  for (int i = 0; i < GP_V4; ++i)
    if (c0 + (int)threadIdx.x + 256 * i < n4) o[c0 + threadIdx.x + 256 * i] = v[i] * coef;
}

void launch_gp_scale(const float* g, int ldg, float* out, int ldo, int rows, int cols, float lam, float* loss,
                     int loss_per_row, float* ws, int64_t ws_n, hipStream_t stream) {
  if (rows == 0) return;
  const ClientBatch cb = client_batch();
  if (cb.k > 1) check_slabs("gp_scale operand", g, out, loss);
  // (16-B alignment of client c's rows follows from client 0's: the slab stride is a multiple of 256 B)
  const bool al = cols % 4 == 0 && ldg % 4 == 0 && ldo % 4 == 0 && reinterpret_cast<uintptr_t>(g) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(out) % 16 == 0;
  const bool v4 = al && cols <= GP_V4 * 256 * 4;
  const dim3 grid(rows, 1, cb.k);
  const int nch = (cols / 4 + GP_CH4 - 1) / GP_CH4;
  if (al && !v4 && ws != nullptr && ws_n >= (int64_t)rows * nch && g_gp_split) {
    if (cb.k > 1) check_slabs("gp_scale workspace", ws);
    const dim3 g2(nch, rows, cb.k);
    hipLaunchKernelGGL((cb.xcd ? gp_partial_kernel<true> : gp_partial_kernel<false>), g2, dim3(256), 0, stream, g, ldg,
                       cols, ws, cb);
    hipLaunchKernelGGL((cb.xcd ? gp_apply_kernel<true> : gp_apply_kernel<false>), g2, dim3(256), 0, stream, g, ldg, out,
                       ldo, rows, cols, lam, loss, loss_per_row, ws, cb);
  } else if (al && !v4)
    hipLaunchKernelGGL((client_batch().xcd ? gp_scale_v4_wide_kernel<true> : gp_scale_v4_wide_kernel<false>), grid, dim3(256), 0, stream, g, ldg, out, ldo, rows, cols, lam, loss,
                       loss_per_row, cb);
  else if (v4 && g_gp_threads == 1024 && cols / 4 <= 2 * 1024)
    hipLaunchKernelGGL((cb.xcd ? gp_scale_v4_kernel<true, 1024, 2> : gp_scale_v4_kernel<false, 1024, 2>), grid, dim3(1024), 0,
                       stream, g, ldg, out, ldo, rows, cols, lam, loss, loss_per_row, cb);
  else if (v4)
    hipLaunchKernelGGL((client_batch().xcd ? gp_scale_v4_kernel<true> : gp_scale_v4_kernel<false>), grid, dim3(256), 0, stream, g, ldg, out, ldo, rows, cols, lam, loss,
                       loss_per_row, cb);
  else
    hipLaunchKernelGGL((client_batch().xcd ? gp_scale_kernel<true> : gp_scale_kernel<false>), grid, dim3(256), 0, stream, g, ldg, out, ldo, rows, cols, lam, loss,
                       loss_per_row, cb);
}

// ============================================================================ one-hot block weight gradient
// Workgroup (r, job): the batch's condition indices are staged in LDS; the workgroup of the FIRST row holding
// index k sums every row with index k in batch order and writes block row k (later rows with the same index
// exit).  With zero != 0 every workgroup clears its row's block row (duplicates store the same zeros).
// The wide table's G.out weight gradient is [7,402 x 7,018] of which the condition block is 6,762 rows: a dense
// GEMM multiplies 500 one-hot rows through it (52 GFLOP, 190 MB of mostly-zero output per step); here at most
// 500 rows of 7,018 floats are written and cleared.
template <bool BT_ = false>
__global__ __launch_bounds__(256) void onehot_wgrad_kernel(OnehotWBatch bt, int zero, ClientBatch cb) {
  const BIdx bi_ = batch_bidx<BT_>(cb.xcd);
  extern __shared__ int oh_smem[];
  OnehotWJob jb = bt.jobs[bi_.y];
  if (bi_.z) {
    const int64_t co = (int64_t)bi_.z * cb.stride;
    jb.dy = cptr(jb.dy, co);
    jb.w = cptr(jb.w, co);
    bt.col = cptr(bt.col, co);
    bt.opt = cptr(bt.opt, co);
    bt.cond_off = cptr(bt.cond_off, co);
  }
  const int r = bi_.x, B = bt.B, tid = threadIdx.x;
  const int my = bt.cond_off[bt.col[r]] + bt.opt[r];
  if (zero) {
    float* w = jb.w + (size_t)my * jb.ldw;
    for (int o = tid; o < jb.n; o += 256) w[o] = 0.f;
    return;
  }
  int* idx = oh_smem;            // [B] condition index of every row
  int* list = oh_smem + B;       // [B] rows holding this workgroup's index, in batch order
  int* flag = oh_smem + 2 * B;   // [2] an earlier row holds it | list length
  if (tid == 0) flag[0] = 0;
  for (int i = tid; i < B; i += 256) idx[i] = bt.cond_off[bt.col[i]] + bt.opt[i];
  __syncthreads();
  for (int i = tid; i < r; i += 256)
    if (idx[i] == my) flag[0] = 1;
  __syncthreads();
  if (flag[0]) return;           // (uniform) another workgroup owns this block row
  if (tid < 64) {                // one wave compacts rows r.. with index `my`, in order
    int cnt = 0;
    for (int i0 = r; i0 < B; i0 += 64) {
      const int i = i0 + tid;
      const bool hit = i < B && idx[i] == my;
      const unsigned long long m = __ballot(hit);
      if (hit) list[cnt + __popcll(m & ((1ull << tid) - 1ull))] = i;
      cnt += __popcll(m);
    }
    if (tid == 0) flag[1] = cnt;
  }
  __syncthreads();
  const int cnt = flag[1];
  float* w = jb.w + (size_t)my * jb.ldw;
  constexpr int U = 4;           // independent columns in flight per thread
  for (int o0 = tid; o0 < jb.n; o0 += 256 * U) {
    float acc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] = 0.f;
    for (int q = 0; q < cnt; ++q) {
      const float* src = jb.dy + (size_t)list[q] * jb.ldy;
#pragma unroll
      for (int u = 0; u < U; ++u) acc[u] += src[min(o0 + 256 * u, jb.n - 1)];
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (o0 + 256 * u < jb.n) w[o0 + 256 * u] = acc[u];
  }
}

void launch_onehot_wgrad(const OnehotWBatch& bt0, int zero, hipStream_t stream) {
  OnehotWBatch bt = bt0;
  bt.n_jobs = std::min(bt.n_jobs, 4);
  if (bt.n_jobs <= 0 || bt.B <= 0) return;
  const ClientBatch cb = client_batch();
  if (cb.k > 1) {
    check_slabs("onehot_wgrad operand", bt.col, bt.opt, bt.cond_off);
    for (int j = 0; j < bt.n_jobs; ++j) check_slabs("onehot_wgrad job", bt.jobs[j].dy, bt.jobs[j].w);
  }
  const size_t lds = zero ? 0 : (size_t)(2 * bt.B + 2) * sizeof(int);
  allow_big_lds(onehot_wgrad_kernel<false>, lds);
  allow_big_lds(onehot_wgrad_kernel<true>, lds);
  hipLaunchKernelGGL((cb.xcd ? onehot_wgrad_kernel<true> : onehot_wgrad_kernel<false>), dim3(bt.B, bt.n_jobs, cb.k),
                     dim3(256), lds, stream, bt, zero, cb);
}

// one wave per row: y = d.v + e ; a = coef * v * ms ; loss += wloss * y
__global__ __launch_bounds__(256) void d_head_kernel(const float* __restrict__ d, int ldd, const float* __restrict__ ms,
                                                     int ldms, const float* __restrict__ v, const float* __restrict__ e,
                                                     const float* __restrict__ coef, const float* __restrict__ wloss,
                                                     float* __restrict__ y, float* __restrict__ a, int lda, int rows,
                                                     int cols, float* loss) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (r >= rows) return;
  const float* dr = d + (size_t)r * ldd;
  const float* mr = ms + (size_t)r * ldms;
  float* ar = a + (size_t)r * lda;
  const float c = coef[r];
  float s = 0.f;
  for (int i = lane; i < cols; i += 64) {
    const float vi = v[i];
    s += dr[i] * vi;
    ar[i] = c * vi * mr[i];
  }
  s = wave_sum(s) + e[0];
  if (lane == 0) {
    y[r] = s;
    const float wl = wloss[r];
    if (wl != 0.f) atomicAdd(loss, wl * s);
  }
}

void launch_d_head(const float* d, int ldd, const float* ms, int ldms, const float* v, const float* e,
                   const float* coef, const float* wloss, float* y, float* a, int lda, int rows, int cols, float* loss,
                   hipStream_t stream) {
  if (rows == 0) return;
  require_unbatched("d_head");
  hipLaunchKernelGGL(d_head_kernel, dim3((rows + 3) / 4), dim3(256), 0, stream, d, ldd, ms, ldms, v, e, coef, wloss, y,
                     a, lda, rows, cols, loss);
}

// ============================================================================ column sums (bias grads)
constexpr int CS_COLS = 64, CS_GROUPS = 16;
struct ColsumBatch {
  ColsumJob jobs[8];
  int n_jobs;
};

template <bool BT_ = false>
__global__ __launch_bounds__(CS_COLS* CS_GROUPS) void colsum_kernel(ColsumBatch bt, ClientBatch cb) {
  const BIdx bi_ = batch_bidx<BT_>(cb.xcd);
  __shared__ float part[2][CS_GROUPS][CS_COLS + 1];
  const ColsumJob jb = client_job(bt.jobs[bi_.y], (int64_t)bi_.z * cb.stride);
  const int c = bi_.x * CS_COLS + (threadIdx.x % CS_COLS);
  const int grp = threadIdx.x / CS_COLS;
  if ((int)(bi_.x * CS_COLS) >= jb.cols) return;
  const int cc = min(c, jb.cols - 1);
  const float* uw = jb.dot_w ? jb.dot_w : jb.w;   // the dot's row weights
  float s = 0.f, s2 = 0.f;
#pragma unroll 8
  for (int r = grp; r < jb.rows; r += CS_GROUPS) {
    const float a = jb.a[(size_t)r * jb.lda + cc];
    s += (jb.w ? jb.w[r] : 1.f) * a;
    if (jb.dot_w) s2 += jb.dot_w[r] * a;
  }
  part[0][grp][threadIdx.x % CS_COLS] = s;
  part[1][grp][threadIdx.x % CS_COLS] = s2;
  __syncthreads();
  if (grp == 0) {   // one wave: the block's 64 columns
    float t = 0.f, t2 = 0.f;
    for (int i = 0; i < CS_GROUPS; ++i) {
      t += part[0][i][threadIdx.x];
      t2 += part[1][i][threadIdx.x];
    }
    if (c < jb.cols && jb.out) jb.out[c] = t;
    if (jb.dot_v) {
      float d = c < jb.cols ? (jb.dot_w ? t2 : t) * jb.dot_v[c] : 0.f;
      if (bi_.x == 0 && jb.dot_e) {   // + e * sum_r u[r], once per job
        float ws = 0.f;
        for (int r = threadIdx.x; r < jb.rows; r += 64) ws += uw ? uw[r] : 1.f;
        d += wave_sum(ws) * (threadIdx.x == 0 ? jb.dot_e[0] : 0.f);
      }
      d = wave_sum(d);
      if (threadIdx.x == 0) atomicAdd(jb.dot_out, d);
    }
  }
}

void launch_colsum(const ColsumJob* jobs, int n_jobs, hipStream_t stream) {
  ColsumBatch bt{};
  int maxc = 0;
  n_jobs = std::min(n_jobs, 8);
  for (int i = 0; i < n_jobs; ++i) {
    bt.jobs[i] = jobs[i];
    maxc = std::max(maxc, jobs[i].cols);
  }
  bt.n_jobs = n_jobs;
  if (n_jobs == 0 || maxc == 0) return;
  const ClientBatch cb = client_batch();
  if (cb.k > 1)
    for (int i = 0; i < n_jobs; ++i)
      check_slabs("colsum job", bt.jobs[i].a, bt.jobs[i].out, bt.jobs[i].w, bt.jobs[i].dot_v, bt.jobs[i].dot_e,
                  bt.jobs[i].dot_out, bt.jobs[i].dot_w);
  hipLaunchKernelGGL((client_batch().xcd ? colsum_kernel<true> : colsum_kernel<false>), dim3((maxc + CS_COLS - 1) / CS_COLS, n_jobs, cb.k), dim3(CS_COLS * CS_GROUPS), 0,
                     stream, bt, cb);
}

// ============================================================================ batch norm + relu
// One 512-thread workgroup owns COLS columns; its 512/COLS row-groups keep up to MAXR rows per
// thread in registers, so statistics, normalisation and the backward need a single pass over
// global memory.  Column reductions are wave64 butterflies (shfl_xor over the row-groups of a
// wave) followed by one 8-entry LDS combine across the waves -- no serial LDS scans.
// Loads use clamped (always valid) addresses and are masked afterwards (no predicated loads).
constexpr int BN_THREADS = 512, BN_WAVES = BN_THREADS / 64;
int g_bn_cols = 8;    // columns per workgroup (tuning knob, see set_tuning)
int g_bn_threads = 512;   // threads per BN workgroup: 512, or 1024 (half the rows per thread; set_tuning("bn_threads"))
// (16 columns for batched launches measured +1.0 ms per 8-client epoch once the clients sit on their own XCDs:
// 47.7 vs 48.7 ms, profiles/batched_r4.md; 8 everywhere)
static int bn_cols_for_launch() { return g_bn_cols; }

// ``groups`` (1 or 2) independent batches of rows/groups consecutive rows each: the D-phase and
// G-phase batches of a step go through the generator as ONE M = 2B GEMM chain, but BatchNorm keeps
// per-batch statistics (`ctgan.py:40-44` runs twice per step) and the running statistics are
// updated batch after batch, in row order -- exactly the reference's two forward passes.
constexpr int BN_MAXG = 2;

// sum over every row-group of the workgroup for this thread's column; NV values at once.
// sh: [NV][BN_WAVES][COLS] LDS; ends with a barrier so sh can be reused right away.
template <int COLS, int NV, int NTH = BN_THREADS>
__device__ __forceinline__ void bn_colsum(float (&v)[NV], float* sh) {
  constexpr int NWV = NTH / 64;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, lc = threadIdx.x % COLS;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
#pragma unroll
    for (int o = COLS; o < 64; o <<= 1) v[k] += __shfl_xor(v[k], o, 64);
    if (lane < COLS) sh[(k * NWV + wv) * COLS + lc] = v[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < NWV; ++w) t += sh[(k * NWV + w) * COLS + lc];
    v[k] = t;
  }
  __syncthreads();
}

template <int COLS, int MAXR, bool BT_ = false, int NTH = BN_THREADS>
__global__ __launch_bounds__(NTH) void bn_relu_train_kernel(
    const float* __restrict__ a, int lda, const float* __restrict__ gamma, const float* __restrict__ beta,
    float* __restrict__ out, int ldo, float* __restrict__ nhat, int ldn, float* __restrict__ mean,
    float* __restrict__ invstd, float* __restrict__ rm, float* __restrict__ rv, int rows, int cols, int groups,
    float momentum, float eps, ClientBatch cb) {
  const BIdx bi_ = batch_bidx<BT_>(cb.xcd);
  if (bi_.z) {
    const int64_t co = (int64_t)bi_.z * cb.stride;
    a = cptr(a, co);
    gamma = cptr(gamma, co);
    beta = cptr(beta, co);
    out = cptr(out, co);
    nhat = cptr(nhat, co);
    mean = cptr(mean, co);
    invstd = cptr(invstd, co);
    rm = cptr(rm, co);
    rv = cptr(rv, co);
  }

  constexpr int GROUPS = NTH / COLS;
  __shared__ float sh[2 * BN_MAXG * (NTH / 64) * COLS];
  const int lc = threadIdx.x % COLS, grp = threadIdx.x / COLS;
  const int c = bi_.x * COLS + lc;
  const bool ok = c < cols;
  const int cc = min(c, cols - 1);
  const int rpg = rows / groups;
  // One-pass statistics around a per-batch shift (the batch's first row): sum(d) and sum(d^2) of
  // d = x - shift reduce together, so the workgroup pays ONE cross-wave reduction instead of two
  // (mean, then centred variance).  The shift keeps E[d^2] - E[d]^2 free of cancellation.
  const float sh0 = a[cc], sh1 = a[(size_t)min(rpg, rows - 1) * lda + cc];
  // the column's affine and running-statistic parameters are requested with the rows (they are consumed
  // after the cross-wave reduction, whose barriers would otherwise leave their round trip exposed)
  const float gm = gamma[cc], bt = beta[cc], rm0 = rm[cc], rv0 = rv[cc];
  float x[MAXR];
  float s[2 * BN_MAXG] = {0.f, 0.f, 0.f, 0.f};   // sum d (batch 0, 1), sum d^2 (batch 0, 1)
#pragma unroll
  for (int i = 0; i < MAXR; ++i) {
    const int r = grp + i * GROUPS;
    const float v = a[(size_t)min(r, rows - 1) * lda + cc];
    x[i] = v;
    const bool g1 = r >= rpg;
    const float d = (r < rows) ? v - (g1 ? sh1 : sh0) : 0.f;
    if (g1) { s[1] += d; s[3] += d * d; } else { s[0] += d; s[2] += d * d; }
  }
  bn_colsum<COLS, 2 * BN_MAXG, NTH>(s, sh);
  const float m0 = s[0] / (float)rpg, m1 = s[1] / (float)rpg;
  const float mu0 = sh0 + m0, mu1 = sh1 + m1;
  const float var0 = fmaxf(s[2] / (float)rpg - m0 * m0, 0.f);   // biased batch variances
  const float var1 = fmaxf(s[3] / (float)rpg - m1 * m1, 0.f);
  const float is0 = rsqrtf(var0 + eps), is1 = rsqrtf(var1 + eps);
  if (grp == 0 && ok) {
    const float unb = (float)rpg / (float)max(rpg - 1, 1);
    float m = rm0, v = rv0;
    mean[c] = mu0;
    invstd[c] = is0;
    m = (1.f - momentum) * m + momentum * mu0;          // batch after batch, in row order
    v = (1.f - momentum) * v + momentum * var0 * unb;
    if (groups > 1) {
      mean[(size_t)cols + c] = mu1;
      invstd[(size_t)cols + c] = is1;
      m = (1.f - momentum) * m + momentum * mu1;
      v = (1.f - momentum) * v + momentum * var1 * unb;
    }
    rm[c] = m;
    rv[c] = v;
  }
  if (!ok) return;
#pragma unroll
  for (int i = 0; i < MAXR; ++i) {
    const int r = grp + i * GROUPS;
    if (r < rows) {
      const bool g1 = r >= rpg;
      const float n = (x[i] - (g1 ? mu1 : mu0)) * (g1 ? is1 : is0);
      nhat[(size_t)r * ldn + c] = n;
      const float y = n * gm + bt;
      out[(size_t)r * ldo + c] = y > 0.f ? y : 0.f;
    }
  }
}

// Large batches (more rows than the register-resident kernel holds): two passes over the
// column block, statistics first, then normalise + ReLU re-reading the GEMM output (L2-resident at
// these sizes).  Same shifted one-pass statistics and running-stat order as above.
template <int COLS, bool BT_ = false>
__global__ __launch_bounds__(BN_THREADS) void bn_relu_train_stream_kernel(
    const float* __restrict__ a, int lda, const float* __restrict__ gamma, const float* __restrict__ beta,
    float* __restrict__ out, int ldo, float* __restrict__ nhat, int ldn, float* __restrict__ mean,
    float* __restrict__ invstd, float* __restrict__ rm, float* __restrict__ rv, int rows, int cols, int groups,
    float momentum, float eps, ClientBatch cb) {
  const BIdx bi_ = batch_bidx<BT_>(cb.xcd);
  if (bi_.z) {
    const int64_t co = (int64_t)bi_.z * cb.stride;
    a = cptr(a, co);
    gamma = cptr(gamma, co);
    beta = cptr(beta, co);
    out = cptr(out, co);
    nhat = cptr(nhat, co);
    mean = cptr(mean, co);
    invstd = cptr(invstd, co);
    rm = cptr(rm, co);
    rv = cptr(rv, co);
  }

  constexpr int GROUPS = BN_THREADS / COLS;
  __shared__ float sh[2 * BN_MAXG * BN_WAVES * COLS];
  const int lc = threadIdx.x % COLS, grp = threadIdx.x / COLS;
  const int c = bi_.x * COLS + lc;
  const bool ok = c < cols;
  const int cc = min(c, cols - 1);
  const int rpg = rows / groups;
  const float sh0 = a[cc], sh1 = a[(size_t)min(rpg, rows - 1) * lda + cc];
  float s[2 * BN_MAXG] = {0.f, 0.f, 0.f, 0.f};
  for (int r = grp; r < rows; r += GROUPS) {
    const float v = a[(size_t)r * lda + cc];
    const bool g1 = r >= rpg;
    const float d = v - (g1 ? sh1 : sh0);
    if (g1) { s[1] += d; s[3] += d * d; } else { s[0] += d; s[2] += d * d; }
  }
  bn_colsum<COLS, 2 * BN_MAXG>(s, sh);
  const float m0 = s[0] / (float)rpg, m1 = s[1] / (float)rpg;
  const float mu0 = sh0 + m0, mu1 = sh1 + m1;
  const float var0 = fmaxf(s[2] / (float)rpg - m0 * m0, 0.f);
  const float var1 = fmaxf(s[3] / (float)rpg - m1 * m1, 0.f);
  const float is0 = rsqrtf(var0 + eps), is1 = rsqrtf(var1 + eps);
  if (grp == 0 && ok) {
    const float unb = (float)rpg / (float)max(rpg - 1, 1);
    float m = rm[c], v = rv[c];
    mean[c] = mu0;
    invstd[c] = is0;
    m = (1.f - momentum) * m + momentum * mu0;
    v = (1.f - momentum) * v + momentum * var0 * unb;
    if (groups > 1) {
      mean[(size_t)cols + c] = mu1;
      invstd[(size_t)cols + c] = is1;
      m = (1.f - momentum) * m + momentum * mu1;
      v = (1.f - momentum) * v + momentum * var1 * unb;
    }
    rm[c] = m;
    rv[c] = v;
  }
  if (!ok) return;
  const float gm = gamma[c], bt = beta[c];
  for (int r = grp; r < rows; r += GROUPS) {
    const bool g1 = r >= rpg;
    const float n = (a[(size_t)r * lda + c] - (g1 ? mu1 : mu0)) * (g1 ? is1 : is0);
    nhat[(size_t)r * ldn + c] = n;
    const float y = n * gm + bt;
    out[(size_t)r * ldo + c] = y > 0.f ? y : 0.f;
  }
}

// BatchNorm(train) + ReLU from the producing GEMM's per-tile partial statistics (GemmArgs::bn_part):
// no reduction over the batch's rows here, so the rows split over many workgroups -- a workgroup
// owns 16 columns x 128 rows (one float4 per thread) instead of 8 columns x every row.
//   1. wave w merges the tile triples (count, mean, M2) of columns 2w, 2w+1 for both batches with
//      Chan's formula, lanes over tiles then a butterfly; lane 0's result is the statistic;
//   2. row block 0 updates the running statistics (batch after batch, like the reference's two
//      forward passes) and writes mean / invstd;
//   3. every thread normalises one float4 of its row and writes nhat and relu(gamma nhat + beta).
constexpr int BNA_THREADS = 512, BNA_COLS = 16, BNA_ROWS = 128;

__device__ __forceinline__ void chan_merge(float& n, float& mu, float& m2, float nb, float mub, float m2b) {
  const float nt = n + nb;
  if (nt > 0.f) {
    const float d = mub - mu;
    mu += d * (nb / nt);
    m2 += m2b + d * d * (n * nb / nt);
    n = nt;
  }
}

template <bool BT_ = false>
__global__ __launch_bounds__(BNA_THREADS) void bn_relu_apply_kernel(
    const float* __restrict__ a, int lda, const float* __restrict__ part, int n_tiles, const float* __restrict__ gamma,
    const float* __restrict__ beta, float* __restrict__ out, int ldo, float* __restrict__ nhat, int ldn,
    float* __restrict__ mean, float* __restrict__ invstd, float* __restrict__ rm, float* __restrict__ rv, int rows,
    int cols, int groups, float momentum, float eps, ClientBatch cb) {
  const BIdx bi_ = batch_bidx<BT_>(cb.xcd);
  if (bi_.z) {
    const int64_t co = (int64_t)bi_.z * cb.stride;
    a = cptr(a, co);
    part = cptr(part, co);
    gamma = cptr(gamma, co);
    beta = cptr(beta, co);
    out = cptr(out, co);
    nhat = cptr(nhat, co);
    mean = cptr(mean, co);
    invstd = cptr(invstd, co);
    rm = cptr(rm, co);
    rv = cptr(rv, co);
  }

  __shared__ float st[BNA_COLS][2][3];   // [col][batch] = (mean, invstd, biased var)
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int c0 = bi_.x * BNA_COLS;
  const int rpg = rows / groups;
  // this thread's float4 of the GEMM output: requested first, in flight during the merge
  const int r = bi_.y * BNA_ROWS + (t >> 2);
  const int cq = (t & 3) * 4;
  float x[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) x[e] = a[(size_t)min(r, rows - 1) * lda + min(c0 + cq + e, cols - 1)];
  // every tile triple this lane merges, all loads issued before the first merge (lane = tile,
  // n_tiles <= 64: the 32/64-tile GEMMs of a <= 4096-row batch pair)
  float pv[2][2][3];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int c = min(c0 + 2 * w + q, cols - 1);
      const float* p = part + ((size_t)(min(lane, n_tiles - 1) * 2 + b) * 3) * cols + c;
      const bool ok = lane < n_tiles;
      pv[q][b][0] = ok ? p[0] : 0.f;
      pv[q][b][1] = ok ? p[cols] : 0.f;
      pv[q][b][2] = ok ? p[2 * (size_t)cols] : 0.f;
    }
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      float n = pv[q][b][0], mu = pv[q][b][1], m2 = pv[q][b][2];
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const float nb = __shfl_xor(n, o, 64), mub = __shfl_xor(mu, o, 64), m2b = __shfl_xor(m2, o, 64);
        chan_merge(n, mu, m2, nb, mub, m2b);
      }
      if (lane == 0) {
        const float var = n > 0.f ? fmaxf(m2 / n, 0.f) : 0.f;
        st[2 * w + q][b][0] = mu;
        st[2 * w + q][b][1] = rsqrtf(var + eps);
        st[2 * w + q][b][2] = var;
      }
    }
  __syncthreads();
  if (bi_.y == 0 && t < BNA_COLS && c0 + t < cols) {
    const int c = c0 + t;
    const float unb = (float)rpg / (float)max(rpg - 1, 1);
    float m = rm[c], v = rv[c];
    for (int b = 0; b < groups; ++b) {
      mean[(size_t)b * cols + c] = st[t][b][0];
      invstd[(size_t)b * cols + c] = st[t][b][1];
      m = (1.f - momentum) * m + momentum * st[t][b][0];      // batch after batch, in row order
      v = (1.f - momentum) * v + momentum * st[t][b][2] * unb;
    }
    rm[c] = m;
    rv[c] = v;
  }
  if (r >= rows) return;
  const int bb = (groups > 1 && r >= rpg) ? 1 : 0;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int cl = cq + e, c = c0 + cl;
    if (c >= cols) break;
    const float nv = (x[e] - st[cl][bb][0]) * st[cl][bb][1];
    nhat[(size_t)r * ldn + c] = nv;
    const float y = nv * gamma[c] + beta[c];
    out[(size_t)r * ldo + c] = y > 0.f ? y : 0.f;
  }
}

void launch_bn_relu_apply(const float* a, int lda, const float* part, int n_tiles, const float* gamma,
                          const float* beta, float* out, int ldo, float* nhat, int ldn, float* mean, float* invstd,
                          float* rm, float* rv, int rows, int cols, int groups, float momentum, float eps,
                          hipStream_t stream) {
  const ClientBatch cb = client_batch();
  if (cb.k > 1) check_slabs("bn_relu_apply operand", a, part, gamma, beta, out, nhat, mean, invstd, rm, rv);
  const dim3 grid((cols + BNA_COLS - 1) / BNA_COLS, (rows + BNA_ROWS - 1) / BNA_ROWS, cb.k);
  hipLaunchKernelGGL((client_batch().xcd ? bn_relu_apply_kernel<true> : bn_relu_apply_kernel<false>), grid, dim3(BNA_THREADS), 0, stream, a, lda, part, n_tiles, gamma, beta,
                     out, ldo, nhat, ldn, mean, invstd, rm, rv, rows, cols, groups, momentum, eps, cb);
}

template <int COLS>
static void bn_train_cols(const float* a, int lda, const float* gamma, const float* beta, float* out, int ldo,
                          float* nhat, int ldn, float* mean, float* invstd, float* rm, float* rv, int rows, int cols,
                          int groups, float momentum, float eps, hipStream_t stream) {
  constexpr int GROUPS = BN_THREADS / COLS;
  const ClientBatch cb = client_batch();
  if (cb.k > 1) check_slabs("bn_relu_train operand", a, gamma, beta, out, nhat, mean, invstd, rm, rv);
  const dim3 grid((cols + COLS - 1) / COLS, 1, cb.k), block(BN_THREADS);
  if (g_bn_threads == 1024 && rows <= 8 * (1024 / COLS)) {   // twice the row groups, half the rows per thread
    hipLaunchKernelGGL((client_batch().xcd ? bn_relu_train_kernel<COLS, 8, true, 1024> : bn_relu_train_kernel<COLS, 8, false, 1024>),
                       grid, dim3(1024), 0, stream, a, lda, gamma, beta, out, ldo, nhat, ldn, mean, invstd, rm, rv, rows,
                       cols, groups, momentum, eps, cb);
    return;
  }
#define BN_TRAIN_LAUNCH(R)                                                                                          \
  hipLaunchKernelGGL((client_batch().xcd ? bn_relu_train_kernel<COLS, R, true> : bn_relu_train_kernel<COLS, R, false>), grid, block, 0, stream, a, lda, gamma, beta, out, ldo, nhat, \
                     ldn, mean, invstd, rm, rv, rows, cols, groups, momentum, eps, cb)
  if (rows <= 4 * GROUPS) BN_TRAIN_LAUNCH(4);
  else if (rows <= 8 * GROUPS) BN_TRAIN_LAUNCH(8);
  else if (rows <= 16 * GROUPS) BN_TRAIN_LAUNCH(16);
  else if (rows <= 32 * GROUPS) BN_TRAIN_LAUNCH(32);
  else if (rows <= 64 * GROUPS) BN_TRAIN_LAUNCH(64);
  else
    hipLaunchKernelGGL((client_batch().xcd ? bn_relu_train_stream_kernel<COLS, true> : bn_relu_train_stream_kernel<COLS, false>), grid, block, 0, stream, a, lda, gamma, beta, out, ldo,
                       nhat, ldn, mean, invstd, rm, rv, rows, cols, groups, momentum, eps, cb);
#undef BN_TRAIN_LAUNCH
}

void launch_bn_relu_train(const float* a, int lda, const float* gamma, const float* beta, float* out, int ldo,
                          float* nhat, int ldn, float* mean, float* invstd, float* rm, float* rv, int rows, int cols,
                          int groups, float momentum, float eps, hipStream_t stream) {
  const int bc = bn_cols_for_launch();
  if (bc == 4)
    bn_train_cols<4>(a, lda, gamma, beta, out, ldo, nhat, ldn, mean, invstd, rm, rv, rows, cols, groups, momentum, eps,
                     stream);
  else if (bc == 16)
    bn_train_cols<16>(a, lda, gamma, beta, out, ldo, nhat, ldn, mean, invstd, rm, rv, rows, cols, groups, momentum,
                      eps, stream);
  else
    bn_train_cols<8>(a, lda, gamma, beta, out, ldo, nhat, ldn, mean, invstd, rm, rv, rows, cols, groups, momentum, eps,
                     stream);
}

template <int COLS, int MAXR, bool BT_ = false, int NTH = BN_THREADS>
__global__ __launch_bounds__(NTH) void bn_relu_bwd_kernel(
    const float* __restrict__ dr, int lddr, const float* __restrict__ r_, int ldr, const float* __restrict__ nhat,
    int ldn, const float* __restrict__ gamma, const float* __restrict__ invstd, float* __restrict__ da, int ldda,
    float* __restrict__ dgamma, float* __restrict__ dbeta, float* __restrict__ dbias, int rows, int cols, ClientBatch cb) {
  const BIdx bi_ = batch_bidx<BT_>(cb.xcd);
  if (bi_.z) {
    const int64_t co = (int64_t)bi_.z * cb.stride;
    dr = cptr(dr, co);
    r_ = cptr(r_, co);
    nhat = cptr(nhat, co);
    gamma = cptr(gamma, co);
    invstd = cptr(invstd, co);
    da = cptr(da, co);
    dgamma = cptr(dgamma, co);
    dbeta = cptr(dbeta, co);
    dbias = cptr(dbias, co);
  }

  constexpr int GROUPS = NTH / COLS;
  __shared__ float sh[3 * (NTH / 64) * COLS];
  const int lc = threadIdx.x % COLS, grp = threadIdx.x / COLS;
  const int c = bi_.x * COLS + lc;
  const bool ok = c < cols;
  const int cc = min(c, cols - 1);
  // gamma * invstd is requested with the rows (consumed after the reduction's barriers)
  const float k = gamma[cc] * invstd[cc];
  float dy[MAXR], nh[MAXR];
  float st[3] = {0.f, 0.f, 0.f};   // sum dy, sum dy * nhat, sum nhat
#pragma unroll
  for (int i = 0; i < MAXR; ++i) {
    const int r = grp + i * GROUPS;
    const size_t rr = (size_t)min(r, rows - 1);
    const float rv = r_[rr * ldr + cc];
    const float dv = dr[rr * lddr + cc];
    const float nv = nhat[rr * ldn + cc];
    const bool in = r < rows;
    const float d = (in && rv > 0.f) ? dv : 0.f;
    const float n = in ? nv : 0.f;
    dy[i] = d;
    nh[i] = n;
    st[0] += d;
    st[1] += d * n;
    st[2] += n;
  }
  bn_colsum<COLS, 3, NTH>(st, sh);
  const float sdy = st[0], sdyn = st[1], snh = st[2];
  const float invn = 1.f / (float)rows;
  // the preceding Linear's bias gradient sum_r da_r, in closed form from the same single
  // reduction: k * (sum dy - rows * sdy / rows - sum nhat * sdyn / rows)
  if (grp == 0 && ok) {
    dbeta[c] = sdy;
    dgamma[c] = sdyn;
    if (dbias) dbias[c] = k * (sdy - sdy * (float)rows * invn - snh * sdyn * invn);
  }
#pragma unroll
  for (int i = 0; i < MAXR; ++i) {
    const int r = grp + i * GROUPS;
    if (r < rows && ok) da[(size_t)r * ldda + c] = k * (dy[i] - sdy * invn - nh[i] * sdyn * invn);
  }
}

// Large-batch backward: the three column sums in a first pass, da in a second (re-reading).
template <int COLS, bool BT_ = false>
__global__ __launch_bounds__(BN_THREADS) void bn_relu_bwd_stream_kernel(
    const float* __restrict__ dr, int lddr, const float* __restrict__ r_, int ldr, const float* __restrict__ nhat,
    int ldn, const float* __restrict__ gamma, const float* __restrict__ invstd, float* __restrict__ da, int ldda,
    float* __restrict__ dgamma, float* __restrict__ dbeta, float* __restrict__ dbias, int rows, int cols, ClientBatch cb) {
  const BIdx bi_ = batch_bidx<BT_>(cb.xcd);
  if (bi_.z) {
    const int64_t co = (int64_t)bi_.z * cb.stride;
    dr = cptr(dr, co);
    r_ = cptr(r_, co);
    nhat = cptr(nhat, co);
    gamma = cptr(gamma, co);
    invstd = cptr(invstd, co);
    da = cptr(da, co);
    dgamma = cptr(dgamma, co);
    dbeta = cptr(dbeta, co);
    dbias = cptr(dbias, co);
  }

  constexpr int GROUPS = BN_THREADS / COLS;
  __shared__ float sh[3 * BN_WAVES * COLS];
  const int lc = threadIdx.x % COLS, grp = threadIdx.x / COLS;
  const int c = bi_.x * COLS + lc;
  const bool ok = c < cols;
  const int cc = min(c, cols - 1);
  float st[3] = {0.f, 0.f, 0.f};
  for (int r = grp; r < rows; r += GROUPS) {
    const size_t rr = (size_t)r;
    const float d = r_[rr * ldr + cc] > 0.f ? dr[rr * lddr + cc] : 0.f;
    const float n = nhat[rr * ldn + cc];
    st[0] += d;
    st[1] += d * n;
    st[2] += n;
  }
  bn_colsum<COLS, 3>(st, sh);
  const float sdy = st[0], sdyn = st[1], snh = st[2];
  const float k = gamma[cc] * invstd[cc];
  const float invn = 1.f / (float)rows;
  if (grp == 0 && ok) {
    dbeta[c] = sdy;
    dgamma[c] = sdyn;
    if (dbias) dbias[c] = k * (sdy - sdy * (float)rows * invn - snh * sdyn * invn);
  }
  if (!ok) return;
  for (int r = grp; r < rows; r += GROUPS) {
    const size_t rr = (size_t)r;
    const float d = r_[rr * ldr + c] > 0.f ? dr[rr * lddr + c] : 0.f;
    da[rr * ldda + c] = k * (d - sdy * invn - nhat[rr * ldn + c] * sdyn * invn);
  }
}

template <int COLS>
static void bn_bwd_cols(const float* dr, int lddr, const float* r, int ldr, const float* nhat, int ldn,
                        const float* gamma, const float* invstd, float* da, int ldda, float* dgamma, float* dbeta,
                        float* dbias, int rows, int cols, hipStream_t stream) {
  constexpr int GROUPS = BN_THREADS / COLS;
  const ClientBatch cb = client_batch();
  if (cb.k > 1) check_slabs("bn_relu_bwd operand", dr, r, nhat, gamma, invstd, da, dgamma, dbeta, dbias);
  const dim3 grid((cols + COLS - 1) / COLS, 1, cb.k), block(BN_THREADS);
  if (g_bn_threads == 1024 && rows <= 8 * (1024 / COLS)) {
    hipLaunchKernelGGL((client_batch().xcd ? bn_relu_bwd_kernel<COLS, 8, true, 1024> : bn_relu_bwd_kernel<COLS, 8, false, 1024>),
                       grid, dim3(1024), 0, stream, dr, lddr, r, ldr, nhat, ldn, gamma, invstd, da, ldda, dgamma, dbeta,
                       dbias, rows, cols, cb);
    return;
  }
#define BN_BWD_LAUNCH(R)                                                                                          \
  hipLaunchKernelGGL((client_batch().xcd ? bn_relu_bwd_kernel<COLS, R, true> : bn_relu_bwd_kernel<COLS, R, false>), grid, block, 0, stream, dr, lddr, r, ldr, nhat, ldn, gamma, \
                     invstd, da, ldda, dgamma, dbeta, dbias, rows, cols, cb)
  if (rows <= 4 * GROUPS) BN_BWD_LAUNCH(4);
  else if (rows <= 8 * GROUPS) BN_BWD_LAUNCH(8);
  else if (rows <= 16 * GROUPS) BN_BWD_LAUNCH(16);
  else if (rows <= 32 * GROUPS) BN_BWD_LAUNCH(32);
  else if (rows <= 64 * GROUPS) BN_BWD_LAUNCH(64);
  else
    hipLaunchKernelGGL((client_batch().xcd ? bn_relu_bwd_stream_kernel<COLS, true> : bn_relu_bwd_stream_kernel<COLS, false>), grid, block, 0, stream, dr, lddr, r, ldr, nhat, ldn, gamma,
                       invstd, da, ldda, dgamma, dbeta, dbias, rows, cols, cb);
#undef BN_BWD_LAUNCH
}

void launch_bn_relu_bwd(const float* dr, int lddr, const float* r, int ldr, const float* nhat, int ldn,
                        const float* gamma, const float* invstd, float* da, int ldda, float* dgamma, float* dbeta,
                        float* dbias, int rows, int cols, hipStream_t stream) {
  const int bc = bn_cols_for_launch();
  if (bc == 4)
    bn_bwd_cols<4>(dr, lddr, r, ldr, nhat, ldn, gamma, invstd, da, ldda, dgamma, dbeta, dbias, rows, cols, stream);
  else if (bc == 16)
    bn_bwd_cols<16>(dr, lddr, r, ldr, nhat, ldn, gamma, invstd, da, ldda, dgamma, dbeta, dbias, rows, cols, stream);
  else
    bn_bwd_cols<8>(dr, lddr, r, ldr, nhat, ldn, gamma, invstd, da, ldda, dgamma, dbeta, dbias, rows, cols, stream);
}

// ============================================================================ Adam
// Store policy of the updated p, m, v (tuning knob "adam_store"): 0 plain stores (dirty in L2, written
// back at the kernel boundary: ~B / 6 TB/s, MI355X_MICROARCH.md "boundary"), otherwise a buffer store
// with these cache bits (2 = nt, 16 = sc1 write-through) so the write-back overlaps the kernel.
int g_adam_store = 16;
int g_adam_max_blocks = 65535;
// set_tuning("adam_u_min").  0: every Adam launch loads ADAM_U float4 per thread.  Measured on the one-client
// Intrusion step (D 1.67 M, G ~0.5 M parameters; tools/gpu_recipes/r5_adamu.sh, 12 samples each): 196.5 ->
// 194.8 us with the unrolled loop also below the old 4 M-element threshold
int64_t g_adam_u_min = 0;

template <int AUX, bool BT_ = false>
__global__ __launch_bounds__(256) void adam_kernel(float4* __restrict__ p, const float4* __restrict__ g,
                                                   float4* __restrict__ m, float4* __restrict__ v,
                                                   const float* __restrict__ step, int64_t n4, float lr, float b1,
                                                   float b2, float eps, float wd, uint64_t* rng_bump, ClientBatch cb) {
  const BIdx bi_ = batch_bidx<BT_>(cb.xcd);
  if (bi_.z) {
    const int64_t co = (int64_t)bi_.z * cb.stride;
    p = cptr(p, co);
    g = cptr(g, co);
    m = cptr(m, co);
    v = cptr(v, co);
    step = cptr(step, co);
    rng_bump = cptr(rng_bump, co);
  }
  const float t = step[0];
  const float bc1 = 1.f - powf(b1, t);
  const float bc2s = sqrtf(1.f - powf(b2, t));
  const float sz = lr / bc1;
  const int bytes = (int)(n4 * 16);
  const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(p, 0, bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rm = __builtin_amdgcn_make_buffer_rsrc(m, 0, bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(v, 0, bytes, 0x00020000);
  for (int64_t i = (int64_t)bi_.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    float4 pp = p[i], gg = g[i], mm = m[i], vv = v[i];
    float* pf = reinterpret_cast<float*>(&pp);
    float* gf = reinterpret_cast<float*>(&gg);
    float* mf = reinterpret_cast<float*>(&mm);
    float* vf = reinterpret_cast<float*>(&vv);
#pragma unroll
    for (int q = 0; q < 4; ++q) adam_elem(gf[q], pf[q], mf[q], vf[q], b1, b2, eps, wd, sz, bc2s);
    adam_store4<AUX>(p, rp, i, pp);
    adam_store4<AUX>(m, rm, i, mm);
    adam_store4<AUX>(v, rv, i, vv);
  }
  if (rng_bump && bi_.x == 0 && threadIdx.x == 0) rng_bump[0] += 1ull;
}

template <bool BT_ = false>
__global__ void adam_tail_kernel(float* p, const float* g, float* m, float* v, const float* step, int64_t start,
                                 int64_t n, float lr, float b1, float b2, float eps, float wd, ClientBatch cb) {
  const BIdx bi_ = batch_bidx<BT_>(cb.xcd);
  if (bi_.z) {
    const int64_t co = (int64_t)bi_.z * cb.stride;
    p = cptr(p, co);
    g = cptr(g, co);
    m = cptr(m, co);
    v = cptr(v, co);
    step = cptr(step, co);
  }
  const int64_t i = start + threadIdx.x;
  if (i >= n) return;
  const float t = step[0];
  const float bc1 = 1.f - powf(b1, t);
  const float bc2s = sqrtf(1.f - powf(b2, t));
  float pe = p[i], me = m[i], ve = v[i];
  adam_elem(g[i], pe, me, ve, b1, b2, eps, wd, lr / bc1, bc2s);
  p[i] = pe;
  m[i] = me;
  v[i] = ve;
}

// ---- Adam with the step's column sums folded in: one launch instead of colsum + Adam.
// The first cs.blk_start[n_jobs] workgroups each reduce ACS_COLS columns of one column-sum job
// (ACS_GROUPS row groups of ACS_COLS lanes, an LDS combine), write the sums (bias gradient or
// metric), and when the job's output lies inside this optimizer's gradient buffer apply Adam to
// exactly those elements straight from registers.  Every other workgroup runs the float4 Adam and
// skips the float4 groups the jobs own: job outputs start 16-B aligned and own ceil4(cols)
// elements (the flat layout stores every tensor that way), so no float4 is shared.
template <int AUX, int U, bool BT_ = false>
__global__ __launch_bounds__(256) void adam_cs_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                      float* __restrict__ m, float* __restrict__ v,
                                                      const float* __restrict__ step, int64_t n4, float lr, float b1,
                                                      float b2, float eps, float wd, uint64_t* rng_bump, AdamColsum cs,
                                                      ClientBatch cb) {
  const BIdx bi_ = batch_bidx<BT_>(cb.xcd);
  const int64_t co = (int64_t)bi_.z * cb.stride;
  if (co) {
    p = cptr(p, co);
    g = cptr(g, co);
    m = cptr(m, co);
    v = cptr(v, co);
    step = cptr(step, co);
    rng_bump = cptr(rng_bump, co);
  }
  adam_cs_body<AUX, U>((int)bi_.x, (int)gridDim.x, p, g, m, v, step, n4, lr, b1, b2, eps, wd, rng_bump, cs, co);
}

void launch_adam_colsum(float* p, const float* g, float* m, float* v, const float* step, int64_t n, float lr, float b1,
                        float b2, float eps, float wd, uint64_t* rng_ctr_bump, const AdamColsum& cs_in,
                        hipStream_t stream) {
  AdamColsum cs = cs_in;
  cs.n_jobs = std::min(cs.n_jobs, 8);
  cs.blk_start[0] = 0;
  for (int k = 0; k < cs.n_jobs; ++k) cs.blk_start[k + 1] = cs.blk_start[k] + (cs.jobs[k].cols + ACS_COLS - 1) / ACS_COLS;
  const int64_t n4 = n / 4;
  const ClientBatch cb = client_batch();
  const int U = adam_unroll(n4, cb.k);
  const int blocks = (int)std::min<int64_t>((n4 + 256 * U - 1) / (256 * U), g_adam_max_blocks);
  const int grid = std::max(blocks, 1) + cs.blk_start[cs.n_jobs];
  if (cb.k > 1) {
    check_slabs("adam operand", p, g, m, v, step, rng_ctr_bump);
    check_slab(cs);
  }
#define FEDTGAN_ADAM_CS(AUX, UU)                                                                                       \
  hipLaunchKernelGGL((client_batch().xcd ? adam_cs_kernel<AUX, UU, true> : adam_cs_kernel<AUX, UU, false>), dim3(grid, 1, cb.k), dim3(256), 0, stream, p, g, m, v, step, n4, lr, b1, \
                     b2, eps, wd, rng_ctr_bump, cs, cb)
#define FEDTGAN_ADAM_CS_U(AUX)                  \
  if (U == ADAM_U) FEDTGAN_ADAM_CS(AUX, ADAM_U); \
  else FEDTGAN_ADAM_CS(AUX, 1);
  if (g_adam_store == 2) { FEDTGAN_ADAM_CS_U(2) }
  else if (g_adam_store == 16) { FEDTGAN_ADAM_CS_U(16) }
  else { FEDTGAN_ADAM_CS_U(0) }
#undef FEDTGAN_ADAM_CS_U
#undef FEDTGAN_ADAM_CS
  if (n4 * 4 < n)
    hipLaunchKernelGGL((client_batch().xcd ? adam_tail_kernel<true> : adam_tail_kernel<false>), dim3(1, 1, cb.k), dim3(64), 0, stream, p, g, m, v, step, n4 * 4, n, lr, b1, b2,
                       eps, wd, cb);
}

void launch_adam(float* p, const float* g, float* m, float* v, const float* step, int64_t n, float lr, float b1,
                 float b2, float eps, float wd, uint64_t* rng_ctr_bump, hipStream_t stream) {
  const int64_t n4 = n / 4;
  // one float4 per thread where possible: a grid-stride loop over few workgroups keeps too few
  // loads in flight for HBM (19.5M-parameter wide-table D: 259 us at 1024 workgroups)
  const int blocks = (int)std::min<int64_t>((n4 + 255) / 256, g_adam_max_blocks);
  const ClientBatch cb = client_batch();
  if (cb.k > 1) check_slabs("adam operand", p, g, m, v, step, rng_ctr_bump);
#define FEDTGAN_ADAM(AUX)                                                                                       \
  hipLaunchKernelGGL((client_batch().xcd ? adam_kernel<AUX, true> : adam_kernel<AUX, false>), dim3(std::max(blocks, 1), 1, cb.k), dim3(256), 0, stream,                 \
                     reinterpret_cast<float4*>(p), reinterpret_cast<const float4*>(g), reinterpret_cast<float4*>(m), \
                     reinterpret_cast<float4*>(v), step, n4, lr, b1, b2, eps, wd, rng_ctr_bump, cb)
  if (g_adam_store == 2) FEDTGAN_ADAM(2);
  else if (g_adam_store == 16) FEDTGAN_ADAM(16);
  else FEDTGAN_ADAM(0);
#undef FEDTGAN_ADAM
  if (n4 * 4 < n)
    hipLaunchKernelGGL((client_batch().xcd ? adam_tail_kernel<true> : adam_tail_kernel<false>), dim3(1, 1, cb.k), dim3(64), 0, stream, p, g, m, v, step, n4 * 4, n, lr, b1, b2,
                       eps, wd, cb);
}

// ============================================================================ generation decode
__global__ __launch_bounds__(256) void sample_decode_kernel(DecodeArgs a) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)a.rows * a.n_cols) return;
  const int r = (int)(idx / a.n_cols), j = (int)(idx % a.n_cols);
  const float* x = a.logits + (size_t)r * a.ldl;
  const int st = a.start[j], w = a.width[j];
  const uint64_t step = a.rng_ctr ? *a.rng_ctr : 0ull;
  RngArgs rng{a.seed, a.rng_ctr, a.rng_stream};
  const int off = a.kind[j] == 0 ? st + 1 : st;
  const uint64_t base = ((uint64_t)r << 20) + (uint64_t)off;
  int best = 0;
  float bv = -INFINITY;
  for (int i = 0; i < w; i += 4) {
    const uint4 u = rng4(rng, step, base + i);
    const uint32_t uu[4] = {u.x, u.y, u.z, u.w};
    for (int q = 0; q < 4 && i + q < w; ++q) {
      const float v = x[off + i + q] + gumbel(uu[q]);
      if (v > bv) { bv = v; best = i + q; }
    }
  }
  double val;
  if (a.kind[j] == 0) {
    double al = (double)tanhf(x[st]);
    al = al < -1.0 ? -1.0 : (al > 1.0 ? 1.0 : al);
    const int c = a.cont[j];
#if FT_CHECKED
    FT_CHECK(&g_check_ops, best >= 0 && best < a.K, CHK_DECODE_MODE);
#endif
    val = al * 4.0 * a.sd[(size_t)c * a.K + best] + a.mu[(size_t)c * a.K + best];
  } else {
#if FT_CHECKED
    FT_CHECK(&g_check_ops, a.code_off[j] + best >= 0 && a.code_off[j] + best < a.n_codes, CHK_DECODE_CODE);
#endif
    val = a.codes[a.code_off[j] + best];
  }
  a.out[(size_t)r * a.n_cols + j] = val;
}

// One wave per row: every lane draws the Gumbel noise of its own logits -- the same Philox word
// per element as sample_decode_kernel (counter (row << 20) + span offset + the 4-aligned position
// in the span, component = position % 4) -- and folds (noisy logit, first index) into its
// column's 64-bit LDS maximum (ds_max_u64: ordered float in the high word, ~index in the low
// word, so ties keep the first index like the serial scan).  Lanes then decode one column each.
// The serial kernel walked each span in one thread: a 70-wide categorical was ~18 dependent
// round trips for one lane of the wave.
constexpr int DEC_WAVES = 4;
__global__ __launch_bounds__(DEC_WAVES * 64) void sample_decode_row_kernel(DecodeArgs a) {
  extern __shared__ unsigned long long dec_best[];   // [DEC_WAVES][n_cols]
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r = blockIdx.x * DEC_WAVES + wv;
  if (r >= a.rows) return;   // (wave-uniform; only wave-level LDS syncs below)
  unsigned long long* best = dec_best + (size_t)wv * a.n_cols;
  for (int j = lane; j < a.n_cols; j += 64) best[j] = 0ull;
  wave_lds_sync();
  const float* x = a.logits + (size_t)r * a.ldl;
  const uint64_t step = a.rng_ctr ? *a.rng_ctr : 0ull;
  RngArgs rng{a.seed, a.rng_ctr, a.rng_stream};
  const uint64_t rbase = (uint64_t)r << 20;
  constexpr int U = 4;   // elements per lane per round trip
  for (int p0 = 0; p0 < a.dim; p0 += U * 64) {
    float xv[U];
    int jc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int p = min(p0 + u * 64 + lane, a.dim - 1);
      xv[u] = x[p];
      jc[u] = a.ecol[p];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int p = p0 + u * 64 + lane;
      const int j = jc[u];
      if (p >= a.dim || j < 0) continue;
      const int off = a.start[j] + (a.kind[j] == 0 ? 1 : 0);
      const int i = p - off;
      const uint4 rw = rng4(rng, step, rbase + (uint64_t)(off + (i & ~3)));
      const uint32_t uu = (i & 3) == 0 ? rw.x : (i & 3) == 1 ? rw.y : (i & 3) == 2 ? rw.z : rw.w;
      const float v = xv[u] + gumbel(uu);
      atomicMax(&best[j], ((unsigned long long)f2ord(v) << 32) | (unsigned long long)(0xFFFFFFFFu - (uint32_t)i));
    }
  }
  wave_lds_sync();
  for (int j = lane; j < a.n_cols; j += 64) {
    const unsigned long long k = best[j];
    const int bi = k ? (int)(0xFFFFFFFFu - (uint32_t)(k & 0xFFFFFFFFull)) : 0;
    double val;
    if (a.kind[j] == 0) {
      double al = (double)tanhf(x[a.start[j]]);
      al = al < -1.0 ? -1.0 : (al > 1.0 ? 1.0 : al);
      const int c = a.cont[j];
#if FT_CHECKED
      FT_CHECK(&g_check_ops, bi >= 0 && bi < a.K, CHK_DECODE_MODE);
#endif
      val = al * 4.0 * a.sd[(size_t)c * a.K + bi] + a.mu[(size_t)c * a.K + bi];
    } else {
#if FT_CHECKED
      FT_CHECK(&g_check_ops, a.code_off[j] + bi >= 0 && a.code_off[j] + bi < a.n_codes, CHK_DECODE_CODE);
#endif
      val = a.codes[a.code_off[j] + bi];
    }
    a.out[(size_t)r * a.n_cols + j] = val;
  }
}

// One wave per row over Philox QUADS: a lane takes a run of up to 4 logits of one column that share
// one Philox word (the same counter and components as the kernels above), adds the 4 Gumbel draws of
// that ONE Philox call, keeps the run's first maximum in registers and folds it into the column's
// LDS maximum with one ds_max_u64 -- a quarter of the Philox calls and LDS atomics of the
// element-per-lane kernel.  Same noise, same ties: bit-identical output.
__global__ __launch_bounds__(DEC_WAVES * 64) void sample_decode_quad_kernel(DecodeArgs a) {
  extern __shared__ unsigned long long dec_best[];   // [DEC_WAVES][n_cols]
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r = blockIdx.x * DEC_WAVES + wv;
  if (r >= a.rows) return;   // (wave-uniform; only wave-level LDS syncs below)
  unsigned long long* best = dec_best + (size_t)wv * a.n_cols;
  for (int j = lane; j < a.n_cols; j += 64) best[j] = 0ull;
  wave_lds_sync();
  const float* x = a.logits + (size_t)r * a.ldl;
  const uint64_t step = a.rng_ctr ? *a.rng_ctr : 0ull;
  RngArgs rng{a.seed, a.rng_ctr, a.rng_stream};
  const uint64_t rbase = (uint64_t)r << 20;
  for (int q = lane; q < a.n_quads; q += 64) {
    const int q0 = a.quads[2 * q], q1 = a.quads[2 * q + 1];
    const int j = q0 & 0xFFFFFF, cnt = q0 >> 24;
    const int i0 = q1 >> 16, p0 = q1 & 0xFFFF;
#if FT_CHECKED
    FT_CHECK(&g_check_ops, j < a.n_cols && cnt >= 1 && cnt <= 4 && p0 + cnt <= a.dim, CHK_DECODE_MODE);
    if (!(j < a.n_cols && cnt >= 1 && cnt <= 4 && p0 + cnt <= a.dim)) continue;
#endif
    float xv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) xv[u] = x[p0 + min(u, cnt - 1)];
    const uint4 rw = rng4(rng, step, rbase + (uint64_t)p0);   // counter = span offset + (i & ~3)
    const uint32_t uu[4] = {rw.x, rw.y, rw.z, rw.w};
    float bv = xv[0] + gumbel(uu[0]);
    int bi = 0;
#pragma unroll
    for (int u = 1; u < 4; ++u) {
      const float v = xv[u] + gumbel(uu[u]);
      if (u < cnt && v > bv) { bv = v; bi = u; }
    }
    const uint32_t i = (uint32_t)(i0 + bi);
    atomicMax(&best[j], ((unsigned long long)f2ord(bv) << 32) | (unsigned long long)(0xFFFFFFFFu - i));
  }
  wave_lds_sync();
  for (int j = lane; j < a.n_cols; j += 64) {
    const unsigned long long k = best[j];
    const int bi = k ? (int)(0xFFFFFFFFu - (uint32_t)(k & 0xFFFFFFFFull)) : 0;
    double val;
    if (a.kind[j] == 0) {
      double al = (double)tanhf(x[a.start[j]]);
      al = al < -1.0 ? -1.0 : (al > 1.0 ? 1.0 : al);
      const int c = a.cont[j];
#if FT_CHECKED
      FT_CHECK(&g_check_ops, bi >= 0 && bi < a.K, CHK_DECODE_MODE);
#endif
      val = al * 4.0 * a.sd[(size_t)c * a.K + bi] + a.mu[(size_t)c * a.K + bi];
    } else {
#if FT_CHECKED
      FT_CHECK(&g_check_ops, a.code_off[j] + bi >= 0 && a.code_off[j] + bi < a.n_codes, CHK_DECODE_CODE);
#endif
      val = a.codes[a.code_off[j] + bi];
    }
    a.out[(size_t)r * a.n_cols + j] = val;
  }
}

// generation decode: 2 = one wave per row over Philox quads, 1 = one wave per row, element per lane,
// 0 = one thread per (row, column)
int g_decode_rows = 2;

void launch_sample_decode(const DecodeArgs& a, hipStream_t stream) {
  const int64_t n = (int64_t)a.rows * a.n_cols;
  if (n == 0) return;
  require_unbatched("sample_decode");
  if (g_decode_rows == 2 && a.quads && a.ecol) {
    const size_t lds = (size_t)DEC_WAVES * a.n_cols * sizeof(unsigned long long);
    hipLaunchKernelGGL(sample_decode_quad_kernel, dim3((unsigned)((a.rows + DEC_WAVES - 1) / DEC_WAVES)),
                       dim3(DEC_WAVES * 64), lds, stream, a);
    return;
  }
  if (g_decode_rows && a.ecol) {
    const size_t lds = (size_t)DEC_WAVES * a.n_cols * sizeof(unsigned long long);
    hipLaunchKernelGGL(sample_decode_row_kernel, dim3((unsigned)((a.rows + DEC_WAVES - 1) / DEC_WAVES)),
                       dim3(DEC_WAVES * 64), lds, stream, a);
    return;
  }
  hipLaunchKernelGGL(sample_decode_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, a);
}

// Generation weight views in one launch (EngineConfig.gen_bf16): for every generator layer, the
// dense columns [0, kd) of W as a bf16 copy (the values the GEMM's staging would round) and the
// one-hot block [kd, kd + C) transposed to [C, N] fp32 (coalesced epilogue gathers).  Replaces six
// small copy launches per generation pass.
__global__ __launch_bounds__(256) void gen_weight_prep_kernel(GenWeightPrep a) {
  int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int j = 0; j < a.n_jobs; ++j) {
    const GenWeightJob& J = a.jobs[j];
    const int64_t nd = (int64_t)J.N * J.kd, nc = (int64_t)J.N * J.C;
    if (e < nd) {
      const int n = (int)(e / J.kd), k = (int)(e % J.kd);
      J.w16[(size_t)n * J.ld16 + k] = f2bf(J.w[(size_t)n * J.ldw + (size_t)k * J.skw]);
      return;
    }
    e -= nd;
    if (e < nc) {
      const int n = (int)(e / J.C), c = (int)(e % J.C);
      J.wt[(size_t)c * J.N + n] = J.w[(size_t)n * J.ldw + (size_t)(J.kd + c) * J.skw];
      return;
    }
    e -= nc;
  }
}

void launch_gen_weight_prep(const GenWeightPrep& a, hipStream_t stream) {
  int64_t total = 0;
  for (int j = 0; j < a.n_jobs; ++j) total += (int64_t)a.jobs[j].N * (a.jobs[j].kd + a.jobs[j].C);
  if (total == 0) return;
  require_unbatched("gen_weight_prep");
  hipLaunchKernelGGL(gen_weight_prep_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, a);
}

template <bool BT_ = false>
__global__ void rng_bump_kernel(uint64_t* ctr, ClientBatch cb) {
  const BIdx bi_ = batch_bidx<BT_>(cb.xcd);
  ctr = cptr(ctr, (int64_t)bi_.z * cb.stride);
  ctr[0] += 1ull;
}

void launch_rng_bump(uint64_t* ctr, hipStream_t stream) {
  const ClientBatch cb = client_batch();
  if (cb.k > 1) check_slab(ctr, "rng counter");
  hipLaunchKernelGGL((client_batch().xcd ? rng_bump_kernel<true> : rng_bump_kernel<false>), dim3(1, 1, cb.k), dim3(1), 0, stream, ctr, cb);
}

}  // namespace fedtgan
