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

#include "common.h"
#include "launch.h"

namespace fedtgan {

// ============================================================================ sampling
constexpr int SAMPLE_THREADS = 256;
constexpr int SAMPLE_ROWS = 8;     // rows per workgroup
constexpr int MAX_PERM = 4096;

__device__ __forceinline__ void draw_cond(const SampleArgs& a, uint64_t step, int b, int& col, int& opt) {
  RngArgs rng{a.seed, a.rng_ctr, a.rng_stream};
  const uint4 r = rng4(rng, step, (uint64_t)b);
  col = min((int)(u01(r.x) * a.n_col), a.n_col - 1);
  const float u = u01(r.y);
  const float* cdf = a.cdf + (size_t)col * a.maxw;
  const int w = a.cond_w[col];
  int o = 0;
  while (o < w - 1 && !(cdf[o] > u)) ++o;
  opt = o;
}

__global__ __launch_bounds__(SAMPLE_THREADS) void sample_kernel(SampleArgs a) {
  __shared__ uint64_t keys[MAX_PERM];
  __shared__ int perm_rows[SAMPLE_ROWS];
  const uint64_t step = a.rng_ctr ? *a.rng_ctr : 0ull;
  const int tid = threadIdx.x;
  if (blockIdx.x == 0 && tid == 0) {
    if (a.step_bump) a.step_bump[0] += 1.0f;
    if (a.zero_metrics && a.metrics) {
      a.metrics[0] = 0.f; a.metrics[1] = 0.f; a.metrics[2] = 0.f; a.metrics[3] = 0.f;
    }
  }
  const int r0 = blockIdx.x * SAMPLE_ROWS;
  const bool with_real = a.xr != nullptr && a.n_col > 0;
  // ---- random permutation of the batch (identical in every workgroup: same Philox keys)
  if (with_real) {
    int p2 = 1;
    while (p2 < a.B) p2 <<= 1;
    RngArgs rk{a.seed, a.rng_ctr, a.rng_stream + 1u};
    for (int i = tid; i < p2; i += blockDim.x) {
      uint64_t k = ~0ull;
      if (i < a.B) k = ((uint64_t)rng4(rk, step, (uint64_t)i).x << 32) | (uint64_t)i;
      keys[i] = k;
    }
    __syncthreads();
    for (int size = 2; size <= p2; size <<= 1) {
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        for (int i = tid; i < p2; i += blockDim.x) {
          const int j = i ^ stride;
          if (j > i) {
            const bool up = (i & size) == 0;
            const uint64_t ki = keys[i], kj = keys[j];
            if ((ki > kj) == up) { keys[i] = kj; keys[j] = ki; }
          }
        }
        __syncthreads();
      }
    }
    if (tid < SAMPLE_ROWS && r0 + tid < a.B) perm_rows[tid] = (int)(keys[r0 + tid] & 0xffffffffu);
    __syncthreads();
  }
  // ---- this workgroup's rows: noise + conditional vector
  for (int rr = 0; rr < SAMPLE_ROWS; ++rr) {
    const int b = r0 + rr;
    if (b >= a.B) break;
    int col = 0, opt = 0;
    if (a.n_col > 0) draw_cond(a, step, b, col, opt);
    const int hot = a.n_col > 0 ? a.cond_off[col] + opt : -1;
    float* hrow = a.h + (size_t)b * a.ldh;
    RngArgs rz{a.seed, a.rng_ctr, a.rng_stream + 2u};
    for (int i = tid; i < (a.E + 1) / 2; i += blockDim.x) {
      const uint4 r = rng4(rz, step, (uint64_t)b * a.E + i);
      const float2 z = box_muller(r.x, r.y);
      hrow[a.zc + 2 * i] = z.x;
      if (2 * i + 1 < a.E) hrow[a.zc + 2 * i + 1] = z.y;
    }
    for (int i = tid; i < a.C; i += blockDim.x) {
      const float v = (i == hot) ? 1.f : 0.f;
      hrow[a.cc + i] = v;
      if (a.xf) a.xf[(size_t)b * a.ldx + a.Dd + i] = v;
    }
    if (tid == 0 && a.col) { a.col[b] = col; a.opt[b] = opt; }
    if (!with_real) continue;
    // real row for the permuted condition
    const int p = perm_rows[rr];
    int pc = 0, po = 0;
    draw_cond(a, step, p, pc, po);
    const int64_t cnt = a.row_cnt[(size_t)pc * a.maxw + po];
    RngArgs rp{a.seed, a.rng_ctr, a.rng_stream + 3u};
    const uint4 rr4 = rng4(rp, step, (uint64_t)b);
    int64_t pick = (int64_t)(u01d(rr4.x, rr4.y) * (double)(cnt > 0 ? cnt : 1));
    if (pick >= cnt) pick = cnt > 0 ? cnt - 1 : 0;
    const int64_t row = a.rows[a.row_off[(size_t)pc * a.maxw + po] + pick];
    const float* src = a.data + (size_t)row * a.Dd;
    float* dst = a.xr + (size_t)b * a.ldx;
    for (int i = tid; i < a.Dd; i += blockDim.x) dst[i] = src[i];
    const int phot = a.cond_off[pc] + po;
    for (int i = tid; i < a.C; i += blockDim.x) dst[a.Dd + i] = (i == phot) ? 1.f : 0.f;
  }
}

void launch_sample(const SampleArgs& a, hipStream_t stream) {
  const int blocks = (a.B + SAMPLE_ROWS - 1) / SAMPLE_ROWS;
  hipLaunchKernelGGL(sample_kernel, dim3(blocks), dim3(SAMPLE_THREADS), 0, stream, a);
}

// ============================================================================ activation
// one thread per (row, span); softmax spans are short (<= a few dozen options)
__global__ __launch_bounds__(256) void activate_kernel(const float* __restrict__ logits, int ldl, float* __restrict__ out,
                                                       int ldo, int rows, SpanTables sp, float inv_tau, uint64_t seed,
                                                       const uint64_t* ctr, uint32_t stream_id) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)rows * sp.n_span) return;
  const int r = (int)(idx / sp.n_span), s = (int)(idx % sp.n_span);
  const int st = sp.start[s], w = sp.width[s];
  const float* x = logits + (size_t)r * ldl + st;
  float* y = out + (size_t)r * ldo + st;
  if (sp.kind[s] == 0) {
    for (int i = 0; i < w; ++i) y[i] = tanhf(x[i]);
    return;
  }
  const uint64_t step = ctr ? *ctr : 0ull;
  RngArgs rng{seed, ctr, stream_id};
  const uint64_t base = ((uint64_t)r << 20) + (uint64_t)st;
  float mx = -INFINITY;
  for (int i = 0; i < w; i += 4) {
    const uint4 u = rng4(rng, step, base + i);
    const uint32_t uu[4] = {u.x, u.y, u.z, u.w};
    for (int q = 0; q < 4 && i + q < w; ++q) {
      const float v = (x[i + q] + gumbel(uu[q])) * inv_tau;
      y[i + q] = v;
      mx = fmaxf(mx, v);
    }
  }
  float sum = 0.f;
  for (int i = 0; i < w; ++i) {
    const float e = __expf(y[i] - mx);
    y[i] = e;
    sum += e;
  }
  const float inv = 1.f / sum;
  for (int i = 0; i < w; ++i) y[i] *= inv;
}

void launch_activate(const float* logits, int ldl, float* out, int ldo, int rows, SpanTables sp, float tau,
                     uint64_t seed, const uint64_t* ctr, uint32_t stream_id, hipStream_t stream) {
  const int64_t n = (int64_t)rows * sp.n_span;
  if (n == 0) return;
  hipLaunchKernelGGL(activate_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, logits, ldl, out, ldo,
                     rows, sp, 1.f / tau, seed, ctr, stream_id);
}

__global__ __launch_bounds__(256) void act_bwd_ce_kernel(const float* __restrict__ dact, int ldd,
                                                         const float* __restrict__ act, int lda,
                                                         const float* __restrict__ logits, int ldl, SpanTables sp,
                                                         const int* __restrict__ col, const int* __restrict__ opt,
                                                         float* __restrict__ dl, int ldg, int rows, float inv_tau,
                                                         float* loss) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)rows * sp.n_span) return;
  const int r = (int)(idx / sp.n_span), s = (int)(idx % sp.n_span);
  const int st = sp.start[s], w = sp.width[s];
  const float* g = dact + (size_t)r * ldd + st;
  const float* y = act + (size_t)r * lda + st;
  float* d = dl + (size_t)r * ldg + st;
  if (sp.kind[s] == 0) {
    for (int i = 0; i < w; ++i) d[i] = g[i] * (1.f - y[i] * y[i]);
    return;
  }
  float dot = 0.f;
  for (int i = 0; i < w; ++i) dot += g[i] * y[i];
  for (int i = 0; i < w; ++i) d[i] = y[i] * (g[i] - dot) * inv_tau;
  const int ci = sp.cond_idx[s];
  if (ci >= 0 && col[r] == ci) {
    const float* x = logits + (size_t)r * ldl + st;
    float mx = -INFINITY;
    for (int i = 0; i < w; ++i) mx = fmaxf(mx, x[i]);
    float sum = 0.f;
    for (int i = 0; i < w; ++i) sum += __expf(x[i] - mx);
    const float lse = mx + __logf(sum);
    const int o = min(opt[r], w - 1);
    const float invB = 1.f / (float)rows;
    for (int i = 0; i < w; ++i) d[i] += (__expf(x[i] - lse) - (i == o ? 1.f : 0.f)) * invB;
    atomicAdd(loss, (lse - x[o]) * invB);
  }
}

void launch_act_bwd_ce(const float* dact, int ldd, const float* act, int lda, const float* logits, int ldl, SpanTables sp,
                       const int* col, const int* opt, float* dlogits, int ldg, int rows, float tau, float* loss,
                       hipStream_t stream) {
  const int64_t n = (int64_t)rows * sp.n_span;
  if (n == 0) return;
  hipLaunchKernelGGL(act_bwd_ce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, dact, ldd, act, lda,
                     logits, ldl, sp, col, opt, dlogits, ldg, rows, 1.f / tau, loss);
}

// ============================================================================ gradient penalty pieces
// one wave per row
__global__ __launch_bounds__(256) void slerp_kernel(const float* __restrict__ real, const float* __restrict__ fake,
                                                    float* __restrict__ out, int rows, int cols, int ld, uint64_t seed,
                                                    const uint64_t* ctr, uint32_t stream_id) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
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
  float cosw = sab / (sqrtf(saa) * sqrtf(sbb));
  cosw = fminf(1.f, fmaxf(-1.f, cosw));
  const float om = acosf(cosw);
  const float so = sinf(om);
  float wa, wb;
  if (so < 1e-6f) { wa = 1.f - alpha; wb = alpha; }
  else { wa = sinf((1.f - alpha) * om) / so; wb = sinf(alpha * om) / so; }
  float* o = out + (size_t)r * ld;
  for (int i = lane; i < cols; i += 64) o[i] = wa * a[i] + wb * b[i];
}

void launch_slerp(const float* real, const float* fake, float* out, int rows, int cols, int ld, uint64_t seed,
                  const uint64_t* ctr, uint32_t stream_id, hipStream_t stream) {
  if (rows == 0) return;
  hipLaunchKernelGGL(slerp_kernel, dim3((rows + 3) / 4), dim3(256), 0, stream, real, fake, out, rows, cols, ld, seed,
                     ctr, stream_id);
}

// one workgroup per packed row
__global__ __launch_bounds__(256) void gp_scale_kernel(const float* __restrict__ g, int ldg, float* __restrict__ out,
                                                       int ldo, int rows, int cols, float lam, float* loss) {
  __shared__ float sh[8];
  const int r = blockIdx.x;
  const float* x = g + (size_t)r * ldg;
  float s = 0.f;
  for (int i = threadIdx.x; i < cols; i += blockDim.x) s += x[i] * x[i];
  s = block_sum(s, sh);
  const float n = sqrtf(s);
  const float coef = lam * 2.f * (n - 1.f) / (fmaxf(n, 1e-30f) * (float)rows);
  float* o = out + (size_t)r * ldo;
  for (int i = threadIdx.x; i < cols; i += blockDim.x) o[i] = coef * x[i];
  if (threadIdx.x == 0) atomicAdd(loss, lam * (n - 1.f) * (n - 1.f) / (float)rows);
}

void launch_gp_scale(const float* g, int ldg, float* out, int ldo, int rows, int cols, float lam, float* loss,
                     hipStream_t stream) {
  if (rows == 0) return;
  hipLaunchKernelGGL(gp_scale_kernel, dim3(rows), dim3(256), 0, stream, g, ldg, out, ldo, rows, cols, lam, loss);
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
  hipLaunchKernelGGL(d_head_kernel, dim3((rows + 3) / 4), dim3(256), 0, stream, d, ldd, ms, ldms, v, e, coef, wloss, y,
                     a, lda, rows, cols, loss);
}

// ============================================================================ column sums (bias grads)
constexpr int CS_COLS = 64, CS_GROUPS = 16;
struct ColsumBatch {
  ColsumJob jobs[8];
  int n_jobs;
};

__global__ __launch_bounds__(CS_COLS* CS_GROUPS) void colsum_kernel(ColsumBatch bt) {
  __shared__ float part[CS_GROUPS][CS_COLS + 1];
  const ColsumJob jb = bt.jobs[blockIdx.y];
  const int c = blockIdx.x * CS_COLS + (threadIdx.x % CS_COLS);
  const int grp = threadIdx.x / CS_COLS;
  if ((int)(blockIdx.x * CS_COLS) >= jb.cols) return;
  float s = 0.f;
  if (c < jb.cols) {
#pragma unroll 8
    for (int r = grp; r < jb.rows; r += CS_GROUPS) s += jb.a[(size_t)r * jb.lda + c];
  }
  part[grp][threadIdx.x % CS_COLS] = s;
  __syncthreads();
  if (grp == 0 && c < jb.cols) {
    float t = 0.f;
    for (int i = 0; i < CS_GROUPS; ++i) t += part[i][threadIdx.x];
    jb.out[c] = t;
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
  hipLaunchKernelGGL(colsum_kernel, dim3((maxc + CS_COLS - 1) / CS_COLS, n_jobs), dim3(CS_COLS * CS_GROUPS), 0, stream,
                     bt);
}

// ============================================================================ batch norm + relu
constexpr int BN_COLS = 32, BN_GROUPS = 16, BN_MAXR = 64;   // rows per thread kept in registers: rows <= 1024

__global__ __launch_bounds__(BN_COLS* BN_GROUPS) void bn_relu_train_kernel(
    const float* __restrict__ a, int lda, const float* __restrict__ gamma, const float* __restrict__ beta,
    float* __restrict__ out, int ldo, float* __restrict__ nhat, int ldn, float* __restrict__ mean,
    float* __restrict__ invstd, float* __restrict__ rm, float* __restrict__ rv, int rows, int cols, float momentum,
    float eps) {
  __shared__ float red[BN_GROUPS][BN_COLS + 1];
  __shared__ float stat[2][BN_COLS];
  const int lc = threadIdx.x % BN_COLS, grp = threadIdx.x / BN_COLS;
  const int c = blockIdx.x * BN_COLS + lc;
  const bool ok = c < cols;
  float x[BN_MAXR];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < BN_MAXR; ++i) {
    const int r = grp + i * BN_GROUPS;
    x[i] = (ok && r < rows) ? a[(size_t)r * lda + c] : 0.f;
    s += x[i];
  }
  red[grp][lc] = s;
  __syncthreads();
  if (grp == 0) {
    float t = 0.f;
    for (int i = 0; i < BN_GROUPS; ++i) t += red[i][lc];
    stat[0][lc] = t / (float)rows;
  }
  __syncthreads();
  const float mu = stat[0][lc];
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < BN_MAXR; ++i) {
    const int r = grp + i * BN_GROUPS;
    const float d = (r < rows) ? x[i] - mu : 0.f;
    q += d * d;
  }
  __syncthreads();
  red[grp][lc] = q;
  __syncthreads();
  if (grp == 0) {
    float t = 0.f;
    for (int i = 0; i < BN_GROUPS; ++i) t += red[i][lc];
    const float var = t / (float)rows;
    stat[1][lc] = rsqrtf(var + eps);
    if (ok) {
      mean[c] = mu;
      invstd[c] = stat[1][lc];
      rm[c] = (1.f - momentum) * rm[c] + momentum * mu;
      rv[c] = (1.f - momentum) * rv[c] + momentum * var * (float)rows / (float)max(rows - 1, 1);
    }
  }
  __syncthreads();
  if (!ok) return;
  const float is = stat[1][lc], gm = gamma[c], bt = beta[c];
#pragma unroll
  for (int i = 0; i < BN_MAXR; ++i) {
    const int r = grp + i * BN_GROUPS;
    if (r < rows) {
      const float n = (x[i] - mu) * is;
      nhat[(size_t)r * ldn + c] = n;
      const float y = n * gm + bt;
      out[(size_t)r * ldo + c] = y > 0.f ? y : 0.f;
    }
  }
}

void launch_bn_relu_train(const float* a, int lda, const float* gamma, const float* beta, float* out, int ldo,
                          float* nhat, int ldn, float* mean, float* invstd, float* rm, float* rv, int rows, int cols,
                          float momentum, float eps, hipStream_t stream) {
  hipLaunchKernelGGL(bn_relu_train_kernel, dim3((cols + BN_COLS - 1) / BN_COLS), dim3(BN_COLS * BN_GROUPS), 0, stream, a,
                     lda, gamma, beta, out, ldo, nhat, ldn, mean, invstd, rm, rv, rows, cols, momentum, eps);
}

__global__ __launch_bounds__(BN_COLS* BN_GROUPS) void bn_relu_bwd_kernel(
    const float* __restrict__ dr, int lddr, const float* __restrict__ r_, int ldr, const float* __restrict__ nhat,
    int ldn, const float* __restrict__ gamma, const float* __restrict__ invstd, float* __restrict__ da, int ldda,
    float* __restrict__ dgamma, float* __restrict__ dbeta, float* __restrict__ dbias, int rows, int cols) {
  __shared__ float red[2][BN_GROUPS][BN_COLS + 1];
  __shared__ float stat[2][BN_COLS];
  const int lc = threadIdx.x % BN_COLS, grp = threadIdx.x / BN_COLS;
  const int c = blockIdx.x * BN_COLS + lc;
  const bool ok = c < cols;
  float dy[BN_MAXR], nh[BN_MAXR];
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int i = 0; i < BN_MAXR; ++i) {
    const int r = grp + i * BN_GROUPS;
    float d = 0.f, n = 0.f;
    if (ok && r < rows) {
      const float rr = r_[(size_t)r * ldr + c];
      d = rr > 0.f ? dr[(size_t)r * lddr + c] : 0.f;
      n = nhat[(size_t)r * ldn + c];
    }
    dy[i] = d;
    nh[i] = n;
    s1 += d;
    s2 += d * n;
  }
  red[0][grp][lc] = s1;
  red[1][grp][lc] = s2;
  __syncthreads();
  if (grp == 0) {
    float t1 = 0.f, t2 = 0.f;
    for (int i = 0; i < BN_GROUPS; ++i) { t1 += red[0][i][lc]; t2 += red[1][i][lc]; }
    stat[0][lc] = t1;
    stat[1][lc] = t2;
    if (ok) { dbeta[c] = t1; dgamma[c] = t2; }
  }
  __syncthreads();
  if (!ok) return;
  const float sdy = stat[0][lc], sdyn = stat[1][lc];
  const float k = gamma[c] * invstd[c];
  const float invn = 1.f / (float)rows;
  float sda = 0.f;
#pragma unroll
  for (int i = 0; i < BN_MAXR; ++i) {
    const int r = grp + i * BN_GROUPS;
    if (r < rows) {
      const float v = k * (dy[i] - sdy * invn - nh[i] * sdyn * invn);
      da[(size_t)r * ldda + c] = v;
      sda += v;
    }
  }
  if (dbias) {
    __syncthreads();
    red[0][grp][lc] = sda;
    __syncthreads();
    if (grp == 0) {
      float t = 0.f;
      for (int i = 0; i < BN_GROUPS; ++i) t += red[0][i][lc];
      dbias[c] = t;
    }
  }
}

void launch_bn_relu_bwd(const float* dr, int lddr, const float* r, int ldr, const float* nhat, int ldn,
                        const float* gamma, const float* invstd, float* da, int ldda, float* dgamma, float* dbeta,
                        float* dbias, int rows, int cols, hipStream_t stream) {
  hipLaunchKernelGGL(bn_relu_bwd_kernel, dim3((cols + BN_COLS - 1) / BN_COLS), dim3(BN_COLS * BN_GROUPS), 0, stream, dr,
                     lddr, r, ldr, nhat, ldn, gamma, invstd, da, ldda, dgamma, dbeta, dbias, rows, cols);
}

// ============================================================================ Adam
__global__ __launch_bounds__(256) void adam_kernel(float4* __restrict__ p, const float4* __restrict__ g,
                                                   float4* __restrict__ m, float4* __restrict__ v,
                                                   const float* __restrict__ step, int64_t n4, float lr, float b1,
                                                   float b2, float eps, float wd, uint64_t* rng_bump) {
  const float t = step[0];
  const float bc1 = 1.f - powf(b1, t);
  const float bc2s = sqrtf(1.f - powf(b2, t));
  const float sz = lr / bc1;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    float4 pp = p[i], gg = g[i], mm = m[i], vv = v[i];
    float* pf = reinterpret_cast<float*>(&pp);
    float* gf = reinterpret_cast<float*>(&gg);
    float* mf = reinterpret_cast<float*>(&mm);
    float* vf = reinterpret_cast<float*>(&vv);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float gq = gf[q] + wd * pf[q];
      mf[q] = b1 * mf[q] + (1.f - b1) * gq;
      vf[q] = b2 * vf[q] + (1.f - b2) * gq * gq;
      pf[q] -= sz * mf[q] / (sqrtf(vf[q]) / bc2s + eps);
    }
    p[i] = pp; m[i] = mm; v[i] = vv;
  }
  if (rng_bump && blockIdx.x == 0 && threadIdx.x == 0) rng_bump[0] += 1ull;
}

__global__ void adam_tail_kernel(float* p, const float* g, float* m, float* v, const float* step, int64_t start,
                                 int64_t n, float lr, float b1, float b2, float eps, float wd) {
  const int64_t i = start + threadIdx.x;
  if (i >= n) return;
  const float t = step[0];
  const float bc1 = 1.f - powf(b1, t);
  const float bc2s = sqrtf(1.f - powf(b2, t));
  const float gq = g[i] + wd * p[i];
  m[i] = b1 * m[i] + (1.f - b1) * gq;
  v[i] = b2 * v[i] + (1.f - b2) * gq * gq;
  p[i] -= (lr / bc1) * m[i] / (sqrtf(v[i]) / bc2s + eps);
}

void launch_adam(float* p, const float* g, float* m, float* v, const float* step, int64_t n, float lr, float b1,
                 float b2, float eps, float wd, uint64_t* rng_ctr_bump, hipStream_t stream) {
  const int64_t n4 = n / 4;
  const int blocks = (int)std::min<int64_t>((n4 + 255) / 256, 1024);
  hipLaunchKernelGGL(adam_kernel, dim3(std::max(blocks, 1)), dim3(256), 0, stream, reinterpret_cast<float4*>(p),
                     reinterpret_cast<const float4*>(g), reinterpret_cast<float4*>(m), reinterpret_cast<float4*>(v),
                     step, n4, lr, b1, b2, eps, wd, rng_ctr_bump);
  if (n4 * 4 < n)
    hipLaunchKernelGGL(adam_tail_kernel, dim3(1), dim3(64), 0, stream, p, g, m, v, step, n4 * 4, n, lr, b1, b2, eps,
                       wd);
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
    val = al * 4.0 * a.sd[(size_t)c * a.K + best] + a.mu[(size_t)c * a.K + best];
  } else {
    val = a.codes[a.code_off[j] + best];
  }
  a.out[(size_t)r * a.n_cols + j] = val;
}

void launch_sample_decode(const DecodeArgs& a, hipStream_t stream) {
  const int64_t n = (int64_t)a.rows * a.n_cols;
  if (n == 0) return;
  hipLaunchKernelGGL(sample_decode_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, a);
}

__global__ void rng_bump_kernel(uint64_t* ctr) { ctr[0] += 1ull; }

void launch_rng_bump(uint64_t* ctr, hipStream_t stream) {
  hipLaunchKernelGGL(rng_bump_kernel, dim3(1), dim3(1), 0, stream, ctr);
}

}  // namespace fedtgan
