// Batched 1-D variational DP-GMM fit (K3): the data passes of the EM loop, for every
// continuous column at once.
//
// Reference: sklearn `BayesianGaussianMixture.fit` with 10 components and a DP prior
// (Server/dtds/features/transformers.py:334-340), one column at a time, plus the federator's
// refit of the global GMM (Server/dtds/distributed.py:725-745). The torch version
// (fed_tgan_amd/features/vgm_fit.py) materialises [n_cols, N, K] fp64 tensors several times
// per iteration. Here every iteration reads the data ONCE:
//
//   vgm_estep_kernel    responsibilities of all K components from the current variational
//                       posterior + the sufficient statistics sum r, sum r x, sum r x^2 and the
//                       entropy term sum r log r, reduced per workgroup (fp64)
//   kmeans_step_kernel  Lloyd assignment (nearest centre, lowest index on ties) + per-centre
//                       count, sum and sum of squares (the last pass seeds the first M-step)
//
// Grid: blockIdx.y = column, blockIdx.x = row chunk. Each workgroup writes one partial record
// [n_cols, n_chunks, R]. The host sums the chunk axis with a fixed-shape reduction, so results
// are deterministic, and runs the tiny [n_cols, K] M-step.
// Data are fp64 and centred per column on the host (numerically like sklearn's centred
// second moments).
//
//   vgm_fit_kernel      the WHOLE fit of a column in one workgroup (seeding, Lloyd, EM loop with
//                       device-side M-step / lower bound / convergence): one launch per fit
#include <algorithm>
#include <stdexcept>
#include <string>

#include "common.h"
#include "launch.h"

namespace fedtgan {

constexpr int FIT_K = 10;
constexpr int FIT_THREADS = 256;

// block-reduce NV doubles per thread into out[0..NV) (deterministic order)
template <int NV>
__device__ __forceinline__ void block_reduce_d(double (&v)[NV], double* out) {
  __shared__ double red[FIT_THREADS / 64][NV];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const double s = wave_sum_d(v[i]);
    if (lane == 0) red[w][i] = s;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < NV; i += blockDim.x) {
    double s = 0.0;
#pragma unroll
    for (int ww = 0; ww < FIT_THREADS / 64; ++ww) s += red[ww][i];
    out[i] = s;
  }
}

__global__ __launch_bounds__(FIT_THREADS) void vgm_estep_kernel(VgmFitArgs a) {
  constexpr int NV = 3 * FIT_K + 1;
  const int j = blockIdx.y;
  const int n = a.n_rows[j];
  const double* x = a.x + (size_t)j * a.ldx;
  double cst[FIT_K], mu[FIT_K], pc[FIT_K];
#pragma unroll
  for (int k = 0; k < FIT_K; ++k) {
    cst[k] = a.consts[j * FIT_K + k];
    mu[k] = a.means[j * FIT_K + k];
    pc[k] = a.prec[j * FIT_K + k];
  }
  double acc[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) acc[i] = 0.0;
  const int r0 = blockIdx.x * a.rows_per_block;
  const int r1 = min(n, r0 + a.rows_per_block);
  for (int r = r0 + threadIdx.x; r < r1; r += blockDim.x) {
    const double xv = x[r];
    double lp[FIT_K], mx = -INFINITY;
#pragma unroll
    for (int k = 0; k < FIT_K; ++k) {
      const double y = (xv - mu[k]) * pc[k];
      lp[k] = cst[k] - 0.5 * y * y;
      mx = fmax(mx, lp[k]);
    }
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < FIT_K; ++k) s += exp(lp[k] - mx);
    const double lse = mx + log(s);
#pragma unroll
    for (int k = 0; k < FIT_K; ++k) {
      const double lr = lp[k] - lse;
      const double rk = exp(lr);
      acc[k] += rk;
      acc[FIT_K + k] += rk * xv;
      acc[2 * FIT_K + k] += rk * xv * xv;
      acc[3 * FIT_K] += rk * lr;
    }
  }
  block_reduce_d<NV>(acc, a.partial + ((size_t)j * gridDim.x + blockIdx.x) * NV);
}

__global__ __launch_bounds__(FIT_THREADS) void kmeans_step_kernel(VgmFitArgs a) {
  constexpr int NV = 3 * FIT_K;
  const int j = blockIdx.y;
  const int n = a.n_rows[j];
  const double* x = a.x + (size_t)j * a.ldx;
  double c[FIT_K];
#pragma unroll
  for (int k = 0; k < FIT_K; ++k) c[k] = a.means[j * FIT_K + k];
  double acc[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) acc[i] = 0.0;
  const int r0 = blockIdx.x * a.rows_per_block;
  const int r1 = min(n, r0 + a.rows_per_block);
  for (int r = r0 + threadIdx.x; r < r1; r += blockDim.x) {
    const double xv = x[r];
    int best = 0;
    double bd = (xv - c[0]) * (xv - c[0]);
#pragma unroll
    for (int k = 1; k < FIT_K; ++k) {
      const double d = (xv - c[k]) * (xv - c[k]);
      if (d < bd) {
        bd = d;
        best = k;
      }
    }
#pragma unroll
    for (int k = 0; k < FIT_K; ++k) {
      const double hit = k == best ? 1.0 : 0.0;
      acc[k] += hit;
      acc[FIT_K + k] += hit * xv;
      acc[2 * FIT_K + k] += hit * xv * xv;
    }
  }
  block_reduce_d<NV>(acc, a.partial + ((size_t)j * gridDim.x + blockIdx.x) * NV);
}

// ============================================================================ whole fit
// The entire fit of one column in ONE workgroup, every column concurrently (grid = n_cols): seeding,
// Lloyd, the hard-assignment M-step, then the variational EM loop with its M-step, lower bound and
// convergence test on the device -- no host round trip per iteration (the per-pass kernels above
// plus torch M-steps cost ~10 fp64 launches and a host sync per iteration).
//
// Math: sklearn BayesianGaussianMixture (weight_concentration_prior_type="dirichlet_process",
// full covariance, n_features = 1), `_initialize` -> loop { `_e_step`, `_m_step`,
// `_compute_lower_bound`; stop when |change| < tol }; priors beta0 = 1, nu0 = 1, m0 = 0 (data
// centred on the host), W0^-1 = var(x, ddof=1), reg_covar.
constexpr int WF_THREADS = 1024, WF_WAVES = WF_THREADS / 64;

// digamma for x > 0: recurrence up to x >= 6, then the asymptotic series (|err| < 1e-14)
__device__ double digamma_d(double x) {
  double r = 0.0;
  while (x < 6.0) {
    r -= 1.0 / x;
    x += 1.0;
  }
  const double f = 1.0 / (x * x);
  return r + log(x) - 0.5 / x -
         f * (1.0 / 12 - f * (1.0 / 120 - f * (1.0 / 252 - f * (1.0 / 240 - f * (1.0 / 132 - f * (691.0 / 32760))))));
}

template <int NV>
__device__ __forceinline__ void wf_reduce(double (&v)[NV], double* red, double* out) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const double s = wave_sum_d(v[i]);
    if (lane == 0) red[w * NV + i] = s;
  }
  __syncthreads();
  if (threadIdx.x < NV) {
    double s = 0.0;
    for (int ww = 0; ww < WF_WAVES; ++ww) s += red[ww * NV + threadIdx.x];
    out[threadIdx.x] = s;
  }
  __syncthreads();
}

struct WfState {
  double a[FIT_K], b[FIT_K], beta[FIT_K], mean[FIT_K], dof[FIT_K], cov[FIT_K], pc[FIT_K], cst[FIT_K];
  double lbk[FIT_K];
};

// M-step from the sufficient statistics st = [nk | sum r x | sum r x^2] (thread k < K owns component k)
__device__ __forceinline__ void wf_mstep(const double* st, WfState& s, double wprior, double cov0, double reg) {
  const int k = threadIdx.x;
  if (k < FIT_K) {
    const double eps10 = 10.0 * 2.220446049250313e-16;
    const double nraw = st[k], nk = nraw + eps10;
    const double xk = st[FIT_K + k] / nk;
    const double sk = fmax(st[2 * FIT_K + k] - 2.0 * xk * st[FIT_K + k] + xk * xk * nraw, 0.0) / nk + reg;
    double tail = 0.0;   // sum_{j > k} nk_j
    for (int j = k + 1; j < FIT_K; ++j) tail += st[j] + eps10;
    s.a[k] = 1.0 + nk;
    s.b[k] = wprior + tail;
    s.beta[k] = 1.0 + nk;
    s.mean[k] = nk * xk / s.beta[k];
    s.dof[k] = 1.0 + nk;
    s.cov[k] = (cov0 + nk * sk + nk / s.beta[k] * xk * xk) / s.dof[k];
    s.pc[k] = 1.0 / sqrt(s.cov[k]);
    // per-component lower-bound terms: -log_wishart_k - log_norm_weight_k - 0.5 log beta_k
    const double logdet = log(s.pc[k]) - 0.5 * log(s.dof[k]);
    const double lw = -(s.dof[k] * logdet + s.dof[k] * 0.5 * 0.6931471805599453 + lgamma(0.5 * s.dof[k]));
    const double betaln = lgamma(s.a[k]) + lgamma(s.b[k]) - lgamma(s.a[k] + s.b[k]);
    s.lbk[k] = -lw + betaln - 0.5 * log(s.beta[k]);
  }
  __syncthreads();
  if (k < FIT_K) {   // E-step constants (need every component's stick terms)
    double pre = 0.0;
    for (int j = 0; j < k; ++j) pre += digamma_d(s.b[j]) - digamma_d(s.a[j] + s.b[j]);
    const double logw = digamma_d(s.a[k]) - digamma_d(s.a[k] + s.b[k]) + pre;
    s.cst[k] = logw - 0.9189385332046727 + log(s.pc[k]) - 0.5 * log(s.dof[k]) +
               0.5 * (0.6931471805599453 + digamma_d(0.5 * s.dof[k]) - 1.0 / s.beta[k]);
  }
  __syncthreads();
}

// Split fit: the E-step statistics of the G workgroups of column j.  Wave 0 publishes this workgroup's record
// with agent-scope stores, thread 0 arrives on the column's counter (agent release) and spins on relaxed loads
// until all G records of this pass are in (one acquire after), then wave 0 sums the G records in workgroup
// order -- the same bits in every workgroup of the column, so all of them take the same M-step and stop at the
// same iteration.  Records are double-buffered by pass: a workgroup can only overwrite a slot after every
// workgroup of its column arrived at the next pass, i.e. finished reading this one.  The spin is bounded; a
// timeout stops waiting (so the grid always drains) and poisons the whole column: the timed-out workgroup
// stores the column's dead flag (sync[32j + 1]) BEFORE its next arrival, so every workgroup whose barrier
// count includes such an arrival sees the flag after its acquire, and workgroup 0 reports the column
// (info[2j+1] = -1) even when it was another workgroup that timed out.
constexpr int VGM_XP = 32;                    // doubles per record (3K + 1 used)
constexpr unsigned VGM_SPIN_LIMIT = 1u << 22;

template <int NV>
__device__ __forceinline__ void cluster_sum(const VgmFitAllArgs& a, int j, int g, int G, int pass, double* tot,
                                            int* dead) {
  double* rec = a.xpart + ((size_t)(j * 2 + (pass & 1)) * G) * VGM_XP;
  const int t = threadIdx.x;
  if (t < NV) __hip_atomic_store(&rec[g * VGM_XP + t], tot[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (t == 0) {
    unsigned* cnt = a.sync + (size_t)j * 32;
    unsigned* col_dead = cnt + 1;
    __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned target = (unsigned)(pass + 1) * (unsigned)G;
    unsigned spins = 0;
    while (!*dead && __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (__hip_atomic_load(col_dead, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) *dead = 1;
      if (++spins > VGM_SPIN_LIMIT) {
        *dead = 1;
        __hip_atomic_store(col_dead, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    if (__hip_atomic_load(col_dead, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) *dead = 1;
  }
  __syncthreads();
  if (t < NV) {
    double s = 0.0;
    for (int q = 0; q < G; ++q) s += __hip_atomic_load(&rec[q * VGM_XP + t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    tot[t] = s;
  }
  __syncthreads();
}

__global__ __launch_bounds__(WF_THREADS) void vgm_fit_kernel(VgmFitAllArgs a) {
  __shared__ double red[WF_WAVES * (3 * FIT_K + 1)];
  __shared__ double tot[3 * FIT_K + 1];
  __shared__ double cen[FIT_K];
  __shared__ double scan[WF_THREADS];
  __shared__ WfState s;
  __shared__ int flag;
  __shared__ int dead;
  const int G = a.split > 1 ? a.split : 1;
  const int j = blockIdx.x / G, g = blockIdx.x % G, t = threadIdx.x;
  const int n = a.n_rows[j];
  // this workgroup's rows of the E-step passes
  const int e_chunk = (n + G - 1) / G;
  const int e_lo = min(n, g * e_chunk), e_hi = min(n, e_lo + e_chunk);
  if (t == 0) dead = 0;
  const double* x = a.x + (size_t)j * a.ldx;
  // ---- prior covariance: var(x, ddof=1) of the centred column
  {
    double v[1] = {0.0};
    for (int r = t; r < n; r += WF_THREADS) v[0] += x[r] * x[r];
    wf_reduce<1>(v, red, tot);
  }
  const double cov0 = tot[0] / (double)max(n - 1, 1);
  const double km_tol = 1e-4 * tot[0] / (double)max(n, 1);
  if (a.init_centers) {
    if (t < FIT_K) cen[t] = a.init_centers[j * FIT_K + t];
    __syncthreads();
  } else {
    // ---- k-means++ seeding (Philox stream per column); d2(r) = min over chosen centres, recomputed
    const RngArgs rng{a.seed, nullptr, 0x5eedu};
    const int seg = (n + WF_THREADS - 1) / WF_THREADS;
    const int lo = min(n, t * seg), hi = min(n, lo + seg);
    for (int c = 0; c < FIT_K; ++c) {
      const uint4 rw = rng4(rng, (uint64_t)j, (uint64_t)c);
      const double u = u01d(rw.x, rw.y);
      if (c == 0) {
        if (t == 0) cen[0] = x[min((int)(u * n), n - 1)];
        __syncthreads();
        continue;
      }
      double part = 0.0;
      for (int r = lo; r < hi; ++r) {
        double d = INFINITY;
        for (int q = 0; q < c; ++q) d = fmin(d, (x[r] - cen[q]) * (x[r] - cen[q]));
        part += d;
      }
      scan[t] = part;
      __syncthreads();
      if (t == 0) {   // exclusive prefix over the 1024 segment sums (sequential: deterministic)
        double run = 0.0;
        for (int i = 0; i < WF_THREADS; ++i) {
          const double v = scan[i];
          scan[i] = run;
          run += v;
        }
        tot[0] = run;
        flag = n - 1;
      }
      __syncthreads();
      const double target = u * tot[0];
      if (target >= scan[t] && (t == WF_THREADS - 1 || target < scan[t + 1]) && lo < hi) {
        double run = scan[t];
        int pick = hi - 1;
        for (int r = lo; r < hi; ++r) {
          double d = INFINITY;
          for (int q = 0; q < c; ++q) d = fmin(d, (x[r] - cen[q]) * (x[r] - cen[q]));
          run += d;
          if (run >= target) {
            pick = r;
            break;
          }
        }
        flag = pick;
      }
      __syncthreads();
      if (t == 0) cen[c] = x[flag];
      __syncthreads();
    }
    // ---- Lloyd
    for (int it = 0; it < a.km_iter; ++it) {
      double v[2 * FIT_K];
#pragma unroll
      for (int k = 0; k < 2 * FIT_K; ++k) v[k] = 0.0;
      double c[FIT_K];
#pragma unroll
      for (int k = 0; k < FIT_K; ++k) c[k] = cen[k];
      for (int r = t; r < n; r += WF_THREADS) {
        const double xv = x[r];
        int best = 0;
        double bd = (xv - c[0]) * (xv - c[0]);
#pragma unroll
        for (int k = 1; k < FIT_K; ++k) {
          const double d = (xv - c[k]) * (xv - c[k]);
          if (d < bd) {
            bd = d;
            best = k;
          }
        }
#pragma unroll
        for (int k = 0; k < FIT_K; ++k) {
          const double hit = k == best ? 1.0 : 0.0;
          v[k] += hit;
          v[FIT_K + k] += hit * xv;
        }
      }
      wf_reduce<2 * FIT_K>(v, red, tot);
      if (t == 0) {
        double shift = 0.0;
        for (int k = 0; k < FIT_K; ++k) {
          const double nc = tot[k] > 0.0 ? tot[FIT_K + k] / tot[k] : cen[k];
          shift += (nc - cen[k]) * (nc - cen[k]);
          cen[k] = nc;
        }
        flag = shift <= km_tol;
      }
      __syncthreads();
      if (flag) break;
    }
  }
  // ---- hard responsibilities of the final centres -> first M-step (sklearn `_initialize`)
  {
    double v[3 * FIT_K];
#pragma unroll
    for (int k = 0; k < 3 * FIT_K; ++k) v[k] = 0.0;
    double c[FIT_K];
#pragma unroll
    for (int k = 0; k < FIT_K; ++k) c[k] = cen[k];
    for (int r = t; r < n; r += WF_THREADS) {
      const double xv = x[r];
      int best = 0;
      double bd = (xv - c[0]) * (xv - c[0]);
#pragma unroll
      for (int k = 1; k < FIT_K; ++k) {
        const double d = (xv - c[k]) * (xv - c[k]);
        if (d < bd) {
          bd = d;
          best = k;
        }
      }
#pragma unroll
      for (int k = 0; k < FIT_K; ++k) {
        const double hit = k == best ? 1.0 : 0.0;
        v[k] += hit;
        v[FIT_K + k] += hit * xv;
        v[2 * FIT_K + k] += hit * xv * xv;
      }
    }
    wf_reduce<3 * FIT_K>(v, red, tot);
  }
  wf_mstep(tot, s, a.wprior, cov0, a.reg_covar);
  // ---- variational EM
  double lb = -INFINITY;
  int iters = 0, converged = 0;
  for (int it = 0; it < a.max_iter; ++it) {
    double cst[FIT_K], mu[FIT_K], pc[FIT_K];
#pragma unroll
    for (int k = 0; k < FIT_K; ++k) {
      cst[k] = s.cst[k];
      mu[k] = s.mean[k];
      pc[k] = s.pc[k];
    }
    double v[3 * FIT_K + 1];
#pragma unroll
    for (int k = 0; k < 3 * FIT_K + 1; ++k) v[k] = 0.0;
    for (int r = e_lo + t; r < e_hi; r += WF_THREADS) {
      const double xv = x[r];
      double lp[FIT_K], mx = -INFINITY;
#pragma unroll
      for (int k = 0; k < FIT_K; ++k) {
        const double y = (xv - mu[k]) * pc[k];
        lp[k] = cst[k] - 0.5 * y * y;
        mx = fmax(mx, lp[k]);
      }
      // (keeping exp(lp_k - mx) for r_k = e_k / sum instead of a second exp measured slower: 33 -> 40 ms per
      // Intrusion fit, 140 -> 157 ms wide; profiles/vgm_split_r5.txt)
      double ssum = 0.0;
#pragma unroll
      for (int k = 0; k < FIT_K; ++k) ssum += exp(lp[k] - mx);
      const double lse = mx + log(ssum);
#pragma unroll
      for (int k = 0; k < FIT_K; ++k) {
        const double lr = lp[k] - lse;
        const double rk = exp(lr);
        v[k] += rk;
        v[FIT_K + k] += rk * xv;
        v[2 * FIT_K + k] += rk * xv * xv;
        v[3 * FIT_K] += rk * lr;
      }
    }
    wf_reduce<3 * FIT_K + 1>(v, red, tot);
    if (G > 1) cluster_sum<3 * FIT_K + 1>(a, j, g, G, it, tot, &dead);
    const double rlr = tot[3 * FIT_K];
    wf_mstep(tot, s, a.wprior, cov0, a.reg_covar);
    double new_lb = -rlr;
#pragma unroll
    for (int k = 0; k < FIT_K; ++k) new_lb += s.lbk[k];
    iters = it + 1;
    const double change = new_lb - lb;
    lb = new_lb;
    if (fabs(change) < a.tol) {
      converged = 1;
      break;
    }
  }
  if (g != 0) return;
  if (t < FIT_K) {
    double* o = a.out + (size_t)j * 6 * FIT_K;
    o[t] = s.a[t];
    o[FIT_K + t] = s.b[t];
    o[2 * FIT_K + t] = s.beta[t];
    o[3 * FIT_K + t] = s.mean[t];
    o[4 * FIT_K + t] = s.dof[t];
    o[5 * FIT_K + t] = s.cov[t];
  }
  if (t == 0) {
    if (G > 1 && __hip_atomic_load(a.sync + (size_t)j * 32 + 1, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT)) dead = 1;
    a.info[2 * j] = iters;
    a.info[2 * j + 1] = dead ? -1 : converged;
    a.lower_bound[j] = lb;
  }
}

int g_vgm_split = 0;

int vgm_fit_split(int n_cols, int max_rows) {
  if (n_cols <= 0 || g_vgm_split == 1) return 1;
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, vgm_fit_kernel, WF_THREADS, 0) != hipSuccess)
    return 1;
  const int cap = cus * std::max(per_cu, 1) / n_cols;     // workgroups per column the device holds at once
  // auto: fill the CUs one workgroup each, >= 2 rows per thread, <= 16 per column (Intrusion 22 x 40k: G = 11,
  // 13.5 ms per fit against 14.1 at G = 9 and 33-40 at G = 1)
  int G = g_vgm_split > 1 ? g_vgm_split : std::min(std::min(16, cus / n_cols), max_rows / (2 * WF_THREADS));
  return std::max(1, std::min(G, cap));
}

void launch_vgm_fit(const VgmFitAllArgs& a, hipStream_t stream) {
  if (a.n_cols == 0) return;
  if (a.split > 1) {
    // The workgroups of a column wait for each other.  The grid is sized to what the device holds at once
    // (vgm_fit_split: <= one workgroup per CU per column at the kernel's occupancy), so on an idle device every
    // workgroup is resident; where one is not, its siblings' bounded spin times out, the column is marked dead
    // (sticky, cluster_sum) and the host refits it unsplit (features/vgm_fit.py).  A plain launch, not
    // hipLaunchCooperativeKernel: a process that had made a cooperative launch segfaulted in libamdhip64's
    // exit-time teardown under rocprofv3 (exit 139 after the tool's finalisation; plain launches exit 0,
    // profiles/exit_r6.txt).
    if (!a.xpart || !a.sync) throw std::runtime_error("vgm_fit: split fit without its record / counter buffers");
    hipLaunchKernelGGL(vgm_fit_kernel, dim3(a.n_cols * a.split), dim3(WF_THREADS), 0, stream, a);
    return;
  }
  hipLaunchKernelGGL(vgm_fit_kernel, dim3(a.n_cols), dim3(WF_THREADS), 0, stream, a);
}

static dim3 fit_grid(const VgmFitArgs& a) { return dim3((a.max_rows + a.rows_per_block - 1) / a.rows_per_block, a.n_cols); }

void launch_vgm_estep(const VgmFitArgs& a, hipStream_t stream) {
  if (a.n_cols == 0 || a.max_rows == 0) return;
  hipLaunchKernelGGL(vgm_estep_kernel, fit_grid(a), dim3(FIT_THREADS), 0, stream, a);
}

void launch_kmeans_step(const VgmFitArgs& a, hipStream_t stream) {
  if (a.n_cols == 0 || a.max_rows == 0) return;
  hipLaunchKernelGGL(kmeans_step_kernel, fit_grid(a), dim3(FIT_THREADS), 0, stream, a);
}

}  // namespace fedtgan
