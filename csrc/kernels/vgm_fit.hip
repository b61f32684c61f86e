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
#include <algorithm>

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
