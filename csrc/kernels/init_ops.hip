// Initialisation-path kernels: the federator's pooled GMM sample and the real-row CSR index of an encoded table.
//
// Both replace short chains of ATen launches (repeat_interleave / randn / gather; argsort / scatter_add / cumsum /
// where) whose first use in a process loads each kernel's code object out of libtorch's fatbin -- tens to hundreds
// of milliseconds apiece in the first GPU process on a box (profiles/init_r5.txt, init_r6.txt).  With these the
// federated initialisation issues only this library's kernels (plus fills and copies).
//
//   pool_sample_kernel   every client's VGM sampled into one pooled [n_cont, N] matrix (the federator's re-fit
//                        sample, `Server/dtds/distributed.py:731-735`): element e of segment s = (column j, client i,
//                        component k) is mean[s] + sd[s] * z_e, z_e a Philox / Box-Muller normal keyed on (seed, e)
//   csr_count_kernel     per (span, row chunk): option histogram of the chunk (LDS)
//   csr_scan_kernel      per span: exclusive offsets of every (option, chunk) block in option-major order, the
//                        per-option totals and row offsets (`Sampler`'s per-option row lists,
//                        `Server/dtds/synthesizers/ctgan.py:205-217`, as CSR)
//   csr_scatter_kernel   per (span, row chunk): each row's index at its block offset + its stable rank among the
//                        chunk's earlier rows of the same option -- rows ascending within every list, deterministic
#include <algorithm>
#include <stdexcept>
#include <string>

#include "common.h"
#include "launch.h"

namespace fedtgan {

constexpr int INIT_THREADS = 256;

__global__ __launch_bounds__(INIT_THREADS) void pool_sample_kernel(PoolSampleArgs a) {
  const RngArgs rng{a.seed, nullptr, 0x9001u};
  for (int64_t e = (int64_t)blockIdx.x * INIT_THREADS + threadIdx.x; e < a.n; e += (int64_t)gridDim.x * INIT_THREADS) {
    // segment of e: the last s with seg_off[s] <= e (segments may be empty)
    int lo = 0, hi = a.nseg - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (a.seg_off[mid] <= e) lo = mid;
      else hi = mid - 1;
    }
    const uint4 r = rng4(rng, 0ull, (uint64_t)e);
    const double u1 = u01d(r.x, r.y), u2 = u01d(r.z, r.w);
    const double z = sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
    a.pool[e] = a.mean[lo] + a.sd[lo] * z;
  }
}

void launch_pool_sample(const PoolSampleArgs& a, hipStream_t stream) {
  if (a.n <= 0) return;
  if (a.nseg <= 0) throw std::runtime_error("pool_sample: no segments");
  const int64_t blocks = std::min<int64_t>((a.n + INIT_THREADS - 1) / INIT_THREADS, 4096);
  hipLaunchKernelGGL(pool_sample_kernel, dim3((unsigned)blocks), dim3(INIT_THREADS), 0, stream, a);
}

// every row of x [rows, n] (contiguous) centred in place on its mean, written to shift[row] (the VGM fit's prior
// mean, sklearn's mean_prior = mean(X)); a fixed-order block reduction, so the same bits every run
__global__ __launch_bounds__(INIT_THREADS) void row_center_kernel(double* x, double* shift, int64_t n) {
  __shared__ double red[INIT_THREADS];
  double* row = x + (size_t)blockIdx.x * n;
  double s = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += INIT_THREADS) s += row[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = INIT_THREADS / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  const double m = red[0] / (double)(n > 0 ? n : 1);
  if (threadIdx.x == 0) shift[blockIdx.x] = m;
  for (int64_t i = threadIdx.x; i < n; i += INIT_THREADS) row[i] -= m;
}

void launch_row_center(double* x, double* shift, int rows, int64_t n, hipStream_t stream) {
  if (rows <= 0) return;
  hipLaunchKernelGGL(row_center_kernel, dim3(rows), dim3(INIT_THREADS), 0, stream, x, shift, n);
}

// ---------------------------------------------------------------------------------------------- CSR row index
// part[(s * chunks + c) * maxw + o] = rows of chunk c whose option in span s is o
__global__ __launch_bounds__(INIT_THREADS) void csr_count_kernel(CsrArgs a) {
  extern __shared__ int hist[];
  const int s = blockIdx.y, c = blockIdx.x;
  for (int o = threadIdx.x; o < a.maxw; o += INIT_THREADS) hist[o] = 0;
  __syncthreads();
  const int r0 = c * a.chunk, r1 = min(a.n, r0 + a.chunk);
  const int w = a.width[s];
  for (int r = r0 + threadIdx.x; r < r1; r += INIT_THREADS) {
    const int o = a.opt[(size_t)r * a.ldo + s];
    if (o >= 0 && o < w) atomicAdd(&hist[o], 1);
  }
  __syncthreads();
  int* out = a.part + ((size_t)s * a.chunks + c) * a.maxw;
  for (int o = threadIdx.x; o < a.maxw; o += INIT_THREADS) out[o] = hist[o];
}

// one thread per span: part -> exclusive block offsets (in place), counts and row offsets
__global__ __launch_bounds__(64) void csr_scan_kernel(CsrArgs a) {
  const int s = blockIdx.x * 64 + threadIdx.x;
  if (s >= a.n_col) return;
  int64_t run = (int64_t)s * a.n;
  const int w = a.width[s];
  for (int o = 0; o < a.maxw; ++o) {
    int64_t tot = 0;
    const int64_t start = run;
    for (int c = 0; c < a.chunks; ++c) {
      int* p = a.part + ((size_t)s * a.chunks + c) * a.maxw + o;
      const int v = *p;
      *p = (int)(run - (int64_t)s * a.n);    // block offset within the span's list
      run += v;
      tot += v;
    }
    a.count[(size_t)s * a.maxw + o] = tot;
    a.offset[(size_t)s * a.maxw + o] = o < w ? start : 0;   // padding slots stay 0
  }
}

// rows of one chunk in INIT_THREADS-row batches: rank = same-option rows earlier in the batch (LDS compare) +
// the chunk's running count of that option (LDS), so every list is in ascending row order
__global__ __launch_bounds__(INIT_THREADS) void csr_scatter_kernel(CsrArgs a) {
  extern __shared__ int sh[];
  int* run = sh;                       // [maxw] running count per option within this chunk
  int* bopt = sh + a.maxw;             // [INIT_THREADS] options of the current batch
  const int s = blockIdx.y, c = blockIdx.x, t = threadIdx.x;
  for (int o = t; o < a.maxw; o += INIT_THREADS) run[o] = 0;
  const int r0 = c * a.chunk, r1 = min(a.n, r0 + a.chunk);
  const int w = a.width[s];
  const int* base = a.part + ((size_t)s * a.chunks + c) * a.maxw;
  int64_t* rows = a.rows + (size_t)s * a.n;
  __syncthreads();
  for (int b0 = r0; b0 < r1; b0 += INIT_THREADS) {
    const int r = b0 + t;
    int o = -1;
    if (r < r1) {
      o = a.opt[(size_t)r * a.ldo + s];
      if (o < 0 || o >= w) o = -1;
    }
    bopt[t] = o;
    __syncthreads();
    int rank = 0;
    bool last = true;
    if (o >= 0) {
      for (int q = 0; q < t; ++q) rank += bopt[q] == o ? 1 : 0;
      for (int q = t + 1; q < INIT_THREADS; ++q)
        if (bopt[q] == o) { last = false; break; }
      rows[base[o] + run[o] + rank] = r;
    }
    __syncthreads();
    // advance the running counts: the batch's last row of each option adds its rank + 1 (one writer per option)
    if (o >= 0 && last) run[o] += rank + 1;
    __syncthreads();
  }
}

void launch_csr_rows(const CsrArgs& a, hipStream_t stream) {
  if (a.n_col <= 0 || a.n <= 0) return;
  if (a.maxw <= 0 || a.chunks <= 0 || a.chunk <= 0) throw std::runtime_error("csr_rows: bad shape");
  const size_t lds_count = (size_t)a.maxw * sizeof(int);
  const size_t lds_scatter = ((size_t)a.maxw + INIT_THREADS) * sizeof(int);
  if (lds_scatter > 64 * 1024) throw std::runtime_error("csr_rows: too many options per span for the LDS tables");
  const dim3 grid(a.chunks, a.n_col);
  hipLaunchKernelGGL(csr_count_kernel, grid, dim3(INIT_THREADS), lds_count, stream, a);
  hipLaunchKernelGGL(csr_scan_kernel, dim3((a.n_col + 63) / 64), dim3(64), 0, stream, a);
  hipLaunchKernelGGL(csr_scatter_kernel, grid, dim3(INIT_THREADS), lds_scatter, stream, a);
}

}  // namespace fedtgan
