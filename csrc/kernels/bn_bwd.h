// BatchNorm(train) + ReLU backward of one workgroup's COLS columns (the generator's Residual layers,
// `Server/dtds/synthesizers/ctgan.py:33-44`): a device function shared by the stand-alone launch
// (ctgan_ops.hip bn_relu_bwd_kernel) and the horizontally fused launch that runs these workgroups beside the
// independent weight-gradient GEMM of the layer above (gemm.hip gemm_bnbwd_kernel).
//
// Per column c (n = rows, k = gamma_c * invstd_c, dy = dr masked by relu'(r)):
//   dbeta = sum dy, dgamma = sum dy * nhat, dbias = k * (sum dy - sum dy - sum nhat * dgamma / n) (the preceding
//   Linear's bias gradient in closed form), da = k * (dy - sum dy / n - nhat * dgamma / n).
// Every thread keeps MAXR of its column's rows in registers (one pass over global memory); the three column sums
// are one wave64 butterfly over the row groups of a wave plus one LDS combine across the waves.
#pragma once

#include "launch.h"

namespace fedtgan {


// sum over every row group of the workgroup for this thread's column, NV values at once.
// sh: [NV][NTH / 64][COLS] floats of LDS; ends with a barrier (sh reusable at once).
template <int COLS, int NV, int NTH>
__device__ __forceinline__ void bnb_colsum(float (&v)[NV], float* sh) {
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

// workgroup `bx` of the backward (columns [bx * COLS, bx * COLS + COLS)); rows <= MAXR * (NTH / COLS).
// sh: >= 3 * (NTH / 64) * COLS floats.
template <int COLS, int MAXR, int NTH>
__device__ __forceinline__ void bn_bwd_block(const BnBwdArgs& a, int bx, float* sh) {
  constexpr int GROUPS = NTH / COLS;
  const int lc = threadIdx.x % COLS, grp = threadIdx.x / COLS;
  const int c = bx * COLS + lc;
  const bool ok = c < a.cols;
  const int cc = min(c, a.cols - 1);
  const int rows = a.rows;
  // gamma * invstd is requested with the rows (consumed after the reduction's barriers)
  const float k = a.gamma[cc] * a.invstd[cc];
  float dy[MAXR], nh[MAXR];
  float st[3] = {0.f, 0.f, 0.f};   // sum dy, sum dy * nhat, sum nhat
#pragma unroll
  for (int i = 0; i < MAXR; ++i) {
    const int r = grp + i * GROUPS;
    const size_t rr = (size_t)min(r, rows - 1);
    const float rv = a.r[rr * a.ldr + cc];
    const float dv = a.dr[rr * a.lddr + cc];
    const float nv = a.nhat[rr * a.ldn + cc];
    const bool in = r < rows;
    const float d = (in && rv > 0.f) ? dv : 0.f;
    const float n = in ? nv : 0.f;
    dy[i] = d;
    nh[i] = n;
    st[0] += d;
    st[1] += d * n;
    st[2] += n;
  }
  bnb_colsum<COLS, 3, NTH>(st, sh);
  const float sdy = st[0], sdyn = st[1], snh = st[2];
  const float invn = 1.f / (float)rows;
  if (grp == 0 && ok) {
    a.dbeta[c] = sdy;
    a.dgamma[c] = sdyn;
    if (a.dbias) a.dbias[c] = k * (sdy - sdy * (float)rows * invn - snh * sdyn * invn);
  }
#pragma unroll
  for (int i = 0; i < MAXR; ++i) {
    const int r = grp + i * GROUPS;
    if (r < rows && ok) a.da[(size_t)r * a.ldda + c] = k * (dy[i] - sdy * invn - nh[i] * sdyn * invn);
  }
}

}  // namespace fedtgan
