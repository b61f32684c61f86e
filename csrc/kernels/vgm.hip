// VGM mode-specific normalisation (CTGAN encode) on the device.
//
// Reference: `BGM_CTGAN_Transformer.transform` (Server/dtds/features/transformers.py:385-428).
// It takes sklearn `predict_proba` per continuous column, adds 1e-6 and renormalises over
// the valid modes, and draws one mode per row with a Python loop over `np.random.choice`.
// It then writes alpha = clip((x - mu_k) / (4 sigma_k), +-0.99) followed by the one-hot of the
// mode among the valid modes; a categorical column becomes a one-hot of its code's position.
//
// Here one thread encodes one (row, column) cell:
//   * continuous: 10 variational log-posteriors in registers, log-sum-exp, +1e-6 on the valid
//     modes, inverse-CDF draw from a Philox uniform, alpha and the one-hot;
//   * categorical: LUT code -> option index, one-hot.
// Every cell also records its option index (the mode, or the category position) into
// opt[row, span], so the per-(span, option) row lists of the real-row sampler can be built on
// the device from one stable sort (fed_tgan_amd/features/encode_gpu.py) with no host round trip.
#include <algorithm>

#include "common.h"
#include "launch.h"

namespace fedtgan {

#if FT_CHECKED
__device__ unsigned g_check_vgm = 0u;
unsigned check_status_vgm() {
  unsigned v = 0u, z = 0u;
  (void)hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_check_vgm), sizeof(v));
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_check_vgm), &z, sizeof(z));
  return v;
}
#else
unsigned check_status_vgm() { return 0u; }
#endif

constexpr int VGM_K = 10;   // components per continuous column (N_CLUSTERS)

__global__ __launch_bounds__(256) void vgm_encode_kernel(VgmEncodeArgs a) {
  const int64_t total = (int64_t)a.n_rows * a.n_cols;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(e / a.n_cols), j = (int)(e % a.n_cols);
    const double xv = a.x[(size_t)r * a.ldx + (size_t)j * a.ldc];
    float* row = a.out + (size_t)r * a.ldo;
    const int pos = a.col_pos[j], aux = a.col_aux[j], span = a.col_span[j];
    int opt;
    if (a.col_kind[j] == 0) {
      const int c = aux;
      const float* cst = a.consts + c * VGM_K;
      const float* mu = a.means + c * VGM_K;
      const float* pc = a.prec + c * VGM_K;
      float lp[VGM_K];
      float mx = -INFINITY;
#pragma unroll
      for (int k = 0; k < VGM_K; ++k) {
        const float y = (float)(xv - (double)mu[k]) * pc[k];
        lp[k] = cst[k] - 0.5f * y * y;
        mx = fmaxf(mx, lp[k]);
      }
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < VGM_K; ++k) s += expf(lp[k] - mx);
      const float inv = 1.f / s;
      float p[VGM_K], tot = 0.f;
#pragma unroll
      for (int k = 0; k < VGM_K; ++k) {
        p[k] = a.vrank[c * VGM_K + k] >= 0 ? expf(lp[k] - mx) * inv + 1e-6f : 0.f;
        tot += p[k];
      }
      RngArgs rng{a.seed, nullptr, a.stream};
      const float u = u01(rng4(rng, 0ull, (uint64_t)e).x) * tot;
      int kk = -1;
      float acc = 0.f;
#pragma unroll
      for (int k = 0; k < VGM_K; ++k) {
        acc += p[k];
        if (kk < 0 && p[k] > 0.f && acc > u) kk = k;
      }
      if (kk < 0) {   // u rounded onto the total, or a NaN cell: last valid mode
#pragma unroll
        for (int k = 0; k < VGM_K; ++k)
          if (a.vrank[c * VGM_K + k] >= 0) kk = k;
      }
      kk = max(kk, 0);    // (the host guarantees every column has a valid mode)
      const float sd = a.stds[c * VGM_K + kk];
      const float al = (float)((xv - (double)mu[kk]) / (4.0 * (double)sd));
      row[pos] = fminf(fmaxf(al, -0.99f), 0.99f);
      opt = a.vrank[c * VGM_K + kk];
      row[pos + 1 + opt] = 1.f;
    } else {
      // codes were range-checked on the host; the clamp keeps a stray value inside the LUT row
#if FT_CHECKED
      FT_CHECK(&g_check_vgm, (int)xv >= 0 && (int)xv < a.col_lut_n[j], CHK_ENCODE_LUT);
#endif
      opt = a.lut[aux + min(max((int)xv, 0), a.col_lut_n[j] - 1)];
      row[pos + opt] = 1.f;
    }
    a.opt[(size_t)r * a.n_span + span] = opt;
  }
}

void launch_vgm_encode(const VgmEncodeArgs& a, hipStream_t stream) {
  const int64_t total = (int64_t)a.n_rows * a.n_cols;
  if (total == 0) return;
  const int blocks = (int)std::min<int64_t>((total + 255) / 256, 8192);
  hipLaunchKernelGGL(vgm_encode_kernel, dim3(blocks), dim3(256), 0, stream, a);
}

}  // namespace fedtgan
