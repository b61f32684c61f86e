// Generic skinny-GEMM for the CTGAN step on CDNA4 MFMA (bf16 operands, fp32 accumulate).
//
//   C[M,N] = epi( alpha * op(A)[M,K] . op(B)[K,N] + beta * C + bias[N] )
//
// op(A) = A or A^T, op(B) = B or B^T, every operand with its own leading dimension so the
// engine can pass column slices of its concat-free activation buffers (the generator's
// residual stack, the packed PacGAN input) without copies.
//
// Tiling: 64x64 output tile per 256-thread workgroup (4 waves in a 2x2 grid, 32x32 per wave
// = 2x2 v_mfma_f32_16x16x32_bf16 tiles), BK = 32.  Operands are read from fp32 global memory
// with coalesced loads along their contiguous dimension, rounded to bf16 and staged in LDS as
// [row][k] images (k contiguous, row stride padded to 40 elements = 80 B so each lane's
// 16-byte fragment is a conflict-light ds_read_b128).  Two LDS buffers: the next k-tile's
// global loads are issued before the current tile's MFMAs (register prefetch), so HBM /
// Infinity-Cache latency hides under the compute of the previous tile.
//
// Split-K (gridDim.z > 1) writes fp32 partial slabs that `gemm_splitk_epilogue` reduces and
// finishes; with gridDim.z == 1 the epilogue is fused.  Epilogues:
//   EPI_NONE            out = v
//   EPI_LRELU_DROPOUT   out = lrelu(v) * keep/(1-p);  ms = lrelu'(v) * keep/(1-p)   (Philox mask)
//   EPI_MASK            out = v * ms
//   EPI_RELU            out = max(v, 0)
#include <algorithm>

#include "common.h"
#include "launch.h"

namespace fedtgan {

typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int BM = 64, BN = 64, BK = 32, KPAD = 40, NT = 256;

__device__ __forceinline__ float apply_epi(const GemmArgs& g, float v, int m, int n, uint64_t step, uint64_t idx) {
  const int epi = g.epi;
  if (epi == EPI_LRELU_DROPOUT) {
    const float s = v > 0.f ? 1.f : g.slope;
    RngArgs rng{g.seed, g.rng_ctr, g.rng_stream};
    const uint4 r = rng4(rng, step, idx);
    const float keep = (u01(r.x) >= g.p_drop) ? 1.f / (1.f - g.p_drop) : 0.f;
    const float f = s * keep;
    g.ms[(size_t)m * g.ldms + n] = f;
    return v * f;
  } else if (epi == EPI_MASK) {
    return v * g.ms[(size_t)m * g.ldms + n];
  } else if (epi == EPI_RELU) {
    return v > 0.f ? v : 0.f;
  } else if (epi == EPI_BN_EVAL_RELU) {
    const float y = (v - g.bn_rm[n]) * rsqrtf(g.bn_rv[n] + g.bn_eps) * g.bn_gamma[n] + g.bn_beta[n];
    return y > 0.f ? y : 0.f;
  }
  return v;
}

// Stage a BM(or BN) x BK tile of an operand into registers (8 fp32 values per thread).
//   ROWMAJ: element (r, k) at p[r*ld + k] (k contiguous)   -> thread: kp = t%16, r = t/16 + 16*i
//   else  : element (r, k) at p[k*ld + r] (r contiguous)   -> thread: r = t%64, kp = t/64 + 4*i
template <bool ROWMAJ>
__device__ __forceinline__ void load_tile(float (&v)[8], const float* __restrict__ p, int ld, int r0, int rmax, int k0,
                                          int kmax) {
  // Every load is issued unconditionally from a clamped (always valid) address and the
  // out-of-range lanes are zeroed afterwards: a predicated load would make hipcc branch
  // around each one and wait vmcnt(0) per element (8 serial round trips per operand).
  const int t = threadIdx.x;
  float x[8];
  bool ok[8];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int r, k;
    if (ROWMAJ) {
      r = r0 + t / 16 + 16 * i;
      k = k0 + 2 * (t % 16);
    } else {
      r = r0 + t % 64;
      k = k0 + 2 * (t / 64 + 4 * i);
    }
    const int rc = min(r, rmax - 1);
    const int kc0 = min(k, kmax - 1), kc1 = min(k + 1, kmax - 1);
    x[2 * i] = ROWMAJ ? p[(size_t)rc * ld + kc0] : p[(size_t)kc0 * ld + rc];
    x[2 * i + 1] = ROWMAJ ? p[(size_t)rc * ld + kc1] : p[(size_t)kc1 * ld + rc];
    ok[2 * i] = r < rmax && k < kmax;
    ok[2 * i + 1] = r < rmax && k + 1 < kmax;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = ok[i] ? x[i] : 0.f;
}

template <bool ROWMAJ>
__device__ __forceinline__ void tile_coords(int i, int& r, int& kp) {
  const int t = threadIdx.x;
  if (ROWMAJ) {
    r = t / 16 + 16 * i;
    kp = t % 16;
  } else {
    r = t % 64;
    kp = t / 64 + 4 * i;
  }
}

// bf16 image: [row][KPAD] (k contiguous), two k per 32-bit store
template <bool ROWMAJ>
__device__ __forceinline__ void store_tile(uint16_t* s, const float (&v)[8]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int r, kp;
    tile_coords<ROWMAJ>(i, r, kp);
    *reinterpret_cast<uint32_t*>(&s[r * KPAD + 2 * kp]) = pack_bf16x2(v[2 * i], v[2 * i + 1]);
  }
}

// fp32 image: [row][KPADF]; odd stride keeps the 16 rows a 16x16x4 fragment reads on distinct banks
constexpr int KPADF = 33;
template <bool ROWMAJ>
__device__ __forceinline__ void store_tile_f32(float* s, const float (&v)[8]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int r, kp;
    tile_coords<ROWMAJ>(i, r, kp);
    s[r * KPADF + 2 * kp] = v[2 * i];
    s[r * KPADF + 2 * kp + 1] = v[2 * i + 1];
  }
}

template <bool TA, bool TB, bool F32>
__global__ __launch_bounds__(NT) void gemm_kernel(GemmArgs g) {
  // one LDS array (two stages of A and B); bf16 mode uses the first half of it
  constexpr int STAGE = F32 ? (BM + BN) * KPADF * 4 : (BM + BN) * KPAD * 2;
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * STAGE];

  const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM;
  const int kb = blockIdx.z * g.kchunk;
  const int ke = min(g.K, kb + g.kchunk);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = w >> 1, wn = w & 1;

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto stage_store = [&](int st, const float (&ra)[8], const float (&rb)[8]) {
    unsigned char* base = smem + st * STAGE;
    if constexpr (F32) {
      store_tile_f32<!TA>(reinterpret_cast<float*>(base), ra);
      store_tile_f32<TB>(reinterpret_cast<float*>(base) + BM * KPADF, rb);
    } else {
      store_tile<!TA>(reinterpret_cast<uint16_t*>(base), ra);
      store_tile<TB>(reinterpret_cast<uint16_t*>(base) + BM * KPAD, rb);
    }
  };

  // A(m,k): TA ? a[k*lda+m] : a[m*lda+k]   -> row-major in k iff !TA
  // B(k,n): TB ? b[n*ldb+k] : b[k*ldb+n]   -> staged as [n][k]; row-major in k iff TB
  float ra[8], rb[8];
  int buf = 0;
  if (kb < ke) {
    load_tile<!TA>(ra, g.a, g.lda, m0, g.M, kb, ke);
    load_tile<TB>(rb, g.b, g.ldb, n0, g.N, kb, ke);
    stage_store(0, ra, rb);
  }
  __syncthreads();
  for (int k0 = kb; k0 < ke; k0 += BK) {
    const bool more = k0 + BK < ke;
    if (more) {
      load_tile<!TA>(ra, g.a, g.lda, m0, g.M, k0 + BK, ke);
      load_tile<TB>(rb, g.b, g.ldb, n0, g.N, k0 + BK, ke);
    }
    if constexpr (F32) {
      const float* A = reinterpret_cast<const float*>(smem + buf * STAGE);
      const float* B = A + BM * KPADF;
#pragma unroll
      for (int s4 = 0; s4 < BK / 4; ++s4) {
        const int kk = 4 * s4 + (lane >> 4);
        float af[2], bfv[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          af[i] = A[(wm * 32 + i * 16 + (lane & 15)) * KPADF + kk];
          bfv[i] = B[(wn * 32 + i * 16 + (lane & 15)) * KPADF + kk];
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfv[j], acc[i][j], 0, 0, 0);
      }
    } else {
      const uint16_t* A = reinterpret_cast<const uint16_t*>(smem + buf * STAGE);
      const uint16_t* B = A + BM * KPAD;
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        af[i] = *reinterpret_cast<const bf16x8*>(&A[(wm * 32 + i * 16 + (lane & 15)) * KPAD + 8 * (lane >> 4)]);
        bfr[i] = *reinterpret_cast<const bf16x8*>(&B[(wn * 32 + i * 16 + (lane & 15)) * KPAD + 8 * (lane >> 4)]);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (more) stage_store(buf ^ 1, ra, rb);
    __syncthreads();
    buf ^= 1;
  }

  const uint64_t step = (g.epi == EPI_LRELU_DROPOUT && g.rng_ctr) ? *g.rng_ctr : 0ull;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 32 + i * 16 + (lane >> 4) * 4 + r;
        const int n = n0 + wn * 32 + j * 16 + (lane & 15);
        if (m >= g.M || n >= g.N) continue;
        const float v0 = acc[i][j][r];
        if (gridDim.z > 1) {
          g.ws[((size_t)blockIdx.z * g.M + m) * g.N + n] = v0;
          continue;
        }
        float v = g.alpha * v0;
        float* cp = g.c + (size_t)m * g.ldc + n;
        if (g.beta != 0.f) v += g.beta * (*cp);
        if (g.bias) v += g.bias[n];
        *cp = apply_epi(g, v, m, n, step, (uint64_t)m * g.N + n);
      }
}

__global__ __launch_bounds__(256) void gemm_splitk_epilogue(GemmArgs g) {
  const int splits = g.splitk;
  const size_t total = (size_t)g.M * g.N;
  const uint64_t step = (g.epi == EPI_LRELU_DROPOUT && g.rng_ctr) ? *g.rng_ctr : 0ull;
  for (size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (size_t)gridDim.x * blockDim.x) {
    const int m = (int)(idx / g.N), n = (int)(idx % g.N);
    // independent partial sums so the slab loads are in flight together
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    int z = 0;
    for (; z + 4 <= splits; z += 4) {
      s0 += g.ws[(size_t)z * total + idx];
      s1 += g.ws[(size_t)(z + 1) * total + idx];
      s2 += g.ws[(size_t)(z + 2) * total + idx];
      s3 += g.ws[(size_t)(z + 3) * total + idx];
    }
    for (; z < splits; ++z) s0 += g.ws[(size_t)z * total + idx];
    float v = g.alpha * ((s0 + s1) + (s2 + s3));
    float* cp = g.c + (size_t)m * g.ldc + n;
    if (g.beta != 0.f) v += g.beta * (*cp);
    if (g.bias) v += g.bias[n];
    *cp = apply_epi(g, v, m, n, step, idx);
  }
}

void launch_gemm(GemmArgs g, hipStream_t stream) {
  if (g.M <= 0 || g.N <= 0) return;
  const int tm = (g.M + BM - 1) / BM, tn = (g.N + BN - 1) / BN;
  if (g.splitk < 1) g.splitk = 1;
  if (g.K <= 0) g.splitk = 1;
  int kchunk = (g.K + g.splitk - 1) / g.splitk;
  kchunk = ((kchunk + BK - 1) / BK) * BK;
  if (kchunk <= 0) kchunk = BK;
  g.splitk = (g.K + kchunk - 1) / kchunk;
  if (g.splitk < 1) g.splitk = 1;
  g.kchunk = kchunk;
  dim3 grid(tn, tm, g.splitk), block(NT);
  if (g.splitk > 1 && g.ws == nullptr) {
    g.splitk = 1;
    g.kchunk = g.K;
    grid.z = 1;
  }
#define FEDTGAN_GEMM_DISPATCH(F)                                                                         \
  if (!g.ta && g.tb) hipLaunchKernelGGL((gemm_kernel<false, true, F>), grid, block, 0, stream, g);       \
  else if (!g.ta && !g.tb) hipLaunchKernelGGL((gemm_kernel<false, false, F>), grid, block, 0, stream, g); \
  else if (g.ta && !g.tb) hipLaunchKernelGGL((gemm_kernel<true, false, F>), grid, block, 0, stream, g);   \
  else hipLaunchKernelGGL((gemm_kernel<true, true, F>), grid, block, 0, stream, g);
  if (g.f32) {
    FEDTGAN_GEMM_DISPATCH(true)
  } else {
    FEDTGAN_GEMM_DISPATCH(false)
  }
#undef FEDTGAN_GEMM_DISPATCH
  if (grid.z > 1) {
    const size_t total = (size_t)g.M * g.N;
    int blocks = (int)std::min<size_t>((total + 255) / 256, 2048);
    hipLaunchKernelGGL(gemm_splitk_epilogue, dim3(blocks), dim3(256), 0, stream, g);
  }
}

}  // namespace fedtgan
