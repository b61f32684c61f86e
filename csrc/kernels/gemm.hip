// Generic skinny-GEMM for the CTGAN step on CDNA4 matrix cores.
//
//   C[M,N] = epi( alpha * op(A)[M,K] . op(B)[K,N] + beta * C + bias[N] )
//
// op(A) = A or A^T, op(B) = B or B^T, every operand with its own leading dimension so the
// engine passes column slices of its concat-free activation buffers (the generator's
// residual stack, the packed PacGAN input) without copies.
//
// The step's GEMMs are small (M <= 500, N <= ~6k, K <= ~6k): what costs is memory latency,
// not FLOPs.  Hence:
//   * 64x64 output tile per 256-thread workgroup (4 waves in a 2x2 grid, 32x32 per wave);
//   * the workgroup's whole K-chunk (KC = 128 bf16 / 64 fp32) is fetched in ONE burst --
//     every thread issues all of its loads back to back from clamped, always-valid
//     addresses (no predicated loads, which hipcc would serialise with vmcnt(0) each), as
//     16-B loads wherever the operand is 16-B aligned with a leading dimension divisible by
//     4 (the engine pads its buffers so that the step's operands are) -- so a chunk costs one
//     memory round trip, and the next chunk's burst is in flight while the current one is
//     multiplied out of LDS;
//   * operands are rounded to bf16 once, while staging into [row][k] LDS images (row stride
//     KC+8 elements: every 16-lane ds_read_b128 group lands on distinct banks), then
//     v_mfma_f32_16x16x32_bf16 with fp32 accumulation; or, with g.f32, kept in fp32 and fed
//     to v_mfma_f32_16x16x4_f32 (exact fp32, same numerics as an fmaf chain);
//   * split-K over gridDim.z spreads a K-heavy GEMM with few output tiles over many CUs
//     (one CU alone pulls only ~60-100 GB/s); fp32 partial slabs are reduced by
//     `gemm_splitk_epilogue`, which also applies the epilogue; with one split it is fused.
// Epilogues:
//   EPI_NONE            out = v
//   EPI_LRELU_DROPOUT   out = lrelu(v) * keep/(1-p);  ms = lrelu'(v) * keep/(1-p)   (Philox mask)
//   EPI_MASK            out = v * ms
//   EPI_RELU            out = max(v, 0)
//   EPI_BN_EVAL_RELU    out = relu((v - rm) * rsqrt(rv + eps) * gamma + beta)   (eval BatchNorm)
// One-hot conditional block (GemmArgs::oh_w): before the epilogue, v += the weight column of the
// row's active condition -- the generator layers multiply only the dense part of [... | z | c]
// and gather the c block's single non-zero product (c is 303 of G0's 431 input columns on Intrusion).
#include <algorithm>
#include <type_traits>

#include "common.h"
#include "launch.h"
#include "adam_cs.h"
#include "bn_bwd.h"

namespace fedtgan {

#if FT_CHECKED
__device__ unsigned g_check_gemm = 0u;
unsigned check_status_gemm() {
  unsigned v = 0u, z = 0u;
  (void)hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_check_gemm), sizeof(v));
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_check_gemm), &z, sizeof(z));
  return v;
}
#else
unsigned check_status_gemm() { return 0u; }
#endif

typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

constexpr int NT = 256;

// largest tile (rows) that keeps two K-bursts in flight (see Cfg::DEPTH)
#ifndef FEDTGAN_GEMM_DEPTH2_MAX_TM
#define FEDTGAN_GEMM_DEPTH2_MAX_TM 64
#endif

// output / split-K slab store: plain, or write-through (sc1) so the kernel boundary finds no dirty
// L2 lines to write back (MI355X_MICROARCH.md "boundary": + bytes / 6 TB/s)
__device__ __forceinline__ void st_out(float* base, size_t idx, float v, int wt) {
  if (wt) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7FFFFFFF, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rs, (int)(idx * 4), 0, 16);
  } else {
    base[idx] = v;
  }
}

// the one-hot block's contribution to output (m, n): one gathered weight (see GemmArgs::oh_w)
__device__ __forceinline__ float onehot_term(const GemmArgs& g, int m, int n) {
  const int idx = g.oh_off[g.oh_col[m]] + g.oh_opt[m];
  return g.oh_trans ? g.oh_w[(size_t)idx * g.oh_ld + n] : g.oh_w[(size_t)n * g.oh_ld + idx];
}

// Eval BatchNorm parameters of one output column, loaded once per column a thread owns (a store
// to C between per-element loads would force the compiler to reload them: it cannot prove that C
// and the BN vectors do not alias -- measured: the 40k-row G0 epilogue 20 -> 54 us)
struct ColEpi {
  float rm, r, gamma, beta;
};

__device__ __forceinline__ ColEpi col_epi(const GemmArgs& g, int n) {
  ColEpi c{0.f, 0.f, 0.f, 0.f};
  if (g.epi == EPI_BN_EVAL_RELU) {
    c.rm = g.bn_rm[n];
    c.r = rsqrtf(g.bn_rv[n] + g.bn_eps);
    c.gamma = g.bn_gamma[n];
    c.beta = g.bn_beta[n];
  }
  return c;
}

// the one BN-eval expression every path uses (bit-identical results across epilogues)
__device__ __forceinline__ float bn_eval_relu(float v, const ColEpi& c) {
  const float y = (v - c.rm) * c.r * c.gamma + c.beta;
  return y > 0.f ? y : 0.f;
}

__device__ __forceinline__ float apply_epi(const GemmArgs& g, float v, int m, int n, uint64_t step, uint64_t idx);

// apply_epi with the column's BN parameters already in registers
__device__ __forceinline__ float apply_epi_c(const GemmArgs& g, float v, int m, int n, uint64_t step, uint64_t idx,
                                             const ColEpi& c) {
  return g.epi == EPI_BN_EVAL_RELU ? bn_eval_relu(v, c) : apply_epi(g, v, m, n, step, idx);
}

__device__ __forceinline__ float apply_epi(const GemmArgs& g, float v, int m, int n, uint64_t step, uint64_t idx) {
  const int epi = g.epi;
  if (epi == EPI_LRELU_DROPOUT) {
    const float s = v > 0.f ? 1.f : g.slope;
    RngArgs rng{g.seed, g.rng_ctr, g.rng_stream};
    const uint4 r = rng4(rng, step, idx);
    const float keep = (u01(r.x) >= g.p_drop) ? 1.f / (1.f - g.p_drop) : 0.f;
    const float f = s * keep;
    g.ms[(size_t)m * g.ldms + n] = f;
    if (g.head_a) g.head_a[(size_t)m * g.ldha + n] = g.head_coef[m] * g.head_v[n] * f;
    return v * f;
  } else if (epi == EPI_MASK) {
    return v * g.ms[(size_t)m * g.ldms + n];
  } else if (epi == EPI_RELU) {
    return v > 0.f ? v : 0.f;
  } else if (epi == EPI_BN_EVAL_RELU) {
    return bn_eval_relu(v, col_epi(g, n));
  }
  return v;
}

// ----------------------------------------------------------------------------- chunk staging
// A chunk is R=64 rows x KC k-values of one operand, held as NV = KC/16 float4 per thread.
//   ROWMAJ (k contiguous in memory): v[i] = row r, k = 4q..4q+3
//       q = t % (KC/4), r = t / (KC/4) + (NT/(KC/4)) * i          (a wave reads 2 rows x KC floats)
//   else   (rows contiguous):        v[2i], v[2i+1] = rows 4rq..4rq+3 at k = 2kp and 2kp+1
//       rq = t % 16,    kp = t / 16 + 16 * i                      (a wave reads 4 k-lines x 64 rows)
// With a 16-B aligned base, a leading dimension and a vector extent divisible by 4 ("vec"),
// every load is a 16-B global_load_dwordx4 (one CU pulls several times more bytes per
// instruction than with dword loads); otherwise every element is a clamped dword load.
// Out-of-range elements are zeroed when the burst is staged into LDS, so nothing waits on a
// burst's loads before its turn comes (PIPE bursts stay in flight).
// bf16 LDS images staged from COLUMN-major operands (rows contiguous in memory) are stored with the
// 16-B k-chunks of a row XOR-permuted by lds_swz(row): the staging writes of 16 lanes then hit 16
// distinct banks instead of 4 (a row is 68 words, 16 words mod 64, so four consecutive row-quads
// alias), and the MFMA fragment reads stay conflict-free (rocprofv3 SQ_LDS_BANK_CONFLICT /
// SQ_LDS_IDX_ACTIVE was 55-75 % on these GEMMs; profiles/pmc_step_r2.txt).  Row-major images are
// stored unpermuted.
template <int KC>
__device__ __forceinline__ int lds_swz(int row) {
  return (3 * (row >> 4)) & (KC / 8 - 1);
}

template <int KC, bool ROWMAJ, int R>
struct Chunk {
  static constexpr int NV = R * KC / (4 * NT);   // float4 per thread
  static constexpr int RQ = R / 4;               // row quads (row-contiguous operands)
  f32x4 v[NV];
  int r0, rmax, k0, kmax;   // bounds of the burst: out-of-range elements are zeroed at staging

  // Issue the burst's loads (and nothing that waits on them, so the burst stays in flight).
  // VEC (a kernel template parameter, so each variant is straight-line code and the compiler's
  // load-counter waits stay exact; decided on the host from the tensor's storage): base 16-B
  // aligned, ld % 4 == 0, and every row's contiguous extent rounded up to 4 still lies inside its
  // ld-long storage row -- so a float4 may run past the logical edge (into padding that staging
  // zeroes) but never past the storage, and its start is clamped to ceil4(extent) - 4.
  template <bool VEC>
  __device__ __forceinline__ void load(const float* __restrict__ p, int ld, int r0_, int rmax_, int k0_, int kmax_) {
    r0 = r0_;
    rmax = rmax_;
    k0 = k0_;
    kmax = kmax_;
    const int t = threadIdx.x;
    if constexpr (ROWMAJ) {
      if constexpr (VEC) {
#pragma unroll
        for (int i = 0; i < NV; ++i) {
          const int rr = r0 + t / (KC / 4) + (NT / (KC / 4)) * i;
          const int k = min(k0 + 4 * (t % (KC / 4)), ((kmax + 3) & ~3) - 4);
          v[i] = *reinterpret_cast<const f32x4*>(p + (size_t)min(rr, rmax - 1) * ld + k);
        }
      } else {
#pragma unroll
        for (int i = 0; i < NV; ++i) {
          const int rr = r0 + t / (KC / 4) + (NT / (KC / 4)) * i;
          const int k = k0 + 4 * (t % (KC / 4));
          const float* row = p + (size_t)min(rr, rmax - 1) * ld;
#pragma unroll
          for (int e = 0; e < 4; ++e) v[i][e] = row[min(k + e, kmax - 1)];
        }
      }
    } else {
      if constexpr (VEC) {
#pragma unroll
        for (int i = 0; i < NV / 2; ++i) {
          const int rr = min(r0 + 4 * (t % RQ), ((rmax + 3) & ~3) - 4);
          const int k = k0 + 2 * (t / RQ + (NT / RQ) * i);
          v[2 * i] = *reinterpret_cast<const f32x4*>(p + (size_t)min(k, kmax - 1) * ld + rr);
          v[2 * i + 1] = *reinterpret_cast<const f32x4*>(p + (size_t)min(k + 1, kmax - 1) * ld + rr);
        }
      } else {
#pragma unroll
        for (int i = 0; i < NV / 2; ++i) {
          const int rr = r0 + 4 * (t % RQ);
          const int k = k0 + 2 * (t / RQ + (NT / RQ) * i);
          const float* l0 = p + (size_t)min(k, kmax - 1) * ld;
          const float* l1 = p + (size_t)min(k + 1, kmax - 1) * ld;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int rc = min(rr + e, rmax - 1);
            v[2 * i][e] = l0[rc];
            v[2 * i + 1][e] = l1[rc];
          }
        }
      }
    }
  }

  // element (i, e) of this thread -> in range?
  __device__ __forceinline__ bool ok_rm(int i, int e) const {
    const int t = threadIdx.x;
    return r0 + t / (KC / 4) + (NT / (KC / 4)) * i < rmax && k0 + 4 * (t % (KC / 4)) + e < kmax;
  }
  __device__ __forceinline__ bool ok_cm(int i, int half, int e) const {
    const int t = threadIdx.x;
    return r0 + 4 * (t % RQ) + e < rmax && k0 + 2 * (t / RQ + (NT / RQ) * i) + half < kmax;
  }

  // bf16 image [row][KC + 8].  A burst wholly inside the operand (every burst but an edge tile's) takes the
  // unchecked body: no per-element bounds selects (counters on the wide G out: VALU instructions ~18x its MFMAs,
  // most of them staging), same bits.
  __device__ __forceinline__ void store_bf16(uint16_t* s) const {
    if (r0 + R <= rmax && k0 + KC <= kmax)
      store_bf16_body<false>(s);
    else
      store_bf16_body<true>(s);
  }
  template <bool CHK>
  __device__ __forceinline__ void store_bf16_body(uint16_t* s) const {
    const int t = threadIdx.x;
    if constexpr (ROWMAJ) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int r = t / (KC / 4) + (NT / (KC / 4)) * i, q = t % (KC / 4);
        float x[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) x[e] = (!CHK || ok_rm(i, e)) ? v[i][e] : 0.f;
        *reinterpret_cast<uint2*>(&s[r * (KC + 8) + 4 * q]) = uint2{pack_bf16x2(x[0], x[1]), pack_bf16x2(x[2], x[3])};
      }
    } else {
#pragma unroll
      for (int i = 0; i < NV / 2; ++i) {
        const int rq = t % RQ, kp = t / RQ + (NT / RQ) * i;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = 4 * rq + e;
          const int pk = (((2 * kp) >> 3) ^ lds_swz<KC>(row)) * 8 + ((2 * kp) & 7);   // swizzled k position
          *reinterpret_cast<uint32_t*>(&s[row * (KC + 8) + pk]) =
              pack_bf16x2((!CHK || ok_cm(i, 0, e)) ? v[2 * i][e] : 0.f, (!CHK || ok_cm(i, 1, e)) ? v[2 * i + 1][e] : 0.f);
        }
      }
    }
  }

  // fp32 image [row][KC + 1]
  __device__ __forceinline__ void store_f32(float* s) const {
    const int t = threadIdx.x;
    if constexpr (ROWMAJ) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int r = t / (KC / 4) + (NT / (KC / 4)) * i, q = t % (KC / 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) s[r * (KC + 1) + 4 * q + e] = ok_rm(i, e) ? v[i][e] : 0.f;
      }
    } else {
#pragma unroll
      for (int i = 0; i < NV / 2; ++i) {
        const int rq = t % RQ, kp = t / RQ + (NT / RQ) * i;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          s[(4 * rq + e) * (KC + 1) + 2 * kp] = ok_cm(i, 0, e) ? v[2 * i][e] : 0.f;
          s[(4 * rq + e) * (KC + 1) + 2 * kp + 1] = ok_cm(i, 1, e) ? v[2 * i + 1][e] : 0.f;
        }
      }
    }
  }
};

// A chunk of a bf16 operand (GemmArgs::bin): R rows x KC k-values, k contiguous in memory, 8 values
// per 16-B load (half the loads and registers of an fp32 chunk); staged into the same [row][KC + 8]
// LDS image without conversion.  The host guarantees a 16-B aligned base, ld % 8 == 0 and storage for
// every row's extent rounded up to 8, so the clamped float4-style addressing of Chunk carries over.
template <int KC, int R>
struct ChunkBF {
  static constexpr int QPR = KC / 8;             // 16-B loads per row
  static constexpr int NV = R * KC / (8 * NT);   // loads per thread
  u32x4 v[NV];
  int r0, rmax, k0, kmax;

  __device__ __forceinline__ void load(const uint16_t* __restrict__ p, int ld, int r0_, int rmax_, int k0_, int kmax_) {
    r0 = r0_;
    rmax = rmax_;
    k0 = k0_;
    kmax = kmax_;
    const int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int rr = r0 + t / QPR + (NT / QPR) * i;
      const int k = min(k0 + 8 * (t % QPR), ((kmax + 7) & ~7) - 8);
      v[i] = *reinterpret_cast<const u32x4*>(p + (size_t)min(rr, rmax - 1) * ld + k);
    }
  }

  __device__ __forceinline__ void store(uint16_t* s) const {
    const int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int r = t / QPR + (NT / QPR) * i, q = t % QPR;
      const int kk = k0 + 8 * q;
      u32x4 x = v[i];
      if (r0 + r >= rmax) {
        x = u32x4{0u, 0u, 0u, 0u};
      } else if (kk + 8 > kmax) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const unsigned lo = kk + 2 * e < kmax ? 0x0000FFFFu : 0u;
          const unsigned hi = kk + 2 * e + 1 < kmax ? 0xFFFF0000u : 0u;
          x[e] &= lo | hi;
        }
      }
      *reinterpret_cast<u32x4*>(&s[r * (KC + 8) + 8 * q]) = x;
    }
  }
};

// Per-tile BatchNorm partials (GemmArgs::bn_part) of the stored values v = acc + bias: for each column
// and batch, the tile's row count, mean and sum of squared deviations (two passes over the
// accumulators: the mean, then the centred squares -- no cancellation), reduced over the 4 lane
// groups of a wave with shuffles and over the 2 row-waves through LDS.  The BN kernel merges the
// tiles' triples (Chan) instead of re-reducing every row of the batch.
template <int MI, int NJ, int TN>
__device__ __forceinline__ void bn_tile_partials(const GemmArgs& g, const f32x4 (&acc)[MI][NJ], int m0, int n0, int by,
                                                 int lane, int wm, int wn, unsigned char* smem) {
  constexpr int WM = 16 * MI, WN = 16 * NJ;
  float* red = reinterpret_cast<float*>(smem);   // [2 wm][TN][2 batch][2] (sum|count), then M2
  float bias[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int n = min(n0 + wn * WN + j * 16 + (lane & 15), g.N - 1);
    bias[j] = g.bias ? g.bias[n] : 0.f;
  }
  float sum[NJ][2], cnt[NJ][2];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    sum[j][0] = sum[j][1] = cnt[j][0] = cnt[j][1] = 0.f;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * WM + i * 16 + (lane >> 4) * 4 + r;
        const float v = acc[i][j][r] + bias[j];
        const bool in = m < g.M, g1 = m >= g.bn_rpg;
        sum[j][0] += (in && !g1) ? v : 0.f;
        sum[j][1] += (in && g1) ? v : 0.f;
        cnt[j][0] += (in && !g1) ? 1.f : 0.f;
        cnt[j][1] += (in && g1) ? 1.f : 0.f;
      }
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int o = 16; o < 64; o <<= 1) {
        sum[j][b] += __shfl_xor(sum[j][b], o, 64);
        cnt[j][b] += __shfl_xor(cnt[j][b], o, 64);
      }
  }
  __syncthreads();   // the stage buffers are free
  if ((lane >> 4) == 0) {
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        float* e = red + (((wm * TN) + wn * WN + j * 16 + lane) * 2 + b) * 2;
        e[0] = sum[j][b];
        e[1] = cnt[j][b];
      }
  }
  __syncthreads();
  float mean[NJ][2], tot[NJ][2], m2[NJ][2];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int col = wn * WN + j * 16 + (lane & 15);
      const float* e0 = red + ((col) * 2 + b) * 2;
      const float* e1 = red + ((TN + col) * 2 + b) * 2;
      tot[j][b] = e0[1] + e1[1];
      mean[j][b] = tot[j][b] > 0.f ? (e0[0] + e1[0]) / tot[j][b] : 0.f;
      m2[j][b] = 0.f;
    }
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * WM + i * 16 + (lane >> 4) * 4 + r;
        const float v = acc[i][j][r] + bias[j];
        const bool in = m < g.M, g1 = m >= g.bn_rpg;
        const float d0 = v - mean[j][0], d1 = v - mean[j][1];
        m2[j][0] += (in && !g1) ? d0 * d0 : 0.f;
        m2[j][1] += (in && g1) ? d1 * d1 : 0.f;
      }
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int o = 16; o < 64; o <<= 1) m2[j][b] += __shfl_xor(m2[j][b], o, 64);
  }
  __syncthreads();
  if ((lane >> 4) == 0) {
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int b = 0; b < 2; ++b) red[((wm * TN) + wn * WN + j * 16 + lane) * 2 + b] = m2[j][b];
  }
  __syncthreads();
  if (wm == 0 && (lane >> 4) == 0) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int col = wn * WN + j * 16 + lane;
      const int n = n0 + col;
      if (n >= g.N) continue;
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        float* o = g.bn_part + ((size_t)(by * 2 + b) * 3) * g.N + n;
        const float q = red[col * 2 + b] + red[(TN + col) * 2 + b];
        o[0] = tot[j][b];
        o[g.N] = mean[j][b];
        o[2 * (size_t)g.N] = q;
      }
    }
  }
}

template <bool F32, int TM, int TN, bool BIN = false>
struct Cfg {
  // K values per burst: (64 + 64) rows x KC fp32 = 64 KB in flight per workgroup.  (KC = 256
  // with 135 KB of LDS raised the per-workgroup rate of long-K GEMMs by 1.36x but cost more on
  // the short-K ones -- padding waste and one workgroup per CU -- so the step got slower.)
  // (128x128 tiles halve the burst: two operands x 128 rows x 128 fp32 in flight would not fit
  // the 256 architectural VGPRs next to the fragments and spill)
  static constexpr int KC = (F32 ? 64 : 128) / (TM >= 128 ? 2 : 1);
  static constexpr int LD = F32 ? KC + 1 : KC + 8;            // LDS row stride (elements)
  static constexpr int ESZ = F32 ? 4 : 2;
  static constexpr int STAGE = (TM + TN) * LD * ESZ;          // bytes per stage (A image + B image)
  // bursts in flight: 2 where the second register slot fits next to the fragments (bf16 path)
  // (bf16 operands: half the registers per burst, so two bursts fit at every tile size)
  static constexpr int DEPTH = (!F32 && (BIN || TM <= FEDTGAN_GEMM_DEPTH2_MAX_TM)) ? 2 : 1;
};

// In-launch split-K reduction (GemmArgs::tile_cnt, 32/64 tiles, N % 4 == 0): the hand-off of
// cdna_hip_programming.md's "projection GEMM" recipe in its write-through form --
//   every K-slice workgroup stages its accumulators through LDS and stores its slab row-contiguously
//   with 16-B write-through (sc1) stores; every wave waits for its stores; after a workgroup barrier
//   one lane takes a ticket (relaxed agent-scope fetch_add on the tile's counter);
//   the workgroup that draws the last ticket resets the counter for the next launch, reads every
//   slab of the tile with sc1 loads (no acquire fence needed: all stores and loads of the slabs are
//   sc1) and applies the epilogue, summing the slabs in the same order as gemm_splitk_epilogue (so
//   both paths give bit-identical outputs).
// Nothing waits on another workgroup (no spinning): every workgroup ends.
template <int TM, int TN, int MI, int NJ, bool PLAIN = false>
__device__ __forceinline__ void splitk_inlaunch(const GemmArgs& g, const f32x4 (&acc)[MI][NJ], int m0, int n0, int tile,
                                                int bz, int gz, int lane, int wm, int wn, unsigned char* smem,
                                                uint64_t step) {
  constexpr int WM = TM / 2, WN = TN / 2;
  constexpr int LDT = TN + 4;   // LDS row stride (floats): float4 rows stay 16-B aligned
  constexpr int Q = TN / 4;     // float4 per tile row
  float* cs = reinterpret_cast<float*>(smem);
  unsigned* last = reinterpret_cast<unsigned*>(smem + TM * LDT * 4);
  __syncthreads();   // the stage buffers are free
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        cs[(wm * WM + i * 16 + (lane >> 4) * 4 + r) * LDT + wn * WN + j * 16 + (lane & 15)] = acc[i][j][r];
  __syncthreads();
  const __amdgpu_buffer_rsrc_t ws = __builtin_amdgcn_make_buffer_rsrc(g.ws, 0, 0x7FFFFFFF, 0x00020000);
  const size_t slab = (size_t)g.M * g.N;
  for (int e = threadIdx.x; e < TM * Q; e += NT) {
    const int ml = e / Q, nl = 4 * (e % Q);
    const int m = m0 + ml, n = n0 + nl;
    if (m < g.M && n < g.N) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(&cs[ml * LDT + nl]);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), ws,
                                             (int)(((size_t)bz * slab + (size_t)m * g.N + n) * 4), 0, 16);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(&g.tile_cnt[tile], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned is_last = t == (unsigned)(gz - 1) ? 1u : 0u;
    if (is_last) __hip_atomic_store(&g.tile_cnt[tile], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *last = is_last;
  }
  __syncthreads();
  if (*last == 0u) return;
  for (int e = threadIdx.x; e < TM * Q; e += NT) {
    const int ml = e / Q, nl = 4 * (e % Q);
    const int m = m0 + ml, n = n0 + nl;
    if (m >= g.M || n >= g.N) continue;
    const int base = (int)(((size_t)m * g.N + n) * 4);
    f32x4 a4[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) a4[q] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int z0 = 0; z0 < gz; z0 += 8) {     // 8 slab loads in flight per pass
      f32x4 part[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int z = min(z0 + q, gz - 1);
        part[q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ws, base + (int)((size_t)z * slab * 4), 0, 16));
      }
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (z0 + q < gz) a4[q & 3] += part[q];   // slab z adds into a4[z & 3] (z0 % 4 == 0)
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float v = g.alpha * ((a4[0][c] + a4[1][c]) + (a4[2][c] + a4[3][c]));
      const int nn = n + c;
      float* cp = g.c + (size_t)m * g.ldc + nn;
      if (g.beta != 0.f) v += g.beta * (*cp);
      if (g.bias) v += g.bias[nn];
      if (g.oh_w) v += onehot_term(g, m, nn);
      st_out(g.c, (size_t)m * g.ldc + nn, PLAIN ? v : apply_epi(g, v, m, nn, step, (uint64_t)m * g.N + nn), g.wt);
    }
  }
}

// TM x TN output tile (64x64; 32x32 for short-K GEMMs that would otherwise need split-K; 128x128
// for large-M x N GEMMs -- generation at M = 40k, wide tables -- where the operand re-reads of
// small tiles make the GEMM L2-bandwidth-bound):
// 4 waves in a 2x2 grid, each owning (TM/2)x(TN/2) = MI x NJ blocks of 16x16 MFMA accumulators.
// The body of one output tile; (bx, by, bz) index the tile within a (gx, gy, gz) tile grid.  Called by
// gemm_kernel (one GEMM per launch) and gemm_pair_kernel (two independent GEMMs in one launch).
// EK (epilogue kind, chosen on the host per launch): 0 = every epilogue (runtime g.epi); 1 = plain (EPI_NONE:
// bias / alpha / beta / one-hot only); 2 = split-K slice whose slab is reduced by a separate launch (raw
// accumulators only); 3 = the mask product (EPI_MASK: the A / R chains).  The Philox / mask / BN epilogue code a launch cannot reach is then not compiled into
// it -- measured on the weight-gradient tiles (op(A) = A^T, always plain): the dW0 || R0 pair 17.7 -> 14.0 us.
template <bool TA, bool TB, bool F32, bool VEC, int TM, int TN, bool BIN = false, bool ADAM = false, int EK = 0>
__device__ __forceinline__ void gemm_tile(const GemmArgs& g, int bx, int by, int bz, int gx, int gy, int gz,
                                          unsigned char* __restrict__ smem) {
  static_assert(!BIN || (!TA && TB && !F32), "bf16 operands: C = A B^T, both k-contiguous, bf16 MFMA");
  using C = Cfg<F32, TM, TN, BIN>;
  constexpr int KC = C::KC;
  constexpr int MI = TM / 32, NJ = TN / 32, WM = TM / 2, WN = TN / 2;

  // XCD-aware tile order: the dispatcher deals workgroups round-robin over the 8 XCDs (each with
  // its own L2), so consecutive workgroup ids -- the N tiles sharing one A row block -- would land
  // on 8 different L2s.  Remap so each XCD gets a contiguous run of logical tiles.
  // Order 2 (host: when it touches fewer operand bytes per XCD, e.g. a wide output over a short M) walks the
  // logical tiles M-fastest, so an XCD's run is a few N column strips over every row block: its L2 then holds a
  // 1/8 slice of B instead of all of it (the tail past 8 * per decodes the same way, so the map stays a bijection).
  if (g.xcd_remap) {
    const int total = gx * gy * gz;
    const int lin = bx + gx * (by + gy * bz);
    const int per = total / 8;
    const int logical = lin < 8 * per ? (lin % 8) * per + lin / 8 : lin;
    if (g.xcd_remap == 2) {
      by = logical % gy;
      bx = (logical / gy) % gx;
    } else {
      bx = logical % gx;
      by = (logical / gx) % gy;
    }
    bz = logical / (gx * gy);
  }
  const int n0 = bx * TN, m0 = by * TM;
  const int kb = bz * g.kchunk;
  const int ke = min(g.K, kb + g.kchunk);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = w >> 1, wn = w & 1;

  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // A(m,k): TA ? a[k*lda+m] : a[m*lda+k]   -> staged [m][k]; k-contiguous in memory iff !TA
  // B(k,n): TB ? b[n*ldb+k] : b[k*ldb+n]   -> staged [n][k]; k-contiguous in memory iff TB
  // one register slot: burst i+1's loads are issued before burst i is multiplied out of LDS
  using CA = std::conditional_t<BIN, ChunkBF<KC, TM>, Chunk<KC, !TA, TM>>;
  using CB = std::conditional_t<BIN, ChunkBF<KC, TN>, Chunk<KC, TB, TN>>;
  auto load_ab = [&](CA& a_, CB& b_, int k0) {
    if constexpr (BIN) {
      a_.load(g.a16, g.lda, m0, g.M, k0, ke);
      b_.load(g.b16, g.ldb, n0, g.N, k0, ke);
    } else {
      a_.template load<VEC>(g.a, g.lda, m0, g.M, k0, ke);
      b_.template load<VEC>(g.b, g.ldb, n0, g.N, k0, ke);
    }
  };
  auto stage_ab = [&](const CA& a_, const CB& b_, int st) {
    unsigned char* base = smem + st * C::STAGE;
    if constexpr (F32) {
      a_.store_f32(reinterpret_cast<float*>(base));
      b_.store_f32(reinterpret_cast<float*>(base) + TM * C::LD);
    } else if constexpr (BIN) {
      a_.store(reinterpret_cast<uint16_t*>(base));
      b_.store(reinterpret_cast<uint16_t*>(base) + TM * C::LD);
    } else {
      a_.store_bf16(reinterpret_cast<uint16_t*>(base));
      b_.store_bf16(reinterpret_cast<uint16_t*>(base) + TM * C::LD);
    }
  };
  CA ca;
  CB cb;
  auto issue = [&](int k0) { load_ab(ca, cb, k0); };
  auto stage = [&](int st) { stage_ab(ca, cb, st); };
  auto compute = [&](int st, int kvalid) {
    if constexpr (F32) {
      const float* A = reinterpret_cast<const float*>(smem + st * C::STAGE);
      const float* B = A + TM * C::LD;
      const int nsteps = (kvalid + 3) / 4;
      for (int s4 = 0; s4 < nsteps; ++s4) {
        const int kk = 4 * s4 + (lane >> 4);
        float af[MI], bfv[NJ];
#pragma unroll
        for (int i = 0; i < MI; ++i) af[i] = A[(wm * WM + i * 16 + (lane & 15)) * C::LD + kk];
#pragma unroll
        for (int j = 0; j < NJ; ++j) bfv[j] = B[(wn * WN + j * 16 + (lane & 15)) * C::LD + kk];
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfv[j], acc[i][j], 0, 0, 0);
      }
    } else {
      const uint16_t* A = reinterpret_cast<const uint16_t*>(smem + st * C::STAGE);
      const uint16_t* B = A + TM * C::LD;
      const int nsteps = (kvalid + 31) / 32;
      for (int s = 0; s < nsteps; ++s) {
        bf16x8 af[MI], bfr[NJ];
        const int ck = 4 * s + (lane >> 4);   // 16-B k-chunk of this lane's fragment
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const int row = wm * WM + i * 16 + (lane & 15);
          const int pc = TA ? (ck ^ lds_swz<KC>(row)) : ck;     // A image staged column-major iff TA
          af[i] = *reinterpret_cast<const bf16x8*>(&A[row * C::LD + 8 * pc]);
        }
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int row = wn * WN + j * 16 + (lane & 15);
          const int pc = TB ? ck : (ck ^ lds_swz<KC>(row));     // B image staged column-major iff !TB
          bfr[j] = *reinterpret_cast<const bf16x8*>(&B[row * C::LD + 8 * pc]);
        }
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
  };
  // per burst: stage the landed burst into LDS buffer st, issue the next burst, multiply.  One
  // barrier per burst: buffer st was last read two bursts ago, before the previous barrier.
  int st = 0;
  if constexpr (C::DEPTH == 2) {
    // two bursts in flight: register slots 0 / 1 alternate, the loop unrolled by two so each
    // slot stays a static register set; a burst's loads are issued two bursts ahead of its use,
    // so a B-burst GEMM costs ~B/2 memory round trips instead of ~B (the compiler's counted
    // vmcnt waits only for the older slot when staging it)
    CA ca2;
    CB cb2;
    auto issue2 = [&](int k0) { load_ab(ca2, cb2, k0); };
    auto stage2 = [&](int s) { stage_ab(ca2, cb2, s); };
    issue(kb);
    if (kb + KC < ke) issue2(kb + KC);
    for (int k0 = kb; k0 < ke; k0 += 2 * KC) {
      stage(st);
      __syncthreads();
      if (k0 + 2 * KC < ke) issue(k0 + 2 * KC);
      compute(st, min(KC, ke - k0));
      st ^= 1;
      if (k0 + KC < ke) {
        stage2(st);
        __syncthreads();
        if (k0 + 3 * KC < ke) issue2(k0 + 3 * KC);
        compute(st, min(KC, ke - k0 - KC));
        st ^= 1;
      }
    }
  } else {
    issue(kb);
    for (int k0 = kb; k0 < ke; k0 += KC) {
      stage(st);
      __syncthreads();
      if (k0 + KC < ke) issue(k0 + KC);
      compute(st, min(KC, ke - k0));
      st ^= 1;
    }
  }

  if constexpr (EK == 2) {   // split-K slice: the raw accumulators to this slice's slab
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * WM + i * 16 + (lane >> 4) * 4 + r;
          const int n = n0 + wn * WN + j * 16 + (lane & 15);
          if (m < g.M && n < g.N) st_out(g.ws, ((size_t)bz * g.M + m) * g.N + n, acc[i][j][r], g.wt);
        }
    return;
  }
  // one-hot block (alpha == 1, checked on the host): every gathered weight of this lane's outputs is
  // loaded in one unrolled loop with no global store in between (all loads in flight together, one
  // memory round trip) and folded into the accumulators before the epilogue.  Split-K slabs leave it
  // to gemm_splitk_epilogue.
  // (the host refuses a one-hot block with op(A) = A^T: weight-gradient instantiations carry none of it)
  if (!TA && g.oh_w && gz == 1) {
    int rows[MI][4];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = min(m0 + wm * WM + i * 16 + (lane >> 4) * 4 + r, g.M - 1);
        rows[i][r] = g.oh_off[g.oh_col[m]] + g.oh_opt[m];
#if FT_CHECKED
        FT_CHECK(&g_check_gemm, rows[i][r] >= 0 && rows[i][r] < g.oh_c, CHK_ONEHOT);
        rows[i][r] = min(max(rows[i][r], 0), g.oh_c - 1);
#endif
      }
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int n = min(n0 + wn * WN + j * 16 + (lane & 15), g.N - 1);
#pragma unroll
        for (int r = 0; r < 4; ++r)
          acc[i][j][r] += g.oh_trans ? g.oh_w[(size_t)rows[i][r] * g.oh_ld + n] : g.oh_w[(size_t)n * g.oh_ld + rows[i][r]];
      }
  }
  // weight-gradient instantiations (op(A) = A^T) have a plain epilogue (host-checked): no epilogue code at all
  constexpr bool PLAIN = TA || EK == 1 || EK == 4;   // (EK 4: BatchNorm partials, plain C + bias)
  constexpr bool MASKED = !TA && EK == 3;
  const uint64_t step = (!PLAIN && g.epi == EPI_LRELU_DROPOUT && g.rng_ctr) ? *g.rng_ctr : 0ull;
  if constexpr (BIN && TM <= 64) if (g.c16) {
    // bf16 output (host: unsplit, beta = 0, epilogue NONE / RELU / BN_EVAL_RELU): the tile goes
    // through LDS and each thread writes 8 consecutive columns of a row as one 16-B store (128x128
    // tiles: in their own LDS epilogue below -- this one would cost them 52 more VGPRs)
    constexpr int LDC = TN + 1;
    static_assert((size_t)(TM * LDC + 5 * TN) * 4 <= (TM <= 64 ? 1 : 2) * C::STAGE,
                  "bf16 epilogue tile must fit the LDS a launch gets");
    __syncthreads();
    float* cs = reinterpret_cast<float*>(smem);
    float* cp = cs + TM * LDC;     // per-column [bias | rm | rsqrt(rv + eps) | gamma | beta] of the tile
    if (threadIdx.x < TN) {        // one load of each parameter per column, by one thread
      const int nn = min(n0 + (int)threadIdx.x, g.N - 1);
      const ColEpi c = col_epi(g, nn);
      cp[threadIdx.x] = g.bias ? g.bias[nn] : 0.f;
      cp[TN + threadIdx.x] = c.rm;
      cp[2 * TN + threadIdx.x] = c.r;
      cp[3 * TN + threadIdx.x] = c.gamma;
      cp[4 * TN + threadIdx.x] = c.beta;
    }
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          cs[(wm * WM + i * 16 + (lane >> 4) * 4 + r) * LDC + wn * WN + j * 16 + (lane & 15)] = acc[i][j][r];
    __syncthreads();
    // a thread's 8 columns are the same in every pass (NT is a multiple of TN / 8)
    static_assert(NT % (TN / 8) == 0, "fixed columns per thread");
    const int nl = 8 * (threadIdx.x % (TN / 8));
    float colb[8];
    ColEpi ce[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      colb[c] = cp[nl + c];
      ce[c] = ColEpi{cp[TN + nl + c], cp[2 * TN + nl + c], cp[3 * TN + nl + c], cp[4 * TN + nl + c]};
    }
#pragma unroll 1
    for (int e = threadIdx.x; e < TM * (TN / 8); e += NT) {
      const int ml = e / (TN / 8);
      const int m = m0 + ml, n = n0 + nl;
      if (m >= g.M || n >= g.N) continue;
      float y[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const int nn = min(n + c, g.N - 1);
        float v = g.alpha * cs[ml * LDC + nl + c];
        if (g.bias) v += colb[c];
        y[c] = apply_epi_c(g, v, m, nn, 0ull, 0ull, ce[c]);
      }
      uint16_t* dst = g.c16 + (size_t)m * g.ldc + n;
      if (n + 8 <= g.N && (reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
        *reinterpret_cast<u32x4*>(dst) = u32x4{pack_bf16x2(y[0], y[1]), pack_bf16x2(y[2], y[3]),
                                               pack_bf16x2(y[4], y[5]), pack_bf16x2(y[6], y[7])};
      } else {
        for (int c = 0; c < 8 && n + c < g.N; ++c) dst[c] = f2bf(y[c]);
      }
    }
    return;
  }
  if constexpr (TM <= 64) {
    if (gz > 1 && g.red_inl) {
      splitk_inlaunch<TM, TN, MI, NJ, PLAIN>(g, acc, m0, n0, by * gx + bx, bz, gz, lane, wm, wn, smem, step);
      return;
    }
  }
  if constexpr (TM >= 128) {
    // 64 accumulators per lane: a fully unrolled epilogue (Philox, loads, stores per element) is
    // past the unroller's budget and the accumulator array would land in scratch, so the tile goes
    // through LDS (the stage buffers are free now) and is written out row-contiguously
    static_assert((size_t)TM * (TN + 1) * 4 <= 2 * C::STAGE, "epilogue tile must fit the stage buffers");
    __syncthreads();
    float* cs = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          cs[(wm * WM + i * 16 + (lane >> 4) * 4 + r) * (TN + 1) + wn * WN + j * 16 + (lane & 15)] = acc[i][j][r];
    // fp32 output, unsplit, 16-B aligned rows: each thread owns a column quad and writes it as one 16-B store (a
    // quarter of the store / index instructions of the per-element loop below; same arithmetic per element)
    if (gz == 1 && !(BIN && g.c16) && (g.ldc & 3) == 0 && (reinterpret_cast<uintptr_t>(g.c) & 15) == 0) {
      static_assert(NT % (TN / 4) == 0, "fixed column quad per thread");
      const int nq = 4 * (threadIdx.x % (TN / 4));
      float cb4[4];
      ColEpi ce4[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int nc = min(n0 + nq + c, g.N - 1);
        cb4[c] = g.bias ? g.bias[nc] : 0.f;
        ce4[c] = col_epi(g, nc);
      }
      __syncthreads();
      const __amdgpu_buffer_rsrc_t crs = __builtin_amdgcn_make_buffer_rsrc(g.c, 0, 0x7FFFFFFF, 0x00020000);
      for (int ml = threadIdx.x / (TN / 4); ml < TM; ml += NT / (TN / 4)) {
        const int m = m0 + ml, n = n0 + nq;
        if (m >= g.M || n >= g.N) continue;
        float y[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          float v = g.alpha * cs[ml * (TN + 1) + nq + c];
          if (g.beta != 0.f && n + c < g.N) v += g.beta * g.c[(size_t)m * g.ldc + n + c];
          if (g.bias) v += cb4[c];
          y[c] = PLAIN ? v : apply_epi_c(g, v, m, n + c, step, (uint64_t)m * g.N + n + c, ce4[c]);
        }
        const size_t e0 = (size_t)m * g.ldc + n;
        if (n + 4 <= g.N) {
          const f32x4 v4 = f32x4{y[0], y[1], y[2], y[3]};
          if (g.wt)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v4), crs, (int)(e0 * 4), 0, 16);
          else
            *reinterpret_cast<f32x4*>(g.c + e0) = v4;
        } else {
#pragma unroll
          for (int c = 0; c < 4; ++c)
            if (n + c < g.N) st_out(g.c, e0 + c, y[c], g.wt);
        }
      }
      return;
    }
    // each thread stays on one column (NT is a multiple of TN): its bias / BN parameters load once
    static_assert(NT % TN == 0, "fixed column per thread");
    const int nl = threadIdx.x % TN;
    const int nc = min(n0 + nl, g.N - 1);
    const float colb = g.bias ? g.bias[nc] : 0.f;
    const ColEpi ce = col_epi(g, nc);
    __syncthreads();
    for (int e = threadIdx.x; e < TM * TN; e += NT) {
      const int ml = e / TN;
      const int m = m0 + ml, n = n0 + nl;
      if (m >= g.M || n >= g.N) continue;
      const float v0 = cs[ml * (TN + 1) + nl];
      if (gz > 1) {
        st_out(g.ws, ((size_t)bz * g.M + m) * g.N + n, v0, g.wt);
        continue;
      }
      float v = g.alpha * v0;
      if constexpr (BIN) {
        if (g.c16) {     // bf16 output (unsplit, beta = 0): consecutive threads, consecutive columns
          if (g.bias) v += colb;
          g.c16[(size_t)m * g.ldc + n] = f2bf(apply_epi_c(g, v, m, n, 0ull, 0ull, ce));
          continue;
        }
      }
      float* cp = g.c + (size_t)m * g.ldc + n;
      if (g.beta != 0.f) v += g.beta * (*cp);
      if (g.bias) v += colb;
      st_out(g.c, (size_t)m * g.ldc + n, PLAIN ? v : apply_epi_c(g, v, m, n, step, (uint64_t)m * g.N + n, ce), g.wt);
    }
    return;
  }
  if constexpr (ADAM) {
    // weight gradient -> Adam (gemm_adam_kernel; unsplit, plain epilogue, checked on the host): each
    // lane's gradients and the same elements' parameter and moments, updated in registers with the
    // float4 Adam's expression (adam_elem); the gradient is also stored (grad-flow diagnostics)
    const float t = g.adam_step[0];
    const float bc1 = 1.f - powf(g.adam_b1, t);
    const float bc2s = sqrtf(1.f - powf(g.adam_b2, t));
    const float sz = g.adam_lr / bc1;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * WM + i * 16 + (lane >> 4) * 4 + r;
          const int n = n0 + wn * WN + j * 16 + (lane & 15);
          if (m >= g.M || n >= g.N) continue;
          const size_t e = (size_t)m * g.ldc + n;
          const float gr = g.alpha * acc[i][j][r];
          float pe = g.adam_p[e], me = g.adam_m[e], ve = g.adam_v[e];
          adam_elem(gr, pe, me, ve, g.adam_b1, g.adam_b2, g.adam_eps, g.adam_wd, sz, bc2s);
          g.c[e] = gr;
          g.adam_m[e] = me;
          g.adam_v[e] = ve;
          g.adam_p[e] = pe;
        }
    return;
  }
  // (the training GEMMs' register epilogue keeps per-element bias loads: hoisting them per column,
  // as the LDS epilogues do, measured 1 us slower per step -- profiles/README.md)
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * WM + i * 16 + (lane >> 4) * 4 + r;
        const int n = n0 + wn * WN + j * 16 + (lane & 15);
        if (m >= g.M || n >= g.N) continue;
        const float v0 = acc[i][j][r];
        if (gz > 1) {
          st_out(g.ws, ((size_t)bz * g.M + m) * g.N + n, v0, g.wt);
          continue;
        }
        float v = g.alpha * v0;
        float* cp = g.c + (size_t)m * g.ldc + n;
        if (g.beta != 0.f) v += g.beta * (*cp);
        if (g.bias) v += g.bias[n];
        st_out(g.c, (size_t)m * g.ldc + n,
               PLAIN ? v : (MASKED ? v * g.ms[(size_t)m * g.ldms + n] : apply_epi(g, v, m, n, step, (uint64_t)m * g.N + n)),
               g.wt);
      }
  if constexpr (EK == 4) {   // (host: BN partials need a plain unsplit C = A op(B) + bias)
    bn_tile_partials<MI, NJ, TN>(g, acc, m0, n0, by, lane, wm, wn, smem);
  }
}

// batched clients (launch.h ClientBatch): client c's copy of every buffer of a GEMM and its Philox seed
__device__ __forceinline__ void client_view(GemmArgs& g, int c) {
  const int64_t o = (int64_t)c * g.cstride;
  g.a = cptr(g.a, o);
  g.b = cptr(g.b, o);
  g.c = cptr(g.c, o);
  g.bias = cptr(g.bias, o);
  g.ms = cptr(g.ms, o);
  g.head_coef = cptr(g.head_coef, o);
  g.head_v = cptr(g.head_v, o);
  g.head_a = cptr(g.head_a, o);
  g.ws = cptr(g.ws, o);
  g.bn_gamma = cptr(g.bn_gamma, o);
  g.bn_beta = cptr(g.bn_beta, o);
  g.bn_rm = cptr(g.bn_rm, o);
  g.bn_rv = cptr(g.bn_rv, o);
  g.rng_ctr = cptr(g.rng_ctr, o);
  g.oh_w = cptr(g.oh_w, o);
  g.oh_col = cptr(g.oh_col, o);
  g.oh_opt = cptr(g.oh_opt, o);
  g.oh_off = cptr(g.oh_off, o);
  g.bn_part = cptr(g.bn_part, o);
  g.tile_cnt = cptr(g.tile_cnt, o);
  g.a16 = cptr(g.a16, o);
  g.b16 = cptr(g.b16, o);
  g.c16 = cptr(g.c16, o);
  g.adam_p = cptr(g.adam_p, o);
  g.adam_m = cptr(g.adam_m, o);
  g.adam_v = cptr(g.adam_v, o);
  g.adam_step = cptr(g.adam_step, o);
  g.seed += (uint64_t)c * g.seed_step;
}

// host: every device pointer of a batched GEMM lies in client 0's slab
static void check_slab(const GemmArgs& g) {
  if (client_batch().k <= 1) return;
  check_slabs("gemm operand", g.a, g.b, g.c, g.bias, g.ms, g.head_coef, g.head_v, g.head_a, g.ws, g.bn_gamma, g.bn_beta,
              g.bn_rm, g.bn_rv, g.rng_ctr, g.oh_w, g.oh_col, g.oh_opt, g.oh_off, g.bn_part, g.tile_cnt, g.a16, g.b16,
              g.c16, g.adam_p, g.adam_m, g.adam_v, g.adam_step);
}

// Every slab load of an output element is issued before the first is consumed (SMAX >= splits
// clamped, always-valid addresses): one memory round trip instead of ceil(splits / 4).
// LDS is sized per launch (gemm_smem_bytes): a GEMM whose K-slice is one burst uses one stage
// buffer, so a 64x64-tile launch over a short K fits 4 workgroups per CU instead of 2.
// BATCH: a batched multi-client launch (grid.z = split-K slices x clients, client-major).  The one-client
// instantiation carries no client prologue at all: even a never-taken client branch costs the step's latency-
// bound GEMMs measurably (the dW0 || R0 pair 17.6 -> 21.6 us, the step 215.5 -> 223 us; profiles/README.md).
template <bool TA, bool TB, bool F32, bool VEC, int TM, int TN, bool BIN = false, bool BATCH = false, int EK = 0>
__global__ __launch_bounds__(NT) void gemm_kernel(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  if constexpr (BATCH) {
    const int sk = (int)gridDim.z / g.nclient;
    const int gx = (int)gridDim.x, gy = (int)gridDim.y;
    int cl, loc;
    if (g.xcd_cl && xcd_client_map((int)(blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z)), gx * gy * sk, g.nclient,
                                   cl, loc)) {
      g.xcd_remap = 0;    // the client's tiles already share one XCD's L2
    } else {
      cl = (int)blockIdx.z / sk;
      loc = (int)blockIdx.x + gx * ((int)blockIdx.y + gy * ((int)blockIdx.z - cl * sk));
    }
    if (cl) client_view(g, cl);
    gemm_tile<TA, TB, F32, VEC, TM, TN, BIN, false, EK>(g, loc % gx, (loc / gx) % gy, loc / (gx * gy), gx, gy, sk, smem);
  } else {
    gemm_tile<TA, TB, F32, VEC, TM, TN, BIN, false, EK>(g, blockIdx.x, blockIdx.y, blockIdx.z, gridDim.x, gridDim.y,
                                                        gridDim.z, smem);
  }
}

// stage buffers a launch needs: two when a K-slice spans several bursts, else one -- unless the
// epilogue stages the whole fp32 tile (128x128 tiles) and needs both
static size_t gemm_smem_bytes(const GemmArgs& g) {
  const int T = g.tile;
  size_t stage;
  if (g.f32) stage = T == 32 ? Cfg<true, 32, 32>::STAGE : (T == 128 ? Cfg<true, 128, 128>::STAGE : Cfg<true, 64, 64>::STAGE);
  else stage = T == 32 ? Cfg<false, 32, 32>::STAGE : (T == 128 ? Cfg<false, 128, 128>::STAGE : Cfg<false, 64, 64>::STAGE);
  const int KC = g.f32 ? Cfg<true, 64, 64>::KC / (T >= 128 ? 2 : 1) : Cfg<false, 64, 64>::KC / (T >= 128 ? 2 : 1);
  const bool one_burst = g.kchunk <= KC;
  return (one_burst && T <= 64) ? stage : 2 * stage;
}

// Two independent GEMMs in ONE launch (horizontal fusion): the first n1 workgroups run GEMM 1's
// tiles, the rest GEMM 2's.  The step has several such pairs (e.g. a weight gradient and the next
// backward product of the same layer); as two launches they pay a kernel boundary and run their
// few dozen workgroups each back to back on an otherwise idle chip.
struct Grid3 {
  int x, y, z;
};

template <class P1, class P2, bool BATCH = false>
__global__ __launch_bounds__(NT) void gemm_pair_kernel(GemmArgs g1, GemmArgs g2, Grid3 grid1, Grid3 grid2) {
  const BIdx bi_ = batch_bidx<BATCH>(g1.xcd_cl);
  constexpr int S1 = 2 * Cfg<false, P1::TM, P1::TM>::STAGE, S2 = 2 * Cfg<false, P2::TM, P2::TM>::STAGE;
  __shared__ __attribute__((aligned(16))) unsigned char smem[S1 > S2 ? S1 : S2];
  if constexpr (BATCH) {
    if (bi_.z) {
      client_view(g1, bi_.z);
      client_view(g2, bi_.z);
    }
  }
  const int n1 = grid1.x * grid1.y * grid1.z;
  int b = bi_.x;
  if (b < n1) {
    gemm_tile<P1::TA, P1::TB, false, P1::VEC, P1::TM, P1::TM>(g1, b % grid1.x, (b / grid1.x) % grid1.y,
                                                               b / (grid1.x * grid1.y), grid1.x, grid1.y, grid1.z, smem);
  } else {
    b -= n1;
    gemm_tile<P2::TA, P2::TB, false, P2::VEC, P2::TM, P2::TM, false, false, P2::EK>(g2, b % grid2.x, (b / grid2.x) % grid2.y,
                                                               b / (grid2.x * grid2.y), grid2.x, grid2.y, grid2.z, smem);
  }
}

template <bool TA_, bool TB_, bool VEC_, int TM_, int EK_ = 0>
struct GemmShape {
  static constexpr bool TA = TA_, TB = TB_, VEC = VEC_;
  static constexpr int TM = TM_, EK = EK_;
};

constexpr int GEMM_MAX_SPLITS = 64;
// 2: every GEMM launch deals its tiles to the XCDs in contiguous runs.  Round 4, same box, two passes of
// tools/microbench.py --step-only: rule-based (1) 207.3-208.1 us per step, always (2) 204.6-205.5 us, off (0)
// 207.6-208.2 us (profiles/knobs_step_r4.txt): the remap's index math is cheaper than the L2 sharing it buys
// even on the short-K step GEMMs (the round-2 measurement that kept it off there predates the pair / chain
// launches)
int g_gemm_xcd_remap = 2;
int g_gemm_xcd_nmajor = 1;
int g_gemm_store_wt = 0;   // 1: write-through (sc1) output / slab stores
int g_gemm_pairs = 1;      // 1: independent GEMM pairs share one launch (launch_gemm_pair)
int g_gemm_pair_max_wg = 0;   // pairs whose two grids together exceed this many workgroups launch separately (0: no limit)
int g_gemm_splitk_inlaunch = 1;   // 1: split-K reduced by the last-arriving slice (GemmArgs::tile_cnt)

// the reduced, epilogue-applied value of output idx = m * N + n (stored to C by the caller)
// MASK: the epilogue is EPI_MASK (host-checked) -- no Philox / BN code in the launch (see gemm_tile's EK)
template <int SMAX, bool MASK = false>
__device__ __forceinline__ float splitk_value(const GemmArgs& g, size_t idx, int m, int n, uint64_t step) {
  const int splits = g.splitk;
  const size_t total = (size_t)g.M * g.N;
  float part[SMAX];
#pragma unroll
  for (int z = 0; z < SMAX; ++z) part[z] = g.ws[(size_t)min(z, splits - 1) * total + idx];
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int z = 0; z < SMAX; ++z)
    if (z < splits) acc[z & 3] += part[z];
  float v = g.alpha * ((acc[0] + acc[1]) + (acc[2] + acc[3]));
  float* cp = g.c + (size_t)m * g.ldc + n;
  if (g.beta != 0.f) v += g.beta * (*cp);
  if (g.bias) v += g.bias[n];
  if (g.oh_w) v += onehot_term(g, m, n);
  if constexpr (MASK) return v * g.ms[(size_t)m * g.ldms + n];
  return apply_epi(g, v, m, n, step, idx);
}

template <int SMAX, bool BT_ = false>
__global__ __launch_bounds__(256) void gemm_splitk_epilogue(GemmArgs g) {
  const BIdx bi_ = batch_bidx<BT_>(g.xcd_cl);
  if (bi_.z) client_view(g, bi_.z);
  const size_t total = (size_t)g.M * g.N;
  const uint64_t step = (g.epi == EPI_LRELU_DROPOUT && g.rng_ctr) ? *g.rng_ctr : 0ull;
  for (size_t idx = (size_t)bi_.x * blockDim.x + threadIdx.x; idx < total; idx += (size_t)gridDim.x * blockDim.x) {
    const int m = (int)(idx / g.N), n = (int)(idx % g.N);
    st_out(g.c, (size_t)m * g.ldc + n, splitk_value<SMAX>(g, idx, m, n, step), g.wt);
  }
}

// Two GEMMs of a chain in one launch (GemmArgs::chain): the head's output row m is final in its split-K
// reduction (SMAX > 0; SMAX = 0: already in C), and the tail -- whose A operand is exactly that output,
// C2[m, :] = epi2(C[m, :] B2^T + bias2) -- needs only that row.  Workgroup (m, s) reduces row m into LDS
// (s == 0 also stores it) and forms C2[m, 64 s .. 64 s + 64): 64 outputs x 4 K-quarters per 256 threads,
// each thread reading 16-B chunks of one B2 row, then the tail's epilogue (bias, LeakyReLU + Philox
// dropout with the same mask indices as the GEMM epilogue, the D head's seed, or the mask product).
// The discriminator's second layer (150 or 50 x 256 x 256) and its R-chain link R1 = (R0 W1^T) . MS1
// were launches of their own after D0's / R0's reduction.
constexpr int CH_MAXK = 1024, CH_COLS = 64;
int g_chain_coalesced = 0;   // chain tail: per-column weight rows read lane-contiguous + wave sums (1) or one row per lane (0)
int g_chain_pre = 1;         // chain tail weights prefetched: 0 never, 1 grids of <= 512 workgroups, 2 always
int g_chain_rows = 2;        // 2: a grid too large for the prefetch runs two head rows per workgroup (with it)
// MASK: head and tail both EPI_MASK (the R chain) -- the launch carries no Philox / BN epilogue code
// PRE: the tail's weights are prefetched (K = 256; host: grids that stay resident at the larger register count).
// ROWS (PRE only): head rows per workgroup -- 2 halves the workgroups and the tail-weight traffic of a grid that
// would not stay resident with one row each (the 150-row D phase).
// ACH: the tail also forms the head's backward link A0 = (A1 W1) . MS0 (GemmArgs::ach_*; one client, per-row
// weights rows, no coalesced variant): A1 = the tail's head seed is in registers of the kq == 0 threads right
// after the tail's epilogue, the W1 rows of the workgroup's 64-column slab are the ones it just multiplied, so
// each workgroup adds a [ROWS, 64] x [64, K] partial and the row group's last arriver sums the nb partials --
// the separate A-chain GEMM launch after the chain is gone.
template <int SMAX, bool MASK = false, bool BT_ = false, bool PRE = false, int ROWS = 1, bool ACH = false>
__global__ __launch_bounds__(256) void chain_epilogue_kernel(GemmArgs g, GemmArgs t) {
  static_assert(ROWS == 1 || PRE, "two rows per workgroup only with the prefetched tail");
  static_assert(!ACH || (!MASK && !BT_), "the fused A-chain takes the D-head chain of one client");
  const BIdx bi_ = batch_bidx<BT_>(g.xcd_cl);
  __shared__ __attribute__((aligned(16))) float row[ROWS][CH_MAXK];
  __shared__ float part[ROWS][4][CH_COLS];
  if (bi_.z) {
    client_view(g, bi_.z);
    client_view(t, bi_.z);
  }
  const int m0 = bi_.x * ROWS, s = bi_.y;
  const uint64_t step = (g.epi == EPI_LRELU_DROPOUT && g.rng_ctr) ? *g.rng_ctr : 0ull;
  // K = 256 (the discriminator's second layer): this thread's 16 float4 of its tail weight row do not depend on
  // the head's row, so all 16 are requested before the slabs are reduced -- one round trip, overlapping the
  // slabs' -- instead of four dependent batches of 4 after the barrier.  (Compile-time trip count: a runtime
  // bound on the register array would put it in scratch.)  The 64 extra VGPRs (130 -> 194) leave room for two
  // workgroups per CU instead of three, so one-row workgroups take it only in grids of <= 512 (host): measured,
  // the 50-row chains 9.9 -> 9.1 and 7.9 -> 6.9 us, the 600-workgroup D-phase chain 11.9 -> 13.1 us.
  constexpr int PQ = 16;
  const bool pre = PRE && !t.chain_co && g.N == 16 * PQ;
  float4 wp[PRE ? PQ : 1];
  if (pre) {
    const int jp = min(s * CH_COLS + (int)(threadIdx.x & (CH_COLS - 1)), t.N - 1);
    const float4* w4 = reinterpret_cast<const float4*>(t.b + (size_t)jp * t.ldb) + (threadIdx.x >> 6) * PQ;
#pragma unroll
    for (int k = 0; k < (PRE ? PQ : 1); ++k) wp[k] = w4[k];
  }
  for (int n = threadIdx.x; n < g.N; n += blockDim.x) {
#pragma unroll
    for (int r = 0; r < ROWS; ++r) {
      const int m = m0 + r;
      float v = 0.f;
      if (ROWS == 1 || m < g.M) {
        if constexpr (SMAX > 0) {
          v = splitk_value<SMAX, MASK>(g, (size_t)m * g.N + n, m, n, step);
          if (s == 0) st_out(g.c, (size_t)m * g.ldc + n, v, g.wt);
        } else {
          v = g.c[(size_t)m * g.ldc + n];
        }
      }
      row[r][n] = v;
    }
  }
  __syncthreads();
  const int jl = threadIdx.x & (CH_COLS - 1), kq = threadIdx.x >> 6;
  const int j = s * CH_COLS + jl;
  if (!PRE && !ACH && t.chain_co) {
    // wave kq owns 16 of the block's 64 output columns; for each, the 64 lanes read the column's weight row as
    // consecutive float4 (one coalesced 1 KB request per 256 K values, instead of 64 rows 1 KB apart per
    // request) and a wave sum finishes the dot product
    constexpr int JW = CH_COLS / 4;
    const int lane = threadIdx.x & 63, m = m0;
    float p[JW];
#pragma unroll
    for (int jj = 0; jj < JW; ++jj) p[jj] = 0.f;
    for (int k0 = 0; k0 < g.N; k0 += 256) {
      const int k = k0 + 4 * lane;
      const bool kin = k < g.N;
      const float4 x = kin ? *reinterpret_cast<const float4*>(row[0] + k) : make_float4(0.f, 0.f, 0.f, 0.f);
      float4 w[JW];
#pragma unroll
      for (int jj = 0; jj < JW; ++jj) {
        const int jc = min(s * CH_COLS + kq * JW + jj, t.N - 1);
        w[jj] = *reinterpret_cast<const float4*>(t.b + (size_t)jc * t.ldb + min(k, g.N - 4));
      }
#pragma unroll
      for (int jj = 0; jj < JW; ++jj)
        if (kin) p[jj] += (w[jj].x * x.x + w[jj].y * x.y) + (w[jj].z * x.z + w[jj].w * x.w);
    }
#pragma unroll
    for (int jj = 0; jj < JW; ++jj) {
      const float tsum = wave_sum(p[jj]);
      if (lane == 0) part[0][0][kq * JW + jj] = tsum;
    }
    __syncthreads();
    if (kq == 0 && j < t.N) {
      float v = t.alpha * part[0][0][jl];
      if (t.bias) v += t.bias[j];
      const uint64_t st = (t.epi == EPI_LRELU_DROPOUT && t.rng_ctr) ? *t.rng_ctr : 0ull;
      if constexpr (MASK) t.c[(size_t)m * t.ldc + j] = v * t.ms[(size_t)m * t.ldms + j];
      else t.c[(size_t)m * t.ldc + j] = apply_epi(t, v, m, j, st, (uint64_t)m * t.N + j);
    }
    return;
  }
  const int q4 = g.N / 16;                       // float4 per K-quarter (host: N % 16 == 0)
  if (pre) {
#pragma unroll
    for (int r = 0; r < ROWS; ++r) {
      const float4* r4 = reinterpret_cast<const float4*>(row[r]) + kq * PQ;
      float a0 = 0.f, a1 = 0.f;
#pragma unroll
      for (int k = 0; k < (PRE ? PQ : 1); ++k) {
        const float4 w = wp[k], x = r4[k];
        a0 = fmaf(w.x, x.x, a0);
        a1 = fmaf(w.y, x.y, a1);
        a0 = fmaf(w.z, x.z, a0);
        a1 = fmaf(w.w, x.w, a1);
      }
      part[r][kq][jl] = a0 + a1;
    }
  } else {
    float a0 = 0.f, a1 = 0.f;
    if (j < t.N) {
      const float4* w4 = reinterpret_cast<const float4*>(t.b + (size_t)j * t.ldb) + kq * q4;
      const float4* r4 = reinterpret_cast<const float4*>(row[0]) + kq * q4;
#pragma unroll 4
      for (int k = 0; k < q4; ++k) {
        const float4 w = w4[k], x = r4[k];
        a0 = fmaf(w.x, x.x, a0);
        a1 = fmaf(w.y, x.y, a1);
        a0 = fmaf(w.z, x.z, a0);
        a1 = fmaf(w.w, x.w, a1);
      }
    }
    part[0][kq][jl] = a0 + a1;
  }
  __syncthreads();
  if (kq == 0 && j < t.N) {
    const uint64_t st = (t.epi == EPI_LRELU_DROPOUT && t.rng_ctr) ? *t.rng_ctr : 0ull;
#pragma unroll
    for (int r = 0; r < ROWS; ++r) {
      const int m = m0 + r;
      if (ROWS > 1 && m >= g.M) break;
      float v = t.alpha * ((part[r][0][jl] + part[r][1][jl]) + (part[r][2][jl] + part[r][3][jl]));
      if (t.bias) v += t.bias[j];
      if constexpr (MASK) t.c[(size_t)m * t.ldc + j] = v * t.ms[(size_t)m * t.ldms + j];
      else t.c[(size_t)m * t.ldc + j] = apply_epi(t, v, m, j, st, (uint64_t)m * t.N + j);
    }
  }
  if constexpr (ACH) {
    __shared__ float a1s[ROWS][CH_COLS];
    __shared__ unsigned ach_last;
    if (kq == 0) {
#pragma unroll
      for (int r = 0; r < ROWS; ++r) {
        const int m = m0 + r;   // the seed this thread's apply_epi just stored (same-thread read-back)
        a1s[r][jl] = (j < t.N && (ROWS == 1 || m < g.M)) ? t.head_a[(size_t)m * t.ldha + j] : 0.f;
      }
    }
    __syncthreads();
    const int jn = min(CH_COLS, t.N - s * CH_COLS);
    for (int i = threadIdx.x; i < g.N; i += blockDim.x) {
      float acc[ROWS];
#pragma unroll
      for (int r = 0; r < ROWS; ++r) acc[r] = 0.f;
      const float* wc = t.b + (size_t)s * CH_COLS * t.ldb + i;   // W1[64 s + c, i]: coalesced over i
      for (int c = 0; c < jn; ++c) {
        const float w = wc[(size_t)c * t.ldb];
#pragma unroll
        for (int r = 0; r < ROWS; ++r) acc[r] = fmaf(a1s[r][c], w, acc[r]);
      }
#pragma unroll
      for (int r = 0; r < ROWS; ++r) {
        const int m = m0 + r;
        if (ROWS == 1 || m < g.M)
          __hip_atomic_store(&t.ach_ws[((size_t)s * g.M + m) * g.N + i], acc[r], __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned tk = __hip_atomic_fetch_add(&t.ach_cnt[bi_.x], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned last = tk == gridDim.y - 1 ? 1u : 0u;
      if (last) __hip_atomic_store(&t.ach_cnt[bi_.x], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      ach_last = last;
    }
    __syncthreads();
    if (ach_last == 0u) return;
    // the slabs in order (the same bits every run); MS0[m, i] was stored by this thread (SMAX > 0: its row loop
    // above covers column i) or by an earlier launch
    for (int i = threadIdx.x; i < g.N; i += blockDim.x) {
#pragma unroll
      for (int r = 0; r < ROWS; ++r) {
        const int m = m0 + r;
        if (ROWS > 1 && m >= g.M) break;
        float sum = 0.f;
        for (int q = 0; q < (int)gridDim.y; ++q)
          sum += __hip_atomic_load(&t.ach_ws[((size_t)q * g.M + m) * g.N + i], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        t.ach_out[(size_t)m * t.ld_ach + i] = sum * g.ms[(size_t)m * g.ldms + i];
      }
    }
  }
}

// A weight-gradient GEMM and its optimizer's Adam in ONE launch: the first nt workgroups are the
// GEMM's tiles, which apply Adam to their own outputs (gemm_tile<..., ADAM>); the rest run the
// flat-buffer Adam with its folded column sums (adam_cs_body), skipping the GEMM's range.  The step's
// last two launches (the generator's first-layer weight gradient, then the generator's Adam) become
// one: none of the other Adam work waits for that gradient.
template <bool VEC, int TM, int AUX, bool BATCH = false, int U = 1>
__global__ __launch_bounds__(NT) void gemm_adam_kernel(GemmArgs g, Grid3 gd, float* p, const float* gr, float* m,
                                                       float* v, const float* step, int64_t n4, float lr, float b1,
                                                       float b2, float eps, float wd, uint64_t* rng_bump,
                                                       AdamColsum cs) {
  const BIdx bi_ = batch_bidx<BATCH>(g.xcd_cl);
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * Cfg<false, TM, TM>::STAGE];
  int64_t co = 0;
  if constexpr (BATCH) {
    co = (int64_t)bi_.z * g.cstride;
    if (co) {   // batched clients: the GEMM's buffers (its Adam pointers included) and the Adam operands
      client_view(g, bi_.z);
      p = cptr(p, co);
      gr = cptr(gr, co);
      m = cptr(m, co);
      v = cptr(v, co);
      step = cptr(step, co);
      rng_bump = cptr(rng_bump, co);
    }
  }
  const int nt = gd.x * gd.y * gd.z;
  const int b = bi_.x;
  if (b < nt) {
    gemm_tile<true, false, false, VEC, TM, TM, false, true>(g, b % gd.x, (b / gd.x) % gd.y, b / (gd.x * gd.y), gd.x,
                                                             gd.y, gd.z, smem);
  } else {
    adam_cs_body<AUX, U>(b - nt, (int)gridDim.x - nt, p, gr, m, v, step, n4, lr, b1, b2, eps, wd, rng_bump, cs, co);
  }
}

int gemm_kc(int f32) { return f32 ? Cfg<true, 64, 64>::KC : Cfg<false, 64, 64>::KC; }

// tile grid, split count, K chunk and per-launch flags of one GEMM
static dim3 gemm_prepare(GemmArgs& g) {
  const ClientBatch& cb = client_batch();
  g.nclient = cb.k > 1 ? cb.k : 1;
  g.cstride = cb.k > 1 ? cb.stride : 0;
  g.xcd_cl = cb.k > 1 ? cb.xcd : 0;
  g.seed_step = cb.k > 1 ? cb.seed_step : 0;
  const int KC = gemm_kc(g.f32);
  const int T = g.tile == 32 ? 32 : (g.tile == 128 ? 128 : 64);   // square output tile
  g.tile = T;
  const int tm = (g.M + T - 1) / T, tn = (g.N + T - 1) / T;
  if (g.splitk < 1 || g.K <= 0 || g.ws == nullptr || g.c16 != nullptr) g.splitk = 1;
  g.splitk = std::min(g.splitk, GEMM_MAX_SPLITS);   // the epilogue holds every slab value in registers
  int kchunk = (std::max(g.K, 1) + g.splitk - 1) / g.splitk;
  kchunk = ((kchunk + KC - 1) / KC) * KC;   // whole bursts per split
  g.splitk = (std::max(g.K, 1) + kchunk - 1) / kchunk;
  g.kchunk = kchunk;
  // (buffer stores take 32-bit byte offsets)
  g.wt = g_gemm_store_wt && (int64_t)g.M * g.ldc * 4 < (int64_t)INT32_MAX &&
         (int64_t)g.splitk * g.M * g.N * 4 < (int64_t)INT32_MAX;
  // measured (profiles/README.md): the XCD-contiguous order pays off on long-K tiles (G-out paired
  // 13.1 -> 10.9 us, split D0 11.9 -> 11.5 us) and costs ~0.2 us of index math on short-K ones;
  // on 128x128-tile GEMMs over >= 8192 rows (generation) the N tiles of one A row block then share
  // an L2 whatever K is (generate_decoded(40000): 375 -> 360 us)
  g.red_inl = g.tile_cnt != nullptr && g_gemm_splitk_inlaunch && g.splitk > 1 && T <= 64 && g.N % 4 == 0 &&
              (int64_t)g.splitk * g.M * g.N * 4 < (int64_t)INT32_MAX;
  // (and on any grid of >= 1024 workgroups: the wide table's GEMMs -- dW_out 3,190 128-tiles over K = 500, dW0,
  // g = A0 W0 over 2,154 tiles -- 0.3256 -> 0.3145 s/epoch with the remap forced, profiles/wide_r4.md)
  g.xcd_remap = g_gemm_xcd_remap == 2 ||
                (g_gemm_xcd_remap == 1 && ((g.splitk > 1 && kchunk >= 512) || (g.splitk == 1 && g.K >= 768) ||
                                           (T == 128 && tm >= 64) || (int64_t)tm * tn * g.splitk >= 1024));
  // M-fastest order when an XCD's run of per = tiles / 8 logical tiles then spans fewer operand rows (row blocks
  // x T of A + column tiles x T of B, both K long): the wide table's G out, 8 x 55 tiles, 7,168 -> 1,920 rows per
  // XCD.  Same tiles, same sums: only which XCD (L2) computes a tile changes.
  if (g.xcd_remap && g_gemm_xcd_nmajor && g.splitk == 1) {
    const int64_t per = std::max<int64_t>((int64_t)tm * tn / 8, 1);
    const int64_t r1 = (per + tn - 1) / tn + 1, c1 = std::min<int64_t>(per, tn);   // N-fastest (order 1)
    const int64_t r2 = std::min<int64_t>(per, tm), c2 = (per + tm - 1) / tm + 1;   // M-fastest (order 2)
    if (4 * (r2 + c2) < 3 * (r1 + c1)) g.xcd_remap = 2;
  }
  return dim3(tn, tm, g.splitk);
}

// epilogue kind of a launch (gemm_tile's EK): a split-K slice reduced by its own launch, a plain epilogue, or any
static int gemm_ek(const GemmArgs& g) {
  if (g.bn_part) return 4;                     // BatchNorm partials of the output
  if (g.splitk > 1 && !g.red_inl) return 2;
  if (g.splitk > 1) return 0;   // (in-launch reduction: the generic body)
  return g.epi == EPI_NONE ? 1 : (g.epi == EPI_MASK ? 3 : 0);
}

template <bool BATCH>
static void gemm_dispatch_t(const GemmArgs& g, dim3 grid, dim3 block, size_t lds, hipStream_t stream) {
  const int T = g.tile;
  if (g.bin) {   // bf16 operands: C = A B^T only (checked on the host)
    if (T == 32) hipLaunchKernelGGL((gemm_kernel<false, true, false, true, 32, 32, true, BATCH>), grid, block, lds, stream, g);
    else if (T == 128) hipLaunchKernelGGL((gemm_kernel<false, true, false, true, 128, 128, true, BATCH>), grid, block, lds, stream, g);
    else hipLaunchKernelGGL((gemm_kernel<false, true, false, true, 64, 64, true, BATCH>), grid, block, lds, stream, g);
    return;
  }
  const bool vec = g.vec != 0;   // both operands qualify for 16-B loads (decided by the caller)
  if constexpr (!BATCH) {
    const int ek = gemm_ek(g);
    if (ek == 4) {   // BatchNorm partials of the output: row-major A, 32 / 64 tiles, 16-B operands (host-checked)
#define FEDTGAN_GEMM_BN(F, TT)                                                                                    \
  if (g.tb) hipLaunchKernelGGL((gemm_kernel<false, true, F, true, TT, TT, false, false, 4>), grid, block, lds, stream, g); \
  else hipLaunchKernelGGL((gemm_kernel<false, false, F, true, TT, TT, false, false, 4>), grid, block, lds, stream, g);
      if (g.f32) {
        if (T == 32) { FEDTGAN_GEMM_BN(true, 32) } else { FEDTGAN_GEMM_BN(true, 64) }
      } else {
        if (T == 32) { FEDTGAN_GEMM_BN(false, 32) } else { FEDTGAN_GEMM_BN(false, 64) }
      }
#undef FEDTGAN_GEMM_BN
      return;
    }
  }
// (op(A) = A^T layouts are plain whatever EK says; a split one keeps the generic body)
#define FEDTGAN_GEMM_LAYOUTS(F, V, TT, EK)                                                                        \
  if (!g.ta && g.tb) hipLaunchKernelGGL((gemm_kernel<false, true, F, V, TT, TT, false, BATCH, EK>), grid, block, lds, stream, g);       \
  else if (!g.ta && !g.tb) hipLaunchKernelGGL((gemm_kernel<false, false, F, V, TT, TT, false, BATCH, EK>), grid, block, lds, stream, g); \
  else if (g.ta && !g.tb) hipLaunchKernelGGL((gemm_kernel<true, false, F, V, TT, TT, false, BATCH>), grid, block, lds, stream, g);   \
  else hipLaunchKernelGGL((gemm_kernel<true, true, F, V, TT, TT, false, BATCH>), grid, block, lds, stream, g);
// EK variants for the bf16 32x32 and 64x64 tiles (the one-client step runs 32-tiles; the batched step 64-tiles)
#define FEDTGAN_GEMM_EK(F, V, TT)                                   \
  if constexpr (!(F)) {                                             \
    const int ek = gemm_ek(g);                                      \
    if (ek == 2) {                                                  \
      FEDTGAN_GEMM_LAYOUTS(F, V, TT, 2)                             \
    } else if (ek == 3) {                                           \
      FEDTGAN_GEMM_LAYOUTS(F, V, TT, 3)                             \
    } else if (ek == 1) {                                           \
      FEDTGAN_GEMM_LAYOUTS(F, V, TT, 1)                             \
    } else {                                                        \
      FEDTGAN_GEMM_LAYOUTS(F, V, TT, 0)                             \
    }                                                               \
  } else {                                                          \
    FEDTGAN_GEMM_LAYOUTS(F, V, TT, 0)                               \
  }
#define FEDTGAN_GEMM_TILES(F, V)                                    \
  if (T == 32) {                                                    \
    FEDTGAN_GEMM_EK(F, V, 32)                                       \
  } else if (T == 128) {                                            \
    FEDTGAN_GEMM_LAYOUTS(F, V, 128, 0)                              \
  } else {                                                          \
    FEDTGAN_GEMM_EK(F, V, 64)                                       \
  }
#define FEDTGAN_GEMM_DISPATCH(F) \
  if (vec) {                     \
    FEDTGAN_GEMM_TILES(F, true)  \
  } else {                       \
    FEDTGAN_GEMM_TILES(F, false) \
  }
  if (g.f32) {
    FEDTGAN_GEMM_DISPATCH(true)
  } else {
    FEDTGAN_GEMM_DISPATCH(false)
  }
#undef FEDTGAN_GEMM_TILES
#undef FEDTGAN_GEMM_EK
#undef FEDTGAN_GEMM_LAYOUTS
#undef FEDTGAN_GEMM_DISPATCH
}

// ------------------------------------------------------------------------ short-K weight gradient
// C [M <= 256, N] = A^T B with A [K, M], B [K, N] both row-major fp32 and K <= 160: the discriminator's
// first-layer weight gradient dW0 = A0^T X of the wide table (256 x 137,800 over the 150 stacked rows).  As a
// tile GEMM that is 2,154 workgroups of 128 x 128 each staging two transposed K = 150 operands and writing a
// 64 KB tile, one round of loads, MFMAs and stores after the other (profiles/wide_r6.md: 100-108 us against
// a 141 MB-write + 83 MB-read bound of ~35 us).  Here one persistent workgroup per CU keeps the whole A^T
// operand resident in LDS (bf16, 80 KB) and walks 64-column strips of B: strip s + 1's loads are in flight
// (registers) while strip s is multiplied and stored.  Both LDS images are row-major [k][column] -- written
// from coalesced float4 loads with 8-B stores -- and read as MFMA operands with gfx950's transposing LDS read
// (ds_read_b64_tr_b16: a 16-lane group gets 16 columns x 4 consecutive k), so neither operand is transposed
// in registers.  The 16-B chunks of a row are XOR-swizzled by the row so that a 32-lane half's two 4-row
// blocks (k rows 8 apart) hit 64 distinct banks.
constexpr int SK_THREADS = 512, SK_NS = 64, SK_KMAX = 160, SK_MMAX = 256;
int g_gemm_shortk = 1;            // 0: the tile GEMM path for every shape
int g_gemm_shortk_min_n = 16384;  // narrower products keep the tile GEMM (and its pairing)

typedef short sk_v4s __attribute__((ext_vector_type(4)));

// byte offset of halfs [c, c + 4) of row r in a row-major bf16 image of W halfs per row (W = 64 or 256):
// chunk (8 halfs) index XOR a per-row slot pattern that separates rows {0..3, 8..11} (mod 16) into 8 bank groups
template <int W>
__device__ __forceinline__ int sk_off(int r, int c) {
  const int sw = W == 32 ? 2 * ((r >> 3) & 1)                                 // 64-B rows: 4 per 64 banks
               : W == 64 ? 2 * (((r >> 1) & 1) | (((r >> 3) & 1) << 1))      // 128-B rows: odd rows sit 32 banks over
                         : 2 * ((r & 3) | (((r >> 3) & 1) << 2));             // 512-B rows: every row on bank 0
  return (r * W + (((c >> 3) ^ sw) << 3) + (c & 7)) * 2;
}

// 8 consecutive k (from k0) of column c0 + (lane & 15), k0 = 8 * (lane >> 4) + kstep: two transposed 4-row reads
template <int W>
__device__ __forceinline__ bf16x8 sk_frag(const unsigned char* img, int kbase, int c0, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int r = kbase + 8 * g + q;
  typedef __attribute__((address_space(3))) sk_v4s lds_v4s;
  const sk_v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(img + sk_off<W>(r, c0 + 4 * p)));
  const sk_v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(img + sk_off<W>(r + 4, c0 + 4 * p)));
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

__global__ __launch_bounds__(SK_THREADS) void gemm_shortk_kernel(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) unsigned char sk_smem[];
  unsigned char* As = sk_smem;                                  // [SK_KMAX][SK_MMAX] bf16
  unsigned char* Bs = sk_smem + SK_KMAX * SK_MMAX * 2;          // [2][SK_KMAX][SK_NS] bf16
  constexpr int BSZ = SK_KMAX * SK_NS * 2;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int K = g.K, M = g.M, N = g.N;
  const int KP = (K + 31) & ~31;                                // MFMA k steps of 32 (rows [K, KP) zero)
  // A image: row k, columns 4 (t % 64) ... ; 8 rows per pass
  for (int k = t >> 6; k < KP; k += SK_THREADS / 64) {
    const int m = 4 * (t & 63);
    f32x4 x = f32x4{0.f, 0.f, 0.f, 0.f};
    if (k < K && m < M) x = *reinterpret_cast<const f32x4*>(g.a + (size_t)k * g.lda + m);
    *reinterpret_cast<uint2*>(As + sk_off<SK_MMAX>(k, m)) = uint2{pack_bf16x2(x[0], x[1]), pack_bf16x2(x[2], x[3])};
  }
  // B strip rows: thread -> column quad t % 16, rows t / 16 + 32 i
  constexpr int NB = SK_KMAX / (SK_THREADS / 16);               // 5 row passes
  const int cq = 4 * (t & 15), r0 = t >> 4;
  f32x4 pf[NB];
  auto load_strip = [&](int s) {
    const int n = s * SK_NS + cq;
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int k = r0 + 32 * i;
      pf[i] = (k < K && n < N) ? *reinterpret_cast<const f32x4*>(g.b + (size_t)k * g.ldb + n) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto stage_strip = [&](unsigned char* img) {
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int k = r0 + 32 * i;
      if (k < KP)
        *reinterpret_cast<uint2*>(img + sk_off<SK_NS>(k, cq)) = uint2{pack_bf16x2(pf[i][0], pf[i][1]),
                                                                      pack_bf16x2(pf[i][2], pf[i][3])};
    }
  };
  const int nstrips = (N + SK_NS - 1) / SK_NS;
  // output store policy (g_gemm_shortk_store, host-checked 32-bit offsets): 0 plain, 1 non-temporal, 2 write-through
  const int pol = g.wt;
  const __amdgpu_buffer_rsrc_t crs = __builtin_amdgcn_make_buffer_rsrc(g.c, 0, 0x7FFFFFFF, 0x00020000);
  int s = blockIdx.x;
  if (s < nstrips) load_strip(s);
  for (int it = 0; s < nstrips; s += gridDim.x, ++it) {
    unsigned char* img = Bs + (it & 1) * BSZ;    // last read two strips ago, before the previous barrier
    stage_strip(img);
    __syncthreads();
    if (s + (int)gridDim.x < nstrips) load_strip(s + gridDim.x);   // in flight through the MFMAs and stores
    // wave w: rows [32 w, 32 w + 32) x the strip's 64 columns
    f32x4 acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kb = 0; kb < KP; kb += 32) {
      bf16x8 af[2], bfr[4];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = sk_frag<SK_MMAX>(As, kb, 32 * w + 16 * i, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = sk_frag<SK_NS>(img, kb, 16 * j, lane);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = s * SK_NS + 16 * j + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = 32 * w + 16 * i + 4 * (lane >> 4) + r;
          if (m < M && n < N) {
            if (pol == 0) g.c[(size_t)m * g.ldc + n] = acc[i][j][r];
            else if (pol == 1) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[i][j][r]), crs,
                                                                     (int)(((size_t)m * g.ldc + n) * 4), 0, 2);
            else __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[i][j][r]), crs,
                                                       (int)(((size_t)m * g.ldc + n) * 4), 0, 16);
          }
        }
      }
  }
}

// The same product with Adam applied to the outputs (a weight gradient inside an optimizer's flat gradient buffer,
// g.adam_* at the same offset as for gemm_adam_kernel), launched right before that optimizer's launch, which skips
// the block: the 141 MB dW0 of the wide table is neither written (unless g.adam_grad) nor re-read.  Per strip the
// kernel now moves 3 x 2 x 32 KB of parameters / moments per 256 x 32 block against 19 KB of B, so it is built for
// bytes in flight: 32-column strips, the accumulators as C^T blocks (operands swapped, so a lane's 4 values are 4
// consecutive columns of one row: float4 parameters / moments), and the NEXT strip's parameters, moments and B
// rows requested before this strip's MFMAs -- two register sets, alternating strip by strip.
constexpr int SKA_NS = 32;
__global__ __launch_bounds__(SK_THREADS) void gemm_shortk_adam_kernel(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) unsigned char ska_smem[];
  unsigned char* As = ska_smem;                                 // [SK_KMAX][SK_MMAX] bf16
  unsigned char* Bs = ska_smem + SK_KMAX * SK_MMAX * 2;         // [2][SK_KMAX][SKA_NS] bf16
  constexpr int BSZ = SK_KMAX * SKA_NS * 2;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int K = g.K, M = g.M, N = g.N;
  const int KP = (K + 31) & ~31;
  for (int k = t >> 6; k < KP; k += SK_THREADS / 64) {
    const int m = 4 * (t & 63);
    f32x4 x = f32x4{0.f, 0.f, 0.f, 0.f};
    if (k < K && m < M) x = *reinterpret_cast<const f32x4*>(g.a + (size_t)k * g.lda + m);
    *reinterpret_cast<uint2*>(As + sk_off<SK_MMAX>(k, m)) = uint2{pack_bf16x2(x[0], x[1]), pack_bf16x2(x[2], x[3])};
  }
  const float tt = g.adam_step[0];   // adam_cs_body's bias corrections, from the same step counter
  const float sz = g.adam_lr / (1.f - powf(g.adam_b1, tt));
  const float bc2s = sqrtf(1.f - powf(g.adam_b2, tt));
  // B strip rows: thread -> column quad t % 8, rows t / 8 + 64 i
  constexpr int RPP = SK_THREADS / (SKA_NS / 4), NB = (SK_KMAX + RPP - 1) / RPP;
  const int cq = 4 * (t & (SKA_NS / 4 - 1)), r0 = t / (SKA_NS / 4);
  // wave w: rows [32 w, 32 w + 32) x 32 columns = 2 x 2 blocks; element (i, j) of a lane: row 32 w + 16 i + lane % 16,
  // columns 16 j + 4 (lane / 16) ... + 3
  struct Set {
    f32x4 x[NB];          // B strip rows
    f32x4 p[2][2], m[2][2], v[2][2];
  };
  auto fetch = [&](Set& st, int s) {
    const int nb = s * SKA_NS;
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int k = r0 + RPP * i;
      st.x[i] = (k < K && nb + cq < N) ? *reinterpret_cast<const f32x4*>(g.b + (size_t)k * g.ldb + nb + cq)
                                       : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int m = min(32 * w + 16 * i + (lane & 15), M - 1);
        const int n = min(nb + 16 * j + 4 * (lane >> 4), N - 4);
        const size_t e = (size_t)m * g.ldc + n;
        st.p[i][j] = *reinterpret_cast<const f32x4*>(g.adam_p + e);
        st.m[i][j] = *reinterpret_cast<const f32x4*>(g.adam_m + e);
        st.v[i][j] = *reinterpret_cast<const f32x4*>(g.adam_v + e);
      }
  };
  // one strip: stage its B rows, request the next strip into the other set, multiply, update, store
  auto strip = [&](Set& cur, Set& nxt, int s, int it, int nstrips) {
    unsigned char* img = Bs + (it & 1) * BSZ;
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int k = r0 + RPP * i;
      if (k < KP)
        *reinterpret_cast<uint2*>(img + sk_off<SKA_NS>(k, cq)) = uint2{pack_bf16x2(cur.x[i][0], cur.x[i][1]),
                                                                        pack_bf16x2(cur.x[i][2], cur.x[i][3])};
    }
    __syncthreads();
    if (s + (int)gridDim.x < nstrips) fetch(nxt, s + gridDim.x);
    f32x4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kb = 0; kb < KP; kb += 32) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = sk_frag<SK_MMAX>(As, kb, 32 * w + 16 * i, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) bfr[j] = sk_frag<SKA_NS>(img, kb, 16 * j, lane);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int m = 32 * w + 16 * i + (lane & 15);
        const int n = s * SKA_NS + 16 * j + 4 * (lane >> 4);
        if (m >= M || n >= N) continue;      // (N % 4 == 0: a float4 is all in or all out)
        const size_t e = (size_t)m * g.ldc + n;
        f32x4 p4 = cur.p[i][j], m4 = cur.m[i][j], v4 = cur.v[i][j];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float pe = p4[r], me = m4[r], ve = v4[r];
          adam_elem(acc[i][j][r], pe, me, ve, g.adam_b1, g.adam_b2, g.adam_eps, g.adam_wd, sz, bc2s);
          p4[r] = pe;
          m4[r] = me;
          v4[r] = ve;
        }
        *reinterpret_cast<f32x4*>(g.adam_p + e) = p4;
        *reinterpret_cast<f32x4*>(g.adam_m + e) = m4;
        *reinterpret_cast<f32x4*>(g.adam_v + e) = v4;
        if (g.adam_grad) *reinterpret_cast<f32x4*>(g.c + e) = acc[i][j];
      }
  };
  const int nstrips = (N + SKA_NS - 1) / SKA_NS;
  Set sa, sb;
  int s = blockIdx.x, it = 0;
  if (s < nstrips) fetch(sa, s);
  while (s < nstrips) {     // two strips per trip: the register sets keep static names
    strip(sa, sb, s, it++, nstrips);
    s += gridDim.x;
    if (s >= nstrips) break;
    strip(sb, sa, s, it++, nstrips);
    s += gridDim.x;
  }
}

// the shapes gemm_shortk_kernel takes (everything else: the tile GEMM)
static bool gemm_shortk_ok(const GemmArgs& g) {
  const auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  return g_gemm_shortk && g.ta && !g.tb && !g.f32 && !g.bin && !g.c16 && g.nclient <= 1 && g.splitk <= 1 &&
         g.epi == EPI_NONE && g.alpha == 1.f && g.beta == 0.f && !g.bias && !g.oh_w && !g.bn_part && !g.chain &&
         !g.head_a && !g.adam_p && g.M <= SK_MMAX && g.M % 4 == 0 && g.K >= 1 && g.K <= SK_KMAX && g.N % 4 == 0 &&
         g.N >= g_gemm_shortk_min_n && g.lda % 4 == 0 && g.ldb % 4 == 0 && al16(g.a) && al16(g.b) && g.N <= g.ldb &&
         g.M <= g.lda && g.N <= g.ldc;
}

int g_gemm_shortk_store = 2;   // write-through: measured best of plain / nt / sc1 (profiles/wide_r6.md)

static void launch_gemm_shortk(GemmArgs g, hipStream_t stream) {
  g.wt = ((int64_t)g.M * g.ldc * 4 < (int64_t)INT32_MAX) ? g_gemm_shortk_store : 0;   // (buffer stores: 32-bit offsets)
  static const size_t lds = (size_t)SK_KMAX * (SK_MMAX + 2 * SK_NS) * 2;   // 120 KB: one workgroup per CU
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_shortk_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_shortk_adam_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  int dev = 0, cus = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int nstrips = (g.N + (g.adam_p ? SKA_NS : SK_NS) - 1) / (g.adam_p ? SKA_NS : SK_NS);
  const dim3 grid(std::min(nstrips, std::max(cus, 1)));
  if (g.adam_p) hipLaunchKernelGGL(gemm_shortk_adam_kernel, grid, dim3(SK_THREADS), lds, stream, g);
  else hipLaunchKernelGGL(gemm_shortk_kernel, grid, dim3(SK_THREADS), lds, stream, g);
}

bool launch_gemm_shortk_adam(GemmArgs g, hipStream_t stream) {
  check_slab(g);
  (void)gemm_prepare(g);
  if (!g.adam_p || !g.adam_m || !g.adam_v || !g.adam_step) return false;
  GemmArgs q = g;
  q.adam_p = nullptr;           // (the shape check excludes Adam GEMMs taken by the generic dispatch)
  if (!gemm_shortk_ok(q)) return false;
  launch_gemm_shortk(g, stream);
  return true;
}

static void gemm_dispatch(const GemmArgs& g, dim3 grid_, hipStream_t stream) {
  if (gemm_shortk_ok(g)) return launch_gemm_shortk(g, stream);
  const dim3 grid(grid_.x, grid_.y, grid_.z * g.nclient);   // split-K slices x clients
  if (g.nclient > 1) gemm_dispatch_t<true>(g, grid, dim3(NT), gemm_smem_bytes(g), stream);
  else gemm_dispatch_t<false>(g, grid, dim3(NT), gemm_smem_bytes(g), stream);
}

static void gemm_epilogue_launch(const GemmArgs& g, hipStream_t stream) {
  if (g.chain) {     // the chained tail GEMM rides on this GEMM's reduction launch (or follows it)
    GemmArgs h = g;
    GemmArgs t = *g.chain;
    h.chain = nullptr;
    t.cstride = g.cstride;      // (the tail was never prepared: it shares the head's client layout)
    t.seed_step = g.seed_step;
    t.nclient = g.nclient;
    // float4 loads from t.b + jc * t.ldb + k: the row stride and the base must keep them 16-B aligned
    t.chain_co = g_chain_coalesced && (g.N % 4 == 0) && (t.ldb % 4 == 0) &&
                 ((reinterpret_cast<uintptr_t>(t.b) & 15) == 0) && !t.ach_out;
    const int nb = (t.N + CH_COLS - 1) / CH_COLS;
    const bool mk = g.epi == EPI_MASK && t.epi == EPI_MASK && t.head_a == nullptr && t.bias == nullptr && t.alpha == 1.f;
    // prefetched tail weights (K = 256) where the grid stays resident at 194 VGPRs (<= 512 workgroups): one row
    // per workgroup, or two when one row each would overflow (g_chain_rows)
    const bool can_pre = g.nclient <= 1 && g.N == 256 && !t.chain_co && g_chain_pre > 0;
    const bool big = (int64_t)g.M * nb > 512;
    const int rows = (can_pre && big && g_chain_rows == 2 && (int64_t)((g.M + 1) / 2) * nb <= 512) ? 2 : 1;
    const bool pre = can_pre && (rows == 2 || !big || g_chain_pre == 2);
    const dim3 grid((g.M + rows - 1) / rows, nb, g.nclient), block(256);
#define FEDTGAN_CHAIN_K(S, MK)                                                                                       \
  do {                                                                                                               \
    if (g.xcd_cl) hipLaunchKernelGGL((chain_epilogue_kernel<S, MK, true>), grid, block, 0, stream, h, t);            \
    else if (rows == 2) hipLaunchKernelGGL((chain_epilogue_kernel<S, MK, false, true, 2>), grid, block, 0, stream, h, t); \
    else if (pre) hipLaunchKernelGGL((chain_epilogue_kernel<S, MK, false, true>), grid, block, 0, stream, h, t);     \
    else hipLaunchKernelGGL((chain_epilogue_kernel<S, MK, false>), grid, block, 0, stream, h, t);                    \
  } while (0)
#define FEDTGAN_CHAIN_ACH(S)                                                                                         \
  do {                                                                                                               \
    if (rows == 2) hipLaunchKernelGGL((chain_epilogue_kernel<S, false, false, true, 2, true>), grid, block, 0, stream, h, t); \
    else if (pre) hipLaunchKernelGGL((chain_epilogue_kernel<S, false, false, true, 1, true>), grid, block, 0, stream, h, t); \
    else hipLaunchKernelGGL((chain_epilogue_kernel<S, false, false, false, 1, true>), grid, block, 0, stream, h, t);       \
  } while (0)
#define FEDTGAN_CHAIN(S)              \
  do {                                \
    if (t.ach_out) FEDTGAN_CHAIN_ACH(S); \
    else if (mk) FEDTGAN_CHAIN_K(S, true);  \
    else FEDTGAN_CHAIN_K(S, false);    \
  } while (0)
    if (t.ach_out && (g.nclient > 1 || g.xcd_cl || !t.head_a || mk))
      throw std::runtime_error("gemm: the fused A-chain needs one client and a chain tail with a head seed");
    if (g.splitk <= 1 || g.red_inl) FEDTGAN_CHAIN(0);
    else if (g.splitk <= 8) FEDTGAN_CHAIN(8);
    else if (g.splitk <= 16) FEDTGAN_CHAIN(16);
    else if (g.splitk <= 32) FEDTGAN_CHAIN(32);
    else FEDTGAN_CHAIN(64);
#undef FEDTGAN_CHAIN
#undef FEDTGAN_CHAIN_ACH
#undef FEDTGAN_CHAIN_K
    return;
  }
  if (g.splitk <= 1 || g.red_inl) return;
  const size_t total = (size_t)g.M * g.N;
  int blocks = (int)std::min<size_t>((total + 255) / 256, 2048);
  const dim3 grid(blocks, 1, g.nclient);
  if (g.splitk <= 8) hipLaunchKernelGGL((g.xcd_cl ? gemm_splitk_epilogue<8, true> : gemm_splitk_epilogue<8, false>), grid, dim3(256), 0, stream, g);
  else if (g.splitk <= 16) hipLaunchKernelGGL((g.xcd_cl ? gemm_splitk_epilogue<16, true> : gemm_splitk_epilogue<16, false>), grid, dim3(256), 0, stream, g);
  else if (g.splitk <= 32) hipLaunchKernelGGL((g.xcd_cl ? gemm_splitk_epilogue<32, true> : gemm_splitk_epilogue<32, false>), grid, dim3(256), 0, stream, g);
  else hipLaunchKernelGGL((g.xcd_cl ? gemm_splitk_epilogue<64, true> : gemm_splitk_epilogue<64, false>), grid, dim3(256), 0, stream, g);
}

void launch_gemm(GemmArgs g, hipStream_t stream) {
  if (g.M <= 0 || g.N <= 0) return;
  check_slab(g);
  if (g.chain) check_slab(*g.chain);
  const dim3 grid = gemm_prepare(g);
  gemm_dispatch(g, grid, stream);
  gemm_epilogue_launch(g, stream);
}

// The instantiated pairs: a weight gradient (op(A) = A^T, 64- or 32-tile) beside the next backward
// product (NT or NN, 32-tile), bf16 -- every pair the training step issues.  Anything else runs as
// two launches.
template <bool V1, bool V2>
static bool gemm_pair_vec(const GemmArgs& g1, Grid3 a, const GemmArgs& g2, Grid3 b, hipStream_t stream) {
  const dim3 grid(a.x * a.y * a.z + b.x * b.y * b.z, 1, g1.nclient), block(NT);
#define FEDTGAN_PAIR_K(T1, TA2, TB2, EK2, BT)                                                                     \
  hipLaunchKernelGGL((gemm_pair_kernel<GemmShape<true, false, V1, T1>, GemmShape<TA2, TB2, V2, 32, EK2>, BT>), grid, \
                     block, 0, stream, g1, g2, a, b)
#define FEDTGAN_PAIR(T1, TA2, TB2)                                         \
  do {                                                                     \
    if (g1.nclient > 1) {                                                  \
      FEDTGAN_PAIR_K(T1, TA2, TB2, 0, true);                               \
    } else if constexpr ((T1) <= 64) {                                     \
      const int ek2 = gemm_ek(g2);                                         \
      if (ek2 == 2) FEDTGAN_PAIR_K(T1, TA2, TB2, 2, false);                \
      else if (ek2 == 3) FEDTGAN_PAIR_K(T1, TA2, TB2, 3, false);           \
      else if (ek2 == 1) FEDTGAN_PAIR_K(T1, TA2, TB2, 1, false);           \
      else FEDTGAN_PAIR_K(T1, TA2, TB2, 0, false);                         \
    } else {                                                               \
      FEDTGAN_PAIR_K(T1, TA2, TB2, 0, false);                              \
    }                                                                      \
  } while (0)
  if (!(g1.ta && !g1.tb) || g2.ta || g2.tile != 32) return false;
  if (g1.tile == 64) {
    if (g2.tb) FEDTGAN_PAIR(64, false, true); else FEDTGAN_PAIR(64, false, false);
  } else if (g1.tile == 32) {
    if (g2.tb) FEDTGAN_PAIR(32, false, true); else FEDTGAN_PAIR(32, false, false);
  } else if (g1.tile == 128) {
    if (g2.tb) FEDTGAN_PAIR(128, false, true); else FEDTGAN_PAIR(128, false, false);
  } else {
    return false;
  }
#undef FEDTGAN_PAIR
#undef FEDTGAN_PAIR_K
  return true;
}

void launch_gemm_pair(GemmArgs g1, GemmArgs g2, hipStream_t stream) {
  if (g1.M <= 0 || g1.N <= 0) return launch_gemm(g2, stream);
  if (g2.M <= 0 || g2.N <= 0) return launch_gemm(g1, stream);
  check_slab(g1);
  check_slab(g2);
  if (g1.chain) check_slab(*g1.chain);
  if (g2.chain) check_slab(*g2.chain);
  const dim3 d1 = gemm_prepare(g1), d2 = gemm_prepare(g2);
  const Grid3 a{(int)d1.x, (int)d1.y, (int)d1.z}, b{(int)d2.x, (int)d2.y, (int)d2.z};
  bool fused = false;
  const int64_t pair_wg = (int64_t)a.x * a.y * a.z + (int64_t)b.x * b.y * b.z;
  if (!g1.f32 && !g2.f32 && !g1.bin && !g2.bin && !g1.c16 && !g2.c16 && g_gemm_pairs &&
      (g_gemm_pair_max_wg <= 0 || pair_wg <= g_gemm_pair_max_wg)) {
    if (g1.vec && g2.vec) fused = gemm_pair_vec<true, true>(g1, a, g2, b, stream);
    else if (g1.vec) fused = gemm_pair_vec<true, false>(g1, a, g2, b, stream);
    else if (g2.vec) fused = gemm_pair_vec<false, true>(g1, a, g2, b, stream);
    else fused = gemm_pair_vec<false, false>(g1, a, g2, b, stream);
  }
  if (!fused) {
    gemm_dispatch(g1, d1, stream);
    gemm_dispatch(g2, d2, stream);
  }
  gemm_epilogue_launch(g1, stream);
  gemm_epilogue_launch(g2, stream);
}

// BN backward workgroups first (the narrow latency-bound part starts at once; g_bnb_first = 0: after the GEMM's
// tiles), COLS columns per BN workgroup (g_bnb_cols: 4 or 8)
int g_bnb_first = 1;
int g_bnb_cols = 4;

template <bool V, int T, int COLS, int MAXR>
__global__ __launch_bounds__(NT) void gemm_bnbwd_kernel(GemmArgs g, Grid3 gd, BnBwdArgs bn, int nbn, int first) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * Cfg<false, T, T>::STAGE];
  const int nt = gd.x * gd.y * gd.z;
  const int b = (int)blockIdx.x;
  const bool is_bn = first ? b < nbn : b >= nt;
  if (is_bn) {
    bn_bwd_block<COLS, MAXR, NT>(bn, first ? b : b - nt, reinterpret_cast<float*>(smem));
    return;
  }
  const int t = first ? b - nbn : b;
  gemm_tile<true, false, false, V, T, T>(g, t % gd.x, (t / gd.x) % gd.y, t / (gd.x * gd.y), gd.x, gd.y, gd.z, smem);
}

bool launch_gemm_bnbwd(GemmArgs g, const BnBwdArgs& b, hipStream_t stream) {
  if (g.M <= 0 || g.N <= 0 || b.rows <= 0 || b.cols <= 0) return false;
  if (client_batch().k > 1 || g.f32 || g.bin || g.c16 || !g.ta || g.tb || g.chain || g.bn_part) return false;
  const int cols = g_bnb_cols == 8 ? 8 : 4;
  const int groups = NT / cols;
  const int maxr = (b.rows + groups - 1) / groups;
  if (maxr > 16) return false;
  static_assert(3 * (NT / 64) * 8 * 4 <= 2 * Cfg<false, 32, 32>::STAGE, "BN scratch fits the GEMM stage buffer");
  check_slab(g);
  const dim3 d = gemm_prepare(g);
  if (g.tile != 32 && g.tile != 64) return false;
  const Grid3 gd{(int)d.x, (int)d.y, (int)d.z};
  const int nbn = (b.cols + cols - 1) / cols;
  const dim3 grid(nbn + gd.x * gd.y * gd.z), block(NT);
  const int first = g_bnb_first;
#define FEDTGAN_BNB(V, T, C, R) \
  hipLaunchKernelGGL((gemm_bnbwd_kernel<V, T, C, R>), grid, block, 0, stream, g, gd, b, nbn, first)
#define FEDTGAN_BNB_R(V, T, C)              \
  if (maxr <= 4) FEDTGAN_BNB(V, T, C, 4);    \
  else if (maxr <= 8) FEDTGAN_BNB(V, T, C, 8); \
  else FEDTGAN_BNB(V, T, C, 16);
#define FEDTGAN_BNB_C(V, T) \
  if (cols == 8) { FEDTGAN_BNB_R(V, T, 8) } else { FEDTGAN_BNB_R(V, T, 4) }
  if (g.vec) {
    if (g.tile == 32) { FEDTGAN_BNB_C(true, 32) } else { FEDTGAN_BNB_C(true, 64) }
  } else {
    if (g.tile == 32) { FEDTGAN_BNB_C(false, 32) } else { FEDTGAN_BNB_C(false, 64) }
  }
#undef FEDTGAN_BNB_C
#undef FEDTGAN_BNB_R
#undef FEDTGAN_BNB
  gemm_epilogue_launch(g, stream);
  return true;
}

bool launch_gemm_adam(GemmArgs g, float* p, const float* gr, float* m, float* v, const float* step, int64_t n,
                      float lr, float b1, float b2, float eps, float wd, uint64_t* rng_ctr_bump,
                      const AdamColsum& cs_in, hipStream_t stream) {
  if (g.M <= 0 || g.N <= 0 || g.f32 || g.bin || g.c16 || !g.ta || g.tb || n % 4 != 0) return false;
  check_slab(g);
  if (client_batch().k > 1) {
    check_slabs("adam operand", p, gr, m, v, step, rng_ctr_bump);
    check_slab(cs_in);
  }
  const dim3 d = gemm_prepare(g);
  if (g.splitk != 1 || (g.tile != 32 && g.tile != 64)) return false;
  g.adam_p = p + (g.c - gr);
  g.adam_m = m + (g.c - gr);
  g.adam_v = v + (g.c - gr);
  g.adam_step = step;
  g.adam_lr = lr;
  g.adam_b1 = b1;
  g.adam_b2 = b2;
  g.adam_eps = eps;
  g.adam_wd = wd;
  AdamColsum cs = cs_in;
  cs.n_jobs = std::min(cs.n_jobs, 8);
  cs.blk_start[0] = 0;
  for (int k = 0; k < cs.n_jobs; ++k) cs.blk_start[k + 1] = cs.blk_start[k] + (cs.jobs[k].cols + ACS_COLS - 1) / ACS_COLS;
  const int64_t n4 = n / 4;
  const int U = adam_unroll(n4, g.nclient);
  const int blocks = (int)std::min<int64_t>((n4 + 256 * U - 1) / (256 * U), g_adam_max_blocks);
  const Grid3 gd{(int)d.x, (int)d.y, (int)d.z};
  const int grid = gd.x * gd.y * gd.z + std::max(blocks, 1) + cs.blk_start[cs.n_jobs];
#define FEDTGAN_GEMM_ADAM_K(V, T, AUX, B, UU)                                                                       \
  hipLaunchKernelGGL((gemm_adam_kernel<V, T, AUX, B, UU>), dim3(grid, 1, g.nclient), dim3(NT), 0, stream, g, gd, p, gr, \
                     m, v, step, n4, lr, b1, b2, eps, wd, rng_ctr_bump, cs)
#define FEDTGAN_GEMM_ADAM(V, T, AUX)                                      \
  do {                                                                   \
    if (g.nclient > 1) {                                                 \
      if (U == ADAM_U) FEDTGAN_GEMM_ADAM_K(V, T, AUX, true, ADAM_U);     \
      else FEDTGAN_GEMM_ADAM_K(V, T, AUX, true, 1);                      \
    } else {                                                             \
      if (U == ADAM_U) FEDTGAN_GEMM_ADAM_K(V, T, AUX, false, ADAM_U);    \
      else FEDTGAN_GEMM_ADAM_K(V, T, AUX, false, 1);                     \
    }                                                                    \
  } while (0)
#define FEDTGAN_GEMM_ADAM_T(V, T)                                 \
  if (g_adam_store == 2) FEDTGAN_GEMM_ADAM(V, T, 2);              \
  else if (g_adam_store == 16) FEDTGAN_GEMM_ADAM(V, T, 16);       \
  else FEDTGAN_GEMM_ADAM(V, T, 0);
  if (g.vec) {
    if (g.tile == 32) { FEDTGAN_GEMM_ADAM_T(true, 32) } else { FEDTGAN_GEMM_ADAM_T(true, 64) }
  } else {
    if (g.tile == 32) { FEDTGAN_GEMM_ADAM_T(false, 32) } else { FEDTGAN_GEMM_ADAM_T(false, 64) }
  }
#undef FEDTGAN_GEMM_ADAM_T
#undef FEDTGAN_GEMM_ADAM
#undef FEDTGAN_GEMM_ADAM_K
  return true;
}

}  // namespace fedtgan
