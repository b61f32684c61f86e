// Generator layer in training: Linear -> BatchNorm(train) -> ReLU as ONE launch, by column ownership
// (the reference's Residual block, `Server/dtds/synthesizers/ctgan.py:33-44`).
//
// The two-launch path (gemm.hip tile GEMM into a scratch matrix, then bn_relu_train / bn_relu_apply)
// needs the whole batch's statistics before any row can be normalised, so the GEMM output makes a
// round trip through memory and a second launch reduces it again.  Here one workgroup owns 16 output
// columns of ONE batch (all of that batch's rows):
//   1. half the workgroup stages its 16 weight rows into LDS as bf16 once, the other half resolves every
//      row's one-hot column (the two dependent index loads) into LDS;
//   2. its 16 waves walk the batch's 16-row blocks: A fragments straight from global memory (fp32,
//      rounded to bf16 in registers -- the same operand rounding as the tile GEMM), B fragments from
//      LDS, v_mfma_f32_16x16x32_bf16 with fp32 accumulation; + bias + the one-hot block's gathered
//      weight; the pre-BN values stay in LDS ([rows][16] fp32), never in HBM;
//   3. two-pass batch statistics from LDS (mean, then centred squares), mean / invstd written out;
//   4. every thread normalises its elements: nhat and relu(gamma nhat + beta) straight to H.
// With two batches in one launch (the paired D/G step, groups = 2) the running statistics must see
// batch 0 before batch 1 (the reference's two forward passes): each batch's workgroup hands its
// (mean, biased var) to a small buffer with write-through (sc1) stores, takes a ticket on the column
// block's counter, and the second arrival applies both updates in order and re-zeroes the counter
// (the hand-off of gemm.hip's in-launch split-K reduction: nothing ever waits on another workgroup).
// The grid is cols/16 x groups x clients workgroups (client = blockIdx.z, see launch.h ClientBatch).
#include "launch.h"

#include "common.h"

namespace fedtgan {

typedef __attribute__((ext_vector_type(8))) short co_bf16x8;
typedef __attribute__((ext_vector_type(4))) float co_f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned co_u32x4;

constexpr int CO_THREADS = 1024, CO_WAVES = CO_THREADS / 64, CO_COLS = 16;
constexpr int CO_LDY = 20;   // LDS row stride of the pre-BN block (floats): the 4 row groups of a
                             // wave's accumulator store land on distinct banks

__device__ __forceinline__ co_bf16x8 co_pack8(const float (&v)[8]) {
  co_u32x4 u{pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7])};
  return __builtin_bit_cast(co_bf16x8, u);
}

// 8 consecutive k values of one row (zero beyond K); VEC: 16-B aligned row starts (two float4)
template <bool VEC>
__device__ __forceinline__ void co_load8(const float* __restrict__ row, int k, int K, float (&v)[8]) {
  if (VEC && k + 8 <= K) {
    const co_f32x4 a = *reinterpret_cast<const co_f32x4*>(row + k);
    const co_f32x4 b = *reinterpret_cast<const co_f32x4*>(row + k + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] = a[e];
      v[4 + e] = b[e];
    }
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = k + e < K ? row[min(k + e, K - 1)] : 0.f;
  }
}

template <bool VEC>
__global__ __launch_bounds__(CO_THREADS) void linear_bn_relu_colown_kernel(ColOwnArgs g) {
  extern __shared__ __align__(16) unsigned char co_smem[];
  const int64_t co = (int64_t)blockIdx.z * g.cstride;
  const float* __restrict__ x = cptr(g.x, co);
  const float* __restrict__ w = cptr(g.w, co);
  const float* bias = cptr(g.bias, co);
  const float* oh_w = cptr(g.oh_w, co);
  const int* oh_col = cptr(g.oh_col, co);
  const int* oh_opt = cptr(g.oh_opt, co);
  const int* oh_off = cptr(g.oh_off, co);
  float* out = cptr(g.out, co);
  float* nhat = cptr(g.nhat, co);

  const int K = g.K, N = g.N, rpg = g.rpg;
  const int KP = (K + 31) / 32 * 32 + 8;   // LDS row stride of the weight slice (bf16)
  uint16_t* ws = reinterpret_cast<uint16_t*>(co_smem);
  float* ys = reinterpret_cast<float*>(co_smem + (size_t)CO_COLS * KP * 2);
  float* red = ys + (size_t)rpg * CO_LDY;             // [CO_THREADS / 16][16] partial sums
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int c0 = blockIdx.x * CO_COLS, b = blockIdx.y;
  const int rbase = b * rpg;                          // first row of this batch

  int* gidx = reinterpret_cast<int*>(red + 2 * CO_THREADS + 4);   // [rpg] one-hot column of each row

  // 1. in parallel: the first half of the workgroup resolves every row's one-hot column (two dependent
  //    loads) into LDS, the second half stages the weight slice W[c0 .. c0+15][0 .. K) into LDS as bf16
  //    (zero-padded to KP, zero rows past N; consecutive threads read consecutive memory: along k for
  //    [out, in] rows, along n for input-major storage)
  constexpr int HALF = CO_THREADS / 2;
  if (g.dbg & 2) {
    // (probe: no staging)
  } else if (t < HALF) {
    if (oh_w)
      for (int r = t; r < rpg; r += HALF) gidx[r] = oh_off[oh_col[rbase + r]] + oh_opt[rbase + r];
  } else {
    // SU elements per thread in flight: every load of a pass is issued before the first LDS store
    // (a load -> convert -> store loop would pay one memory round trip per element)
    constexpr int SU = 16;
    const int total = CO_COLS * KP;
    const bool im = g.w_sn == 1;
    for (int e0 = t - HALF; e0 < total; e0 += SU * HALF) {
      float v[SU];
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const int e = e0 + u * HALF;
        const int n = im ? e % CO_COLS : e / KP, k = im ? e / CO_COLS : e % KP;
        const bool ok = e < total && c0 + n < N && k < K;
        v[u] = ok ? w[(size_t)min(c0 + n, N - 1) * g.w_sn + (size_t)min(k, K - 1) * g.w_sk] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const int e = e0 + u * HALF;
        const int n = im ? e % CO_COLS : e / KP, k = im ? e / CO_COLS : e % KP;
        if (e < total) ws[n * KP + k] = f2bf(v[u]);
      }
    }
  }
  __syncthreads();

  // 2. 16-row blocks of this batch, round-robin over the waves; a block's A loads and its rows' one-hot
  //    gathers are issued together (one memory round trip per K chunk)
  const int nrb = (rpg + 15) / 16;
  const int n_l = lane & 15, kq = 8 * (lane >> 4);
  const int n_g = min(c0 + n_l, N - 1);
  const float bv = bias ? bias[n_g] : 0.f;
  for (int rb = wv; rb < nrb; rb += CO_WAVES) {
    if (g.dbg & 1) {   // (probe: no GEMM)
      for (int i = 0; i < 4; ++i) {
        const int r = 16 * rb + 4 * (lane >> 4) + i;
        if (r < rpg) ys[r * CO_LDY + n_l] = bv + (float)r;
      }
      continue;
    }
    const int lr = min(16 * rb + n_l, rpg - 1);       // this lane's A row (fragment row = lane & 15)
    const float* xr = x + (size_t)(rbase + lr) * g.ldx;
    float gv[4] = {0.f, 0.f, 0.f, 0.f};
    if (oh_w) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = min(16 * rb + 4 * (lane >> 4) + i, rpg - 1);
        gv[i] = oh_w[(size_t)n_g * g.oh_sn + (size_t)gidx[r] * g.oh_sc];
      }
    }
    co_f32x4 acc{0.f, 0.f, 0.f, 0.f};
    constexpr int KU = 8;   // k-steps of 32 whose loads are issued together
    for (int k0 = 0; k0 < K; k0 += 32 * KU) {
      float av[KU][8];
#pragma unroll
      for (int u = 0; u < KU; ++u) co_load8<VEC>(xr, k0 + 32 * u + kq, K, av[u]);
#pragma unroll
      for (int u = 0; u < KU; ++u) {
        const int k = k0 + 32 * u;
        if (k < K) {
          const co_bf16x8 af = co_pack8(av[u]);
          const co_bf16x8 bf = *reinterpret_cast<const co_bf16x8*>(&ws[n_l * KP + k + kq]);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf, acc, 0, 0, 0);
        }
      }
    }
    // acc[i] = row 16 rb + 4 (lane >> 4) + i, column c0 + (lane & 15)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = 16 * rb + 4 * (lane >> 4) + i;
      if (r < rpg) {
        ys[r * CO_LDY + n_l] = acc[i] + bv + gv[i];
      }
    }
  }
  __syncthreads();

  // 3. batch statistics of the 16 columns, two passes over the LDS block
  const int col = t & 15, part = t >> 4;   // CO_THREADS / 16 row slices per column
  float s = 0.f;
  for (int r = part; r < rpg; r += CO_THREADS / CO_COLS) s += ys[r * CO_LDY + col];
  red[part * CO_COLS + col] = s;
  __syncthreads();
  float mu = 0.f;
#pragma unroll 16
  for (int p = 0; p < CO_THREADS / CO_COLS; ++p) mu += red[p * CO_COLS + col];
  mu /= (float)rpg;
  __syncthreads();
  float q = 0.f;
  for (int r = part; r < rpg; r += CO_THREADS / CO_COLS) {
    const float d = ys[r * CO_LDY + col] - mu;
    q += d * d;
  }
  red[part * CO_COLS + col] = q;
  __syncthreads();
  float m2 = 0.f;
#pragma unroll 16
  for (int p = 0; p < CO_THREADS / CO_COLS; ++p) m2 += red[p * CO_COLS + col];
  const float var = m2 / (float)rpg;   // biased batch variance
  const float is = rsqrtf(var + g.eps);
  const int c = c0 + col;
  const bool okc = c < N;

  // running statistics (batch after batch, in row order) and the per-batch outputs
  if (t < CO_COLS && okc) {
    float* mean = cptr(g.mean, co);
    float* invstd = cptr(g.invstd, co);
    mean[(size_t)b * N + c] = mu;
    invstd[(size_t)b * N + c] = is;
  }
  const float unb = (float)rpg / (float)max(rpg - 1, 1);
  if (g.groups == 1) {
    if (t < CO_COLS && okc) {
      float* rm = cptr(g.rm, co);
      float* rv = cptr(g.rv, co);
      rm[c] = (1.f - g.momentum) * rm[c] + g.momentum * mu;
      rv[c] = (1.f - g.momentum) * rv[c] + g.momentum * var * unb;
    }
  } else {
    unsigned* flag = reinterpret_cast<unsigned*>(red + 2 * CO_THREADS);   // past the partial sums
    const __amdgpu_buffer_rsrc_t st = __builtin_amdgcn_make_buffer_rsrc(cptr(g.stat, co), 0, 0x7FFFFFFF, 0x00020000);
    if (t < CO_COLS && okc) {
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(mu), st, (int)(((size_t)(2 * b) * N + c) * 4), 0, 16);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(var), st, (int)(((size_t)(2 * b + 1) * N + c) * 4), 0, 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) {
      unsigned* cnt = cptr(g.cnt, co) + blockIdx.x;
      const unsigned tk = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned last = tk == (unsigned)(g.groups - 1) ? 1u : 0u;
      if (last) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = last;
    }
    __syncthreads();
    if (*flag && t < CO_COLS && okc) {
      float* rm = cptr(g.rm, co);
      float* rv = cptr(g.rv, co);
      float m = rm[c], v = rv[c];
      for (int bb = 0; bb < g.groups; ++bb) {
        const float mb = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(st, (int)(((size_t)(2 * bb) * N + c) * 4), 0, 16));
        const float vb =
            __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(st, (int)(((size_t)(2 * bb + 1) * N + c) * 4), 0, 16));
        m = (1.f - g.momentum) * m + g.momentum * mb;
        v = (1.f - g.momentum) * v + g.momentum * vb * unb;
      }
      rm[c] = m;
      rv[c] = v;
    }
  }

  // 4. normalise: consecutive threads write consecutive columns of a row (the thread's column is fixed)
  if (!okc || (g.dbg & 4)) return;
  const float gm = cptr(g.gamma, co)[c], bt = cptr(g.beta, co)[c];
  for (int r = part; r < rpg; r += CO_THREADS / CO_COLS) {
    const float nv = (ys[r * CO_LDY + col] - mu) * is;
    const size_t R = (size_t)(rbase + r);
    nhat[R * g.ldn + c] = nv;
    const float y = nv * gm + bt;
    out[R * g.ldo + c] = y > 0.f ? y : 0.f;
  }
}

size_t colown_smem_bytes(int K, int rpg) {
  const int KP = (K + 31) / 32 * 32 + 8;
  return (size_t)CO_COLS * KP * 2 + ((size_t)rpg * CO_LDY + 2 * CO_THREADS + 4 + rpg) * 4;
}

int g_colown_dbg = 0;

void launch_linear_bn_relu_colown(ColOwnArgs g, bool vec, hipStream_t stream) {
  const ClientBatch& cb = client_batch();
  g.dbg = g_colown_dbg;
  g.cstride = cb.k > 1 ? cb.stride : 0;
  if (cb.k > 1) {
    check_slabs("linear_bn_relu_colown operand", g.x, g.w, g.bias, g.oh_w, g.oh_col, g.oh_opt, g.oh_off, g.gamma,
                g.beta, g.out, g.nhat, g.mean, g.invstd, g.rm, g.rv, g.stat, g.cnt);
  }
  const dim3 grid((g.N + CO_COLS - 1) / CO_COLS, g.groups, cb.k > 1 ? cb.k : 1);
  const size_t lds = colown_smem_bytes(g.K, g.rpg);
  if (vec) hipLaunchKernelGGL((linear_bn_relu_colown_kernel<true>), grid, dim3(CO_THREADS), lds, stream, g);
  else hipLaunchKernelGGL((linear_bn_relu_colown_kernel<false>), grid, dim3(CO_THREADS), lds, stream, g);
}

}  // namespace fedtgan
