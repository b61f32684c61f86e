// Shared device helpers for the gfx950 (CDNA4) kernels of fed_tgan_amd.
//
// * Philox4x32-10 counter-based RNG.  Every random draw in the training step is addressed by
//   (seed, stream id, step counter, element index); the step counter lives in device memory
//   and is bumped by the last kernel of a step, so a captured hipGraph produces fresh numbers
//   on every replay without any host involvement.
// * bf16 packing for the MFMA operands (round-to-nearest-even).
// * wave64 reductions (DPP/shuffle based, 64 lanes -- never 32).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fedtgan {

constexpr int WAVE = 64;

// ---- checked build (csrc/build.py --checked -> _C_checked.so, FEDTGAN_CHECKED=1 at run time): every
// data-dependent index a kernel derives from its tables (CSR row picks, condition options, decode
// codes, one-hot gathers, encode lookups) is verified; a violation sets a bit in the translation
// unit's flag word with a vector atomic (no trap: the access itself is clamped so the kernel never
// faults) and the host raises after the launch sequence (`fedtgan_check_status`).  Release builds
// compile the checks away.
enum CheckCode : unsigned {
  CHK_CSR_PICK = 0,      // sampler: CSR entry outside the row-list array
  CHK_DATA_ROW = 1,      // sampler: data row outside the training matrix
  CHK_COND = 2,          // sampler: drawn column / option outside the span tables
  CHK_DECODE_CODE = 3,   // decode: categorical code index outside the code table
  CHK_DECODE_MODE = 4,   // decode: mode index >= K
  CHK_ONEHOT = 5,        // GEMM one-hot gather: condition index outside the block
  CHK_ENCODE_LUT = 6,    // encode: label lookup outside the table
};
#ifdef FEDTGAN_CHECKED
#define FT_CHECK(flag, cond, code)                                  \
  do {                                                              \
    if (!(cond)) atomicOr((flag), 1u << (unsigned)(code));          \
  } while (0)
#define FT_CHECKED 1
#else
#define FT_CHECK(flag, cond, code) ((void)0)
#define FT_CHECKED 0
#endif

// batched clients (launch.h ClientBatch): client copy of a buffer, `off` bytes after client 0's
template <class T>
__device__ __forceinline__ T* cptr(T* p, int64_t off) {
  return p ? (T*)((const char*)p + off) : p;
}

// Batched clients, XCD-aware: the dispatcher deals a grid's workgroups round-robin over the 8 XCDs by linear id
// (MI355X_MICROARCH.md "Workgroup dispatch"), so in a client-major grid every client's tiles land on all 8 XCDs
// and each XCD's 4 MB L2 holds pieces of all K clients' operands -- the tiles' re-reads of a client's
// activations and weights (a few MB per client) then miss L2.  Remapped, the workgroups of XCD x (linear id
// % 8 == x) serve clients {x / (8 / K)} (K <= 8) or {x * (K / 8) + ...} (K >= 8): a client's whole launch
// runs on its own XCD(s), and every kernel of a step places the client there, so its data stays in that L2
// from kernel to kernel.  lin = the workgroup's linear id in a grid of K * T workgroups, T per client
// (client-major); valid when K divides 8 or 8 divides K, and 8 divides K * T.  Returns false otherwise
// (then client = lin / T).
__device__ __forceinline__ bool xcd_client_map(int lin, int T, int K, int& client, int& local) {
  if (K > 1 && ((K * T) & 7) == 0 && ((8 % K) == 0 || (K & 7) == 0)) {
    const int x = lin & 7, slot = lin >> 3;
    if (K <= 8) {
      const int xpc = 8 / K;                  // XCDs per client
      client = x / xpc;
      local = slot * xpc + x % xpc;
    } else {
      const int cpx = K >> 3;                 // clients per XCD
      client = x * cpx + slot / T;
      local = slot % T;
    }
    return true;
  }
  client = lin / T;
  local = lin - client * T;
  return false;
}

// the block coordinates a workgroup serves in a batched grid (gridDim.x, gridDim.y, K clients = gridDim.z):
// blockIdx itself, or with `xcd` (ClientBatch::xcd) the XCD-aware client placement above.  Every batched kernel
// reads its (x, y, client) from here, so a client's producer and consumer kernels run on the same XCD(s).
struct BIdx {
  int x, y, z;
};
// B: the batched instantiation of the kernel (the launchers pick it when ClientBatch::xcd is set, i.e. only in
// batched launches); the one-client instantiation reads nothing -- even a never-taken runtime branch on a kernel
// argument put a scalar load and a wait in front of every kernel's first loads, +3.5 us over the latency-bound
// one-client step's 25 launches (profiles/xcd_clients_r4.txt)
template <bool B>
__device__ __forceinline__ BIdx batch_bidx(int xcd) {
  BIdx b{(int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z};
  if constexpr (B) {
    if (xcd) {
      const int gx = (int)gridDim.x, T = gx * (int)gridDim.y;
      int cl, loc;
      if (xcd_client_map(b.x + T * b.z + gx * b.y, T, (int)gridDim.z, cl, loc)) {
        b.x = loc % gx;
        b.y = loc / gx;
        b.z = cl;
      }
    }
  }
  return b;
}

struct RngArgs {
  uint64_t seed;
  const uint64_t* ctr;  // device-resident step counter
  uint32_t stream;      // per-call-site stream id
};

__device__ __forceinline__ uint32_t mulhilo(uint32_t a, uint32_t b, uint32_t& hi) {
  uint64_t p = (uint64_t)a * (uint64_t)b;
  hi = (uint32_t)(p >> 32);
  return (uint32_t)p;
}

__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint2 k) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0, hi1;
    uint32_t lo0 = mulhilo(0xD2511F53u, c.x, hi0);
    uint32_t lo1 = mulhilo(0xCD9E8D57u, c.z, hi1);
    c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
    k.x += 0x9E3779B9u;
    k.y += 0xBB67AE85u;
  }
  return c;
}

// 4 random words for element `idx` of stream `rng.stream` at the current step.
__device__ __forceinline__ uint4 rng4(const RngArgs& rng, uint64_t step, uint64_t idx) {
  uint4 c = make_uint4((uint32_t)idx, (uint32_t)(idx >> 32), rng.stream, (uint32_t)step);
  uint2 k = make_uint2((uint32_t)rng.seed, (uint32_t)(rng.seed >> 32) ^ (uint32_t)(step >> 32));
  return philox4x32_10(c, k);
}

// uniform in (0, 1): never exactly 0 or 1 (safe for log(-log(u)) and Box-Muller)
__device__ __forceinline__ float u01(uint32_t x) { return ((float)(x >> 8) + 0.5f) * (1.0f / 16777216.0f); }

__device__ __forceinline__ double u01d(uint32_t a, uint32_t b) {
  uint64_t v = ((uint64_t)a << 21) ^ (uint64_t)b;
  v &= ((1ull << 53) - 1);
  return ((double)v + 0.5) * (1.0 / 9007199254740992.0);
}

// NOTE: the fast __logf is not monotone-safe next to 1.0 (it can return +0 or a tiny positive
// value for u = 1 - 2^-25), which would turn -log(u) into <= 0 and poison Box-Muller / Gumbel
// with NaN.  The accurate logf is used for log(u) and the results are clamped.
__device__ __forceinline__ float neg_log_u(uint32_t x) { return fmaxf(-logf(u01(x)), 1e-30f); }

__device__ __forceinline__ float2 box_muller(uint32_t a, uint32_t b) {
  const float r = sqrtf(2.0f * neg_log_u(a));
  float s, c;
  __sincosf(6.283185307179586f * u01(b), &s, &c);
  return make_float2(r * c, r * s);
}

__device__ __forceinline__ float gumbel(uint32_t x) { return -logf(neg_log_u(x)); }

// round-to-nearest-even fp32 -> bf16 bits
// fp32 -> bf16, round to nearest even: gfx950's v_cvt_pk_bf16_f32 (one VALU op per PAIR; fp32 denormals are kept,
// amdhsa_float_denorm_mode_32 = 3) -- the same bits as the integer form (u + 0x7FFF + lsb) >> 16 it replaces for
// every non-NaN input (a NaN now stays a quiet NaN instead of possibly rounding to infinity)
typedef __bf16 bf16x2_hw __attribute__((ext_vector_type(2)));
typedef float f32x2_hw __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint16_t f2bf(float f) {
  return __builtin_bit_cast(uint16_t, (__bf16)f);
}

__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_hw){a, b}, bf16x2_hw));
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, WAVE);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, WAVE));
  return v;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, WAVE);
  return v;
}

// block-wide sum for blockDim.x multiple of 64 (<= 1024); `sh` needs blockDim.x/64 floats
__device__ __forceinline__ float block_sum(float v, float* sh) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if (lane == 0) sh[w] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += sh[i];
  return t;
}

}  // namespace fedtgan
