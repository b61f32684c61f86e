// Adam over a flat buffer with column-sum jobs folded in: the body shared by adam_cs_kernel
// (ctgan_ops.hip) and gemm_adam_kernel (gemm.hip, where a weight-gradient GEMM's tiles run in the
// same launch and apply Adam to their own outputs).  See ctgan_ops.hip for the scheme.
#pragma once
#include "common.h"
#include "launch.h"

namespace fedtgan {

// batched clients (launch.h ClientBatch): a client's copy of a column-sum job / of every job of an Adam launch
__device__ __forceinline__ ColsumJob client_job(ColsumJob jb, int64_t o) {
  jb.a = cptr(jb.a, o);
  jb.out = cptr(jb.out, o);
  jb.w = cptr(jb.w, o);
  jb.dot_v = cptr(jb.dot_v, o);
  jb.dot_e = cptr(jb.dot_e, o);
  jb.dot_out = cptr(jb.dot_out, o);
  jb.dot_w = cptr(jb.dot_w, o);
  return jb;
}
inline void check_slab(const AdamColsum& cs) {
  for (int k = 0; k < cs.n_jobs && k < 8; ++k)
    check_slabs("adam column-sum job", cs.jobs[k].a, cs.jobs[k].out, cs.jobs[k].w, cs.jobs[k].dot_v, cs.jobs[k].dot_e,
                cs.jobs[k].dot_out, cs.jobs[k].dot_w);
}

// One Adam element update, with explicit fmaf so every kernel that applies it (the float4 Adam, the
// column-sum jobs, a fused GEMM's epilogue) rounds identically whatever the compiler contracts:
//   gq = g + wd p ; m = b1 m + (1 - b1) gq ; v = b2 v + (1 - b2) gq^2 ; p -= sz m / (sqrt(v) / bc2s + eps)
__device__ __forceinline__ void adam_elem(float g, float& p, float& m, float& v, float b1, float b2, float eps, float wd,
                                          float sz, float bc2s) {
  const float gq = fmaf(wd, p, g);
  m = fmaf(b1, m, (1.f - b1) * gq);
  v = fmaf(b2, v, ((1.f - b2) * gq) * gq);
  p = p - (sz * m) / (sqrtf(v) / bc2s + eps);
}

template <int AUX>
__device__ __forceinline__ void adam_store4(float4* base, __amdgpu_buffer_rsrc_t rs, int64_t i, float4 x) {
  if constexpr (AUX == 0) {
    base[i] = x;
  } else {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 u = *reinterpret_cast<const u32x4*>(&x);
    __builtin_amdgcn_raw_buffer_store_b128(u, rs, (int)(i * 16), 0, AUX);
  }
}

// The first cs.blk_start[n_jobs] workgroups each reduce ACS_COLS columns of one column-sum job
// (ACS_GROUPS row groups of ACS_COLS lanes, an LDS combine), write the sums (bias gradient or
// metric), and when the job's output lies inside this optimizer's gradient buffer apply Adam to
// exactly those elements straight from registers.  Every other workgroup runs the float4 Adam and
// skips the float4 groups the jobs own (and [skip_lo, skip_hi), a fused GEMM's): job outputs start
// 16-B aligned and own ceil4(cols) elements (the flat layout stores every tensor that way), so no
// float4 is shared.  bid / nblk: this workgroup's index and the count among the launch's Adam ones.
// U: float4 per thread and operand per pass of the Adam loop (1, or ADAM_U for large optimizers: adam_unroll)
constexpr int ADAM_U = 4;
// the launchers' choice of U: the unrolled loop from g_adam_u_min float4 over the launch's clients (default: always)
inline int adam_unroll(int64_t n4, int clients) { return n4 * (clients > 1 ? clients : 1) >= g_adam_u_min ? ADAM_U : 1; }

template <int AUX, int U = 1>
__device__ __forceinline__ void adam_cs_body(int bid, int nblk, float* __restrict__ p, const float* __restrict__ g,
                                             float* __restrict__ m, float* __restrict__ v,
                                             const float* __restrict__ step, int64_t n4, float lr, float b1, float b2,
                                             float eps, float wd, uint64_t* rng_bump, const AdamColsum& cs,
                                             int64_t co = 0) {
  const float t = step[0];
  const float bc1 = 1.f - powf(b1, t);
  const float bc2s = sqrtf(1.f - powf(b2, t));
  const float sz = lr / bc1;
  const int nb = cs.blk_start[cs.n_jobs];
  if (bid < nb) {
    // 4 float4 column quads x 64 row groups; a 500-row job is 8 loads per thread
    __shared__ float part[2][ACS_GROUPS][ACS_COLS + 1];
    int j = 0;
    while (j + 1 < cs.n_jobs && bid >= cs.blk_start[j + 1]) ++j;
    // (co: batched clients -- this client's copy of the job; applied to the one job read here, never to the
    // whole by-value AdamColsum, which would then live in scratch memory)
    const ColsumJob jb = co ? client_job(cs.jobs[j], co) : cs.jobs[j];
    const int cb = bid - cs.blk_start[j];
    const int qd = threadIdx.x & 3, grp = threadIdx.x >> 2;
    const int c0 = cb * ACS_COLS + qd * 4;
    // the Adam operands of this block's owned elements are fetched first, so their round trip
    // overlaps the column-sum loads instead of following them
    const int64_t e = cs.own_lo[j] + cb * ACS_COLS + (int)threadIdx.x;
    const bool upd = threadIdx.x < ACS_COLS && e < cs.own_hi[j];
    float pe = 0.f, me = 0.f, ve = 0.f;
    if (upd) {
      pe = p[e];
      me = m[e];
      ve = v[e];
    }
    float4 s4 = make_float4(0.f, 0.f, 0.f, 0.f), d4 = make_float4(0.f, 0.f, 0.f, 0.f);
    const bool two = jb.dot_w != nullptr;   // a second column sum with the dot's row weights
    if (cs.vec[j]) {   // 16-B aligned rows padded to >= ceil4(cols): whole quads are in bounds
      const int cq = min(c0, ((jb.cols + 3) & ~3) - 4);
#pragma unroll 4
      for (int r = grp; r < jb.rows; r += ACS_GROUPS) {
        const float wr = jb.w ? jb.w[r] : 1.f;
        const float ur = two ? jb.dot_w[r] : 0.f;
        const float4 x = *reinterpret_cast<const float4*>(jb.a + (size_t)r * jb.lda + cq);
        s4.x += wr * x.x;
        s4.y += wr * x.y;
        s4.z += wr * x.z;
        s4.w += wr * x.w;
        d4.x += ur * x.x;
        d4.y += ur * x.y;
        d4.z += ur * x.z;
        d4.w += ur * x.w;
      }
    } else {
      const int last = jb.cols - 1;
      for (int r = grp; r < jb.rows; r += ACS_GROUPS) {
        const float wr = jb.w ? jb.w[r] : 1.f;
        const float ur = two ? jb.dot_w[r] : 0.f;
        const float* ar = jb.a + (size_t)r * jb.lda;
        const float x0 = ar[min(c0, last)], x1 = ar[min(c0 + 1, last)];
        const float x2 = ar[min(c0 + 2, last)], x3 = ar[min(c0 + 3, last)];
        s4.x += wr * x0;
        s4.y += wr * x1;
        s4.z += wr * x2;
        s4.w += wr * x3;
        d4.x += ur * x0;
        d4.y += ur * x1;
        d4.z += ur * x2;
        d4.w += ur * x3;
      }
    }
    part[0][grp][qd * 4 + 0] = s4.x;
    part[0][grp][qd * 4 + 1] = s4.y;
    part[0][grp][qd * 4 + 2] = s4.z;
    part[0][grp][qd * 4 + 3] = s4.w;
    part[1][grp][qd * 4 + 0] = d4.x;
    part[1][grp][qd * 4 + 1] = d4.y;
    part[1][grp][qd * 4 + 2] = d4.z;
    part[1][grp][qd * 4 + 3] = d4.w;
    __syncthreads();
    if (threadIdx.x >= 64) return;
    const int lane = threadIdx.x;   // wave 0: lane = column (lane & 15) x quarter of the row groups
    float tsum = 0.f, tdot = 0.f;
#pragma unroll
    for (int i = 0; i < ACS_GROUPS / 4; ++i) {
      tsum += part[0][(lane >> 4) * (ACS_GROUPS / 4) + i][lane & 15];
      tdot += part[1][(lane >> 4) * (ACS_GROUPS / 4) + i][lane & 15];
    }
    tsum += __shfl_xor(tsum, 16);
    tsum += __shfl_xor(tsum, 32);
    tdot += __shfl_xor(tdot, 16);
    tdot += __shfl_xor(tdot, 32);
    if (!two) tdot = tsum;
    const int col = cb * ACS_COLS + lane;
    const bool live = lane < ACS_COLS && col < jb.cols;
    if (live && jb.out) jb.out[col] = tsum;
    if (jb.dot_v) {
      // a dot over this job's own parameters reads them as they were before this launch (the
      // prefetched value of the lane that updates them): no other workgroup writes them
      const float vc = live ? (cs.dot_self[j] ? pe : jb.dot_v[col]) : 0.f;
      float d = tdot * vc;
      if (cb == 0 && jb.dot_e) {   // + e * sum_r u[r], once per job
        const float* uw = two ? jb.dot_w : jb.w;
        float ws = 0.f;
        for (int r = lane; r < jb.rows; r += 64) ws += uw ? uw[r] : 1.f;
        d += wave_sum(ws) * (lane == 0 ? jb.dot_e[0] : 0.f);
      }
      d = wave_sum(d);
      if (lane == 0) atomicAdd(jb.dot_out, d);
    }
    if (upd) {
      adam_elem(live ? tsum : 0.f, pe, me, ve, b1, b2, eps, wd, sz, bc2s);
      m[e] = me;
      v[e] = ve;
      p[e] = pe;
    }
    return;
  }
  const int bytes = (int)(n4 * 16);
  float4* p4 = reinterpret_cast<float4*>(p);
  float4* m4 = reinterpret_cast<float4*>(m);
  float4* v4 = reinterpret_cast<float4*>(v);
  const float4* g4 = reinterpret_cast<const float4*>(g);
  const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(p4, 0, bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rm = __builtin_amdgcn_make_buffer_rsrc(m4, 0, bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(v4, 0, bytes, 0x00020000);
  const int64_t stride = (int64_t)(nblk - nb) * blockDim.x;
  if constexpr (U > 1) {
    // U float4 of each operand per thread, all 4U loads issued before the first update: the bytes in flight
    // per wave no longer depend on how many workgroups share a CU (a fused GEMM launch keeps the tile's LDS
    // for every workgroup -- 2 per CU -- which left the one-float4-per-thread loop HBM-starved on the wide
    // table's 35 M-parameter D).  The fused GEMM's range [skip_lo, skip_hi) is cut out of the index space
    // (no wasted loads); the column-sum jobs' few elements are loaded and left to the jobs.
    // (and a second range, [skip2_lo, skip2_hi) above the first: a short-K weight gradient's, updated ahead)
    const int64_t lo4 = cs.skip_lo >> 2, hi4 = max(cs.skip_hi >> 2, lo4);
    const int64_t lo4b = cs.skip2_lo >> 2, hi4b = max(cs.skip2_hi >> 2, lo4b);
    const int64_t nn = n4 - (hi4 - lo4) - (hi4b - lo4b);
    for (int64_t i0 = (int64_t)(bid - nb) * blockDim.x + threadIdx.x; i0 < nn; i0 += U * stride) {
      float4 pp[U], gg[U], mm[U], vv[U];
      int64_t ix[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t j = min(i0 + u * stride, nn - 1);
        const int64_t j1 = j < lo4 ? j : j + (hi4 - lo4);
        ix[u] = j1 < lo4b ? j1 : j1 + (hi4b - lo4b);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        pp[u] = p4[ix[u]];
        gg[u] = g4[ix[u]];
        mm[u] = m4[ix[u]];
        vv[u] = v4[ix[u]];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t e = ix[u] * 4;
        bool skip = i0 + u * stride >= nn;
        for (int k = 0; k < cs.n_jobs; ++k) skip |= e >= cs.own_lo[k] && e < cs.own_hi[k];
        if (skip) continue;
        float* pf = reinterpret_cast<float*>(&pp[u]);
        float* gf = reinterpret_cast<float*>(&gg[u]);
        float* mf = reinterpret_cast<float*>(&mm[u]);
        float* vf = reinterpret_cast<float*>(&vv[u]);
#pragma unroll
        for (int q = 0; q < 4; ++q) adam_elem(gf[q], pf[q], mf[q], vf[q], b1, b2, eps, wd, sz, bc2s);
        adam_store4<AUX>(p4, rp, ix[u], pp[u]);
        adam_store4<AUX>(m4, rm, ix[u], mm[u]);
        adam_store4<AUX>(v4, rv, ix[u], vv[u]);
      }
    }
    if (rng_bump && bid == nb && threadIdx.x == 0) rng_bump[0] += 1ull;
    return;
  }
  for (int64_t i = (int64_t)(bid - nb) * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const int64_t e = i * 4;
    bool owned = false;
    for (int k = 0; k < cs.n_jobs; ++k) owned |= e >= cs.own_lo[k] && e < cs.own_hi[k];
    owned |= e >= cs.skip_lo && e < cs.skip_hi;     // updated by a fused GEMM's epilogue (gemm_adam_kernel)
    owned |= e >= cs.skip2_lo && e < cs.skip2_hi;   // by a short-K weight gradient's, ahead of this launch
    if (owned) continue;
    float4 pp = p4[i], gg = g4[i], mm = m4[i], vv = v4[i];
    float* pf = reinterpret_cast<float*>(&pp);
    float* gf = reinterpret_cast<float*>(&gg);
    float* mf = reinterpret_cast<float*>(&mm);
    float* vf = reinterpret_cast<float*>(&vv);
#pragma unroll
    for (int q = 0; q < 4; ++q) adam_elem(gf[q], pf[q], mf[q], vf[q], b1, b2, eps, wd, sz, bc2s);
    adam_store4<AUX>(p4, rp, i, pp);
    adam_store4<AUX>(m4, rm, i, mm);
    adam_store4<AUX>(v4, rv, i, vv);
  }
  if (rng_bump && bid == nb && threadIdx.x == 0) rng_bump[0] += 1ull;
}


}  // namespace fedtgan
