// Shared device building blocks for the P-DivGNN hot path on gfx950 (CDNA4).
//
// Data layout (DESIGN.md "Layout"): every latent tensor is a plain row-major
// (rows x 128) fp32 array in HBM, natural feature order, 512 B per row.
//
// Wave tile: one 64-lane wave owns 32 consecutive rows.  Lane l holds row
// (l & 31) and the half h = l >> 5, i.e. features [64h, 64h+64) of that row, in
// a 64-float register fragment `v[s]` = feature 64h + s.  Loading a fragment is
// 16 x 16-byte loads of one contiguous 256-byte half row.
//
// GEMM on the matrix cores (v_mfma_f32_32x32x2_f32, exact fp32): for a 128x128
// weight W (nn.Linear layout, out x in) the fragment is the B operand and the
// weight the A operand read from LDS.  Step s of the 64-step K loop sums the
// two inputs {s, 64+s} (lane halves h = 0, 1).  The LDS image of W holds in row
// R = nb*32 + i the weight row pi(nb, i) = 64*((i>>2)&1) + 16*nb + 4*(i>>3) + (i&3),
// which makes the accumulator layout of output block nb equal to the fragment
// layout: accumulator register `reg` of block nb of lane l is output feature
// 64h + 16*nb + reg of row (l & 31).  Chained layers therefore stay in
// registers with no LDS transpose.  Rows are padded to 132 floats so the
// per-lane 16-byte A reads (ds_read_b128) are bank-conflict free.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/pdivgnn.h"

namespace pdg {

constexpr int L = 128;                  // latent size (the reference's configs all use 128)
constexpr int TILE = 32;                // rows per wave tile
constexpr int WPAD = 132;               // LDS row stride of a 128x128 weight block (floats)
constexpr int WBLK = 128 * WPAD;        // floats per weight block in LDS (67,584 B)
constexpr float LN_EPS = 1e-5f;         // torch_geometric LayerNorm default eps

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// Graph-LayerNorm statistics of one call (written by pdg_ln_finalize) and the
// backward scalars of one call: include/pdivgnn.h.
typedef pdg_ln_stat LNStat;
typedef pdg_ln_bwd LNBwd;

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }

// An offset the compiler cannot prove loop-invariant: loads addressed with it
// stay inside the tile loop instead of being hoisted (and kept live in
// registers, or spilled) across the whole persistent loop.
__device__ __forceinline__ int opaque(int x) {
  asm volatile("" : "+v"(x));
  return x;
}

// Per-lane offset of the lane's half row: 64 * h.
__device__ __forceinline__ int half_off() { return opaque(64 * (lane_id() >> 5)); }

// x / den as the reference computes it (models.py LayerNorm: out = x / (std + eps)),
// via the reciprocal and one Newton correction: 3 instructions instead of the
// ~10-instruction IEEE division sequence, within 1 ulp of the quotient.
__device__ __forceinline__ float div_den(float x, float den, float rstd) {
  const float q = x * rstd;
  const float r = fmaf(-q, den, x);
  return fmaf(r, rstd, q);
}

__device__ __forceinline__ int wperm(int nb, int i) {
  return 64 * ((i >> 2) & 1) + 16 * nb + 4 * (i >> 3) + (i & 3);
}

// Copy a 128x128 block W[o][col0 + k] (row stride ld floats) into the LDS A-image.
__device__ __forceinline__ void load_wblock(float* __restrict__ lds, const float* __restrict__ W,
                                            int ld, int col0) {
  for (int idx = threadIdx.x; idx < 128 * 32; idx += blockDim.x) {
    const int R = idx >> 5, c4 = idx & 31;
    const int o = wperm(R >> 5, R & 31);
    const f32x4 val = *reinterpret_cast<const f32x4*>(W + (size_t)o * ld + col0 + 4 * c4);
    *reinterpret_cast<f32x4*>(lds + R * WPAD + 4 * c4) = val;
  }
}

// acc[nb] += W * v over K = 128 (256 MFMAs).  The A fragments of step group t+1
// are read from LDS while the 16 MFMAs of group t issue; the scheduling
// barriers keep the compiler from hoisting all 64 LDS reads (which would need
// 256 registers) so a wave stays within the 256-register budget of 2 waves/SIMD.
__device__ __forceinline__ void read_a(f32x4 (&a)[4], const float* __restrict__ base, int t) {
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) a[nb] = *reinterpret_cast<const f32x4*>(base + nb * 32 * WPAD + 4 * t);
}

__device__ __forceinline__ void mfma_group(f32x16 (&acc)[4], const f32x4 (&a)[4], const float (&v)[64], int t) {
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
      acc[nb] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[nb][j], v[4 * t + j], acc[nb], 0, 0, 0);
}

__device__ __forceinline__ void gemm128(f32x16 (&acc)[4], const float* __restrict__ wl,
                                        const float (&v)[64]) {
  const int l = lane_id();
  const float* base = wl + opaque((l & 31) * WPAD + 64 * (l >> 5));
  f32x4 a0[4], a1[4];
  read_a(a0, base, 0);
#pragma unroll
  for (int t = 0; t < 16; t += 2) {
    read_a(a1, base, t + 1);
    mfma_group(acc, a0, v, t);
    __builtin_amdgcn_sched_barrier(0);
    if (t + 2 < 16) read_a(a0, base, t + 2);
    mfma_group(acc, a1, v, t + 1);
    __builtin_amdgcn_sched_barrier(0);
  }
}

__device__ __forceinline__ void zero_acc(f32x16 (&acc)[4]) {
#pragma unroll
  for (int nb = 0; nb < 4; ++nb)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[nb][r] = 0.f;
}

// Fragment <-> accumulator element mapping: v[16*nb + reg] <-> acc[nb][reg].
#define PDG_FOR_FRAG(s) _Pragma("unroll") for (int s = 0; s < 64; ++s)
#define ACC(acc, s) (acc)[(s) >> 4][(s) & 15]

__device__ __forceinline__ void load_frag(float (&v)[64], const float* __restrict__ row) {
  const f32x4* p = reinterpret_cast<const f32x4*>(row + 64 * (lane_id() >> 5));
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    const f32x4 x = p[t];
    v[4 * t + 0] = x[0]; v[4 * t + 1] = x[1]; v[4 * t + 2] = x[2]; v[4 * t + 3] = x[3];
  }
}

__device__ __forceinline__ void store_frag(float* __restrict__ row, const float (&v)[64]) {
  f32x4* p = reinterpret_cast<f32x4*>(row + 64 * (lane_id() >> 5));
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    f32x4 x; x[0] = v[4 * t]; x[1] = v[4 * t + 1]; x[2] = v[4 * t + 2]; x[3] = v[4 * t + 3];
    p[t] = x;
  }
}

__device__ __forceinline__ void store_acc(float* __restrict__ row, const f32x16 (&acc)[4]) {
  f32x4* p = reinterpret_cast<f32x4*>(row + 64 * (lane_id() >> 5));
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    f32x4 x;
    x[0] = ACC(acc, 4 * t); x[1] = ACC(acc, 4 * t + 1); x[2] = ACC(acc, 4 * t + 2); x[3] = ACC(acc, 4 * t + 3);
    p[t] = x;
  }
}

// Chunked fragment access: chunk q in {0,1} covers v[32q .. 32q+32) (8 x 16 B).
// Kernels fence the scheduler between chunks (PDG_FENCE) so at most one chunk of
// each source row is in flight per wave, bounding register use.
#define PDG_FENCE() __builtin_amdgcn_sched_barrier(0)

__device__ __forceinline__ void load_chunk(float* __restrict__ dst32, const float* __restrict__ row, int q) {
  const f32x4* p = reinterpret_cast<const f32x4*>(row + 64 * (lane_id() >> 5) + 32 * q);
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const f32x4 x = p[t];
    dst32[4 * t + 0] = x[0]; dst32[4 * t + 1] = x[1]; dst32[4 * t + 2] = x[2]; dst32[4 * t + 3] = x[3];
  }
}

__device__ __forceinline__ void store_chunk(float* __restrict__ row, const float* __restrict__ src32, int q) {
  f32x4* p = reinterpret_cast<f32x4*>(row + 64 * (lane_id() >> 5) + 32 * q);
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    f32x4 x; x[0] = src32[4 * t]; x[1] = src32[4 * t + 1]; x[2] = src32[4 * t + 2]; x[3] = src32[4 * t + 3];
    p[t] = x;
  }
}

// v[s] (op)= vec[64h + s] for a 128-vector in global memory (bias, LN params).
__device__ __forceinline__ void load_vec_half(float (&v)[64], const float* __restrict__ vec) {
  load_frag(v, vec);
}

// ----------------------------------------------------------------------------- reductions
__device__ __forceinline__ double wave_sum(double x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  return x;
}

// Block-wide sum of two doubles; result valid in thread 0.  `red` needs 2*nwaves doubles.
__device__ __forceinline__ void block_sum2(double& a, double& b, double* red) {
  a = wave_sum(a);
  b = wave_sum(b);
  const int w = wave_id(), nw = blockDim.x >> 6;
  __syncthreads();
  if (lane_id() == 0) { red[2 * w] = a; red[2 * w + 1] = b; }
  __syncthreads();
  if (threadIdx.x == 0) {
    a = 0; b = 0;
    for (int i = 0; i < nw; ++i) { a += red[2 * i]; b += red[2 * i + 1]; }
  }
}

// Apply graph-LayerNorm in place: v = (v - mean) / (std + eps) * g + beta (models.py LayerNorm).
__device__ __forceinline__ void ln_apply(float (&v)[64], const LNStat& st, const float* __restrict__ g,
                                         const float* __restrict__ beta) {
  const f32x4* gp = reinterpret_cast<const f32x4*>(g + half_off());
  const f32x4* bp = reinterpret_cast<const f32x4*>(beta + half_off());
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    const f32x4 gg = gp[t], bb = bp[t];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[4 * t + j] = div_den(v[4 * t + j] - st.mean, st.den, st.rstd) * gg[j] + bb[j];
  }
}

}  // namespace pdg
