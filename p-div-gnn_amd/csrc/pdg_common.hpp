// Shared device building blocks for the P-DivGNN hot path on gfx950 (CDNA4).
//
// Data layout (DESIGN.md "Layout"): every latent tensor is a plain row-major
// (rows x 128) fp32 array in HBM, natural feature order, 512 B per row.
//
// Wave tile: one 64-lane wave owns 16 consecutive rows.  Lane l holds row
// (l & 15) and the quarter q = l >> 4, i.e. features [32q, 32q+32) of that row,
// in a 32-float register fragment `v[s]` = feature 32q + s.  Loading a fragment
// is 8 x 16-byte loads of one contiguous 128-byte quarter row.
//
// GEMM on the matrix cores (v_mfma_f32_16x16x4_f32, exact fp32, 32 cycles per
// instruction per SIMD): for a 128x128 weight W (nn.Linear layout, out x in) the
// fragment is the B operand (B[k][j]: k = lane quarter, j = row) and the weight
// the A operand, read from an LDS image.  Step s of the 32-step K loop sums the
// four inputs {32q + s : q = 0..3}.  The image holds in row R = 16*ob + i the
// weight row pi(ob, i) = 32*(i>>2) + 4*ob + (i&3), which makes the accumulator
// layout equal to the fragment layout: register r of output block ob in lane
// quarter q is output feature 32q + 4*ob + r.  Chained layers therefore stay in
// registers with no LDS transpose.  Fragment (32) + accumulator (32) + A
// fragments (16) leave room for 3 waves per SIMD.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/pdivgnn.h"

namespace pdg {

constexpr int L = 128;                  // latent size (the reference's configs all use 128)
constexpr int TILE = 16;                // rows per wave tile
constexpr int FRAG = 32;                // fragment floats per lane
constexpr int WPAD = 132;               // LDS row stride of a 128x128 weight block (floats)
constexpr int WBLK = 128 * WPAD;        // floats per weight block in LDS (67,584 B)
constexpr float LN_EPS = 1e-5f;         // torch_geometric LayerNorm default eps

typedef float f32x4 __attribute__((ext_vector_type(4)));

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

// Per-lane offset of the lane's quarter row: 32 * q.
__device__ __forceinline__ int quarter_off() { return opaque(32 * (lane_id() >> 4)); }

// x / den as the reference computes it (models.py LayerNorm: out = x / (std + eps)),
// via the reciprocal and one Newton correction: 3 instructions instead of the
// ~10-instruction IEEE division sequence, within 1 ulp of the quotient.
__device__ __forceinline__ float div_den(float x, float den, float rstd) {
  const float q = x * rstd;
  const float r = fmaf(-q, den, x);
  return fmaf(r, rstd, q);
}

__device__ __forceinline__ int wperm(int ob, int i) { return 32 * (i >> 2) + 4 * ob + (i & 3); }

// Copy a 128x128 block W[o][col0 + k] (row stride ld floats) into the LDS A-image.
__device__ __forceinline__ void load_wblock(float* __restrict__ lds, const float* __restrict__ W,
                                            int ld, int col0) {
  for (int idx = threadIdx.x; idx < 128 * 32; idx += blockDim.x) {
    const int R = idx >> 5, c4 = idx & 31;
    const int o = wperm(R >> 4, R & 15);
    const f32x4 val = *reinterpret_cast<const f32x4*>(W + (size_t)o * ld + col0 + 4 * c4);
    *reinterpret_cast<f32x4*>(lds + R * WPAD + 4 * c4) = val;
  }
}

// Accumulator: 8 output blocks of 16 features x 16 rows, 4 registers per lane each.
struct Acc {
  f32x4 b[8];
};
#define ACC(acc, s) (acc).b[(s) >> 2][(s) & 3]
#define PDG_FOR_FRAG(s) _Pragma("unroll") for (int s = 0; s < FRAG; ++s)
#define PDG_FENCE() __builtin_amdgcn_sched_barrier(0)

__device__ __forceinline__ void zero_acc(Acc& acc) {
#pragma unroll
  for (int ob = 0; ob < 8; ++ob) acc.b[ob] = f32x4{0.f, 0.f, 0.f, 0.f};
}

// acc += W * v over K = 128: 8 input groups t x 4 output-block pairs x 8 MFMAs
// (256 MFMAs).  The A fragments of the next (t, pair) are read from LDS while
// the current pair's 8 MFMAs issue; the two accumulators of a pair alternate so
// each dependent chain has a 64-cycle spacing (> the 40-cycle MFMA latency).
// Scheduling barriers keep the compiler from hoisting all 64 LDS reads.
__device__ __forceinline__ void gemm128(Acc& acc, const float* __restrict__ wl, const float (&v)[FRAG]) {
  const int l = lane_id();
  const float* base = wl + opaque((l & 15) * WPAD + 32 * (l >> 4));
  f32x4 a0[2], a1[2];
  a0[0] = *reinterpret_cast<const f32x4*>(base + 0 * 16 * WPAD);
  a0[1] = *reinterpret_cast<const f32x4*>(base + 1 * 16 * WPAD);
#pragma unroll
  for (int it = 0; it < 32; it += 2) {
    // iteration it: input group t = it >> 2, output-block pair p = it & 3 (blocks 2p, 2p+1)
    {
      const int nt = (it + 1) >> 2, np = (it + 1) & 3;
      a1[0] = *reinterpret_cast<const f32x4*>(base + (2 * np) * 16 * WPAD + 4 * nt);
      a1[1] = *reinterpret_cast<const f32x4*>(base + (2 * np + 1) * 16 * WPAD + 4 * nt);
      const int t = it >> 2, p = it & 3;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc.b[2 * p] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[0][j], v[4 * t + j], acc.b[2 * p], 0, 0, 0);
        acc.b[2 * p + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[1][j], v[4 * t + j], acc.b[2 * p + 1], 0, 0, 0);
      }
    }
    PDG_FENCE();
    {
      if (it + 2 < 32) {
        const int nt = (it + 2) >> 2, np = (it + 2) & 3;
        a0[0] = *reinterpret_cast<const f32x4*>(base + (2 * np) * 16 * WPAD + 4 * nt);
        a0[1] = *reinterpret_cast<const f32x4*>(base + (2 * np + 1) * 16 * WPAD + 4 * nt);
      }
      const int t = (it + 1) >> 2, p = (it + 1) & 3;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc.b[2 * p] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[0][j], v[4 * t + j], acc.b[2 * p], 0, 0, 0);
        acc.b[2 * p + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[1][j], v[4 * t + j], acc.b[2 * p + 1], 0, 0, 0);
      }
    }
    PDG_FENCE();
  }
}

// ----------------------------------------------------------------------------- fragment I/O
__device__ __forceinline__ void load_frag(float (&v)[FRAG], const float* __restrict__ row) {
  const f32x4* p = reinterpret_cast<const f32x4*>(row + quarter_off());
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const f32x4 x = p[t];
    v[4 * t + 0] = x[0]; v[4 * t + 1] = x[1]; v[4 * t + 2] = x[2]; v[4 * t + 3] = x[3];
  }
}

__device__ __forceinline__ void store_frag(float* __restrict__ row, const float (&v)[FRAG]) {
  f32x4* p = reinterpret_cast<f32x4*>(row + quarter_off());
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    f32x4 x; x[0] = v[4 * t]; x[1] = v[4 * t + 1]; x[2] = v[4 * t + 2]; x[3] = v[4 * t + 3];
    p[t] = x;
  }
}

__device__ __forceinline__ void store_acc(float* __restrict__ row, const Acc& acc) {
  f32x4* p = reinterpret_cast<f32x4*>(row + quarter_off());
#pragma unroll
  for (int t = 0; t < 8; ++t) p[t] = acc.b[t];
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

}  // namespace pdg
