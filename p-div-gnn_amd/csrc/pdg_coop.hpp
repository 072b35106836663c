// The block-cooperative layout shared by the edge / node kernels of pdg_ebw.hip (backward) and pdg_efwd.hip
// (forward): one block of 8 waves per CU, wave w owns output features [16w, 16w + 16) of a product with the
// weights stationary in registers as bf16 terms, operands as bf16x6 row images in LDS, whole-row HBM access
// through fp32 row tiles (see pdg_ebw.hip's header).
#pragma once
#include "pdg_common.hpp"
#include "pdg_runtime.hpp"
#include "pdg_x6.hpp"

using namespace pdg;

namespace {

constexpr int EBW_WAVES = 8;
constexpr int EBW_THREADS = 64 * EBW_WAVES;
constexpr int EBW_IMG = 3 * X6_TERM;        // one bf16x6 image of 32 rows (24 KB)
// relu mask bytes of 32 rows, row stride MSK_STRIDE: the epilogue reads one 4-byte word per lane
// from 16 rows at a time, which a 128-B stride put on 2 of the 32 banks of a ds_read_b32 lane
// group (16-way conflicts); 136 B (34 words) spreads them over all 32.  The staging writes (32
// consecutive words of a row per lane group) stay conflict free.
// the cooperative edge forward's C = Wc e as an unbiased bf16x6 product (gemm_x6f, the lo terms of Wc's
// K chunks 0-1 in LDS) instead of fp32 MFMAs (0: A/B only).  Round 5: edge_fwd 211.4-212.9 -> 205.3-206.3 us
// per config-2 call, the step -0.07 ms in two same-box pairs; every parity gate green (EXPERIMENTS §4).
#ifndef PDG_MSK_STRIDE
#define PDG_MSK_STRIDE 136
#endif
constexpr int MSK_STRIDE = PDG_MSK_STRIDE;
constexpr int EBW_MASK = X6_ROWS * MSK_STRIDE;
constexpr int WSLAB = L * L + L;            // floats per slab (weight + bias sums)
// fp32 row tile in LDS that turns the product's output layout (16 rows x 64 B per wave
// instruction: 25 % below whole-row access in an isolated stream, tools/membench.hip) into
// row-major global accesses: 32 rows, stride 132 floats (the 16-row column writes of the
// output layout then hit 64 distinct banks).  Used by pdg_edge_gout_wc (-2 %); in
// pdg_edge_bwd_w2 the three extra tiles measured +2 % and are not used.
constexpr int OT_STRIDE = L + 4;

// 16-row images (pdg_edge_bwd_w2's two-round register pipeline): term planes of 16 rows
constexpr int R16 = 16;
constexpr int T16 = R16 * X6_ROWB;          // bytes per term plane (4 KB)
constexpr int IMG16 = 3 * T16;              // one bf16x6 image of 16 rows (12 KB)
constexpr int MSK16 = R16 * MSK_STRIDE;

// Columns 4cg .. 4cg+3 of image row r, split into the three terms (term planes TERM bytes apart).
template <int TERM = X6_TERM>
__device__ __forceinline__ void img_store4(unsigned char* img, int r, int cg, const f32x4& v) {
  unsigned h0, m0, l0, h1, m1, l1;
  split3_pair(v[0], v[1], h0, m0, l0);
  split3_pair(v[2], v[3], h1, m1, l1);
  const int off = x6_addr(r, 8 * cg);
  *reinterpret_cast<u32x2*>(img + off) = u32x2{h0, h1};
  *reinterpret_cast<u32x2*>(img + TERM + off) = u32x2{m0, m1};
  *reinterpret_cast<u32x2*>(img + 2 * TERM + off) = u32x2{l0, l1};
}

__device__ __forceinline__ unsigned relu_mask4(const f32x4& a) {
  return (a[0] > 0.f ? 0x1u : 0u) | (a[1] > 0.f ? 0x100u : 0u) | (a[2] > 0.f ? 0x10000u : 0u) |
         (a[3] > 0.f ? 0x1000000u : 0u);
}

// gz2 = LN_bwd(gy) * [a2 > 0] for 4 features (ln_relu_bwd, pdg_bwd.hip, element by element).
__device__ __forceinline__ f32x4 ln_relu_bwd4(const f32x4& gy, const f32x4& a2, const LNStat& st,
                                              const pdg_ln_bwd& lb, const f32x4& g) {
  f32x4 z;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float xhat = div_den(a2[e] - st.mean, st.den, st.rstd);
    const float ga = st.rstd * (g[e] * gy[e] - lb.c1) - xhat * lb.c2;
    z[e] = a2[e] > 0.f ? ga : 0.f;
  }
  return z;
}

// slab += G^T X over the 32 staged rows (K = rows): wave w owns o in 32 (w & 3) + [0, 32),
// i in 64 (w >> 2) + [0, 64) as two 32x32 accumulators (wgrad_x6_kernel's operand reads).
// KS 16-row K steps per call (2: a 32-row image, 1: a 16-row one, term planes TERM bytes apart).
template <int KS = 2, int TERM = X6_TERM>
__device__ __forceinline__ void wgrad_round(f32x16 (&acc)[2], const unsigned char* gimg, const unsigned char* ximg) {
  const int l = lane_id(), w = wave_id(), h = l >> 5;
  const int ob = 32 * (w & 3), ib = 64 * (w >> 2);
  const int lrow = 8 * h + ((l & 15) >> 2);
  const int lcolb = 2 * (16 * ((l >> 4) & 1) + 4 * (l & 3));
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int row = 16 * ks + lrow;
    bf16x8 A[3], B[2][3];
    const int g0 = x6_addr(row, lcolb + 2 * ob), g1 = x6_addr(row + 4, lcolb + 2 * ob);
#pragma unroll
    for (int p = 0; p < 3; ++p) A[p] = x6_operand(gimg + p * TERM, g0, g1);
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int x0 = x6_addr(row, lcolb + 2 * (ib + 32 * b)), x1 = x6_addr(row + 4, lcolb + 2 * (ib + 32 * b));
#pragma unroll
      for (int p = 0; p < 3; ++p) B[b][p] = x6_operand(ximg + p * TERM, x0, x1);
    }
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      f32x16 t = acc[b];
      t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[2], B[b][0], t, 0, 0, 0);
      t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[1], B[b][1], t, 0, 0, 0);
      t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[0], B[b][2], t, 0, 0, 0);
      t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[1], B[b][0], t, 0, 0, 0);
      t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[0], B[b][1], t, 0, 0, 0);
      acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[0], B[b][0], t, 0, 0, 0);
    }
  }
}

// d[nb] = (W^T-slice x image rows 16 nb .. 16 nb + 15): D row = output feature 16w + 4(l >> 4) + j,
// column = staged row 16 nb + (l & 15).  NI images share the weight operands.
template <int NI, int NB = 2, int TERM = X6_TERM>
__device__ __forceinline__ void gemm_round(f32x4 (&d)[NI][NB], const WSlice& ws, const unsigned char* const (&img)[NI]) {
  const int l = lane_id(), n = l & 15, kg = l >> 4;
#pragma unroll
  for (int u = 0; u < NI; ++u)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) d[u][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
#pragma unroll
    for (int u = 0; u < NI; ++u)
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        const int off = x6_addr(16 * nb + n, 64 * ks + 16 * kg);
        bf16x8 B[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) B[p] = *reinterpret_cast<const bf16x8*>(img[u] + p * TERM + off);
        f32x4 t = d[u][nb];
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ws.a[ks][2], B[0], t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ws.a[ks][1], B[1], t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ws.a[ks][0], B[2], t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ws.a[ks][1], B[0], t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ws.a[ks][0], B[1], t, 0, 0, 0);
        d[u][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ws.a[ks][0], B[0], t, 0, 0, 0);
      }
  }
}

// Block's row range: contiguous, a multiple of 32 rows except at the end.
__device__ __forceinline__ void block_rows(int M, int& r0, int& r1) {
  const int nb = gridDim.x;
  int per = (M + nb - 1) / nb;
  per = (per + X6_ROWS - 1) / X6_ROWS * X6_ROWS;
  r0 = min(M, per * (int)blockIdx.x);
  r1 = min(M, per * ((int)blockIdx.x + 1));
}

// The rows a block walks, in 32-row units: [r0, r1) is the range its buffer resources span and its
// loads clamp to, its units start at `first` and are `stride` rows apart.  XI (XCD-interleaved): the
// blocks that share an XCD's L2 (b and b + 8, MI355X_MICROARCH.md 'Workgroup dispatch'; the grid a
// multiple of 8) sweep one contiguous eighth of the rows together, taking its units round-robin,
// instead of each block owning one contiguous range (block_rows).  Rows gathered by index (the edge
// forward's P / Q rows, reused by the edges of the mesh neighbours of a node, ~+-13 units apart in dst
// order) then have one live window per XCD instead of one per block.
// The interleaved form is compiled for a grid of XCD_GRID blocks (one per CU of MI355X: the stride is then
// a constant; a runtime stride cost the edge backward 13 spilled VGPRs); the launchers check the grid.
constexpr int XCD_GRID = 256;
__device__ __forceinline__ void row_schedule(bool xi, int M, int& r0, int& r1, int& first, int& stride) {
  if (xi) {
    const int units = (M + X6_ROWS - 1) / X6_ROWS, perx = (units + 7) / 8;
    const int x = blockIdx.x & 7, j = blockIdx.x >> 3;
    r0 = min(M, x * perx * X6_ROWS);
    r1 = min(M, (x + 1) * perx * X6_ROWS);
    first = min(M, r0 + j * X6_ROWS);
    stride = (XCD_GRID >> 3) * X6_ROWS;
  } else {
    block_rows(M, r0, r1);
    first = r0;
    stride = X6_ROWS;
  }
}

// XCD-interleaved units in the edge backward kernels (pdg_edge_bwd_w2, pdg_edge_gout_wc; the grid of
// XCD_GRID blocks).  Off: 195-198 vs 195-198 us per edge_bwd_w2 call (no gather whose reuse it could
// help: gaggr[dst] is read in dst order), and the slab sums change order.

// slab += acc (the block's own slab, fixed block -> slab map) and the bias sums:
// thread (cg, rg) holds column sums of columns 4cg .. 4cg+3 over its rows; reduced over
// the 16 row groups in order through LDS (`red`, 8 KB, the images being dead).
__device__ __forceinline__ void slab_accumulate(float* __restrict__ slab, const f32x16 (&acc)[2], const f32x4& bsum,
                                                float* red, int init) {
  const int l = lane_id(), w = wave_id(), h = l >> 5, c = l & 31;
  const int ob = 32 * (w & 3), ib = 64 * (w >> 2);
  // every load before any store: vmcnt counts loads and stores together in issue order, so a
  // load behind a store cannot be waited for alone; interleaved (slab[] += acc), the compiler
  // emitted ~25 load -> wait -> store round trips, one slab line at a time
  float old[2][16];
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int o = ob + (r & 3) + 8 * (r >> 2) + 4 * h, i = ib + 32 * b + c;
      old[b][r] = init ? 0.f : slab[o * L + i];   // init: the first call of a backward writes (no fill)
    }
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int o = ob + (r & 3) + 8 * (r >> 2) + 4 * h, i = ib + 32 * b + c;
      slab[o * L + i] = old[b][r] + acc[b][r];
    }
  const int cg = threadIdx.x & 31, rg = threadIdx.x >> 5;
  *reinterpret_cast<f32x4*>(red + rg * L + 4 * cg) = bsum;
  __syncthreads();
  if (threadIdx.x < L) {
    float s = 0.f;
#pragma unroll
    for (int g = 0; g < 16; ++g) s += red[g * L + threadIdx.x];
    slab[L * L + threadIdx.x] = (init ? 0.f : slab[L * L + threadIdx.x]) + s;
  }
}

// fp32 row tile of 32 rows (stride OT_STRIDE) and the e tile's row stride of the cooperative edge forward
constexpr int EFC_TILE = X6_ROWS * OT_STRIDE;   // floats per fp32 row tile
constexpr int EFC_ES = L + 8;                    // e tile row stride: the C operand reads are conflict free

}  // namespace
