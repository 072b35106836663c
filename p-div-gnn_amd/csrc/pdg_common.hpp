// Shared device building blocks for the P-DivGNN hot path on gfx950 (CDNA4).
//
// Data layout (DESIGN.md "Layout"): every latent tensor is a plain row-major
// (rows x 128) fp32 array in HBM, natural feature order, 512 B per row.
//
// Wave tile: one 64-lane wave owns 16 consecutive rows.  Lane l holds row
// (l & 15) and, with q = l >> 4, the 32 features {16T + 4q + j : T < 8, j < 4}
// of that row in a register fragment v[4T + j]: eight 16-byte chunks, chunk T
// at byte 64T + 16q of the row.  One fragment-load instruction therefore reads
// 64 contiguous bytes of each of the 16 rows (16 half-lines; the next chunk
// reads the other halves), and a row is covered by 4 lanes side by side.
//
// GEMM on the matrix cores (v_mfma_f32_16x16x4_f32, exact fp32, 32 cycles per
// instruction per SIMD): for a 128x128 weight W (nn.Linear layout, out x in) the
// fragment is the B operand (B[k][j]: k = lane quarter, j = row) and the weight
// the A operand, read from a plain row-major LDS copy of W.  MFMA (T, j) sums
// the four inputs {16T + 4k + j : k < 4}; output block ob's D row i = 4q + r is
// output feature 16 ob + i, so register r of accumulator block ob in lane
// quarter q is feature 16 ob + 4q + r: the accumulator layout equals the
// fragment layout and chained layers stay in registers.  Fragment (32) +
// accumulator (32) + A fragments (16) leave room for 3 waves per SIMD.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/pdivgnn.h"
#include "pdg_runtime.hpp"

namespace pdg {

constexpr int L = 128;                  // latent size (the reference's configs all use 128)
constexpr int TILE = 16;                // rows per wave tile
constexpr int FRAG = 32;                // fragment floats per lane
constexpr int WPAD = 136;               // LDS row stride of a 128x128 weight block (floats): 136 = 8 mod 64
                                        // makes the ds_read_b128 A reads of gemm128 bank-conflict free
constexpr int WBLK = 128 * WPAD;        // floats per weight block in LDS (69,632 B)
#ifndef PDG_EDGE_WAVES
#define PDG_EDGE_WAVES 12
#endif
constexpr int EDGE_WAVES = PDG_EDGE_WAVES;
constexpr float LN_EPS = 1e-5f;         // torch_geometric LayerNorm default eps

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

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

// XCD-aware block order: blocks are dealt round-robin over the 8 XCDs (b and
// b + 8 share one L2), so logical block (b & 7) * (G / 8) + (b >> 3) gives each
// XCD a contiguous range of tiles per round of the persistent loop.  Edges are
// dst-sorted and mesh-local, so the P/Q rows one XCD gathers for its range stay
// in that XCD's L2.  Speed only: any order is correct.
__device__ __forceinline__ int xcd_block() {
  const int g = gridDim.x, b = blockIdx.x;
  return (g & 7) ? b : (b & 7) * (g >> 3) + (b >> 3);
}

// Persistent wave-tile loop over tiles_of(M) tiles of 16 rows.
#define PDG_TILE_LOOP(M)                                                              \
  const int nw_ = blockDim.x >> 6;                                                    \
  const int ntiles_ = tiles_of(M);                                                    \
  for (int tile = xcd_block() * nw_ + wave_id(); tile < ntiles_; tile += gridDim.x * nw_)

// Per-lane feature offset 4q of every fragment chunk (chunk T adds 16T).
__device__ __forceinline__ int lane_col() { return opaque(4 * (lane_id() >> 4)); }

// Chunk T (4 floats) of a row or feature vector, `p` already offset by lane_col().
__device__ __forceinline__ f32x4 ld4(const float* __restrict__ p, int T) {
  return *reinterpret_cast<const f32x4*>(p + 16 * T);
}
// Row stores are nontemporal (streamed past the caches' normal allocation): measured -0.08 ms per
// config-2 step, all from pdg_segment_sum re-reading the edge forward's a2m rows; nontemporal
// LOADS of whole rows made pdg_edge_fwd 4 % slower and are off.
__device__ __forceinline__ void st4(float* __restrict__ p, int T, const f32x4& x) {
  __builtin_nontemporal_store(x, reinterpret_cast<f32x4*>(p + 16 * T));
}
// A 16-byte row store outside the fragment helpers (nontemporal: measured +0.2 ms
// per config-2 step, the P / Q rows the edge forward gathers and the gaggr rows the edge backward
// gathers then miss the caches; plain stores).
__device__ __forceinline__ void stg4(float* __restrict__ p, const f32x4& x) {
  *reinterpret_cast<f32x4*>(p) = x;
}
// A 16-byte load through a global-address-space pointer: for row pointers the compiler cannot
// place (read from an LDS table), which it would otherwise load with FLAT instructions; those
// count in both vmcnt and lgkmcnt, so every later LDS wait also waits for them.
__device__ __forceinline__ f32x4 ldg4(const float* p) {
  typedef __attribute__((address_space(1))) const f32x4 g_f32x4;
  return *(g_f32x4*)p;
}
// Branch-free row access for loops whose vmcnt waits must be counted exactly (a load or store skipped on
// some path makes the compiler wait for every outstanding memory operation, vmcnt(0), at the merge).
__device__ __forceinline__ int clamp_row(int r, int r1) { return r < r1 ? r : r1 - 1; }

// An empty asm that reads x: its load has completed here, and cannot be sunk past this point.
template <class T>
__device__ __forceinline__ void pin_vgpr(const T& x) {
  asm volatile("" ::"v"(x));
}

// Buffer resource over rows [r0, r1) of a (rows, 128) fp32 array: stores past row r1 fall outside
// num_records and are dropped by the hardware range check (no branch around them).  A null array
// gets an empty range (every store dropped).
// P / Q of the node pre-pass (node_pq -> edge forward gathers).  PDG_PQ_BLOCKED (default since round 5):
// one N x 256 array whose row holds, per 16-feature block b, P[16b .. 16b + 15] then Q[16b .. 16b + 15]
// (Q's pointer = P's + 16 floats), so the 64 B of P and of Q a wave of the cooperative edge forward gathers
// for one node share one 128-B line: edge_fwd 191.9-196.7 -> 188.3-191.1 us per config-2 call, bitwise the
// same outputs (two same-box pairs).  0: two N x 128 arrays (the layout pdg_edge_fwd reads).
#ifndef PDG_PQ_BLOCKED
#define PDG_PQ_BLOCKED 1
#endif
constexpr int PQ_LD = PDG_PQ_BLOCKED ? 2 * 128 : 128;   // row stride of P / Q (floats)
// offset of feature c (a multiple of 4: one 16-byte chunk) in a P / Q row
__device__ __forceinline__ int pq_col(int c) { return PDG_PQ_BLOCKED ? c + (c & ~15) : c; }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rows_rsrc(float* base, int r0, int r1) {
  return __builtin_amdgcn_make_buffer_rsrc(base ? base + (size_t)r0 * L : nullptr, (short)0,
                                           base ? (r1 - r0) * L * 4 : 0, 0x00020000);
}
// 16-byte store of columns c .. c+3 of block-relative row r (dropped when r is past the range).
__device__ __forceinline__ void rows_store4(__amdgpu_buffer_rsrc_t rs, int r, int c, const f32x4& v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rs, (r * L + c) * 4, 0, 0);
}
// The same, nontemporal (aux nt: the policy of stnt4).
__device__ __forceinline__ void rows_store4_nt(__amdgpu_buffer_rsrc_t rs, int r, int c, const f32x4& v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rs, (r * L + c) * 4, 0, 2);
}

// A 16-byte row store with the fragment stores' policy (nontemporal).
__device__ __forceinline__ void stnt4(float* __restrict__ p, const f32x4& x) { st4(p, 0, x); }
// x / den as the reference computes it (models.py LayerNorm: out = x / (std + eps)),
// via the reciprocal and one Newton correction: 3 instructions instead of the
// ~10-instruction IEEE division sequence, within 1 ulp of the quotient.
__device__ __forceinline__ float div_den(float x, float den, float rstd) {
  const float q = x * rstd;
  const float r = fmaf(-q, den, x);
  return fmaf(r, rstd, q);
}

// Copy a 128x128 block W[o][col0 + k] (row stride ld floats) into LDS, row stride WPAD.
__device__ __forceinline__ void load_wblock(float* __restrict__ lds, const float* __restrict__ W,
                                            int ld, int col0) {
  for (int idx = threadIdx.x; idx < 128 * 32; idx += blockDim.x) {
    const int o = idx >> 5, c4 = idx & 31;
    const f32x4 val = *reinterpret_cast<const f32x4*>(W + (size_t)o * ld + col0 + 4 * c4);
    *reinterpret_cast<f32x4*>(lds + o * WPAD + 4 * c4) = val;
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

// A loop-invariant per-feature vector (bias, LayerNorm weight / bias) kept in two
// VGPRs: lane l holds p[l] and p[64 + l].  Chunk T of the fragment layout (features
// 16T + 4q + j of lane quarter q) is fetched with ds_bpermute through the LDS
// crossbar: no LDS allocation and no vector-memory counter, so reading it never
// waits for this wave's outstanding global stores (vmcnt counts loads and stores
// together on CDNA, in issue order).
struct FeatVec {
  float lo, hi;
};
__device__ __forceinline__ FeatVec load_featvec(const float* __restrict__ p) {
  const int l = lane_id();
  return FeatVec{p[l], p[64 + l]};
}
__device__ __forceinline__ f32x4 featvec_chunk(const FeatVec& fv, int T) {
  const int addr = opaque(4 * (16 * (T & 3) + 4 * (lane_id() >> 4)));   // kept inside the tile loop
  const int src = __float_as_int(T < 4 ? fv.lo : fv.hi);
  f32x4 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) r[j] = __int_as_float(__builtin_amdgcn_ds_bpermute(addr + 4 * j, src));
  return r;
}
// acc += W * v over K = 128: 8 input groups t x 4 output-block pairs x 8 MFMAs
// (256 MFMAs).  The A fragments of the next (t, pair) are read from LDS while
// the current pair's 8 MFMAs issue; the two accumulators of a pair alternate so
// each dependent chain has a 64-cycle spacing (> the 40-cycle MFMA latency).
// Scheduling barriers keep the compiler from hoisting all 64 LDS reads.
__device__ __forceinline__ void gemm128(Acc& acc, const float* __restrict__ wl, const float (&v)[FRAG]) {
  const int l = lane_id();
  const float* base = wl + opaque((l & 15) * WPAD + 4 * (l >> 4));
  f32x4 a0[2], a1[2];
  a0[0] = *reinterpret_cast<const f32x4*>(base + 0 * 16 * WPAD);
  a0[1] = *reinterpret_cast<const f32x4*>(base + 1 * 16 * WPAD);
  // A fragment of output block ob, input chunk t: W[16 ob + i][16 t + 4 k .. + 3]
#pragma unroll
  for (int it = 0; it < 32; it += 2) {
    // iteration it: input group t = it >> 2, output-block pair p = it & 3 (blocks 2p, 2p+1)
    {
      const int nt = (it + 1) >> 2, np = (it + 1) & 3;
      a1[0] = *reinterpret_cast<const f32x4*>(base + (2 * np) * 16 * WPAD + 16 * nt);
      a1[1] = *reinterpret_cast<const f32x4*>(base + (2 * np + 1) * 16 * WPAD + 16 * nt);
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
        a0[0] = *reinterpret_cast<const f32x4*>(base + (2 * np) * 16 * WPAD + 16 * nt);
        a0[1] = *reinterpret_cast<const f32x4*>(base + (2 * np + 1) * 16 * WPAD + 16 * nt);
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

#define PDG_GEMM_W2(acc, w, v) gemm128(acc, w, v)

// ----------------------------------------------------------------------------- edge-kernel weights
// The fused edge kernels hold two weights in LDS: Wc (or Wc^T) in fp32 and W2 (or W2^T) as
// three bf16 term planes for the bf16x6 product below; 64 KB + 96 KB = the whole 160 KB,
// so neither image is padded: 16-byte chunks are XOR-swizzled by the row's low 4 bits.
// Both layouts make every ds_read_b128 lane group of the A reads hit 16 distinct slots.
constexpr int EDGE_LDS_BYTES = 128 * 128 * 4 + 3 * 128 * 128 * 2;   // 163,840

// fp32 image, unpadded: element (o, c) at float o*128 + 4*((c >> 2) ^ (o & 15)) + (c & 3).
__device__ __forceinline__ void load_wblock_swz(float* __restrict__ lds, const float* __restrict__ W, int ld,
                                                int col0) {
  for (int idx = threadIdx.x; idx < 128 * 32; idx += blockDim.x) {
    const int o = idx >> 5, c4 = idx & 31;
    const f32x4 val = *reinterpret_cast<const f32x4*>(W + (size_t)o * ld + col0 + 4 * c4);
    *reinterpret_cast<f32x4*>(lds + o * 128 + 4 * (c4 ^ (o & 15))) = val;
  }
}

// gemm128 on the swizzled fp32 image (same MFMA order and pipelining, so the same results).
__device__ __forceinline__ void gemm128_swz(Acc& acc, const float* __restrict__ wl, const float (&v)[FRAG]) {
  const int l = lane_id(), i = l & 15, q = l >> 4;
  // chunk (4t + q) ^ i = 4 (t ^ (i >> 2)) + (q ^ (i & 3))
  const float* base = wl + opaque(i * 128 + 4 * (q ^ (i & 3)));
  const int ti = i >> 2;
  f32x4 a0[2], a1[2];
  a0[0] = *reinterpret_cast<const f32x4*>(base + 0 * 16 * 128 + 16 * (0 ^ ti));
  a0[1] = *reinterpret_cast<const f32x4*>(base + 1 * 16 * 128 + 16 * (0 ^ ti));
#pragma unroll
  for (int it = 0; it < 32; it += 2) {
    {
      const int nt = (it + 1) >> 2, np = (it + 1) & 3;
      a1[0] = *reinterpret_cast<const f32x4*>(base + (2 * np) * 16 * 128 + 16 * (nt ^ ti));
      a1[1] = *reinterpret_cast<const f32x4*>(base + (2 * np + 1) * 16 * 128 + 16 * (nt ^ ti));
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
        a0[0] = *reinterpret_cast<const f32x4*>(base + (2 * np) * 16 * 128 + 16 * (nt ^ ti));
        a0[1] = *reinterpret_cast<const f32x4*>(base + (2 * np + 1) * 16 * 128 + 16 * (nt ^ ti));
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

// bf16x6 product on the matrix cores, fp32 accuracy: W = W0 + W1 + W2 and v = v0 + v1 + v2
// split exactly into bf16 terms (round-to-nearest, 24 significant bits), six products
// Wi vj (i + j <= 2) summed in fp32 smallest first (dropped terms < 2^-24 |W||v|).
// v_mfma_f32_16x16x32_bf16, K chunk m sums the lane's fragment elements v[8m .. 8m+7]
// (features 32m + 4q + {0..3} and 32m + 16 + 4q + {0..3}); the plane images store each
// 32-feature block of a weight row permuted to match: position 8q + 4 half + e.
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void split3_pair_u(float x0, float x1, unsigned& h, unsigned& m, unsigned& lo) {
  h = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2_t){x0, x1}, bf16x2_t));
  const float r0 = x0 - __uint_as_float(h << 16), r1 = x1 - __uint_as_float(h & 0xffff0000u);
  m = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2_t){r0, r1}, bf16x2_t));
  const float q0 = r0 - __uint_as_float(m << 16), q1 = r1 - __uint_as_float(m & 0xffff0000u);
  lo = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2_t){q0, q1}, bf16x2_t));
}

constexpr int PLANE_BYTES = 128 * 128 * 2;

// Byte offset of weight (o, f) in a plane image.
__device__ __forceinline__ int plane_off(int o, int f) {
  const int m = f >> 5, fl = f & 31, half = fl >> 4, qq = (fl & 15) >> 2, e = fl & 3;
  const int chunk = 4 * m + qq;
  return o * 256 + 16 * (chunk ^ (o & 15)) + 2 * (4 * half + e);
}

// Build the three term planes of W[o][col0 + f] (row stride ld) at `planes` (bytes).
__device__ __forceinline__ void load_wplanes(unsigned char* __restrict__ planes, const float* __restrict__ W,
                                             int ld, int col0) {
  for (int idx = threadIdx.x; idx < 128 * 64; idx += blockDim.x) {
    const int o = idx >> 6, f = 2 * (idx & 63);   // features f, f + 1 (same chunk, adjacent positions)
    const float* wr = W + (size_t)o * ld + col0 + f;
    unsigned h, m, lo;
    split3_pair_u(wr[0], wr[1], h, m, lo);
    const int off = plane_off(o, f);
    *reinterpret_cast<unsigned*>(planes + off) = h;
    *reinterpret_cast<unsigned*>(planes + PLANE_BYTES + off) = m;
    *reinterpret_cast<unsigned*>(planes + 2 * PLANE_BYTES + off) = lo;
  }
}

__device__ __forceinline__ void gemm128_x6(Acc& acc, const unsigned char* __restrict__ planes,
                                           const float (&v)[FRAG]) {
  const int l = lane_id(), i = l & 15, q = l >> 4;
  // chunk (4m + q) ^ i = 4 (m ^ (i >> 2)) + (q ^ (i & 3))
  const unsigned char* base = planes + opaque(i * 256 + 16 * (q ^ (i & 3)));
  const int mi = i >> 2;
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    unsigned h[4], md[4], lo[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) split3_pair_u(v[8 * m + 2 * p], v[8 * m + 2 * p + 1], h[p], md[p], lo[p]);
    const bf16x8_t B0 = __builtin_bit_cast(bf16x8_t, (u32x4_t){h[0], h[1], h[2], h[3]});
    const bf16x8_t B1 = __builtin_bit_cast(bf16x8_t, (u32x4_t){md[0], md[1], md[2], md[3]});
    const bf16x8_t B2 = __builtin_bit_cast(bf16x8_t, (u32x4_t){lo[0], lo[1], lo[2], lo[3]});
    const int co = 64 * (m ^ mi);
#pragma unroll
    for (int pr = 0; pr < 4; ++pr) {   // output blocks 2pr, 2pr+1: two independent chains
      bf16x8_t A[2][3];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const unsigned char* a = base + (2 * pr + u) * 16 * 256 + co;
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) A[u][pl] = *reinterpret_cast<const bf16x8_t*>(a + pl * PLANE_BYTES);
      }
      f32x4 t0 = acc.b[2 * pr], t1 = acc.b[2 * pr + 1];
      t0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[0][2], B0, t0, 0, 0, 0);
      t1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[1][2], B0, t1, 0, 0, 0);
      t0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[0][1], B1, t0, 0, 0, 0);
      t1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[1][1], B1, t1, 0, 0, 0);
      t0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[0][0], B2, t0, 0, 0, 0);
      t1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[1][0], B2, t1, 0, 0, 0);
      t0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[0][1], B0, t0, 0, 0, 0);
      t1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[1][1], B0, t1, 0, 0, 0);
      t0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[0][0], B1, t0, 0, 0, 0);
      t1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[1][0], B1, t1, 0, 0, 0);
      acc.b[2 * pr] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[0][0], B0, t0, 0, 0, 0);
      acc.b[2 * pr + 1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[1][0], B0, t1, 0, 0, 0);
      PDG_FENCE();
    }
  }
}

// ----------------------------------------------------------------------------- fragment I/O
__device__ __forceinline__ void load_frag(float (&v)[FRAG], const float* __restrict__ row) {
  const float* p = row + lane_col();
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const f32x4 x = ld4(p, t);
    v[4 * t + 0] = x[0]; v[4 * t + 1] = x[1]; v[4 * t + 2] = x[2]; v[4 * t + 3] = x[3];
  }
}

__device__ __forceinline__ void store_frag(float* __restrict__ row, const float (&v)[FRAG]) {
  float* p = row + lane_col();
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    f32x4 x; x[0] = v[4 * t]; x[1] = v[4 * t + 1]; x[2] = v[4 * t + 2]; x[3] = v[4 * t + 3];
    st4(p, t, x);
  }
}

__device__ __forceinline__ void store_acc(float* __restrict__ row, const Acc& acc) {
  float* p = row + lane_col();
#pragma unroll
  for (int t = 0; t < 8; ++t) st4(p, t, acc.b[t]);
}

// ----------------------------------------------------------------------------- reductions
__device__ __forceinline__ double wave_sum(double x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  return x;
}

// ----------------------------------------------------------------------------- LayerNorm backward
// scalars without finalize launches.  The backward of the graph LayerNorm y = xhat*g + b needs
// per-channel sums over all rows of gy and gy*xhat (the g / b gradients) and two scalars
// S1 = sum_c g_c sum gy_c, S2 = sum_c g_c sum (gy xhat)_c for the input gradient.  Each producer
// block emits its column-partial row (256 doubles, added into a per-block accumulator that spans
// all message-passing steps; pdg_ln_param_grads reduces it once) and its own pair
// (sum_c g_c row_c, sum_c g_c row_128+c).  The consumer reduces the <= MAX_BLOCKS pairs itself
// (lnb_resolve), so no launch sits between producer and consumer.

// All threads of the block (>= 128) call this with the block's complete row in LDS; `tmp` is a
// 256-double LDS scratch.  accumulate ? part[b] += row : part[b] = row; sp[b] = the pair.
__device__ __forceinline__ void lnb_emit(const double* row, const float* __restrict__ g, double* __restrict__ part,
                                         int accumulate, double* __restrict__ sp, double* tmp) {
  const int t = threadIdx.x, b = blockIdx.x;
  for (int i = t; i < 256; i += blockDim.x) {
    double* dst = part + (size_t)b * 256 + i;
    *dst = accumulate ? *dst + row[i] : row[i];
  }
  if (sp == nullptr) return;
  if (t < 128) {
    tmp[t] = (double)g[t] * row[t];
    tmp[128 + t] = (double)g[t] * row[128 + t];
  }
  __syncthreads();
  for (int o = 64; o > 0; o >>= 1) {
    if (t < o) {
      tmp[t] += tmp[t + o];
      tmp[128 + t] += tmp[128 + t + o];
    }
    __syncthreads();
  }
  if (t == 0) {
    sp[2 * b] = tmp[0];
    sp[2 * b + 1] = tmp[128];
  }
}

// The backward scalars of one LayerNorm call: *lbp (precomputed), or, when sp != NULL, from the
// producers' np pairs.  Every wave computes them with the same lane order and xor butterfly (float
// addition commutes, so all lanes of all waves of all blocks get bit-identical values).
__device__ __forceinline__ pdg_ln_bwd lnb_resolve(const pdg_ln_bwd* __restrict__ lbp, const double* __restrict__ sp,
                                                  int np, const pdg_ln_stat* __restrict__ stp) {
  if (sp == nullptr) return *lbp;
  double s1 = 0, s2 = 0;
  for (int b = lane_id(); b < np; b += 64) {
    const double2 v = reinterpret_cast<const double2*>(sp)[b];
    s1 += v.x;
    s2 += v.y;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s1 += __shfl_xor(s1, o);
    s2 += __shfl_xor(s2, o);
  }
  const double M = stp->count, sd = stp->std_d;
  pdg_ln_bwd r;
  r.S1 = s1;
  r.S2 = s2;
  r.c1 = (float)(s1 / M);
  r.c2 = sd > 0 ? (float)(s2 / (M * sd)) : 0.f;
  return r;
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

// Graph-LayerNorm statistics from per-block (sum, sumsq) partials in the fixed pdg_ln_finalize
// order: threads 0..255 accumulate strided by 256, waves beyond the fourth add +0, so any block of
// >= 256 threads gives bit-identical statistics.  Thread 0 writes *out (global or LDS).
__device__ __forceinline__ void ln_stat_from_partials(const double* __restrict__ part, int n, double count,
                                                      pdg_ln_stat* out, double* red) {
  double a = 0, b = 0;
  if (threadIdx.x < 256)
    for (int i = threadIdx.x; i < n; i += 256) { a += part[2 * i]; b += part[2 * i + 1]; }
  block_sum2(a, b, red);
  if (threadIdx.x == 0) {
    const double mean = a / count;
    double var = b / count - mean * mean;
    if (var < 0) var = 0;
    const double sd = sqrt(var);
    pdg_ln_stat s;
    s.mean = (float)mean;
    s.std_ = (float)sd;
    s.den = s.std_ + LN_EPS;
    s.rstd = 1.0f / s.den;
    s.mean_d = mean;
    s.std_d = sd;
    s.count = count;
    *out = s;
  }
}

}  // namespace pdg
