// bf16x6 row images in LDS (shared by the weight-gradient passes, pdg_wgrad.hip and
// pdg_ebw.hip): 32 rows x 128 features of fp32 data split exactly into three bf16 terms,
// each term a row-major [32][256 B] image with XOR-swizzled 16-B chunks, read either
// transposed (ds_read_b64_tr_b16: 8 consecutive rows of one column per lane, the
// operand of a K = rows product) or straight (16 B of one row: 8 consecutive features).
#pragma once
#include "pdg_common.hpp"

namespace pdg {

typedef float f32x16 __attribute__((ext_vector_type(16)));   // 32x32 MFMA accumulator
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

constexpr int X6_ROWS = 32;                       // rows staged per round
constexpr int X6_ROWB = 256;                      // bytes per row of one term image
constexpr int X6_TERM = X6_ROWS * X6_ROWB;        // bytes per term image (8 KB)

// Byte address of byte `b` (0..255) of image row `r`: 16-B chunk index XOR (4 (r & 3) + t((r >> 2) & 3)).
// (measured: 1.9e7 -> 0 LDS bank-conflict cycles per edge_bwd_w2 launch with the mask stride below,
// bitwise the same results, time unchanged within noise; the transposed reads stay conflict free)
__device__ __forceinline__ int x6_addr(int r, int b) {
  // t = (0, 2, 3, 1): the straight 16-B operand reads of the edge backward (row = lane & 15,
  // chunk + (lane >> 4)) then hit 16 distinct chunks in every ds_read_b128 lane group
  const int t = (0x78 >> (2 * ((r >> 2) & 3))) & 3;
  return r * X6_ROWB + (b ^ (((r & 3) << 6) | (t << 4)));
}

// (x0, x1) = hi + mid + lo exactly, per element: bf16 round-to-nearest-even of x, of the
// remainder and of the rest, two elements per v_cvt_pk_bf16_f32 (a bf16 widens to float by
// a 16-bit shift); each term comes out as a packed pair (x0 in the low half).
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void split3_pair(float x0, float x1, unsigned& h, unsigned& m, unsigned& lo) {
  h = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){x0, x1}, bf16x2));
  const float r0 = x0 - __uint_as_float(h << 16), r1 = x1 - __uint_as_float(h & 0xffff0000u);
  m = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){r0, r1}, bf16x2));
  const float q0 = r0 - __uint_as_float(m << 16), q1 = r1 - __uint_as_float(m & 0xffff0000u);
  lo = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){q0, q1}, bf16x2));
}

// MFMA operand of columns col0 + (l & 31), rows 16 ks + 8 (l >> 5) + 0..7, from term image `img`:
// two transposed reads of 4 rows each, at the lane's addresses ofs0 / ofs1 (row
// 16 ks + 8 (l >> 5) + ((l & 15) >> 2) [+ 4], columns col0 + 16 ((l >> 4) & 1) + 4 (l & 3) .. +3).
__device__ __forceinline__ bf16x8 x6_operand(const unsigned char* img, int ofs0, int ofs1) {
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + ofs0));
  const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + ofs1));
  s16x4 v0 = a, v1 = b;
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 r = s16x8{v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
  return __builtin_bit_cast(bf16x8, r);
}

// A operand of rows 16w .. 16w+15 of a 128x128 matrix WT (o' x k, row-major), K chunk ks
// (k = 32 ks + 8 (l >> 4) + 0..7), three bf16 terms.
struct WSlice {
  bf16x8 a[4][3];
};

__device__ __forceinline__ void load_wslice(WSlice& ws, const float* __restrict__ WT, int w, int ld = L) {
  const int l = lane_id();
  const float* row = WT + (size_t)(16 * w + (l & 15)) * ld + 8 * (l >> 4);
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const f32x4 x0 = *reinterpret_cast<const f32x4*>(row + 32 * ks);
    const f32x4 x1 = *reinterpret_cast<const f32x4*>(row + 32 * ks + 4);
    unsigned h[4], m[4], lo[4];
    split3_pair(x0[0], x0[1], h[0], m[0], lo[0]);
    split3_pair(x0[2], x0[3], h[1], m[1], lo[1]);
    split3_pair(x1[0], x1[1], h[2], m[2], lo[2]);
    split3_pair(x1[2], x1[3], h[3], m[3], lo[3]);
    ws.a[ks][0] = __builtin_bit_cast(bf16x8, (u32x4){h[0], h[1], h[2], h[3]});
    ws.a[ks][1] = __builtin_bit_cast(bf16x8, (u32x4){m[0], m[1], m[2], m[3]});
    ws.a[ks][2] = __builtin_bit_cast(bf16x8, (u32x4){lo[0], lo[1], lo[2], lo[3]});
  }
}

// d[nb] += (W^T-slice x rows 16 nb .. 16 nb + 15 of a straight-read image), the layout of pdg_ebw.hip's
// gemm_round (D row = output feature 16w + 4 (l >> 4) + j, column = image row 16 nb + (l & 15)), with an
// UNBIASED accumulation: per 32-wide K chunk the five small products are chained from zero and hi x hi
// is formed from zero, and both are added to d by fp32 VALU adds.  The bf16 MFMA adds its accumulator
// input with a rounding biased by about -6e-10 of the magnitude (tools/mfma_round.py); formed from zero
// it is unbiased, and over K = 128 this scheme measured a mean error of -2.7e-11 of the product scale
// (fp32 MFMA chain: -2.9e-11; one bf16x6 chain: -1.1e-9) at 3.6x less rms error than the fp32 MFMA
// chain.  Six bf16 MFMAs per chunk cost 2.7x less matrix time than the fp32 MFMAs of the same K.
// CHAIN: the five small products of all four K chunks in ONE chain (its accumulator bias is relative to
// the small terms, 2^-8 of the product) added to d once at the end, hi x hi still from zero per chunk:
// one VALU add per element and chunk instead of two.  node_net: 37.2-37.7 -> 33.9-34.4 us per config-2
// call (two same-box A/B pairs; op tests against fp64 with the bias check green); node_pq measured
// 26.7-26.9 -> 28.0-28.4 us with it and keeps the per-chunk form.
template <int NB, int TERM, bool CHAIN = false>
__device__ __forceinline__ void gemm_x6f(f32x4 (&d)[NB], const WSlice& ws, const unsigned char* img) {
  const int l = lane_id(), n = l & 15, kg = l >> 4;
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
  f32x4 smc[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) smc[nb] = z;
#pragma unroll
  for (int ks = 0; ks < 4; ++ks)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const int off = x6_addr(16 * nb + n, 64 * ks + 16 * kg);
      bf16x8 B[3];
#pragma unroll
      for (int p = 0; p < 3; ++p) B[p] = *reinterpret_cast<const bf16x8*>(img + p * TERM + off);
      if (CHAIN) {
        f32x4 t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ws.a[ks][2], B[0], smc[nb], 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ws.a[ks][1], B[1], t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ws.a[ks][0], B[2], t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ws.a[ks][1], B[0], t, 0, 0, 0);
        smc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ws.a[ks][0], B[1], t, 0, 0, 0);
        const f32x4 hh = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ws.a[ks][0], B[0], z, 0, 0, 0);
#pragma unroll
        for (int j = 0; j < 4; ++j) d[nb][j] += hh[j];
        continue;
      }
      f32x4 sm = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ws.a[ks][2], B[0], z, 0, 0, 0);
      sm = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ws.a[ks][1], B[1], sm, 0, 0, 0);
      sm = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ws.a[ks][0], B[2], sm, 0, 0, 0);
      sm = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ws.a[ks][1], B[0], sm, 0, 0, 0);
      sm = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ws.a[ks][0], B[1], sm, 0, 0, 0);
      const f32x4 hh = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ws.a[ks][0], B[0], z, 0, 0, 0);
#pragma unroll
      for (int j = 0; j < 4; ++j) d[nb][j] += hh[j] + sm[j];
    }
  if (CHAIN)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) d[nb] += smc[nb];
}

// Columns 4cg .. 4cg+3 of image row r, split into the three terms (term planes TERM bytes apart).
template <int TERM>
__device__ __forceinline__ void x6_store4(unsigned char* img, int r, int cg, const f32x4& v) {
  unsigned h0, m0, l0, h1, m1, l1;
  split3_pair(v[0], v[1], h0, m0, l0);
  split3_pair(v[2], v[3], h1, m1, l1);
  const int off = x6_addr(r, 8 * cg);
  *reinterpret_cast<u32x2*>(img + off) = u32x2{h0, h1};
  *reinterpret_cast<u32x2*>(img + TERM + off) = u32x2{m0, m1};
  *reinterpret_cast<u32x2*>(img + 2 * TERM + off) = u32x2{l0, l1};
}

}  // namespace pdg
