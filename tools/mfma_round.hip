// Rounding of the MFMA accumulation on gfx950 (diagnostic, tools/mfma_round.py): D = A B + C for
// one 16x16 tile per wave, bf16 inputs (v_mfma_f32_16x16x32_bf16) or fp32 inputs
// (v_mfma_f32_16x16x4_f32), written out for comparison with the exactly rounded fp64 result.
//   hipcc -O3 --offload-arch=gfx950 -shared -fPIC tools/mfma_round.hip -o tools/_mfma_round.so
#include <hip/hip_runtime.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// A: ntiles x 16 x 32 bf16 (row-major, row = output row m, col = k); B: ntiles x 32 x 16 (k, n);
// C, D: ntiles x 16 x 16 fp32.  Lane l holds A[m = l & 15][k = 8 (l >> 4) .. +7], B[k = 8 (l >> 4) ..][n = l & 15]
// and D[m = 4 (l >> 4) + j][n = l & 15].
__global__ void mfma_bf16_kernel(const __bf16* A, const __bf16* B, const float* C, float* D) {
  const int t = blockIdx.x, l = threadIdx.x;
  const __bf16* a = A + (size_t)t * 512 + (l & 15) * 32 + 8 * (l >> 4);
  bf16x8 av, bv;
  for (int i = 0; i < 8; ++i) {
    av[i] = a[i];
    bv[i] = B[(size_t)t * 512 + (8 * (l >> 4) + i) * 16 + (l & 15)];
  }
  f32x4 c;
  for (int j = 0; j < 4; ++j) c[j] = C[(size_t)t * 256 + (4 * (l >> 4) + j) * 16 + (l & 15)];
  const f32x4 d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, c, 0, 0, 0);
  for (int j = 0; j < 4; ++j) D[(size_t)t * 256 + (4 * (l >> 4) + j) * 16 + (l & 15)] = d[j];
}

// A: ntiles x 16 x 4 fp32, B: ntiles x 4 x 16; lane l holds A[l & 15][l >> 4], B[l >> 4][l & 15].
__global__ void mfma_f32_kernel(const float* A, const float* B, const float* C, float* D) {
  const int t = blockIdx.x, l = threadIdx.x;
  const float av = A[(size_t)t * 64 + (l & 15) * 4 + (l >> 4)];
  const float bv = B[(size_t)t * 64 + (l >> 4) * 16 + (l & 15)];
  f32x4 c;
  for (int j = 0; j < 4; ++j) c[j] = C[(size_t)t * 256 + (4 * (l >> 4) + j) * 16 + (l & 15)];
  const f32x4 d = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, c, 0, 0, 0);
  for (int j = 0; j < 4; ++j) D[(size_t)t * 256 + (4 * (l >> 4) + j) * 16 + (l & 15)] = d[j];
}

extern "C" int mfma_round_bf16(int ntiles, const void* A, const void* B, const float* C, float* D) {
  hipLaunchKernelGGL(mfma_bf16_kernel, dim3(ntiles), dim3(64), 0, 0, (const __bf16*)A, (const __bf16*)B, C, D);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}

extern "C" int mfma_round_f32(int ntiles, const float* A, const float* B, const float* C, float* D) {
  hipLaunchKernelGGL(mfma_f32_kernel, dim3(ntiles), dim3(64), 0, 0, A, B, C, D);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}

// ---- fp32-accurate products over K = 128 (one 16x16 tile per wave; A: 16 x 128, B: 128 x 16, fp32)
// mode 0: bf16x6, one accumulation chain through all six products of every K chunk (gemm_round's order)
// mode 1: bf16x6, per K chunk the five small products chained from zero and hi*hi from zero, added to
//         the running sum by fp32 VALU adds (round-to-nearest-even)
// mode 2: bf16x9 (all nine products), one chain
// mode 3: fp32 MFMA 16x16x4, one chain
#include "pdg_x6.hpp"
using namespace pdg;

__device__ __forceinline__ void split8(const float* p, bf16x8 (&t)[3]) {
  unsigned h[4], m[4], lo[4];
  for (int i = 0; i < 4; ++i) split3_pair(p[2 * i], p[2 * i + 1], h[i], m[i], lo[i]);
  t[0] = __builtin_bit_cast(bf16x8, (u32x4){h[0], h[1], h[2], h[3]});
  t[1] = __builtin_bit_cast(bf16x8, (u32x4){m[0], m[1], m[2], m[3]});
  t[2] = __builtin_bit_cast(bf16x8, (u32x4){lo[0], lo[1], lo[2], lo[3]});
}

__global__ void x6_chain_kernel(const float* A, const float* B, float* D, int mode) {
  const int t = blockIdx.x, l = threadIdx.x;
  const float* a = A + (size_t)t * 2048;   // 16 x 128
  const float* b = B + (size_t)t * 2048;   // 128 x 16
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
  if (mode == 3) {
    for (int s = 0; s < 32; ++s) {
      const int k = 4 * s + (l >> 4);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[(l & 15) * 128 + k], b[k * 16 + (l & 15)], acc, 0, 0, 0);
    }
  } else {
    for (int ks = 0; ks < 4; ++ks) {
      float av[8], bv[8];
      for (int i = 0; i < 8; ++i) {
        const int k = 32 * ks + 8 * (l >> 4) + i;
        av[i] = a[(l & 15) * 128 + k];
        bv[i] = b[k * 16 + (l & 15)];
      }
      bf16x8 A3[3], B3[3];
      split8(av, A3);
      split8(bv, B3);
      if (mode == 0 || mode == 2) {
        f32x4 x = acc;
        if (mode == 2) {
          x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A3[2], B3[2], x, 0, 0, 0);
          x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A3[1], B3[2], x, 0, 0, 0);
          x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A3[2], B3[1], x, 0, 0, 0);
        }
        x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A3[2], B3[0], x, 0, 0, 0);
        x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A3[1], B3[1], x, 0, 0, 0);
        x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A3[0], B3[2], x, 0, 0, 0);
        x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A3[1], B3[0], x, 0, 0, 0);
        x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A3[0], B3[1], x, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A3[0], B3[0], x, 0, 0, 0);
      } else {
        f32x4 s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A3[2], B3[0], z, 0, 0, 0);
        s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A3[1], B3[1], s, 0, 0, 0);
        s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A3[0], B3[2], s, 0, 0, 0);
        s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A3[1], B3[0], s, 0, 0, 0);
        s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A3[0], B3[1], s, 0, 0, 0);
        const f32x4 h = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A3[0], B3[0], z, 0, 0, 0);
        for (int j = 0; j < 4; ++j) acc[j] = acc[j] + (h[j] + s[j]);
      }
    }
  }
  for (int j = 0; j < 4; ++j) D[(size_t)t * 256 + (4 * (l >> 4) + j) * 16 + (l & 15)] = acc[j];
}

extern "C" int x6_chain(int ntiles, const float* A, const float* B, float* D, int mode) {
  hipLaunchKernelGGL(x6_chain_kernel, dim3(ntiles), dim3(64), 0, 0, A, B, D, mode);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
