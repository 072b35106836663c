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
