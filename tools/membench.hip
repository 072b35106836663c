// Streaming-bandwidth probe for the access shapes of the edge kernels (not part of the
// library): R arrays read and W arrays written, E rows of 512 B each, one persistent
// block per CU (512 threads), rounds of 32 rows.  Shapes:
//   rowmajor: a wave instruction covers 2 whole rows (64 lanes x 16 B)
//   dlayout:  a wave instruction covers 16 rows x 64 B (the 16x16 MFMA output layout)
// Prints GB/s for each (shape, R, W).  Build: hipcc -O3 --offload-arch=gfx950 -o membench membench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int L = 128;

template <int R, int W, bool DL>
__global__ __launch_bounds__(512, 1) void probe(const float* const* __restrict__ in, float* const* __restrict__ out,
                                                int E) {
  const int nb = gridDim.x;
  int per = (E + nb - 1) / nb;
  per = (per + 31) / 32 * 32;
  const int r0 = min(E, per * (int)blockIdx.x), r1 = min(E, per * ((int)blockIdx.x + 1));
  const int t = threadIdx.x, l = t & 63, w = t >> 6;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int base = r0; base < r1; base += 32) {
    f32x4 v[R][2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      int row, col;
      if (DL) {   // wave w: rows 16u + (l & 15), features 16w + 4(l >> 4)
        row = base + 16 * u + (l & 15);
        col = 16 * w + 4 * (l >> 4);
      } else {    // thread t: row (t >> 5) + 16u, features 4 (t & 31)
        row = base + (t >> 5) + 16 * u;
        col = 4 * (t & 31);
      }
      row = row < r1 ? row : r1 - 1;
#pragma unroll
      for (int a = 0; a < R; ++a) v[a][u] = *reinterpret_cast<const f32x4*>(in[a] + (size_t)row * L + col);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int a = 0; a < R; ++a) acc += v[a][u];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      int row, col;
      if (DL) {
        row = base + 16 * u + (l & 15);
        col = 16 * w + 4 * (l >> 4);
      } else {
        row = base + (t >> 5) + 16 * u;
        col = 4 * (t & 31);
      }
      if (row < r1)
#pragma unroll
        for (int a = 0; a < W; ++a) *reinterpret_cast<f32x4*>(out[a] + (size_t)row * L + col) = acc + (float)a;
    }
  }
}

template <int R, int W, bool DL>
void run(int E, float** d_in, float** d_out, int cus) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int it = 0; it < 3; ++it) hipLaunchKernelGGL((probe<R, W, DL>), dim3(cus), dim3(512), 0, 0, d_in, d_out, E);
  (void)hipEventRecord(a);
  const int reps = 20;
  for (int it = 0; it < reps; ++it) hipLaunchKernelGGL((probe<R, W, DL>), dim3(cus), dim3(512), 0, 0, d_in, d_out, E);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  const double bytes = (double)E * 512.0 * (R + W);
  printf("{\"shape\": \"%s\", \"reads\": %d, \"writes\": %d, \"us\": %.1f, \"GBps\": %.0f}\n", DL ? "dlayout" : "rowmajor",
         R, W, ms / reps * 1e3, bytes / (ms / reps * 1e-3) / 1e9);
}

int main() {
  const int E = 241920;
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  std::vector<float*> bufs(16);
  for (auto& p : bufs) {
    (void)hipMalloc(&p, (size_t)E * 512);
    (void)hipMemset(p, 0, (size_t)E * 512);
  }
  float **d_in, **d_out;
  (void)hipMalloc(&d_in, 8 * sizeof(float*));
  (void)hipMalloc(&d_out, 8 * sizeof(float*));
  (void)hipMemcpy(d_in, bufs.data(), 8 * sizeof(float*), hipMemcpyHostToDevice);
  (void)hipMemcpy(d_out, bufs.data() + 8, 8 * sizeof(float*), hipMemcpyHostToDevice);
  run<1, 1, false>(E, d_in, d_out, cus);
  run<5, 3, false>(E, d_in, d_out, cus);
  run<5, 3, true>(E, d_in, d_out, cus);
  run<8, 0, false>(E, d_in, d_out, cus);
  run<1, 7, false>(E, d_in, d_out, cus);
  run<1, 7, true>(E, d_in, d_out, cus);
  run<3, 1, false>(E, d_in, d_out, cus);
  run<3, 1, true>(E, d_in, d_out, cus);
  run<4, 4, false>(E, d_in, d_out, cus);
  return 0;
}
