// Fused node_net of one message-passing step (models.py:240-243: update =
// node_net(cat[aggr, x]) = Linear(256->128) ReLU Linear(128->128) ReLU, plus
// the LayerNorm partials of the output); aggr comes from pdg_segment_sum.
//
// Node rows are few (N ~ E/6): the separate layer kernels ran one 16-row tile
// per wave and were dominated by launch fill/drain and exposed load latency.
// Here the weights are STATIONARY IN REGISTERS instead of LDS: a block has 8
// compute waves, wave w owns output features [16w, 16w+16) of both layers and
// keeps its 16 rows of W1 (16 x 256) and W2 (16 x 128) as MFMA A fragments
// (96 VGPRs).  Activations pass through LDS: a tile of 16 nodes' [aggr | x]
// rows (the B operand, read with ds_read_b128), then the layer-1 output tile.
// Four loader waves stream the NEXT tile's [aggr | x] rows (coalesced 1-KB
// wave loads) into a second buffer while the compute waves run the current one.
//
// MFMA (v_mfma_f32_16x16x4_f32): step (T, j) sums inputs 16T + 4k + j (k = lane
// quarter), exactly the order of gemm128, so a1/a2 are bitwise those of the
// separate pdg_node_mlp1 / pdg_mlp2_fwd kernels.
#include "pdg_common.hpp"
#include "pdg_runtime.hpp"

using namespace pdg;

namespace {

constexpr int NU_COMPUTE = 8;                 // compute waves (16 output features each)
constexpr int NU_LOADERS = 4;                 // loader waves
constexpr int NU_THREADS = 64 * (NU_COMPUTE + NU_LOADERS);
constexpr int XS = 2 * L + 8;                 // [aggr | x] tile row stride (floats): 264 = 8 mod 64 dwords
constexpr int AS = L + 8;                     // layer-1 tile row stride: 136
constexpr int XBUF = TILE * XS;               // floats per [aggr | x] buffer

// Loader waves (256 lanes): copy rows 16 t .. 16 t + 15 of aggr and x into the
// tile buffer; lane (row lr = lane >> 5 (+8), chunk j = lane & 31), 4 independent
// 16-B loads per lane.  Rows past N are zero.
__device__ __forceinline__ void load_tile(float* __restrict__ xb, int t, int N, int lt,
                                          const float* __restrict__ aggr, const float* __restrict__ x) {
  const int j = lt & 31, lr = lt >> 5;
  f32x4 v[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int r = lr + 8 * (u >> 1), node = t * TILE + r;
    const float* src = (u & 1) ? x : aggr;
    v[u] = node < N ? reinterpret_cast<const f32x4*>(src + (size_t)node * L)[j] : f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int r = lr + 8 * (u >> 1);
    *reinterpret_cast<f32x4*>(xb + r * XS + (u & 1) * L + 4 * j) = v[u];
  }
}

__device__ __forceinline__ int nu_tile(int i) { return xcd_block() + i * (int)gridDim.x; }

}  // namespace

__global__ __launch_bounds__(NU_THREADS, 1) void node_net_kernel(
    int N, const float* __restrict__ aggr, const float* __restrict__ x, const float* __restrict__ W1,
    const float* __restrict__ b1, const float* __restrict__ W2, const float* __restrict__ b2,
    float* __restrict__ a1_out, float* __restrict__ a2_out, double* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) float xin[2 * XBUF];
  __shared__ __attribute__((aligned(16))) float a1t[TILE * AS];
  const int w = wave_id(), l = lane_id();
  const bool loader = w >= NU_COMPUTE;
  const int ntiles = tiles_of(N);
  const int lt = threadIdx.x - 64 * NU_COMPUTE;   // loader lane
  // compute state: lane row r = l & 15, quarter q = l >> 4; weights of output rows 16w + (l & 15)
  const int r = l & 15, q = l >> 4;
  f32x4 w1f[16], w2f[8];
  if (!loader) {
    const float* w1r = W1 + (size_t)(16 * w + r) * (2 * L) + 4 * q;
    const float* w2r = W2 + (size_t)(16 * w + r) * L + 4 * q;
#pragma unroll
    for (int T = 0; T < 16; ++T) w1f[T] = *reinterpret_cast<const f32x4*>(w1r + 16 * T);
#pragma unroll
    for (int T = 0; T < 8; ++T) w2f[T] = *reinterpret_cast<const f32x4*>(w2r + 16 * T);
  }
  double s1 = 0, s2 = 0;
  if (loader && nu_tile(0) < ntiles) load_tile(xin, nu_tile(0), N, lt, aggr, x);
  __syncthreads();
  for (int i = 0;; ++i) {
    const int tile = nu_tile(i);
    if (tile >= ntiles) break;   // uniform across the block
    const float* xb = xin + (i & 1) * XBUF;
    const int row = tile * TILE + r;
    const bool valid = row < N;
    f32x4 a1 = {0.f, 0.f, 0.f, 0.f};
    if (loader) {
      const int nt = nu_tile(i + 1);
      if (nt < ntiles) load_tile(xin + ((i + 1) & 1) * XBUF, nt, N, lt, aggr, x);
    } else {
      // layer 1: a1 = relu(W1 [aggr | x] + b1), K = 256
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      const float* xr = xb + r * XS + 4 * q;
#pragma unroll
      for (int T = 0; T < 16; ++T) {
        const f32x4 bv = *reinterpret_cast<const f32x4*>(xr + 16 * T);
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(w1f[T][jj], bv[jj], acc, 0, 0, 0);
      }
      const f32x4 bias1 = *reinterpret_cast<const f32x4*>(b1 + 16 * w + 4 * q);
#pragma unroll
      for (int c = 0; c < 4; ++c) a1[c] = fmaxf(acc[c] + bias1[c], 0.f);
      // D row 4q + c of this wave's block = feature 16w + 4q + c of node row r
      *reinterpret_cast<f32x4*>(a1t + r * AS + 16 * w + 4 * q) = a1;
      if (valid && a1_out) *reinterpret_cast<f32x4*>(a1_out + (size_t)row * L + 16 * w + 4 * q) = a1;
    }
    __syncthreads();
    if (!loader) {
      // layer 2: a2 = relu(W2 a1 + b2) + LayerNorm partials
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      const float* ar = a1t + r * AS + 4 * q;
#pragma unroll
      for (int T = 0; T < 8; ++T) {
        const f32x4 bv = *reinterpret_cast<const f32x4*>(ar + 16 * T);
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(w2f[T][jj], bv[jj], acc, 0, 0, 0);
      }
      const f32x4 bias2 = *reinterpret_cast<const f32x4*>(b2 + 16 * w + 4 * q);
      f32x4 a2;
#pragma unroll
      for (int c = 0; c < 4; ++c) a2[c] = fmaxf(acc[c] + bias2[c], 0.f);
      if (valid) {
        *reinterpret_cast<f32x4*>(a2_out + (size_t)row * L + 16 * w + 4 * q) = a2;
        const float p1 = (a2[0] + a2[1]) + (a2[2] + a2[3]);
        const float p2 = (a2[0] * a2[0] + a2[1] * a2[1]) + (a2[2] * a2[2] + a2[3] * a2[3]);
        s1 += (double)p1;
        s2 += (double)p2;
      }
    }
    __syncthreads();
  }
  __shared__ double red[2 * (NU_THREADS / 64)];
  block_sum2(s1, s2, red);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = s1;
    part[2 * blockIdx.x + 1] = s2;
  }
}

extern "C" int pdg_node_net(int n_nodes, const float* aggr, const float* x, const float* Wn1, const float* bn1,
                            const float* Wn2, const float* bn2, float* a1n, float* a2n, double* partials,
                            int* nparts, void* stream) {
  PDG_CHECK_ARG(n_nodes > 0, "pdg_node_net: n_nodes must be > 0");
  PDG_CHECK_ARG(aggr && x && a2n, "pdg_node_net: aggr, x and a2n are required");
  PDG_CHECK_ARG(PDG_ALIGNED(aggr) && PDG_ALIGNED(x) && PDG_ALIGNED(Wn1) && PDG_ALIGNED(Wn2) && PDG_ALIGNED(a2n) &&
                    PDG_ALIGNED(a1n) && PDG_ALIGNED(bn1) && PDG_ALIGNED(bn2),
                "pdg_node_net: misaligned pointer");
  const int tiles = tiles_of(n_nodes);
  const int cap = device_cus() < MAX_BLOCKS ? device_cus() : MAX_BLOCKS;
  const int grid = tiles < cap ? tiles : cap;
  hipLaunchKernelGGL(node_net_kernel, dim3(grid), dim3(NU_THREADS), 0, (hipStream_t)stream, n_nodes, aggr, x, Wn1,
                     bn1, Wn2, bn2, a1n, a2n, partials);
  PDG_CHECK_LAUNCH("pdg_node_net");
  if (nparts) *nparts = grid;
  return PDG_OK;
}
