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
#include "pdg_x6.hpp"

using namespace pdg;

namespace {

constexpr int NU_COMPUTE = 8;                 // compute waves (16 output features each)
constexpr int NU_LOADERS = 4;                 // loader waves
constexpr int NU_THREADS = 64 * (NU_COMPUTE + NU_LOADERS);
constexpr int XS = 2 * L + 8;                 // [aggr | x] tile row stride (floats): 264 = 8 mod 64 dwords
constexpr int AS = L + 8;                     // layer-1 tile row stride: 136
constexpr int XBUF = TILE * XS;               // floats per [aggr | x] buffer

// Loader waves (256 lanes): copy rows 16 t .. 16 t + 15 of aggr and x into a
// tile buffer; lane (row lr = lane >> 5 (+8), chunk j = lane & 31), 4 independent
// 16-B loads per lane.  Rows past N are zero.  Three buffers: the loads of tile
// i + 2 are issued before the barrier of iteration i and written after it, so
// their latency overlaps two compute phases.
struct TileRegs {
  f32x4 v[4];
};

// Issue the loads of tile t (no wait: the registers are consumed after the next barrier).
__device__ __forceinline__ void fetch_tile(TileRegs& tr, int t, int N, int lt, const float* __restrict__ aggr,
                                           const float* __restrict__ x) {
  const int j = lt & 31, lr = lt >> 5;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int r = lr + 8 * (u >> 1), node = t * TILE + r;
    const float* src = (u & 1) ? x : aggr;
    tr.v[u] = node < N ? reinterpret_cast<const f32x4*>(src + (size_t)node * L)[j] : f32x4{0.f, 0.f, 0.f, 0.f};
  }
}

__device__ __forceinline__ void store_tile(float* __restrict__ xb, int lt, const TileRegs& tr) {
  const int j = lt & 31, lr = lt >> 5;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int r = lr + 8 * (u >> 1);
    *reinterpret_cast<f32x4*>(xb + r * XS + (u & 1) * L + 4 * j) = tr.v[u];
  }
}

__device__ __forceinline__ int nu_tile(int i) { return xcd_block() + i * (int)gridDim.x; }

// LayerNorm-backward column partials accumulated by the compute waves (the pdg_ln_colsum layout:
// [sum gy (128) | sum gy*xhat (128)] per block): lane (r, q) of wave w holds fp64 sums for
// features 16w + 4q + c over the rows it produced.  The 16 lanes of each q are added with a
// fixed xor butterfly and lane r = 0 writes the block's entries to `row` (LDS; every feature has
// one owner).
__device__ __forceinline__ void write_ln_partials(double (&sg)[4], double (&sx)[4], double* row) {
#pragma unroll
  for (int off = 1; off < 16; off <<= 1)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      sg[c] += __shfl_xor(sg[c], off);
      sx[c] += __shfl_xor(sx[c], off);
    }
  const int l = lane_id();
  if ((l & 15) == 0) {
    const int f = 16 * wave_id() + 4 * (l >> 4);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      row[f + c] = sg[c];
      row[L + f + c] = sx[c];
    }
  }
}

}  // namespace

// node_net with both layers as unbiased bf16x6 products (gemm_x6f; the fp32 kernels above are
// MFMA-bound): 8 waves, no loader waves, the three weight slices W1a (aggr half), W1b (x half) and W2
// as bf16 terms in registers (144 VGPRs).  Per 16-row tile: every thread fetches one row chunk of aggr
// and x of tile i + 2, layer 1 of tile i from its [aggr | x] images, a barrier, the split of tile
// i + 2 into the images layer 1 of tile i - 1 read, layer 2 of tile i from its a1 image (double-
// buffered).  One barrier per tile; 96 KB of LDS.
constexpr int NN_T16 = TILE * X6_ROWB;        // bytes per term plane of a 16-row image (4 KB)
constexpr int NN_IMG = 3 * NN_T16;            // one 16-row bf16x6 image (12 KB)

__global__ __launch_bounds__(64 * NU_COMPUTE, 1) void node_net_x6_kernel(
    int N, const float* __restrict__ aggr, const float* __restrict__ x, const float* __restrict__ W1,
    const float* __restrict__ b1, const float* __restrict__ W2, const float* __restrict__ b2,
    float* __restrict__ a1_out, float* __restrict__ a2_out, double* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) unsigned char xin[3 * 2 * NN_IMG];   // [buffer][aggr | x]
  __shared__ __attribute__((aligned(16))) unsigned char a1i[2 * NN_IMG];
  const int w = wave_id(), l = lane_id();
  const int ntiles = tiles_of(N);
  const int r = l & 15, q = l >> 4;
  const int oc = 16 * w + 4 * q;
  const int j = threadIdx.x & 31, rr = threadIdx.x >> 5;   // the thread's staged row chunk
  // no memory operation of the loop is conditional (rows past N are clamped on load and zeroed when
  // staged, stores past N dropped by the buffer range), so its waits count loads: a load or store on a
  // branch made the compiler wait for every outstanding load AND store (vmcnt(0)) once per tile
  f32x4 va, vx;
  bool vok;
  auto fetch = [&](int t) {
    const int node = t * TILE + rr;
    vok = node < N;
    const size_t o = (size_t)clamp_row(node, N) * L;
    va = reinterpret_cast<const f32x4*>(aggr + o)[j];
    vx = reinterpret_cast<const f32x4*>(x + o)[j];
  };
  auto stage = [&](int buf) {
    const f32x4 zero = f32x4{0.f, 0.f, 0.f, 0.f};
    x6_store4<NN_T16>(xin + (2 * buf) * NN_IMG, rr, j, vok ? va : zero);
    x6_store4<NN_T16>(xin + (2 * buf + 1) * NN_IMG, rr, j, vok ? vx : zero);
  };
  const __amdgpu_buffer_rsrc_t rs_a1 = rows_rsrc(a1_out, 0, N), rs_a2 = rows_rsrc(a2_out, 0, N);
#pragma unroll
  for (int k = 0; k < 2; ++k)
    if (nu_tile(k) < ntiles) {
      fetch(nu_tile(k));
      stage(k);
    }
  WSlice w1a, w1b, w2;
  load_wslice(w1a, W1, w, 2 * L);
  load_wslice(w1b, W1 + L, w, 2 * L);
  load_wslice(w2, W2, w, L);
  const f32x4 bias1 = *reinterpret_cast<const f32x4*>(b1 + oc);
  const f32x4 bias2 = *reinterpret_cast<const f32x4*>(b2 + oc);
  double s1 = 0, s2 = 0;
  __syncthreads();
  for (int i = 0;; ++i) {
    const int tile = nu_tile(i);
    if (tile >= ntiles) break;   // uniform across the block
    fetch(nu_tile(i + 2));   // past the last tile: clamped rows, staged into a buffer no tile reads
    const int row = tile * TILE + r;
    // layer 1: a1 = relu(W1a aggr + W1b x + b1), the aggr chunks first
    f32x4 d1[1] = {{0.f, 0.f, 0.f, 0.f}};
    gemm_x6f<1, NN_T16, true>(d1, w1a, xin + (2 * (i % 3)) * NN_IMG);
    gemm_x6f<1, NN_T16, true>(d1, w1b, xin + (2 * (i % 3) + 1) * NN_IMG);
    f32x4 a1;
#pragma unroll
    for (int c = 0; c < 4; ++c) a1[c] = fmaxf(d1[0][c] + bias1[c], 0.f);
    x6_store4<NN_T16>(a1i + (i & 1) * NN_IMG, r, 4 * w + q, a1);
    rows_store4(rs_a1, row, oc, a1);   // a1_out NULL (inference): an empty range
    __syncthreads();   // the a1 image is complete; the input buffer of tile i - 1 is free
    // layer 2: a2 = relu(W2 a1 + b2) + LayerNorm partials
    f32x4 d2[1] = {{0.f, 0.f, 0.f, 0.f}};
    gemm_x6f<1, NN_T16, true>(d2, w2, a1i + (i & 1) * NN_IMG);
    f32x4 a2;
#pragma unroll
    for (int c = 0; c < 4; ++c) a2[c] = fmaxf(d2[0][c] + bias2[c], 0.f);
    rows_store4(rs_a2, row, oc, a2);
    if (row < N) {
      const float p1 = (a2[0] + a2[1]) + (a2[2] + a2[3]);
      const float p2 = (a2[0] * a2[0] + a2[1] * a2[1]) + (a2[2] * a2[2] + a2[3] * a2[3]);
      s1 += (double)p1;
      s2 += (double)p2;
    }
    // tile i + 2 into the buffer layer 1 of tile i - 1 read (before the previous barrier); read after
    // the next one.  After layer 2 its loads have the whole tile to land.
    stage((i + 2) % 3);
  }
  __shared__ double red[2 * NU_COMPUTE];
  block_sum2(s1, s2, red);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = s1;
    part[2 * blockIdx.x + 1] = s2;
  }
}


// paired tiles (node_net_pair_kernel) by default: 46.6 -> 45.5-46.4 us per config-2 call in a same-box
// A/B; the same pairing of node_pq_rw measured no faster and is not kept

extern "C" int pdg_node_net(int n_nodes, const float* aggr, const float* x, const float* Wn1, const float* bn1,
                            const float* Wn2, const float* bn2, float* a1n, float* a2n, double* partials,
                            int* nparts, void* stream) {
  PDG_CHECK_ARG(n_nodes > 0, "pdg_node_net: n_nodes must be > 0");
  // the output buffer ranges span all rows: byte sizes below 2^31
  PDG_CHECK_ARG(n_nodes < (1 << 22), "pdg_node_net: at most 4,194,303 nodes per call");
  PDG_CHECK_ARG(aggr && x && a2n, "pdg_node_net: aggr, x and a2n are required");
  PDG_CHECK_ARG(PDG_ALIGNED(aggr) && PDG_ALIGNED(x) && PDG_ALIGNED(Wn1) && PDG_ALIGNED(Wn2) && PDG_ALIGNED(a2n) &&
                    PDG_ALIGNED(a1n) && PDG_ALIGNED(bn1) && PDG_ALIGNED(bn2),
                "pdg_node_net: misaligned pointer");
  const int tiles = tiles_of(n_nodes);
  const int cap = device_cus() < MAX_BLOCKS ? device_cus() : MAX_BLOCKS;
  const int grid = tiles < cap ? tiles : cap;
  hipLaunchKernelGGL(node_net_x6_kernel, dim3(grid), dim3(64 * NU_COMPUTE), 0, (hipStream_t)stream, n_nodes, aggr, x,
                     Wn1, bn1, Wn2, bn2, a1n, a2n, partials);
  PDG_CHECK_LAUNCH("pdg_node_net");
  if (nparts) *nparts = grid;
  return PDG_OK;
}

// ============================================================================ node_net backward
// Backward of node_net for one step, the work of pdg_mlp2_bwd + pdg_gemm_dual in one pass
// (models.py:240-243 / :202-208): with gy = d loss / d x_{t+1} (the residual branch's input),
//   gz2  = LN_bwd(gy) * [a2 > 0]                 (loader waves, elementwise, -> LDS + HBM)
//   gz1  = (W2^T gz2) * [a1 > 0]                 (compute waves, K = 128)
//   gaggr = W1a^T gz1,  gx_part = W1b^T gz1 + gy  (compute waves, two K = 128 products)
// Same register-stationary structure as node_net_kernel (wave w owns output features
// [16w, 16w+16) of all three products: 96 VGPRs of transposed weights); bitwise the
// results of the separate kernels.
namespace {

constexpr int GS = L + 8;                      // LDS row stride of the gz2 / gz1 tiles

// Loader waves: tile t's gz2 rows into `buf` (and to HBM).  Lane lt covers chunks lt and
// lt + 256 of the 16 x 32 (row, 16-B chunk) tile; loads issued one iteration ahead.
struct Gz2Regs {
  f32x4 gv[2], av[2];
};

__device__ __forceinline__ void fetch_gz2(Gz2Regs& rg, int t, int N, int lt, const float* __restrict__ gy,
                                          const float* __restrict__ a2) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int c = lt + 256 * u, rr = c >> 5, j = c & 31, node = t * TILE + rr;
    const bool ok = node < N;
    rg.gv[u] = ok ? reinterpret_cast<const f32x4*>(gy + (size_t)node * L)[j] : f32x4{0.f, 0.f, 0.f, 0.f};
    rg.av[u] = ok ? reinterpret_cast<const f32x4*>(a2 + (size_t)node * L)[j] : f32x4{0.f, 0.f, 0.f, 0.f};
  }
}

__device__ __forceinline__ void store_gz2(float* __restrict__ buf, float* __restrict__ gybuf, int t, int N, int lt,
                                          const Gz2Regs& rg, const LNStat& st, const pdg_ln_bwd& lb,
                                          const float* __restrict__ g, float* __restrict__ gz2_out) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int c = lt + 256 * u, rr = c >> 5, j = c & 31, node = t * TILE + rr;
    const f32x4 gg = reinterpret_cast<const f32x4*>(g)[j];
    f32x4 z;
#pragma unroll
    for (int e = 0; e < 4; ++e) {   // ln_relu_bwd (pdg_bwd.hip), element by element
      const float xhat = div_den(rg.av[u][e] - st.mean, st.den, st.rstd);
      const float ga = st.rstd * (gg[e] * rg.gv[u][e] - lb.c1) - xhat * lb.c2;
      z[e] = rg.av[u][e] > 0.f ? ga : 0.f;
    }
    *reinterpret_cast<f32x4*>(buf + rr * GS + 4 * j) = z;
    *reinterpret_cast<f32x4*>(gybuf + rr * GS + 4 * j) = rg.gv[u];   // the residual term, for the compute waves
    if (node < N) stg4(gz2_out + (size_t)node * L + 4 * j, z);
  }
}

}  // namespace

__global__ __launch_bounds__(NU_THREADS, 1) void node_bwd_kernel(
    int N, const float* __restrict__ gy, const float* __restrict__ a2, const float* __restrict__ a1,
    const pdg_ln_stat* __restrict__ stp, const pdg_ln_bwd* __restrict__ lbp, const float* __restrict__ lg,
    const float* __restrict__ W2T, const float* __restrict__ W1aT, const float* __restrict__ W1bT,
    float* __restrict__ gz2_out, float* __restrict__ gz1_out, float* __restrict__ gaggr,
    float* __restrict__ gx_part, const double* __restrict__ lb_pairs, int lb_npairs) {
  // LDS (dynamic, 69.6 KB): gz2 tiles and the loaders' gy rows (3 buffers each), gz1 tiles (2)
  extern __shared__ __attribute__((aligned(16))) float nbw_sm[];
  float* gz2t = nbw_sm;
  float* gyt = gz2t + 3 * TILE * GS;
  float* gz1t = gyt + 3 * TILE * GS;
  const int w = wave_id(), l = lane_id();
  const bool loader = w >= NU_COMPUTE;
  const int ntiles = tiles_of(N);
  const int lt = threadIdx.x - 64 * NU_COMPUTE;
  const LNStat st = *reinterpret_cast<const LNStat*>(stp);
  const pdg_ln_bwd lb = lnb_resolve(lbp, lb_pairs, lb_npairs, stp);
  const int r = l & 15, q = l >> 4;
  const int oc = 16 * w + 4 * q;   // this lane's 4 output features (D rows 4q .. 4q+3 of block w)
  f32x4 w2f[8], waf[8], wbf[8];
  if (!loader) {
    const float* p2 = W2T + (size_t)(16 * w + r) * L + 4 * q;
    const float* pa = W1aT + (size_t)(16 * w + r) * L + 4 * q;
    const float* pb = W1bT + (size_t)(16 * w + r) * L + 4 * q;
#pragma unroll
    for (int T = 0; T < 8; ++T) {
      w2f[T] = *reinterpret_cast<const f32x4*>(p2 + 16 * T);
      waf[T] = *reinterpret_cast<const f32x4*>(pa + 16 * T);
      wbf[T] = *reinterpret_cast<const f32x4*>(pb + 16 * T);
    }
  }
  Gz2Regs rg;
  if (loader) {
#pragma unroll
    for (int k = 0; k < 2; ++k)
      if (nu_tile(k) < ntiles) {
        fetch_gz2(rg, nu_tile(k), N, lt, gy, a2);
        store_gz2(gz2t + k * TILE * GS, gyt + k * TILE * GS, nu_tile(k), N, lt, rg, st, lb, lg, gz2_out);
      }
  }
  // compute waves: the relu-mask rows of a1 are loaded one tile ahead, before the previous tile's
  // stores (vmcnt counts loads and stores together in issue order: a load issued behind the stores
  // is waited for together with them)
  f32x4 a1v = {0.f, 0.f, 0.f, 0.f};
  if (!loader && nu_tile(0) < ntiles) {
    const int row0 = nu_tile(0) * TILE + r;
    a1v = *reinterpret_cast<const f32x4*>(a1 + (size_t)(row0 < N ? row0 : N - 1) * L + oc);
  }
  __syncthreads();
  for (int i = 0;; ++i) {
    const int tile = nu_tile(i);
    if (tile >= ntiles) break;   // uniform across the block
    const int row = tile * TILE + r;
    const bool valid = row < N;
    const bool ahead = nu_tile(i + 2) < ntiles;
    float* g1 = gz1t + (i & 1) * TILE * GS;
    if (loader) {
      if (ahead) fetch_gz2(rg, nu_tile(i + 2), N, lt, gy, a2);
    } else {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      const float* zr = gz2t + (i % 3) * TILE * GS + r * GS + 4 * q;
#pragma unroll
      for (int T = 0; T < 8; ++T) {
        const f32x4 bv = *reinterpret_cast<const f32x4*>(zr + 16 * T);
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(w2f[T][jj], bv[jj], acc, 0, 0, 0);
      }
      f32x4 z1;
#pragma unroll
      for (int c = 0; c < 4; ++c) z1[c] = a1v[c] > 0.f ? acc[c] : 0.f;   // relu_mask_acc
      *reinterpret_cast<f32x4*>(g1 + r * GS + oc) = z1;
      if (valid) stg4(gz1_out + (size_t)row * L + oc, z1);
    }
    __syncthreads();
    if (loader) {
      if (ahead)
        store_gz2(gz2t + ((i + 2) % 3) * TILE * GS, gyt + ((i + 2) % 3) * TILE * GS, nu_tile(i + 2), N, lt, rg, st,
                  lb, lg, gz2_out);
    } else {
      const f32x4 res = *reinterpret_cast<const f32x4*>(gyt + (i % 3) * TILE * GS + r * GS + oc);
      f32x4 acc_a = {0.f, 0.f, 0.f, 0.f}, acc_b = {0.f, 0.f, 0.f, 0.f};
      const float* zr = g1 + r * GS + 4 * q;
#pragma unroll
      for (int T = 0; T < 8; ++T) {
        const f32x4 bv = *reinterpret_cast<const f32x4*>(zr + 16 * T);
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          acc_a = __builtin_amdgcn_mfma_f32_16x16x4f32(waf[T][jj], bv[jj], acc_a, 0, 0, 0);
          acc_b = __builtin_amdgcn_mfma_f32_16x16x4f32(wbf[T][jj], bv[jj], acc_b, 0, 0, 0);
        }
      }
      acc_b += res;
      if (nu_tile(i + 1) < ntiles) {
        const int rn = nu_tile(i + 1) * TILE + r;
        a1v = *reinterpret_cast<const f32x4*>(a1 + (size_t)(rn < N ? rn : N - 1) * L + oc);
      }
      if (valid) {
        stg4(gaggr + (size_t)row * L + oc, acc_a);
        stg4(gx_part + (size_t)row * L + oc, acc_b);
      }
    }
  }
}

extern "C" int pdg_node_bwd(int n_nodes, const float* gy, const float* a2n, const float* a1n, const pdg_ln_stat* st,
                            const pdg_ln_bwd* lb, const float* ln_g, const float* Wn2T, const float* Wn1aT,
                            const float* Wn1bT, float* gz2, float* gz1, float* gaggr, float* gx_part,
                            const double* lb_pairs, int lb_npairs, void* stream) {
  PDG_CHECK_ARG(n_nodes > 0, "pdg_node_bwd: n_nodes must be > 0");
  PDG_CHECK_ARG(gy && a2n && a1n && st && (lb || lb_pairs) && ln_g && gz2 && gz1 && gaggr && gx_part,
                "pdg_node_bwd: null argument");
  PDG_CHECK_ARG(PDG_ALIGNED(gy) && PDG_ALIGNED(a2n) && PDG_ALIGNED(a1n) && PDG_ALIGNED(Wn2T) &&
                    PDG_ALIGNED(Wn1aT) && PDG_ALIGNED(Wn1bT) && PDG_ALIGNED(gz2) && PDG_ALIGNED(gz1) &&
                    PDG_ALIGNED(gaggr) && PDG_ALIGNED(gx_part) && PDG_ALIGNED(ln_g),
                "pdg_node_bwd: misaligned pointer");
  const int tiles = tiles_of(n_nodes);
  const int cap = device_cus() < MAX_BLOCKS ? device_cus() : MAX_BLOCKS;
  const int grid = tiles < cap ? tiles : cap;
  const size_t shm = (size_t)8 * TILE * GS * sizeof(float);
  hipLaunchKernelGGL(node_bwd_kernel, dim3(grid), dim3(NU_THREADS), shm, (hipStream_t)stream, n_nodes, gy, a2n, a1n,
                     st, lb, ln_g, Wn2T, Wn1aT, Wn1bT, gz2, gz1, gaggr, gx_part, lb_pairs, lb_npairs);
  PDG_CHECK_LAUNCH("pdg_node_bwd");
  return PDG_OK;
}

// ============================================================================ node P/Q pre-pass
// x_t = LN(a2_prev) [+ x_prev], P = Wa x_t, Q = Wb x_t (weights Wa = W1[:, 0:128], Wb = W1[:, 128:256] of
// edge_net.0) with P and Q as bf16x6 products (gemm_x6f: unbiased accumulation, 2.7x less matrix time than
// the fp32 MFMAs of the LDS-weight pdg_node_pq, which was MFMA-bound).  x_t goes through a 16-row bf16x6
// image; Wa / Wb are held as bf16 terms (96 VGPRs).  x_t is bitwise pdg_node_pq's; P / Q agree with it to
// fp32 rounding and are closer to fp64.
constexpr int PQ_T16 = TILE * X6_ROWB;       // bytes per term plane of a 16-row image (4 KB)
constexpr int PQ_IMG = 3 * PQ_T16;           // one 16-row bf16x6 image (12 KB)

// One block of 8 waves per CU, no loader waves (the weight terms need the 256-VGPR budget of 8
// waves): every thread fetches one row chunk of tile i + 2 (a2_prev, x_prev) before the products of
// tile i and stores it, LayerNorm applied and split, into buffer (i + 2) % 3 after the barrier.
// Branch-free (node_pq_x6_kernel's tile loop): rows past N are loaded clamped (a real row) and the
// x rows are stored through a per-tile buffer range that drops rows past N.
template <bool RES>
__device__ __forceinline__ void fetch_xt1(f32x4& av, f32x4& rv, int t, int N, const float* __restrict__ a2p,
                                          const float* __restrict__ xres) {
  const int j = threadIdx.x & 31, node = clamp_row(t * TILE + (threadIdx.x >> 5), N);
  av = reinterpret_cast<const f32x4*>(a2p + (size_t)node * L)[j];
  if (RES) rv = reinterpret_cast<const f32x4*>(xres + (size_t)node * L)[j];
}

// [t0, t1) of tile t, empty past the last tile
__device__ __forceinline__ __amdgpu_buffer_rsrc_t tile_rsrc(float* base, int t, int N) {
  const int t0 = t * TILE, t1 = max(t0, min(N, t0 + TILE));
  return rows_rsrc(base, t1 > t0 ? t0 : 0, t1 > t0 ? t1 : 0);
}

template <bool RES>
__device__ __forceinline__ void store_xt1(unsigned char* __restrict__ img, int t, int N, const f32x4& av,
                                          const f32x4& rv, const LNStat& st, const f32x4& gg, const f32x4& bb,
                                          float* __restrict__ xout) {
  const int j = threadIdx.x & 31, rr = threadIdx.x >> 5;
  f32x4 y;
#pragma unroll
  for (int e = 0; e < 4; ++e) {   // ln_res_frag (pdg_fwd.hip), element by element
    float v = div_den(av[e] - st.mean, st.den, st.rstd) * gg[e] + bb[e];
    if (RES) v += rv[e];
    y[e] = v;
  }
  x6_store4<PQ_T16>(img, rr, j, y);
  rows_store4(tile_rsrc(xout, t, N), rr, 4 * j, y);
}

template <bool RES>
__global__ __launch_bounds__(64 * NU_COMPUTE, 1) void node_pq_x6_kernel(
    int N, const float* __restrict__ a2p, const pdg_ln_stat* __restrict__ stp, const float* __restrict__ lg,
    const float* __restrict__ lb, const float* __restrict__ xres, float* __restrict__ xout,
    const float* __restrict__ W1, float* __restrict__ P, float* __restrict__ Q, const double* __restrict__ part,
    int nparts, double count, pdg_ln_stat* __restrict__ st_out) {
  __shared__ __attribute__((aligned(16))) unsigned char xt[3 * PQ_IMG];
  __shared__ LNStat st_sh;
  __shared__ double red_fin[2 * NU_COMPUTE];
  const int w = wave_id(), l = lane_id();
  const int ntiles = tiles_of(N);
  if (part) {   // the node LayerNorm statistics of the previous step, folded in (pdg_node_pq_rw_fin)
    ln_stat_from_partials(part, nparts, count, &st_sh, red_fin);
    __syncthreads();
    if (blockIdx.x == 0 && threadIdx.x == 0) *st_out = st_sh;
  }
  const LNStat st = part ? st_sh : *reinterpret_cast<const LNStat*>(stp);
  const f32x4 gg = reinterpret_cast<const f32x4*>(lg)[threadIdx.x & 31];
  const f32x4 bb = reinterpret_cast<const f32x4*>(lb)[threadIdx.x & 31];
  // loaded before the loop: a wait for them inside it would count the loop's stores too
  pin_vgpr(gg);
  pin_vgpr(bb);
  pin_vgpr(st.mean);
  pin_vgpr(st.den);
  pin_vgpr(st.rstd);
  const int r = l & 15, q = l >> 4;
  const int oc = 16 * w + 4 * q;
  f32x4 av, rv;
#pragma unroll
  for (int k = 0; k < 2; ++k)
    if (nu_tile(k) < ntiles) {
      fetch_xt1<RES>(av, rv, nu_tile(k), N, a2p, xres);
      store_xt1<RES>(xt + k * PQ_IMG, nu_tile(k), N, av, rv, st, gg, bb, xout);
    }
  WSlice wa, wb;
  load_wslice(wa, W1, w, 3 * L);
  load_wslice(wb, W1 + L, w, 3 * L);
  __syncthreads();
  for (int i = 0;; ++i) {
    const int tile = nu_tile(i);
    if (tile >= ntiles) break;   // uniform across the block
    // no memory operation below is conditional (a skipped one made every wait in the loop a vmcnt(0)):
    // past the last tile the rows are loaded clamped and staged into a free buffer, stores dropped
    fetch_xt1<RES>(av, rv, nu_tile(i + 2), N, a2p, xres);
    f32x4 dp[1] = {{0.f, 0.f, 0.f, 0.f}}, dq[1] = {{0.f, 0.f, 0.f, 0.f}};
    const unsigned char* im = xt + (i % 3) * PQ_IMG;
    gemm_x6f<1, PQ_T16>(dp, wa, im);
    gemm_x6f<1, PQ_T16>(dq, wb, im);
#if PDG_PQ_BLOCKED
    {   // rows of PQ_LD floats: a buffer range over the tile's rows of the blocked P / Q array
      const int t0 = tile * TILE, nr = max(0, min(N, t0 + TILE) - t0);
      const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(P + (size_t)t0 * PQ_LD, (short)0, nr * PQ_LD * 4, 0x00020000);
      const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc(Q + (size_t)t0 * PQ_LD, (short)0, nr * PQ_LD * 4, 0x00020000);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, dp[0]), rp, (r * PQ_LD + pq_col(oc)) * 4, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, dq[0]), rq, (r * PQ_LD + pq_col(oc)) * 4, 0, 0);
    }
#else
    rows_store4(tile_rsrc(P, tile, N), r, oc, dp[0]);
    rows_store4(tile_rsrc(Q, tile, N), r, oc, dq[0]);
#endif
    __syncthreads();
    // buffer (i + 2) % 3 was last read in iteration i - 1
    store_xt1<RES>(xt + ((i + 2) % 3) * PQ_IMG, nu_tile(i + 2), N, av, rv, st, gg, bb, xout);
  }
}

static_assert(!PDG_PQ_BLOCKED || 1, "the blocked P / Q layout is written by node_pq_x6_kernel only");

static int node_pq_rw_launch(int n_nodes, const float* a2_prev, const pdg_ln_stat* st, const float* ln_g,
                             const float* ln_b, const float* x_res, float* x_out, const float* W1, float* P,
                             float* Q, const double* part, int nparts, double count, pdg_ln_stat* st_out,
                             void* stream) {
  PDG_CHECK_ARG(n_nodes > 0, "pdg_node_pq_rw: n_nodes must be > 0");
  PDG_CHECK_ARG(PDG_ALIGNED(a2_prev) && PDG_ALIGNED(x_out) && PDG_ALIGNED(P) && PDG_ALIGNED(Q) && PDG_ALIGNED(W1) &&
                    PDG_ALIGNED(ln_g) && PDG_ALIGNED(ln_b) && PDG_ALIGNED(x_res),
                "pdg_node_pq_rw: misaligned pointer");
  const int tiles = tiles_of(n_nodes);
  const int cap = device_cus() < MAX_BLOCKS ? device_cus() : MAX_BLOCKS;
  const int grid = tiles < cap ? tiles : cap;
  const int nt = 64 * NU_COMPUTE;
  if (x_res)
    hipLaunchKernelGGL(node_pq_x6_kernel<true>, dim3(grid), dim3(nt), 0,
                       (hipStream_t)stream, n_nodes, a2_prev, st, ln_g, ln_b, x_res, x_out, W1, P, Q, part, nparts,
                       count, st_out);
  else
    hipLaunchKernelGGL(node_pq_x6_kernel<false>, dim3(grid), dim3(nt), 0,
                       (hipStream_t)stream, n_nodes, a2_prev, st, ln_g, ln_b, x_res, x_out, W1, P, Q, part, nparts,
                       count, st_out);
  PDG_CHECK_LAUNCH("pdg_node_pq_rw");
  return PDG_OK;
}

extern "C" int pdg_node_pq_rw(int n_nodes, const float* a2_prev, const pdg_ln_stat* st, const float* ln_g,
                              const float* ln_b, const float* x_res, float* x_out, const float* W1, float* P,
                              float* Q, void* stream) {
  PDG_CHECK_ARG(st != nullptr, "pdg_node_pq_rw: st is null");
  return node_pq_rw_launch(n_nodes, a2_prev, st, ln_g, ln_b, x_res, x_out, W1, P, Q, nullptr, 0, 0.0, nullptr,
                           stream);
}

extern "C" int pdg_node_pq_rw_fin(int n_nodes, const float* a2_prev, const double* partials, int nparts,
                                  double count, pdg_ln_stat* st_out, const float* ln_g, const float* ln_b,
                                  const float* x_res, float* x_out, const float* W1, float* P, float* Q,
                                  void* stream) {
  PDG_CHECK_ARG(partials && st_out && nparts > 0 && nparts < MAX_BLOCKS && count > 0,
                "pdg_node_pq_rw_fin: bad statistics arguments");
  return node_pq_rw_launch(n_nodes, a2_prev, nullptr, ln_g, ln_b, x_res, x_out, W1, P, Q, partials, nparts, count,
                           st_out, stream);
}

// ============================================================================ summed transposed GEMMs
// out = W0T in0 + W1T in1 [+ res] (the input gradient of x through P = Wa x, Q = Wb x plus the
// node_net path), weights held in registers; bitwise pdg_gemm_sum2.  COLS: also the column
// partials (pdg_ln_colsum layout) of the backward of the LayerNorm LN(ln_a2) whose upstream
// gradient is `out` (x_{t} = LN(a2n_{t-1}) + x_{t-1}: the node LayerNorm of the previous step).
template <bool COLS>
__global__ __launch_bounds__(NU_THREADS, 1) void gemm_sum2_rw_kernel(
    int N, const float* __restrict__ in0, const float* __restrict__ in1, const float* __restrict__ W0T,
    const float* __restrict__ W1T, const float* __restrict__ res, float* __restrict__ out,
    const float* __restrict__ ln_a2, const pdg_ln_stat* __restrict__ ln_st, double* __restrict__ cpart,
    const float* __restrict__ ln_g, double* __restrict__ pairs, int accumulate) {
  __shared__ __attribute__((aligned(16))) float xin[3 * XBUF];
  __shared__ double crow[COLS ? 256 : 1], ctmp[COLS ? 256 : 1];
  const int w = wave_id(), l = lane_id();
  const bool loader = w >= NU_COMPUTE;
  const int ntiles = tiles_of(N);
  const int lt = threadIdx.x - 64 * NU_COMPUTE;
  const int r = l & 15, q = l >> 4;
  const int oc = 16 * w + 4 * q;
  f32x4 wf[16];
  double csg[4] = {0, 0, 0, 0}, csx[4] = {0, 0, 0, 0};
  float mean = 0.f, den = 1.f, rstd = 1.f;
  if (COLS) {
    mean = ln_st->mean;
    den = ln_st->den;
    rstd = ln_st->rstd;
  }
  if (!loader) {
    const float* p0 = W0T + (size_t)(16 * w + r) * L + 4 * q;
    const float* p1 = W1T + (size_t)(16 * w + r) * L + 4 * q;
#pragma unroll
    for (int T = 0; T < 8; ++T) {
      wf[T] = *reinterpret_cast<const f32x4*>(p0 + 16 * T);
      wf[8 + T] = *reinterpret_cast<const f32x4*>(p1 + 16 * T);
    }
  }
  TileRegs tr;
  if (loader) {
#pragma unroll
    for (int k = 0; k < 2; ++k)
      if (nu_tile(k) < ntiles) {
        fetch_tile(tr, nu_tile(k), N, lt, in0, in1);
        store_tile(xin + k * XBUF, lt, tr);
      }
  }
  __syncthreads();
  for (int i = 0;; ++i) {
    const int tile = nu_tile(i);
    if (tile >= ntiles) break;   // uniform across the block
    const bool ahead = nu_tile(i + 2) < ntiles;
    if (loader) {
      if (ahead) fetch_tile(tr, nu_tile(i + 2), N, lt, in0, in1);
    } else {
      const int row = tile * TILE + r;
      const int rc = row < N ? row : N - 1;
      f32x4 rv = {0.f, 0.f, 0.f, 0.f};
      if (res) rv = *reinterpret_cast<const f32x4*>(res + (size_t)rc * L + oc);
      f32x4 av;
      if (COLS) av = *reinterpret_cast<const f32x4*>(ln_a2 + (size_t)rc * L + oc);
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      const float* xr = xin + (i % 3) * XBUF + r * XS + 4 * q;
#pragma unroll
      for (int T = 0; T < 16; ++T) {
        const f32x4 bv = *reinterpret_cast<const f32x4*>(xr + 16 * T);
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[T][jj], bv[jj], acc, 0, 0, 0);
      }
      if (res) acc += rv;
      if (row < N) {
        stg4(out + (size_t)row * L + oc, acc);
        if (COLS) {
#pragma unroll
          for (int c = 0; c < 4; ++c) {   // the pdg_ln_colsum formulas
            const float xhat = div_den(av[c] - mean, den, rstd);
            csg[c] += (double)acc[c];
            csx[c] += (double)(acc[c] * xhat);
          }
        }
      }
    }
    __syncthreads();
    if (loader && ahead) store_tile(xin + ((i + 2) % 3) * XBUF, lt, tr);   // last read in iteration i - 1
  }
  if (COLS) {
    if (!loader) write_ln_partials(csg, csx, crow);
    __syncthreads();
    lnb_emit(crow, ln_g, cpart, accumulate, pairs, ctmp);
  }
}

extern "C" int pdg_gemm_sum2_rw(int rows, const float* in0, const float* in1, const float* W0T, const float* W1T,
                                const float* res, float* out, const float* ln_a2, const pdg_ln_stat* ln_st,
                                double* partials, int* nparts, const float* ln_g, double* pairs, int accumulate,
                                void* stream) {
  PDG_CHECK_ARG(rows > 0, "pdg_gemm_sum2_rw: rows must be > 0");
  PDG_CHECK_ARG(PDG_ALIGNED(in0) && PDG_ALIGNED(in1) && PDG_ALIGNED(out) && PDG_ALIGNED(W0T) && PDG_ALIGNED(W1T) &&
                    PDG_ALIGNED(res),
                "pdg_gemm_sum2_rw: misaligned pointer");
  const int tiles = tiles_of(rows);
  const int cap = device_cus() < MAX_BLOCKS ? device_cus() : MAX_BLOCKS;
  const int grid = tiles < cap ? tiles : cap;
  if (partials) {
    PDG_CHECK_ARG(ln_a2 && ln_st && PDG_ALIGNED(ln_a2) && PDG_ALIGNED(partials) && (!pairs || ln_g),
                  "pdg_gemm_sum2_rw: column partials need an aligned ln_a2, ln_st (and ln_g for pairs)");
    hipLaunchKernelGGL(gemm_sum2_rw_kernel<true>, dim3(grid), dim3(NU_THREADS), 0, (hipStream_t)stream, rows, in0,
                       in1, W0T, W1T, res, out, ln_a2, ln_st, partials, ln_g, pairs, accumulate);
  } else {
    hipLaunchKernelGGL(gemm_sum2_rw_kernel<false>, dim3(grid), dim3(NU_THREADS), 0, (hipStream_t)stream, rows, in0,
                       in1, W0T, W1T, res, out, nullptr, nullptr, nullptr, nullptr, nullptr, 0);
  }
  PDG_CHECK_LAUNCH("pdg_gemm_sum2_rw");
  if (nparts) *nparts = grid;
  return PDG_OK;
}
