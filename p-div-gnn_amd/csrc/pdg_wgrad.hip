// Weight gradients of the shared 128x128 Linears (autograd of addmm in
// gnn_local_stress/models.py:194-208, :260-286), deterministic split-K.
//
// dW[o][i] = sum_k G[k][o] X[k][i] is a K = rows reduction (rows = edges, up
// to ~10^6).  Each block owns a contiguous row range and accumulates into its
// own fp32 slab (128x128 + 128 bias sums) with += (no atomics), so the shared
// weights of the 10 weight-tied message-passing steps accumulate across calls
// in a fixed order; pdg_wgrad_reduce sums the slabs in block order.
//
// MFMA mapping (v_mfma_f32_32x32x2_f32): A = G^T (o on the lane, k = lane half),
// B = X (i on the lane, k = lane half): both operands are plain 128-byte
// row segments, read straight from global memory.  4 waves per block, wave w
// owns outputs o in [32w, 32w+32) and all 128 inputs (4 accumulators).
#include "pdg_common.hpp"
#include "pdg_runtime.hpp"
#include "pdg_x6.hpp"

using namespace pdg;

constexpr int SLAB = L * L + L;   // floats per slab

__device__ __forceinline__ void zero_acc16(f32x16 (&acc)[4]) {
#pragma unroll
  for (int nb = 0; nb < 4; ++nb)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[nb][r] = 0.f;
}

__device__ __forceinline__ void wgrad_pass(int M, int r0, int r1, const float* __restrict__ G,
                                           const float* __restrict__ X, f32x16 (&acc)[4], double& bsum) {
  const int l = lane_id(), h = l >> 5, c = l & 31, w = wave_id();
  const float* gcol = G + 32 * w + c;
  const float* xcol = X + c;
  int k = r0;
  for (; k + 8 <= r1; k += 8) {
    float ga[4], xb[4][4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const size_t kk = (size_t)(k + 2 * u + h) * L;
      ga[u] = gcol[kk];
#pragma unroll
      for (int ib = 0; ib < 4; ++ib) xb[u][ib] = xcol[kk + 32 * ib];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      bsum += (double)ga[u];
#pragma unroll
      for (int ib = 0; ib < 4; ++ib)
        acc[ib] = __builtin_amdgcn_mfma_f32_32x32x2f32(ga[u], xb[u][ib], acc[ib], 0, 0, 0);
    }
  }
  for (; k < r1; k += 2) {
    const int kr = k + h;
    const bool ok = kr < r1;
    const size_t kk = (size_t)(ok ? kr : r0) * L;
    const float ga = ok ? gcol[kk] : 0.f;
    bsum += (double)ga;
#pragma unroll
    for (int ib = 0; ib < 4; ++ib) {
      const float xb = ok ? xcol[kk + 32 * ib] : 0.f;
      acc[ib] = __builtin_amdgcn_mfma_f32_32x32x2f32(ga, xb, acc[ib], 0, 0, 0);
    }
  }
  (void)M;
}

__global__ __launch_bounds__(256) void wgrad_accum_kernel(int M, const float* __restrict__ G,
                                                          const float* __restrict__ X,
                                                          const float* __restrict__ G2,
                                                          const float* __restrict__ X2,
                                                          float* __restrict__ slabs) {
  const int nb = gridDim.x;
  const long chunk = (((long)M + nb - 1) / nb + 1) & ~1L;
  const int r0 = (int)min((long)M, chunk * blockIdx.x);
  const int r1 = (int)min((long)M, chunk * (blockIdx.x + 1));
  f32x16 acc[4];
  zero_acc16(acc);
  double bsum = 0;
  wgrad_pass(M, r0, r1, G, X, acc, bsum);
  if (G2) wgrad_pass(M, r0, r1, G2, X2, acc, bsum);
  const int l = lane_id(), h = l >> 5, w = wave_id();
  float* slab = slabs + (size_t)blockIdx.x * SLAB;
#pragma unroll
  for (int ib = 0; ib < 4; ++ib)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int o = 32 * w + (r & 3) + 8 * (r >> 2) + 4 * h;
      const int i = 32 * ib + (l & 31);
      slab[o * L + i] += acc[ib][r];
    }
  const double other = __shfl_xor(bsum, 32);
  if (h == 0) slab[L * L + 32 * w + (l & 31)] += (float)(bsum + other);
}

extern "C" int pdg_wgrad_accum(int rows, const float* G, const float* X, const float* G2, const float* X2,
                               float* slabs, int nslabs, void* stream) {
  PDG_CHECK_ARG(rows > 0 && nslabs > 0 && nslabs <= MAX_BLOCKS, "pdg_wgrad_accum: bad sizes");
  PDG_CHECK_ARG((G2 == nullptr) == (X2 == nullptr), "pdg_wgrad_accum: G2/X2 must both be set or NULL");
  hipLaunchKernelGGL(wgrad_accum_kernel, dim3(nslabs), dim3(256), 0, (hipStream_t)stream, rows, G, X, G2, X2,
                     slabs);
  PDG_CHECK_LAUNCH("pdg_wgrad_accum");
  return PDG_OK;
}

// Two-level slab reduction (fixed order): pass 1 sums each chunk of WR_CHUNK slabs into
// the chunk's first slab (only the thread owning element e touches column e of those
// slabs), pass 2 adds the chunk sums in chunk order into the gradient.
constexpr int WR_CHUNK = 32;

__global__ __launch_bounds__(256) void wgrad_chunk_kernel(float* __restrict__ slabs, int n) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= SLAB) return;
  const int b0 = blockIdx.y * WR_CHUNK, b1 = min(n, b0 + WR_CHUNK);
  float p0 = 0.f, p1 = 0.f, p2 = 0.f, p3 = 0.f;
  int b = b0;
  for (; b + 4 <= b1; b += 4) {
    p0 += slabs[(size_t)b * SLAB + e];
    p1 += slabs[(size_t)(b + 1) * SLAB + e];
    p2 += slabs[(size_t)(b + 2) * SLAB + e];
    p3 += slabs[(size_t)(b + 3) * SLAB + e];
  }
  for (; b < b1; ++b) p0 += slabs[(size_t)b * SLAB + e];
  slabs[(size_t)b0 * SLAB + e] = (p0 + p1) + (p2 + p3);
}

__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ slabs, int nch,
                                                           float* __restrict__ gW, int ld, int col0,
                                                           float* __restrict__ gb) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= SLAB) return;
  float s = 0.f;
  for (int c = 0; c < nch; ++c) s += slabs[(size_t)c * WR_CHUNK * SLAB + e];
  if (e < L * L) {
    const int o = e / L, i = e % L;
    gW[(size_t)o * ld + col0 + i] += s;
  } else if (gb) {
    gb[e - L * L] += s;
  }
}

extern "C" int pdg_wgrad_reduce(float* slabs, int nslabs, float* grad_W, int ld, int col0, float* grad_b,
                                void* stream) {
  PDG_CHECK_ARG(nslabs > 0 && grad_W != nullptr, "pdg_wgrad_reduce: bad args");
  const int nch = (nslabs + WR_CHUNK - 1) / WR_CHUNK;
  hipLaunchKernelGGL(wgrad_chunk_kernel, dim3((SLAB + 255) / 256, nch), dim3(256), 0, (hipStream_t)stream, slabs,
                     nslabs);
  PDG_CHECK_LAUNCH("pdg_wgrad_reduce(chunks)");
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((SLAB + 255) / 256), dim3(256), 0, (hipStream_t)stream, slabs,
                     nch, grad_W, ld, col0, grad_b);
  PDG_CHECK_LAUNCH("pdg_wgrad_reduce");
  return PDG_OK;
}

// Every weight's slab reduction of a backward pass in one launch (the two-pass pdg_wgrad_reduce
// per weight cost 2 launches of ~6 us each, mostly fixed cost).  Block (x, job): elements
// 32 x .. 32 x + 31 of the job's slab; thread (e = t & 31, group g = t >> 5) sums slabs g, g + 8, ..
// (8 loads in flight), then the 8 group sums are added in group order and added into gW / gb.
constexpr int WRB_MAX = 16;
struct WgradReduceJobs {
  const float* slabs[WRB_MAX];
  float* gW[WRB_MAX];
  float* gb[WRB_MAX];
  int nslabs[WRB_MAX], ld[WRB_MAX], col0[WRB_MAX];
};

__global__ __launch_bounds__(256) void wgrad_reduce_batch_kernel(WgradReduceJobs jobs) {
  __shared__ float red[8][33];
  const int j = blockIdx.y;
  const float* __restrict__ slabs = jobs.slabs[j];
  const int n = jobs.nslabs[j];
  const int el = threadIdx.x & 31, g = threadIdx.x >> 5;
  const int e = blockIdx.x * 32 + el;
  float acc = 0.f;
  if (e < SLAB) {
    for (int b0 = g; b0 < n; b0 += 64) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = b0 + 8 * u < n ? slabs[(size_t)(b0 + 8 * u) * SLAB + e] : 0.f;
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
  }
  red[g][el] = acc;
  __syncthreads();
  if (g == 0 && e < SLAB) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += red[k][el];
    if (e < L * L) {
      const int o = e / L, i = e % L;
      jobs.gW[j][(size_t)o * jobs.ld[j] + jobs.col0[j] + i] += s;
    } else if (jobs.gb[j]) {
      jobs.gb[j][e - L * L] += s;
    }
  }
}

extern "C" int pdg_wgrad_reduce_batch(int njobs, const float* const* slabs, const int* nslabs, float* const* grad_W,
                                      const int* ld, const int* col0, float* const* grad_b, void* stream) {
  PDG_CHECK_ARG(njobs > 0 && njobs <= WRB_MAX && slabs && nslabs && grad_W && ld && col0 && grad_b,
                "pdg_wgrad_reduce_batch: bad arguments");
  WgradReduceJobs jobs;
  for (int i = 0; i < njobs; ++i) {
    PDG_CHECK_ARG(slabs[i] && grad_W[i] && nslabs[i] > 0 && nslabs[i] <= MAX_BLOCKS && ld[i] >= L &&
                      col0[i] >= 0 && col0[i] + L <= ld[i],
                  "pdg_wgrad_reduce_batch: bad job");
    jobs.slabs[i] = slabs[i];
    jobs.gW[i] = grad_W[i];
    jobs.gb[i] = grad_b[i];
    jobs.nslabs[i] = nslabs[i];
    jobs.ld[i] = ld[i];
    jobs.col0[i] = col0[i];
  }
  hipLaunchKernelGGL(wgrad_reduce_batch_kernel, dim3((SLAB + 31) / 32, njobs), dim3(256), 0, (hipStream_t)stream,
                     jobs);
  PDG_CHECK_LAUNCH("pdg_wgrad_reduce_batch");
  return PDG_OK;
}

// ============================================================================ narrow weight gradient
// T[c][i] = sum_k Wide[k][c] * Narrow[k][i], c < 128, i < K <= 8.  Half-wave per row.
template <int K>
__global__ __launch_bounds__(256) void wgrad_narrow_kernel(int M, const float* __restrict__ wide,
                                                           const float* __restrict__ narrow,
                                                           double* __restrict__ part) {
  constexpr int NP = 4 * K + 4 + K;   // per-lane partials: 4 channels x K, 4 wide sums, K narrow sums
  __shared__ double red[8][32][NP];
  const int hw = threadIdx.x >> 5, j = threadIdx.x & 31;
  const int nhw = blockDim.x >> 5;
  double acc[NP];
#pragma unroll
  for (int p = 0; p < NP; ++p) acc[p] = 0;
  for (int k = blockIdx.x * nhw + hw; k < M; k += gridDim.x * nhw) {
    const f32x4 w = reinterpret_cast<const f32x4*>(wide + (size_t)k * L)[j];
    float nv[K];
#pragma unroll
    for (int i = 0; i < K; ++i) nv[i] = narrow[(size_t)k * K + i];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
#pragma unroll
      for (int i = 0; i < K; ++i) acc[c * K + i] += (double)(w[c] * nv[i]);
      acc[4 * K + c] += (double)w[c];
    }
#pragma unroll
    for (int i = 0; i < K; ++i) acc[4 * K + 4 + i] += (double)nv[i];
  }
#pragma unroll
  for (int p = 0; p < NP; ++p) red[hw][j][p] = acc[p];
  __syncthreads();
  // block partial layout: [T (128*K) | wide sums (128) | narrow sums (K)]
  double* out = part + (size_t)blockIdx.x * (L * K + L + K);
  for (int e = threadIdx.x; e < L * K + L + K; e += blockDim.x) {
    double s = 0;
    if (e < L * K) {
      const int c = e / K, i = e % K;
      for (int w = 0; w < nhw; ++w) s += red[w][c >> 2][(c & 3) * K + i];
    } else if (e < L * K + L) {
      const int c = e - L * K;
      for (int w = 0; w < nhw; ++w) s += red[w][c >> 2][4 * K + (c & 3)];
    } else {
      const int i = e - L * K - L;
      for (int w = 0; w < nhw; ++w) s += red[w][0][4 * K + 4 + i];   // same in every lane
    }
    out[e] = s;
  }
}

// One block per output element: 256 threads sum the per-block partials, fixed-order tree.
__global__ __launch_bounds__(256) void wgrad_narrow_finalize_kernel(const double* __restrict__ part, int n, int K,
                                                                    int transpose, float* __restrict__ gW,
                                                                    float* __restrict__ gbw,
                                                                    float* __restrict__ gbn) {
  __shared__ double red[256];
  const int e = blockIdx.x;
  const int tot = L * K + L + K;
  double s = 0;
  for (int b = threadIdx.x; b < n; b += blockDim.x) s += part[(size_t)b * tot + e];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = blockDim.x >> 1; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x != 0) return;
  s = red[0];
  if (e < L * K) {
    const int c = e / K, i = e % K;
    if (transpose) gW[i * L + c] += (float)s;
    else gW[c * K + i] += (float)s;
  } else if (e < L * K + L) {
    if (gbw) gbw[e - L * K] += (float)s;
  } else {
    if (gbn) gbn[e - L * K - L] += (float)s;
  }
}

extern "C" int pdg_wgrad_narrow(int rows, const float* wide, const float* narrow, int k_narrow, int transpose,
                                double* partials, float* grad_W, float* grad_b_wide, float* grad_b_narrow,
                                void* stream) {
  PDG_CHECK_ARG(rows > 0, "pdg_wgrad_narrow: rows must be > 0");
  PDG_CHECK_ARG(k_narrow == 1 || k_narrow == 3 || k_narrow == 6, "pdg_wgrad_narrow: k_narrow must be 1, 3 or 6");
  PDG_CHECK_ARG(PDG_ALIGNED(wide), "pdg_wgrad_narrow: misaligned pointer");
  long want = (rows + 7) / 8;
  long cap = (long)device_cus();
  const int grid = (int)(want < cap ? want : cap);
  hipStream_t s = (hipStream_t)stream;
  if (k_narrow == 1)
    hipLaunchKernelGGL(wgrad_narrow_kernel<1>, dim3(grid), dim3(256), 0, s, rows, wide, narrow, partials);
  else if (k_narrow == 3)
    hipLaunchKernelGGL(wgrad_narrow_kernel<3>, dim3(grid), dim3(256), 0, s, rows, wide, narrow, partials);
  else
    hipLaunchKernelGGL(wgrad_narrow_kernel<6>, dim3(grid), dim3(256), 0, s, rows, wide, narrow, partials);
  PDG_CHECK_LAUNCH("pdg_wgrad_narrow");
  const int tot = L * k_narrow + L + k_narrow;
  hipLaunchKernelGGL(wgrad_narrow_finalize_kernel, dim3(tot), dim3(256), 0, s, partials, grid, k_narrow, transpose,
                     grad_W, grad_b_wide, grad_b_narrow);
  PDG_CHECK_LAUNCH("pdg_wgrad_narrow(finalize)");
  return PDG_OK;
}

// The finalize of pdg_wgrad_narrow alone, for block partials formed inside another kernel
// (pdg_mlp2_bwd_coop / pdg_decoder_bwd_coop with narrow_partials).
extern "C" int pdg_wgrad_narrow_finalize(const double* partials, int nparts, int k_narrow, int transpose,
                                         float* grad_W, float* grad_b_wide, float* grad_b_narrow, void* stream) {
  PDG_CHECK_ARG(nparts > 0 && nparts <= MAX_BLOCKS && partials && grad_W, "pdg_wgrad_narrow_finalize: bad arguments");
  PDG_CHECK_ARG(k_narrow == 1 || k_narrow == 3 || k_narrow == 6, "pdg_wgrad_narrow_finalize: k_narrow must be 1, 3 or 6");
  const int tot = L * k_narrow + L + k_narrow;
  hipLaunchKernelGGL(wgrad_narrow_finalize_kernel, dim3(tot), dim3(256), 0, (hipStream_t)stream, partials, nparts,
                     k_narrow, transpose, grad_W, grad_b_wide, grad_b_narrow);
  PDG_CHECK_LAUNCH("pdg_wgrad_narrow_finalize");
  return PDG_OK;
}

// ============================================================================ backward epilogue
// Every end-of-backward reduction in one launch (pdg_bwd_epilogue): the deferred slab reductions
// (pdg_wgrad_reduce_batch), the LayerNorm parameter gradients (pdg_ln_param_grads), up to two narrow
// weight-gradient finalizes (pdg_wgrad_narrow_finalize) and the edge encoder's first-layer sums
// (pdg_enc_narrow_reduce).  Blocks are dealt to the parts by index; each part's block does what the
// separate kernel's block did, in the same order (bitwise the same gradients; the encoder sums use
// 256 threads in place of 512 and add their rows in another fixed order).  Four launches fewer per step.
constexpr int EPI_NARROW_MAX = 2;
struct EpilogueJobs {
  WgradReduceJobs wr;
  int n_wr;
  const double* ln_acc[4];
  int ln_rows[4];
  float* ln_g[4];
  float* ln_b[4];
  int n_ln;
  const double* np[EPI_NARROW_MAX];
  int np_n[EPI_NARROW_MAX], np_k[EPI_NARROW_MAX], np_t[EPI_NARROW_MAX];
  float* np_W[EPI_NARROW_MAX];
  float* np_bw[EPI_NARROW_MAX];
  float* np_bn[EPI_NARROW_MAX];
  int n_np;
  const double* enc;   // edge encoder narrow sums (nslabs x 256), or NULL
  int enc_n;
  float* enc_w0;
  float* enc_b0;
};

__global__ __launch_bounds__(256) void bwd_epilogue_kernel(EpilogueJobs J) {
  __shared__ double dred[256];
  __shared__ float fred[8][33];
  int b = blockIdx.x;
  constexpr int WR_X = (SLAB + 31) / 32;
  if (b < J.n_wr * WR_X) {   // a slab reduction block (wgrad_reduce_batch_kernel)
    const int j = b / WR_X, bx = b % WR_X;
    const float* __restrict__ slabs = J.wr.slabs[j];
    const int n = J.wr.nslabs[j];
    const int el = threadIdx.x & 31, g = threadIdx.x >> 5;
    const int e = bx * 32 + el;
    float acc = 0.f;
    if (e < SLAB) {
      for (int b0 = g; b0 < n; b0 += 64) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = b0 + 8 * u < n ? slabs[(size_t)(b0 + 8 * u) * SLAB + e] : 0.f;
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += v[u];
      }
    }
    fred[g][el] = acc;
    __syncthreads();
    if (g == 0 && e < SLAB) {
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) s += fred[k][el];
      if (e < L * L) {
        const int o = e / L, i = e % L;
        J.wr.gW[j][(size_t)o * J.wr.ld[j] + J.wr.col0[j] + i] += s;
      } else if (J.wr.gb[j]) {
        J.wr.gb[j][e - L * L] += s;
      }
    }
    return;
  }
  b -= J.n_wr * WR_X;
  if (b < J.n_ln * 256) {   // a LayerNorm parameter column (ln_param_grads_kernel)
    const int grp = b / 256, col = b % 256;
    double s = 0;
    for (int r = threadIdx.x; r < J.ln_rows[grp]; r += blockDim.x) s += J.ln_acc[grp][(size_t)r * 256 + col];
    dred[threadIdx.x] = s;
    __syncthreads();
    for (int o = blockDim.x >> 1; o > 0; o >>= 1) {
      if ((int)threadIdx.x < o) dred[threadIdx.x] += dred[threadIdx.x + o];
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      float* g = col < 128 ? J.ln_b[grp] : J.ln_g[grp];
      if (g) g[col & 127] += (float)dred[0];
    }
    return;
  }
  b -= J.n_ln * 256;
  for (int q = 0; q < J.n_np; ++q) {   // a narrow weight-gradient element (wgrad_narrow_finalize_kernel)
    const int K = J.np_k[q], tot = L * K + L + K;
    if (b >= tot) {
      b -= tot;
      continue;
    }
    double s = 0;
    for (int r = threadIdx.x; r < J.np_n[q]; r += blockDim.x) s += J.np[q][(size_t)r * tot + b];
    dred[threadIdx.x] = s;
    __syncthreads();
    for (int o = blockDim.x >> 1; o > 0; o >>= 1) {
      if ((int)threadIdx.x < o) dred[threadIdx.x] += dred[threadIdx.x + o];
      __syncthreads();
    }
    if (threadIdx.x != 0) return;
    s = dred[0];
    if (b < L * K) {
      const int c = b / K, i = b % K;
      if (J.np_t[q]) J.np_W[q][i * L + c] += (float)s;
      else J.np_W[q][c * K + i] += (float)s;
    } else if (b < L * K + L) {
      if (J.np_bw[q]) J.np_bw[q][b - L * K] += (float)s;
    } else {
      if (J.np_bn[q]) J.np_bn[q][b - L * K - L] += (float)s;
    }
    return;
  }
  if (J.enc && b < 2) {   // the edge encoder's w0 (b = 0) / b0 (b = 1) sums (enc_narrow_reduce_kernel's job)
    const int col = threadIdx.x & (L - 1), grp = threadIdx.x >> 7, e = L * b + col;
    double s0 = 0, s1 = 0, s2 = 0, s3 = 0;
    int r = grp;
    for (; r + 6 < J.enc_n; r += 8) {
      s0 += J.enc[(size_t)r * 2 * L + e];
      s1 += J.enc[(size_t)(r + 2) * 2 * L + e];
      s2 += J.enc[(size_t)(r + 4) * 2 * L + e];
      s3 += J.enc[(size_t)(r + 6) * 2 * L + e];
    }
    for (; r < J.enc_n; r += 2) s0 += J.enc[(size_t)r * 2 * L + e];
    dred[threadIdx.x] = (s0 + s1) + (s2 + s3);
    __syncthreads();
    if (grp == 0) {
      const double t = dred[col] + dred[L + col];
      if (b == 0) J.enc_w0[col] += (float)t;
      else J.enc_b0[col] += (float)t;
    }
  }
}

extern "C" int pdg_bwd_epilogue(int n_reduce, const float* const* slabs, const int* nslabs, float* const* grad_W,
                                const int* ld, const int* col0, float* const* grad_b, int n_ln, const double* const* ln_acc,
                                const int* ln_rows, float* const* ln_grad_g, float* const* ln_grad_b, int n_narrow,
                                const double* const* narrow_partials, const int* narrow_nparts, const int* narrow_k,
                                const int* narrow_transpose, float* const* narrow_gW, float* const* narrow_gb_wide,
                                float* const* narrow_gb_narrow, const double* enc_sums, int enc_nslabs,
                                float* enc_grad_w0, float* enc_grad_b0, void* stream) {
  PDG_CHECK_ARG(n_reduce >= 0 && n_reduce <= WRB_MAX && n_ln >= 0 && n_ln <= 4 && n_narrow >= 0 &&
                    n_narrow <= EPI_NARROW_MAX,
                "pdg_bwd_epilogue: bad job counts");
  EpilogueJobs J{};
  J.n_wr = n_reduce;
  for (int i = 0; i < n_reduce; ++i) {
    PDG_CHECK_ARG(slabs[i] && grad_W[i] && nslabs[i] > 0 && nslabs[i] <= MAX_BLOCKS && ld[i] >= L &&
                      col0[i] >= 0 && col0[i] + L <= ld[i],
                  "pdg_bwd_epilogue: bad reduction job %d", i);
    J.wr.slabs[i] = slabs[i];
    J.wr.gW[i] = grad_W[i];
    J.wr.gb[i] = grad_b[i];
    J.wr.nslabs[i] = nslabs[i];
    J.wr.ld[i] = ld[i];
    J.wr.col0[i] = col0[i];
  }
  J.n_ln = n_ln;
  for (int i = 0; i < n_ln; ++i) {
    PDG_CHECK_ARG(ln_acc[i] && ln_rows[i] > 0 && ln_rows[i] <= MAX_BLOCKS, "pdg_bwd_epilogue: bad LayerNorm group %d", i);
    J.ln_acc[i] = ln_acc[i];
    J.ln_rows[i] = ln_rows[i];
    J.ln_g[i] = ln_grad_g[i];
    J.ln_b[i] = ln_grad_b[i];
  }
  J.n_np = n_narrow;
  long nb = (long)n_reduce * ((SLAB + 31) / 32) + (long)n_ln * 256;
  for (int i = 0; i < n_narrow; ++i) {
    PDG_CHECK_ARG(narrow_partials[i] && narrow_nparts[i] > 0 && narrow_nparts[i] <= MAX_BLOCKS && narrow_gW[i] &&
                      (narrow_k[i] == 1 || narrow_k[i] == 3 || narrow_k[i] == 6),
                  "pdg_bwd_epilogue: bad narrow job %d", i);
    J.np[i] = narrow_partials[i];
    J.np_n[i] = narrow_nparts[i];
    J.np_k[i] = narrow_k[i];
    J.np_t[i] = narrow_transpose[i];
    J.np_W[i] = narrow_gW[i];
    J.np_bw[i] = narrow_gb_wide[i];
    J.np_bn[i] = narrow_gb_narrow[i];
    nb += L * narrow_k[i] + L + narrow_k[i];
  }
  PDG_CHECK_ARG(!enc_sums || (enc_nslabs > 0 && enc_grad_w0 && enc_grad_b0), "pdg_bwd_epilogue: bad encoder sums");
  J.enc = enc_sums;
  J.enc_n = enc_nslabs;
  J.enc_w0 = enc_grad_w0;
  J.enc_b0 = enc_grad_b0;
  if (enc_sums) nb += 2;
  if (nb == 0) return PDG_OK;
  hipLaunchKernelGGL(bwd_epilogue_kernel, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream, J);
  PDG_CHECK_LAUNCH("pdg_bwd_epilogue");
  return PDG_OK;
}

// ============================================================================ segmented, LDS-staged wgrad
// One launch per weight and backward: the row segments of every message-passing
// step (and both edge_net evaluations) form one virtual K = sum(rows) reduction.
// Block b owns a contiguous range of virtual rows, staged 32 rows at a time into
// LDS (G and X tiles, double buffered, coalesced 16-byte loads), and keeps the
// whole 128x128 partial in registers: wave w owns the 64x64 quadrant
// (o in 64*(w>>1) + [0,64), i in 64*(w&1) + [0,64)) as 2x2 MFMA 32x32 tiles.
struct WgradSegs {
  const float* G[PDG_MAX_SEGS];
  const float* X[PDG_MAX_SEGS];
  long start[PDG_MAX_SEGS + 1];
  int nseg;
};

constexpr int WG_ROWS = 32;
constexpr int WG_TILE = WG_ROWS * L;   // floats per staged tile

// Segment table copied to LDS once per block (the kernel-argument copy would be
// read with dependent per-lane global loads).  Each thread stages rows
// r_i = base + (tid >> 5) + 8 i (i < 4) of every 32-row tile and tracks the
// segment of each of them incrementally (tiles advance monotonically).
struct WgTable {
  long start[PDG_MAX_SEGS + 1];
  const float* G[PDG_MAX_SEGS];
  const float* X[PDG_MAX_SEGS];
};
constexpr int WG_TABLE_FLOATS = (sizeof(WgTable) + 15) / 16 * 4;

// Several weights' segment passes in one launch (blockIdx.y = job; each job its own slab set):
// the node_net.2 / decoder / node encoder passes were three launches, the two single-segment ones
// ~19 us each for 41 MB (fill / drain).
constexpr int WGJ_MAX = 3;
struct WgradJobs {
  WgradSegs s[WGJ_MAX];
  long total[WGJ_MAX];
  float* slabs[WGJ_MAX];
};

constexpr int WG16 = 16 * X6_ROWB;   // bytes per term plane of a 16-row image (4 KB)
constexpr int WIMG16 = 3 * WG16;     // one 16-row bf16x6 image (12 KB)

// Split one row's 4 columns 4cg .. 4cg + 3 into image row r of a 16-row image.
__device__ __forceinline__ void x6_store1(unsigned char* img, int cg, int r, const f32x4& v) {
  unsigned h0, m0, l0, h1, m1, l1;
  split3_pair(v[0], v[1], h0, m0, l0);
  split3_pair(v[2], v[3], h1, m1, l1);
  const int off = x6_addr(r, 8 * cg);
  *reinterpret_cast<u32x2*>(img + off) = u32x2{h0, h1};
  *reinterpret_cast<u32x2*>(img + WG16 + off) = u32x2{m0, m1};
  *reinterpret_cast<u32x2*>(img + 2 * WG16 + off) = u32x2{l0, l1};
}

// Two-deep form (default; the structure of wgrad_x6_pair2_kernel for one product): one block of 8 waves
// per slab, 16-row rounds with two rounds of (G, X) row loads in flight by round parity, double-
// buffered 16-row images, one barrier per round.  Wave w owns o in 32 (w & 3) + [0, 32), i in
// 64 (w >> 2) + [0, 64) as two 32x32 accumulators.  The block's K steps run in row order (the grouped
// form above summed three row thirds and added them at the end: the same products in another order).
__device__ __forceinline__ void wgrad_x6_body2(const WgradSegs& sg, long total, float* __restrict__ slabs) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem7[];   // [table | parity x (G | X)]
  WgTable* tb = reinterpret_cast<WgTable*>(smem7);
  unsigned char* img = smem7 + WG_TABLE_FLOATS * 4;
  const int nseg = sg.nseg;
  for (int i = threadIdx.x; i <= PDG_MAX_SEGS; i += blockDim.x) tb->start[i] = sg.start[i];
  for (int i = threadIdx.x; i < PDG_MAX_SEGS; i += blockDim.x) {
    tb->G[i] = sg.G[i];
    tb->X[i] = sg.X[i];
  }
  __syncthreads();
  const int nb = gridDim.x;
  long per = (total + nb - 1) / nb;
  per = (per + X6_ROWS - 1) / X6_ROWS * X6_ROWS;
  const long r0 = min(total, per * blockIdx.x), r1 = min(total, per * (blockIdx.x + 1));
  const int l = lane_id(), h = l >> 5, c = l & 31, w = wave_id();
  const int cg = threadIdx.x & 31, rg = threadIdx.x >> 5;   // staged row rg, columns 4 cg ..
  const int ob = 32 * (w & 3), ib = 64 * (w >> 2);
  const int lrow = 8 * h + ((l & 15) >> 2);
  const int lcolb = 2 * (16 * ((l >> 4) & 1) + 4 * (l & 3));
  f32x16 acc[2];
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[b][r] = 0.f;
  f32x4 bs = f32x4{0.f, 0.f, 0.f, 0.f};   // column sums of G
  if (r0 < r1) {
    int seg;
    {
      int lo = 0, hi = nseg;
      while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (tb->start[mid] <= r0) lo = mid; else hi = mid;
      }
      seg = lo;
    }
    f32x4 vg[2], vx[2];
    auto issue = [&](const int s, long base) {   // rows past r1 read row r1 - 1 (zeroed when staged)
      const long vr = min(base + rg, r1 - 1);
      while (seg + 1 < nseg && vr >= tb->start[seg + 1]) ++seg;
      const long r = vr - tb->start[seg];
      vg[s] = ldg4(tb->G[seg] + r * L + 4 * cg);
      vx[s] = ldg4(tb->X[seg] + r * L + 4 * cg);
    };
    auto round = [&](const int s, long base) {
      unsigned char* gimg = img + s * 2 * WIMG16;
      unsigned char* ximg = gimg + WIMG16;
      {
        const bool ok = base + rg < r1;
        const f32x4 zero = f32x4{0.f, 0.f, 0.f, 0.f};
        const f32x4 g = ok ? vg[s] : zero, x = ok ? vx[s] : zero;
        bs += g;
        x6_store1(gimg, cg, rg, g);
        x6_store1(ximg, cg, rg, x);
      }
      issue(s, base + 32);   // the set is free: the round after next
      __syncthreads();       // this round's images complete (the other parity's are the previous round's)
      bf16x8 A[3], B[2][3];
      const int g0 = x6_addr(lrow, lcolb + 2 * ob), g1 = x6_addr(lrow + 4, lcolb + 2 * ob);
#pragma unroll
      for (int p = 0; p < 3; ++p) A[p] = x6_operand(gimg + p * WG16, g0, g1);
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int x0 = x6_addr(lrow, lcolb + 2 * (ib + 32 * b)), x1 = x6_addr(lrow + 4, lcolb + 2 * (ib + 32 * b));
#pragma unroll
        for (int p = 0; p < 3; ++p) B[b][p] = x6_operand(ximg + p * WG16, x0, x1);
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
    };
    issue(0, r0);
    __builtin_amdgcn_sched_barrier(0);
    issue(1, r0 + 16);
    __builtin_amdgcn_sched_barrier(0);
    for (long base = r0; base < r1; base += 32) {   // both rounds always run (a round past r1 adds zeros)
      round(0, base);
      round(1, base + 16);
    }
    __syncthreads();   // the last round's image reads precede the LDS reuse below
  }
  float* slab = slabs + (size_t)blockIdx.x * SLAB;
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int o = ob + (r & 3) + 8 * (r >> 2) + 4 * h;
      const int i = ib + 32 * b + c;
      slab[o * L + i] = acc[b][r];
    }
  // bias sums: the 16 row groups of each column group, in row-group order (the images are dead)
  float* red = reinterpret_cast<float*>(img);
  *reinterpret_cast<f32x4*>(red + 4 * threadIdx.x) = bs;
  __syncthreads();
  if (threadIdx.x < L) {
    const int col = threadIdx.x, g = col >> 2, j = col & 3;
    float sum = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) sum += red[4 * (32 * q + g) + j];
    slab[L * L + col] = sum;
  }
}

__global__ __launch_bounds__(512, 1) void wgrad_x6_kernel2(WgradSegs sg, long total, float* __restrict__ slabs) {
  wgrad_x6_body2(sg, total, slabs);
}

__global__ __launch_bounds__(512, 1) void wgrad_x6_jobs_kernel2(WgradJobs jobs) {
  const int j = blockIdx.y;
  wgrad_x6_body2(jobs.s[j], jobs.total[j], jobs.slabs[j]);
}

constexpr size_t WGJ2_SHM = WG_TABLE_FLOATS * 4 + 2 * 2 * WIMG16;

extern "C" int pdg_wgrad_slabs_per_cu(void) { return 3 / 3; }

extern "C" int pdg_wgrad_segments(int nseg, const float* const* g_ptrs, const float* const* x_ptrs, const int* rows,
                                  float* slabs, int nslabs, void* stream) {
  PDG_CHECK_ARG(nseg > 0 && nseg <= PDG_MAX_SEGS, "pdg_wgrad_segments: 1..%d segments", PDG_MAX_SEGS);
  PDG_CHECK_ARG(nslabs > 0 && nslabs <= MAX_BLOCKS, "pdg_wgrad_segments: bad nslabs");
  WgradSegs sg;
  long tot = 0;
  for (int i = 0; i < nseg; ++i) {
    PDG_CHECK_ARG(rows[i] >= 0, "pdg_wgrad_segments: negative rows");
    PDG_CHECK_ARG(PDG_ALIGNED(g_ptrs[i]) && PDG_ALIGNED(x_ptrs[i]), "pdg_wgrad_segments: misaligned pointer");
    sg.G[i] = g_ptrs[i];
    sg.X[i] = x_ptrs[i];
    sg.start[i] = tot;
    tot += rows[i];
  }
  sg.start[nseg] = tot;
  for (int i = nseg + 1; i <= PDG_MAX_SEGS; ++i) sg.start[i] = tot;
  sg.nseg = nseg;
  PDG_CHECK_ARG(tot > 0, "pdg_wgrad_segments: no rows");
  hipLaunchKernelGGL(wgrad_x6_kernel2, dim3(nslabs), dim3(512), WGJ2_SHM, (hipStream_t)stream, sg, tot, slabs);
  PDG_CHECK_LAUNCH("pdg_wgrad_segments");
  return PDG_OK;
}

extern "C" int pdg_wgrad_segments_batch(int njobs, const int* nseg, const float* const* g_ptrs,
                                        const float* const* x_ptrs, const int* rows, float* const* slabs, int nslabs,
                                        void* stream) {
  PDG_CHECK_ARG(njobs > 0 && njobs <= WGJ_MAX && nseg && g_ptrs && x_ptrs && rows && slabs,
                "pdg_wgrad_segments_batch: 1..%d jobs", WGJ_MAX);
  PDG_CHECK_ARG(nslabs > 0 && nslabs <= MAX_BLOCKS, "pdg_wgrad_segments_batch: bad nslabs");
  WgradJobs jobs;
  int k = 0;
  for (int j = 0; j < njobs; ++j) {
    PDG_CHECK_ARG(nseg[j] > 0 && nseg[j] <= PDG_MAX_SEGS && slabs[j], "pdg_wgrad_segments_batch: bad job");
    WgradSegs& sg = jobs.s[j];
    long tot = 0;
    for (int i = 0; i < nseg[j]; ++i, ++k) {
      PDG_CHECK_ARG(rows[k] >= 0, "pdg_wgrad_segments_batch: negative rows");
      PDG_CHECK_ARG(PDG_ALIGNED(g_ptrs[k]) && PDG_ALIGNED(x_ptrs[k]), "pdg_wgrad_segments_batch: misaligned pointer");
      sg.G[i] = g_ptrs[k];
      sg.X[i] = x_ptrs[k];
      sg.start[i] = tot;
      tot += rows[k];
    }
    sg.start[nseg[j]] = tot;
    for (int i = nseg[j] + 1; i <= PDG_MAX_SEGS; ++i) sg.start[i] = tot;
    sg.nseg = nseg[j];
    PDG_CHECK_ARG(tot > 0, "pdg_wgrad_segments_batch: a job has no rows");
    jobs.total[j] = tot;
    jobs.slabs[j] = slabs[j];
  }
  hipLaunchKernelGGL(wgrad_x6_jobs_kernel2, dim3(nslabs, njobs), dim3(512), WGJ2_SHM, (hipStream_t)stream, jobs);
  PDG_CHECK_LAUNCH("pdg_wgrad_segments_batch");
  return PDG_OK;
}

// ---------------------------------------------------------------------------- pairs
// Two weight gradients that share an operand in one pass (the shared array is read once):
//   SHX (shared X):  dW0 = A0^T A2, dW1 = A1^T A2   (edge_net.0's Wa / Wb: gP, gQ against x)
//   !SHX (shared G): dW0 = A0^T A1, dW1 = A0^T A2   (node_net.0's two halves: gz1n against aggr, x)
// 8 waves: waves 0-3 the 64x64 quadrants of product 0, waves 4-7 those of product 1, each with the
// bf16x6 operand reads of wgrad_x6_kernel; 3 x 24 KB of images, two blocks per CU.  Block b writes
// slab b of slabs0 and of slabs1 (weight + the column sums of that product's G), reduced by
// pdg_wgrad_reduce like pdg_wgrad_segments' slabs.
struct WgradSegs3 {
  const float* A[3][PDG_MAX_SEGS];
  long start[PDG_MAX_SEGS + 1];
  int nseg;
};
struct WgTable3 {
  long start[PDG_MAX_SEGS + 1];
  const float* A[3][PDG_MAX_SEGS];
};
constexpr int WG3_TABLE_BYTES = (sizeof(WgTable3) + 15) / 16 * 16;

// Two-deep form (default): 16-row rounds with TWO rounds of row loads in flight, in the registers one
// 32-row round used to take (two sets of one row x three arrays per thread, by round parity): set s
// is staged for round n and re-issued for round n + 2 at once, so rows are landing while the CU
// multiplies (the form above issues the next round's rows at the top of a round and waits for them
// after its MFMAs).  The images are double-buffered by round parity, one barrier per round.  No
// load is conditional (rows past the block are clamped on load and zeroed when staged).  The weight
// products accumulate the same K steps in the same order (bitwise the same dW); the column sums
// are formed per thread over other rows (fp32, another order).  Per config-2 call 174-179 -> 164-168 us
// (rocprofv3, same box); three sets in flight (PDG_WGP_DEPTH=3, triple-buffered images) measured the
// same as two: what is left is the round's MFMA phase (two waves per SIMD) in series with its stage.
#ifndef PDG_WGP_DEPTH
#define PDG_WGP_DEPTH 2
#endif
constexpr int WGP_DEPTH = PDG_WGP_DEPTH;   // row sets (and image buffers) in flight
template <bool SHX>
__global__ __launch_bounds__(512, 1) void wgrad_x6_pair2_kernel(WgradSegs3 sg, long total, float* __restrict__ slabs0,
                                                               float* __restrict__ slabs1) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem3[];   // [table | parity x A0 | A1 | A2]
  WgTable3* tb = reinterpret_cast<WgTable3*>(smem3);
  unsigned char* img = smem3 + WG3_TABLE_BYTES;
  const int nseg = sg.nseg;
  for (int i = threadIdx.x; i <= PDG_MAX_SEGS; i += blockDim.x) tb->start[i] = sg.start[i];
  for (int i = threadIdx.x; i < 3 * PDG_MAX_SEGS; i += blockDim.x) tb->A[i / PDG_MAX_SEGS][i % PDG_MAX_SEGS] =
      sg.A[i / PDG_MAX_SEGS][i % PDG_MAX_SEGS];
  __syncthreads();
  const int nb = gridDim.x;
  long per = (total + nb - 1) / nb;
  per = (per + X6_ROWS - 1) / X6_ROWS * X6_ROWS;
  const long r0 = min(total, per * blockIdx.x), r1 = min(total, per * (blockIdx.x + 1));
  const int l = lane_id(), h = l >> 5, c = l & 31, w = wave_id();
  const int pw = w >> 2, w4 = w & 3;                      // product, quadrant
  const int cg = threadIdx.x & 31, rg = threadIdx.x >> 5;  // staged row rg, columns 4 cg ..
  const int ob = 64 * (w4 >> 1), ib = 64 * (w4 & 1);
  const int lrow = 8 * h + ((l & 15) >> 2);
  const int lcolb = 2 * (16 * ((l >> 4) & 1) + 4 * (l & 3));
  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  f32x4 bs0 = f32x4{0.f, 0.f, 0.f, 0.f}, bs1 = f32x4{0.f, 0.f, 0.f, 0.f};   // column sums of A0 (and A1)
  if (r0 < r1) {
    int seg;
    {
      int lo = 0, hi = nseg;
      while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (tb->start[mid] <= r0) lo = mid; else hi = mid;
      }
      seg = lo;
    }
    f32x4 v[WGP_DEPTH][3];
    auto issue = [&](const int s, long base) {   // rows past r1 read row r1 - 1 (zeroed when staged)
      const long vr = min(base + rg, r1 - 1);
      while (seg + 1 < nseg && vr >= tb->start[seg + 1]) ++seg;
      const long r = vr - tb->start[seg];
#pragma unroll
      for (int a = 0; a < 3; ++a) v[s][a] = ldg4(tb->A[a][seg] + r * L + 4 * cg);
    };
    auto round = [&](const int s, long base) {
      unsigned char* im = img + s * 3 * WIMG16;
      {
        const bool ok = base + rg < r1;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
          const f32x4 x = ok ? v[s][a] : f32x4{0.f, 0.f, 0.f, 0.f};
          if (a == 0) bs0 += x;
          if (SHX && a == 1) bs1 += x;
          x6_store1(im + a * WIMG16, cg, rg, x);
        }
      }
      issue(s, base + 16 * WGP_DEPTH);   // the set is free: the round WGP_DEPTH ahead
      __syncthreads();       // this round's images complete (the other parity's are the previous round's)
      const unsigned char* gimg = im + (SHX ? pw : 0) * WIMG16;
      const unsigned char* ximg = im + (SHX ? 2 : 1 + pw) * WIMG16;
      bf16x8 A[2][3], B[2][3];
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        const int g0 = x6_addr(lrow, lcolb + 2 * (ob + 32 * a)), g1 = x6_addr(lrow + 4, lcolb + 2 * (ob + 32 * a));
        const int x0 = x6_addr(lrow, lcolb + 2 * (ib + 32 * a)), x1 = x6_addr(lrow + 4, lcolb + 2 * (ib + 32 * a));
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          A[a][p] = x6_operand(gimg + p * WG16, g0, g1);
          B[a][p] = x6_operand(ximg + p * WG16, x0, x1);
        }
      }
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          f32x16 t = acc[a][b];
          t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[a][2], B[b][0], t, 0, 0, 0);
          t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[a][1], B[b][1], t, 0, 0, 0);
          t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[a][0], B[b][2], t, 0, 0, 0);
          t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[a][1], B[b][0], t, 0, 0, 0);
          t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[a][0], B[b][1], t, 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[a][0], B[b][0], t, 0, 0, 0);
        }
    };
    // each set's loads strictly before the next set's, in the order the loop re-issues them
#pragma unroll
    for (int d = 0; d < WGP_DEPTH; ++d) {
      issue(d, r0 + 16 * d);
      __builtin_amdgcn_sched_barrier(0);
    }
    for (long base = r0; base < r1; base += 16 * WGP_DEPTH) {   // every round of a step runs (past r1: zeros)
#pragma unroll
      for (int d = 0; d < WGP_DEPTH; ++d) round(d, base + 16 * d);
    }
    __syncthreads();   // the last round's image reads precede the LDS reuse below
  }
  float* slab = (pw ? slabs1 : slabs0) + (size_t)blockIdx.x * SLAB;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int o = ob + 32 * a + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int i = ib + 32 * b + c;
        slab[o * L + i] = acc[a][b][r];
      }
  float* red = reinterpret_cast<float*>(img);
  *reinterpret_cast<f32x4*>(red + 4 * threadIdx.x) = bs0;
  *reinterpret_cast<f32x4*>(red + 2048 + 4 * threadIdx.x) = SHX ? bs1 : bs0;
  __syncthreads();
  if (threadIdx.x < 2 * L) {
    const int p = threadIdx.x >> 7, col = threadIdx.x & 127, g = col >> 2, j = col & 3;
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) s += red[2048 * p + 4 * (32 * q + g) + j];
    (p ? slabs1 : slabs0)[(size_t)blockIdx.x * SLAB + L * L + col] = s;
  }
}

extern "C" int pdg_wgrad_pairs(int nseg, const float* const* a0_ptrs, const float* const* a1_ptrs,
                               const float* const* a2_ptrs, const int* rows, int shared_x, float* slabs0,
                               float* slabs1, int nslabs, void* stream) {
  PDG_CHECK_ARG(nseg > 0 && nseg <= PDG_MAX_SEGS, "pdg_wgrad_pairs: 1..%d segments", PDG_MAX_SEGS);
  PDG_CHECK_ARG(nslabs > 0 && nslabs <= MAX_BLOCKS && slabs0 && slabs1 && slabs0 != slabs1,
                "pdg_wgrad_pairs: bad slabs");
  WgradSegs3 sg;
  long tot = 0;
  for (int i = 0; i < nseg; ++i) {
    PDG_CHECK_ARG(rows[i] >= 0, "pdg_wgrad_pairs: negative rows");
    PDG_CHECK_ARG(rows[i] == 0 || (a0_ptrs[i] && a1_ptrs[i] && a2_ptrs[i] && PDG_ALIGNED(a0_ptrs[i]) &&
                                   PDG_ALIGNED(a1_ptrs[i]) && PDG_ALIGNED(a2_ptrs[i])),
                  "pdg_wgrad_pairs: null or misaligned pointer");
    sg.A[0][i] = a0_ptrs[i];
    sg.A[1][i] = a1_ptrs[i];
    sg.A[2][i] = a2_ptrs[i];
    sg.start[i] = tot;
    tot += rows[i];
  }
  for (int i = nseg; i < PDG_MAX_SEGS; ++i) sg.A[0][i] = sg.A[1][i] = sg.A[2][i] = nullptr;
  sg.start[nseg] = tot;
  for (int i = nseg + 1; i <= PDG_MAX_SEGS; ++i) sg.start[i] = tot;
  sg.nseg = nseg;
  PDG_CHECK_ARG(tot > 0, "pdg_wgrad_pairs: no rows");
  const size_t shm = WG3_TABLE_BYTES + WGP_DEPTH * 3 * WIMG16;
  if (shared_x)
    hipLaunchKernelGGL(wgrad_x6_pair2_kernel<true>, dim3(nslabs), dim3(512), shm, (hipStream_t)stream, sg, tot, slabs0,
                       slabs1);
  else
    hipLaunchKernelGGL(wgrad_x6_pair2_kernel<false>, dim3(nslabs), dim3(512), shm, (hipStream_t)stream, sg, tot, slabs0,
                       slabs1);
  PDG_CHECK_LAUNCH("pdg_wgrad_pairs");
  return PDG_OK;
}
