// Backward kernels of the P-DivGNN hot path (autograd of gnn_local_stress/models.py:288-326).
//
// Conventions: pdg_common.hpp.  Transposed weights (W^T) are passed explicitly
// (pdg_transpose), so every LDS image is built with contiguous 16-byte loads.
//
// graph-LayerNorm backward (PyG LayerNorm mode="graph", y = g*xhat + b,
// xhat = (a - mean)/(std + eps)), over all M = rows*128 elements of a call:
//   ga = rstd * (g*gy - S1/M) - xhat * S2 / (M*std),  S1 = sum g*gy,  S2 = sum g*gy*xhat
// S1/S2 come from the per-channel sums (pdg_ln_colsum*), which are also the
// LayerNorm parameter gradients.
#include "pdg_common.hpp"
#include "pdg_runtime.hpp"

using namespace pdg;

// ga2 -> gz2 for one fragment (in place on gy): LN backward and relu mask.
__device__ __forceinline__ void ln_relu_bwd(float (&gy)[FRAG], const float (&a2)[FRAG], const LNStat& st,
                                            const pdg_ln_bwd& lb, const float* __restrict__ g) {
  const float* gp = g + lane_col();
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const f32x4 gg = ld4(gp, t);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int s = 4 * t + j;
      const float xhat = div_den(a2[s] - st.mean, st.den, st.rstd);
      const float ga = st.rstd * (gg[j] * gy[s] - lb.c1) - xhat * lb.c2;
      gy[s] = a2[s] > 0.f ? ga : 0.f;
    }
    if ((t & 3) == 3) PDG_FENCE();
  }
}

// ln_relu_bwd with the LayerNorm weight as a FeatVec (no vector-memory access).
__device__ __forceinline__ void ln_relu_bwd_fv(float (&gy)[FRAG], const float (&a2)[FRAG], const LNStat& st,
                                               const pdg_ln_bwd& lb, const FeatVec& g) {
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const f32x4 gg = featvec_chunk(g, t);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int s = 4 * t + j;
      const float xhat = div_den(a2[s] - st.mean, st.den, st.rstd);
      const float ga = st.rstd * (gg[j] * gy[s] - lb.c1) - xhat * lb.c2;
      gy[s] = a2[s] > 0.f ? ga : 0.f;
    }
  }
}

__device__ __forceinline__ void relu_mask_acc(float (&v)[FRAG], const Acc& acc, const float (&a)[FRAG]) {
  PDG_FOR_FRAG(s) v[s] = a[s] > 0.f ? ACC(acc, s) : 0.f;
}

// ============================================================================ decoder backward
__global__ __launch_bounds__(384, 3) void decoder_bwd_kernel(int N, const float* __restrict__ gy,
                                                              const float* __restrict__ a1d,
                                                              const float* __restrict__ Wd2,
                                                              const float* __restrict__ Wd1T,
                                                              float* __restrict__ gz1d,
                                                              float* __restrict__ gx) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* w2l = lds + WBLK;   // Wd2 (3 x 128)
  load_wblock(lds, Wd1T, L, 0);
  for (int i = threadIdx.x; i < 3 * L; i += blockDim.x) w2l[i] = Wd2[i];
  __syncthreads();
  const int l = lane_id();
  PDG_TILE_LOOP(N) {
    const int row = tile * TILE + (l & 15);
    const bool valid = row < N;
    const int rc = valid ? row : N - 1;
    const float g0 = gy[(size_t)rc * 3], g1 = gy[(size_t)rc * 3 + 1], g2 = gy[(size_t)rc * 3 + 2];
    float v[FRAG];
    const int lc = lane_col();
    const float* w0 = w2l + lc;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      f32x4 a[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) a[t] = ld4(a1d + (size_t)rc * L + lc, 4 * q + t);
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int s = 16 * q + 4 * t + j;
          const int f = 16 * (4 * q + t) + j;   // feature offset beyond lane_col()
          const float ga = fmaf(g2, w0[2 * L + f], fmaf(g1, w0[L + f], g0 * w0[f]));
          v[s] = a[t][j] > 0.f ? ga : 0.f;
        }
      PDG_FENCE();
    }
    if (valid) store_frag(gz1d + (size_t)row * L, v);
    Acc acc;
    zero_acc(acc);
    gemm128(acc, lds, v);
    if (valid) store_acc(gx + (size_t)row * L, acc);
  }
}

extern "C" int pdg_decoder_bwd(int n_nodes, const float* gy, const float* a1d, const float* Wd2,
                               const float* Wd1T, float* gz1d, float* gx, void* stream) {
  PDG_CHECK_ARG(n_nodes > 0, "pdg_decoder_bwd: n_nodes must be > 0");
  PDG_CHECK_ARG(PDG_ALIGNED(a1d) && PDG_ALIGNED(gz1d) && PDG_ALIGNED(gx) && PDG_ALIGNED(Wd1T),
                "pdg_decoder_bwd: misaligned pointer");
  const int grid = persistent_grid(n_nodes, 6, 2);
  hipLaunchKernelGGL(decoder_bwd_kernel, dim3(grid), dim3(384), (WBLK + 3 * L) * sizeof(float), (hipStream_t)stream,
                     n_nodes, gy, a1d, Wd2, Wd1T, gz1d, gx);
  PDG_CHECK_LAUNCH("pdg_decoder_bwd");
  return PDG_OK;
}

// ============================================================================ LN column sums
// Half-wave per row (lane j: channels 4j..4j+3); fp64 accumulation; block partial
// = [sum gy (128) | sum gy*xhat (128)].
__global__ __launch_bounds__(256) void ln_colsum_kernel(int M, const float* __restrict__ gyr,
                                                        const int* __restrict__ gidx,
                                                        const float* __restrict__ a2,
                                                        const pdg_ln_stat* __restrict__ stp,
                                                        double* __restrict__ part, const float* __restrict__ lg,
                                                        double* __restrict__ sp, int accumulate) {
  __shared__ double red[8][256];
  __shared__ double row[256], tmp[256];
  const int hw = threadIdx.x >> 5, j = threadIdx.x & 31;
  const int nhw = blockDim.x >> 5;
  const float mean = stp->mean, den = stp->den, rstd = stp->rstd;
  double sg[4] = {0, 0, 0, 0}, sx[4] = {0, 0, 0, 0};
  for (int k = blockIdx.x * nhw + hw; k < M; k += gridDim.x * nhw) {
    const int gr = gidx ? gidx[k] : k;
    const f32x4 g = reinterpret_cast<const f32x4*>(gyr + (size_t)gr * L)[j];
    const f32x4 a = reinterpret_cast<const f32x4*>(a2 + (size_t)k * L)[j];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float xhat = div_den(a[c] - mean, den, rstd);
      sg[c] += (double)g[c];
      sx[c] += (double)(g[c] * xhat);
    }
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    red[hw][4 * j + c] = sg[c];
    red[hw][128 + 4 * j + c] = sx[c];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 256; i += blockDim.x) {
    double s = 0;
    for (int w = 0; w < nhw; ++w) s += red[w][i];
    row[i] = s;
  }
  __syncthreads();
  lnb_emit(row, lg, part, accumulate, sp, tmp);
}

extern "C" int pdg_ln_colsum(int rows, const float* gy_rows, const int* gidx, const float* a2,
                             const pdg_ln_stat* st, double* partials, int* nparts, const float* ln_g,
                             double* pairs, int accumulate, void* stream) {
  PDG_CHECK_ARG(rows > 0, "pdg_ln_colsum: rows must be > 0");
  PDG_CHECK_ARG(PDG_ALIGNED(gy_rows) && PDG_ALIGNED(a2), "pdg_ln_colsum: misaligned pointer");
  long want = (rows + 7) / 8;
  long cap = (long)device_cus() * 2;
  if (cap > MAX_BLOCKS) cap = MAX_BLOCKS;
  const int grid = (int)(want < cap ? want : cap);
  PDG_CHECK_ARG(!pairs || ln_g, "pdg_ln_colsum: pairs need ln_g");
  hipLaunchKernelGGL(ln_colsum_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, rows, gy_rows, gidx, a2, st,
                     partials, ln_g, pairs, accumulate);
  PDG_CHECK_LAUNCH("pdg_ln_colsum");
  if (nparts) *nparts = grid;
  return PDG_OK;
}

#ifndef PDG_COLSUM_NODES_BPC
#define PDG_COLSUM_NODES_BPC 2   // 2 blocks per CU: config-2 step -0.008..-0.018 ms in 3 of 3 same-box A/B pairs
#endif
// every block adds its partial row into the caller's LayerNorm accumulator group, whose capacity is
// 2 rows per CU (pdg_ln_colsum in include/pdivgnn.h; EPDEngine._acc_rows): a larger grid would write
// into the next group's rows
static_assert(PDG_COLSUM_NODES_BPC >= 1 && PDG_COLSUM_NODES_BPC <= 2,
              "ln_colsum_nodes: the accumulator holds 2 partial rows per CU");
__global__ __launch_bounds__(256) void ln_colsum_nodes_kernel(int N, const float* __restrict__ gaggr,
                                                              const int* __restrict__ rowptr,
                                                              const float* __restrict__ xs,
                                                              double* __restrict__ part, const float* __restrict__ lg,
                                                              double* __restrict__ sp, int accumulate) {
  __shared__ double red[8][256];
  __shared__ double row[256], tmp[256];
  const int hw = threadIdx.x >> 5, j = threadIdx.x & 31;
  const int nhw = blockDim.x >> 5;
  double sg[4] = {0, 0, 0, 0}, sx[4] = {0, 0, 0, 0};
  for (int v = blockIdx.x * nhw + hw; v < N; v += gridDim.x * nhw) {
    const float deg = (float)(rowptr[v + 1] - rowptr[v]);
    const f32x4 g = reinterpret_cast<const f32x4*>(gaggr + (size_t)v * L)[j];
    const f32x4 x = reinterpret_cast<const f32x4*>(xs + (size_t)v * L)[j];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      sg[c] += (double)deg * (double)g[c];
      sx[c] += (double)g[c] * (double)x[c];
    }
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    red[hw][4 * j + c] = sg[c];
    red[hw][128 + 4 * j + c] = sx[c];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 256; i += blockDim.x) {
    double s = 0;
    for (int w = 0; w < nhw; ++w) s += red[w][i];
    row[i] = s;
  }
  __syncthreads();
  lnb_emit(row, lg, part, accumulate, sp, tmp);
}

extern "C" int pdg_ln_colsum_nodes(int n_nodes, const float* gaggr, const int* rowptr, const float* xhat_sum,
                                   double* partials, int* nparts, const float* ln_g, double* pairs, int accumulate,
                                   void* stream) {
  PDG_CHECK_ARG(n_nodes > 0, "pdg_ln_colsum_nodes: n_nodes must be > 0");
  PDG_CHECK_ARG(PDG_ALIGNED(gaggr) && PDG_ALIGNED(xhat_sum), "pdg_ln_colsum_nodes: misaligned pointer");
  long want = (n_nodes + 7) / 8;
  long cap = (long)device_cus() * PDG_COLSUM_NODES_BPC;   // partial rows: the engine keeps 2 per CU
  if (cap > MAX_BLOCKS) cap = MAX_BLOCKS;
  const int grid = (int)(want < cap ? want : cap);
  PDG_CHECK_ARG(!pairs || ln_g, "pdg_ln_colsum_nodes: pairs need ln_g");
  hipLaunchKernelGGL(ln_colsum_nodes_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, n_nodes, gaggr, rowptr,
                     xhat_sum, partials, ln_g, pairs, accumulate);
  PDG_CHECK_LAUNCH("pdg_ln_colsum_nodes");
  if (nparts) *nparts = grid;
  return PDG_OK;
}

// Two-level reduction of the per-block partials (P x 256 doubles): one block per
// column sums its P partials with 256 threads and a fixed-order tree, then a
// single block turns the 256 column sums into parameter gradients and S1/S2.
__device__ __forceinline__ double block_tree_sum(double x, double* red) {
  red[threadIdx.x] = x;
  __syncthreads();
  for (int o = blockDim.x >> 1; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  return red[0];
}

__global__ __launch_bounds__(256) void colsum_reduce_kernel(const double* __restrict__ part, int n, int width,
                                                            double* __restrict__ out) {
  __shared__ double red[256];
  const int col = blockIdx.x;
  double s = 0;
  for (int b = threadIdx.x; b < n; b += blockDim.x) s += part[(size_t)b * width + col];
  const double t = block_tree_sum(s, red);
  if (threadIdx.x == 0) out[col] = t;
}

__global__ __launch_bounds__(128) void ln_colsum_finalize_kernel(const double* __restrict__ cols,
                                                                 const float* __restrict__ g,
                                                                 const pdg_ln_stat* __restrict__ stp,
                                                                 float* __restrict__ grad_g,
                                                                 float* __restrict__ grad_b,
                                                                 pdg_ln_bwd* __restrict__ out) {
  __shared__ double red2[2 * 16];
  const int c = threadIdx.x;
  const double sg = cols[c], sx = cols[128 + c];
  if (grad_b) grad_b[c] += (float)sg;
  if (grad_g) grad_g[c] += (float)sx;
  double s1 = (double)g[c] * sg, s2 = (double)g[c] * sx;
  block_sum2(s1, s2, red2);
  if (threadIdx.x == 0) {
    const double M = stp->count;
    const double sd = stp->std_d;
    pdg_ln_bwd r;
    r.S1 = s1;
    r.S2 = s2;
    r.c1 = (float)(s1 / M);
    r.c2 = sd > 0 ? (float)(s2 / (M * sd)) : 0.f;
    *out = r;
  }
}

extern "C" int pdg_ln_colsum_finalize(const double* partials, int nparts, const float* ln_g,
                                      const pdg_ln_stat* st, float* grad_g, float* grad_b, pdg_ln_bwd* out,
                                      void* stream) {
  PDG_CHECK_ARG(nparts > 0 && nparts < MAX_BLOCKS, "pdg_ln_colsum_finalize: bad nparts");
  // the 256 column sums go into the row right after the last partial (see the header)
  double* cols = const_cast<double*>(partials) + (size_t)nparts * 256;
  hipLaunchKernelGGL(colsum_reduce_kernel, dim3(256), dim3(256), 0, (hipStream_t)stream, partials, nparts, 256, cols);
  PDG_CHECK_LAUNCH("pdg_ln_colsum_finalize(reduce)");
  hipLaunchKernelGGL(ln_colsum_finalize_kernel, dim3(1), dim3(128), 0, (hipStream_t)stream, cols, ln_g, st, grad_g,
                     grad_b, out);
  PDG_CHECK_LAUNCH("pdg_ln_colsum_finalize");
  return PDG_OK;
}

// End of the backward: the LayerNorm parameter gradients from the per-block column accumulators
// (lnb_emit), one block per (group, column): grad_b[c] += sum of column c, grad_g[c] += column
// 128 + c, summed over the group's rows in a fixed order.
constexpr int LNP_MAX = 4;
struct LnParamJobs {
  const double* acc[LNP_MAX];
  int rows[LNP_MAX];
  float* grad_g[LNP_MAX];
  float* grad_b[LNP_MAX];
};

__global__ __launch_bounds__(256) void ln_param_grads_kernel(LnParamJobs jb) {
  __shared__ double red[256];
  const int grp = blockIdx.y, col = blockIdx.x;          // col < 256: 0..127 sum gy, 128..255 sum gy*xhat
  double s = 0;
  for (int b = threadIdx.x; b < jb.rows[grp]; b += blockDim.x) s += jb.acc[grp][(size_t)b * 256 + col];
  const double t = block_tree_sum(s, red);
  if (threadIdx.x == 0) {
    float* g = col < 128 ? jb.grad_b[grp] : jb.grad_g[grp];
    if (g) g[col & 127] += (float)t;
  }
}

extern "C" int pdg_ln_param_grads(int ngroups, const double* const* acc, const int* rows, float* const* grad_g,
                                  float* const* grad_b, void* stream) {
  PDG_CHECK_ARG(ngroups > 0 && ngroups <= LNP_MAX, "pdg_ln_param_grads: 1..%d groups", LNP_MAX);
  LnParamJobs jb{};
  for (int i = 0; i < ngroups; ++i) {
    PDG_CHECK_ARG(acc[i] && rows[i] > 0 && rows[i] <= MAX_BLOCKS, "pdg_ln_param_grads: bad group %d", i);
    jb.acc[i] = acc[i];
    jb.rows[i] = rows[i];
    jb.grad_g[i] = grad_g[i];
    jb.grad_b[i] = grad_b[i];
  }
  hipLaunchKernelGGL(ln_param_grads_kernel, dim3(256, ngroups), dim3(256), 0, (hipStream_t)stream, jb);
  PDG_CHECK_LAUNCH("pdg_ln_param_grads");
  return PDG_OK;
}

// ============================================================================ MLP tail backward
__global__ __launch_bounds__(384, 3) void mlp2_bwd_kernel(int M, const float* __restrict__ gyr,
                                                           const int* __restrict__ gidx,
                                                           const float* __restrict__ a2,
                                                           const float* __restrict__ a1,
                                                           const pdg_ln_stat* __restrict__ stp,
                                                           const pdg_ln_bwd* __restrict__ lbp,
                                                           const float* __restrict__ lg,
                                                           const float* __restrict__ W2T,
                                                           float* __restrict__ gz2, float* __restrict__ gz1,
                                                           const double* __restrict__ lb_pairs, int lb_npairs) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  load_wblock(lds, W2T, L, 0);
  __syncthreads();
  const LNStat st = *reinterpret_cast<const LNStat*>(stp);
  const pdg_ln_bwd lb = lnb_resolve(lbp, lb_pairs, lb_npairs, stp);
  const int l = lane_id();
  PDG_TILE_LOOP(M) {
    const int row = tile * TILE + (l & 15);
    const bool valid = row < M;
    const int rc = valid ? row : M - 1;
    const int gr = gidx ? gidx[rc] : rc;
    float v[FRAG], a[FRAG];
    load_frag(v, gyr + (size_t)gr * L);
    load_frag(a, a2 + (size_t)rc * L);
    ln_relu_bwd(v, a, st, lb, lg);
    if (valid) store_frag(gz2 + (size_t)row * L, v);
    Acc acc;
    zero_acc(acc);
    gemm128(acc, lds, v);
    load_frag(a, a1 + (size_t)rc * L);
    relu_mask_acc(v, acc, a);
    if (valid) store_frag(gz1 + (size_t)row * L, v);
  }
}

extern "C" int pdg_mlp2_bwd(int rows, const float* gy_rows, const int* gidx, const float* a2, const float* a1,
                            const pdg_ln_stat* st, const pdg_ln_bwd* lb, const float* ln_g, const float* W2T,
                            float* gz2, float* gz1, const double* lb_pairs, int lb_npairs, void* stream) {
  PDG_CHECK_ARG(rows > 0, "pdg_mlp2_bwd: rows must be > 0");
  PDG_CHECK_ARG(lb || lb_pairs, "pdg_mlp2_bwd: need lb or lb_pairs");
  PDG_CHECK_ARG(PDG_ALIGNED(gy_rows) && PDG_ALIGNED(a2) && PDG_ALIGNED(a1) && PDG_ALIGNED(gz2) &&
                    PDG_ALIGNED(gz1) && PDG_ALIGNED(W2T),
                "pdg_mlp2_bwd: misaligned pointer");
  const int grid = persistent_grid(rows, 6, 2);
  hipLaunchKernelGGL(mlp2_bwd_kernel, dim3(grid), dim3(384), WBLK * sizeof(float), (hipStream_t)stream, rows,
                     gy_rows, gidx, a2, a1, st, lb, ln_g, W2T, gz2, gz1, lb_pairs, lb_npairs);
  PDG_CHECK_LAUNCH("pdg_mlp2_bwd");
  return PDG_OK;
}

// ============================================================================ dual / summed GEMMs
__global__ __launch_bounds__(768, 3) void gemm_dual_kernel(int M, const float* __restrict__ in,
                                                            const float* __restrict__ W0T,
                                                            const float* __restrict__ W1T,
                                                            const float* __restrict__ res0,
                                                            const float* __restrict__ res1,
                                                            float* __restrict__ out0, float* __restrict__ out1) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  load_wblock(lds, W0T, L, 0);
  load_wblock(lds + WBLK, W1T, L, 0);
  __syncthreads();
  const int l = lane_id();
  PDG_TILE_LOOP(M) {
    const int row = tile * TILE + (l & 15);
    const bool valid = row < M;
    const int rc = valid ? row : M - 1;
    float v[FRAG], r[FRAG];
    load_frag(v, in + (size_t)rc * L);
    Acc acc;
    zero_acc(acc);
    gemm128(acc, lds, v);
    if (res0) {
      load_frag(r, res0 + (size_t)rc * L);
      PDG_FOR_FRAG(s) ACC(acc, s) += r[s];
    }
    if (valid) store_acc(out0 + (size_t)row * L, acc);
    zero_acc(acc);
    gemm128(acc, lds + WBLK, v);
    if (res1) {
      load_frag(r, res1 + (size_t)rc * L);
      PDG_FOR_FRAG(s) ACC(acc, s) += r[s];
    }
    if (valid) store_acc(out1 + (size_t)row * L, acc);
  }
}

extern "C" int pdg_gemm_dual(int rows, const float* in, const float* W0T, const float* W1T, const float* res0,
                             const float* res1, float* out0, float* out1, void* stream) {
  PDG_CHECK_ARG(rows > 0, "pdg_gemm_dual: rows must be > 0");
  PDG_CHECK_ARG(PDG_ALIGNED(in) && PDG_ALIGNED(out0) && PDG_ALIGNED(out1) && PDG_ALIGNED(W0T) &&
                    PDG_ALIGNED(W1T) && (!res0 || PDG_ALIGNED(res0)) && (!res1 || PDG_ALIGNED(res1)),
                "pdg_gemm_dual: misaligned pointer");
  const int grid = persistent_grid(rows, 12, 1);
  hipLaunchKernelGGL(gemm_dual_kernel, dim3(grid), dim3(768), 2 * WBLK * sizeof(float), (hipStream_t)stream, rows,
                     in, W0T, W1T, res0, res1, out0, out1);
  PDG_CHECK_LAUNCH("pdg_gemm_dual");
  return PDG_OK;
}

__global__ __launch_bounds__(768, 3) void gemm_sum2_kernel(int M, const float* __restrict__ in0,
                                                            const float* __restrict__ in1,
                                                            const float* __restrict__ W0T,
                                                            const float* __restrict__ W1T,
                                                            const float* __restrict__ res,
                                                            float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  load_wblock(lds, W0T, L, 0);
  load_wblock(lds + WBLK, W1T, L, 0);
  __syncthreads();
  const int l = lane_id();
  PDG_TILE_LOOP(M) {
    const int row = tile * TILE + (l & 15);
    const bool valid = row < M;
    const int rc = valid ? row : M - 1;
    float v[FRAG];
    Acc acc;
    zero_acc(acc);
    load_frag(v, in0 + (size_t)rc * L);
    gemm128(acc, lds, v);
    load_frag(v, in1 + (size_t)rc * L);
    gemm128(acc, lds + WBLK, v);
    if (res) {
      load_frag(v, res + (size_t)rc * L);
      PDG_FOR_FRAG(s) ACC(acc, s) += v[s];
    }
    if (valid) store_acc(out + (size_t)row * L, acc);
  }
}

extern "C" int pdg_gemm_sum2(int rows, const float* in0, const float* in1, const float* W0T, const float* W1T,
                             const float* res, float* out, void* stream) {
  PDG_CHECK_ARG(rows > 0, "pdg_gemm_sum2: rows must be > 0");
  PDG_CHECK_ARG(PDG_ALIGNED(in0) && PDG_ALIGNED(in1) && PDG_ALIGNED(out) && PDG_ALIGNED(W0T) &&
                    PDG_ALIGNED(W1T) && (!res || PDG_ALIGNED(res)),
                "pdg_gemm_sum2: misaligned pointer");
  const int grid = persistent_grid(rows, 12, 1);
  hipLaunchKernelGGL(gemm_sum2_kernel, dim3(grid), dim3(768), 2 * WBLK * sizeof(float), (hipStream_t)stream, rows,
                     in0, in1, W0T, W1T, res, out);
  PDG_CHECK_LAUNCH("pdg_gemm_sum2");
  return PDG_OK;
}

// ============================================================================ fused edge backward
// Memory-order discipline as in edge_fwd_kernel (pdg_fwd.hip): vmcnt counts loads and
// stores together in issue order, so each row a later step needs is loaded before
// the stores that precede that step (a1m before gz2m is stored, ge_next / a2e before
// gz1m, a1e before gz2e, ge_next as the ge_out accumulator before gz1e), and the
// next tile's gathered gaggr row and a2m row before this tile's last store.
#ifndef PDG_EDGE_BWD_WAVES
#define PDG_EDGE_BWD_WAVES PDG_EDGE_WAVES
#endif
constexpr int EB_WAVES = PDG_EDGE_BWD_WAVES;

template <bool EU>
__global__ __launch_bounds__(64 * EB_WAVES, EB_WAVES / 4) void edge_bwd_kernel(
    int E, const int* __restrict__ dst, const float* __restrict__ gaggr, const float* __restrict__ ge_next,
    const float* __restrict__ a2m, const float* __restrict__ a1m, const float* __restrict__ a2e,
    const float* __restrict__ a1e, const pdg_ln_stat* __restrict__ stm_p, const pdg_ln_stat* __restrict__ ste_p,
    const pdg_ln_bwd* __restrict__ lbm_p, const pdg_ln_bwd* __restrict__ lbe_p, const float* __restrict__ lg,
    const float* __restrict__ W2T, const float* __restrict__ WcT, float* __restrict__ gz2m,
    float* __restrict__ gz1m, float* __restrict__ gz2e, float* __restrict__ gz1e, float* __restrict__ gC,
    float* __restrict__ ge_out, const double* __restrict__ pm, int npm, const double* __restrict__ pe, int npe) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  load_wblock_swz(lds, WcT, L, 0);                                   // Wc^T (fp32)
  unsigned char* w2p = reinterpret_cast<unsigned char*>(lds + 128 * 128);
  load_wplanes(w2p, W2T, L, 0);                                      // W2^T as bf16 term planes
#define PDG_GEMM_2(acc, v) gemm128_x6(acc, w2p, v)
#define PDG_GEMM_C(acc, v) gemm128_swz(acc, lds, v)
  const FeatVec fg = load_featvec(lg);
  __syncthreads();
  const LNStat stm = *reinterpret_cast<const LNStat*>(stm_p);
  const LNStat ste = *reinterpret_cast<const LNStat*>(EU ? ste_p : stm_p);
  const pdg_ln_bwd lbm = lnb_resolve(lbm_p, pm, npm, stm_p);
  const pdg_ln_bwd lbe = EU ? lnb_resolve(lbe_p, pe, npe, ste_p) : lbm;
  const int l = lane_id();
  const int lc = lane_col();
  const int nw = blockDim.x >> 6, ntiles = tiles_of(E), stride = gridDim.x * nw;
  int tile = xcd_block() * nw + wave_id();
  // rows are clamped, so the prefetches below are unconditional (never live across the loop)
  auto rowc = [&](int t) {
    const int r = t * TILE + (l & 15);
    return r < E ? r : E - 1;
  };
  float gm[FRAG], a[FRAG];   // this tile's gaggr[dst] and a2m rows
  {
    const int rc = rowc(tile);
    load_frag(gm, gaggr + (size_t)dst[rc] * L);
    load_frag(a, a2m + (size_t)rc * L);
  }
  int d_next = dst[rowc(tile + stride)];
  for (; tile < ntiles; tile += stride) {
    const int row = tile * TILE + (l & 15);
    const bool valid = row < E;
    const int rc = valid ? row : E - 1;
    float A[FRAG];
    Acc Z;
    // ---- message path: gy = gaggr[dst]   (scatter_add_ backward = gather)
    ln_relu_bwd_fv(gm, a, stm, lbm, fg);                   // gm := gz2m
    load_frag(A, a1m + (size_t)rc * L);
    if (valid) store_frag(gz2m + (size_t)row * L, gm);
    zero_acc(Z);
    PDG_GEMM_2(Z, gm);
    float v[FRAG];
    relu_mask_acc(v, Z, A);                                // v := gz1m
    if (EU) {
      // ---- edge-update path: gy = ge_next
      float G[FRAG];
      load_frag(G, ge_next + (size_t)rc * L);
      load_frag(A, a2e + (size_t)rc * L);
      if (valid) store_frag(gz1m + (size_t)row * L, v);
      ln_relu_bwd_fv(G, A, ste, lbe, fg);                  // G := gz2e
      zero_acc(Z);
      PDG_GEMM_2(Z, G);
      load_frag(A, a1e + (size_t)rc * L);
      if (valid) store_frag(gz2e + (size_t)row * L, G);
      relu_mask_acc(G, Z, A);                              // G := gz1e
      // ge_out = ge_next + Wc^T gC: the accumulator starts as ge_next
      {
        const float* gp = ge_next + (size_t)rc * L + lc;
#pragma unroll
        for (int T = 0; T < 8; ++T) Z.b[T] = ld4(gp, T);
      }
      if (valid) store_frag(gz1e + (size_t)row * L, G);
      PDG_FOR_FRAG(s) v[s] = v[s] + G[s];                  // gC = gz1m + gz1e
    } else {
      if (valid) store_frag(gz1m + (size_t)row * L, v);
      zero_acc(Z);
    }
    // ---- ge_out = [ge_next +] Wc^T gC
    if (valid) store_frag(gC + (size_t)row * L, v);
    PDG_GEMM_C(Z, v);
    // next tile's rows before this tile's last store
    {
      const int rcn = rowc(tile + stride);
      load_frag(gm, gaggr + (size_t)d_next * L);
      load_frag(a, a2m + (size_t)rcn * L);
      d_next = dst[rowc(tile + 2 * stride)];
    }
    PDG_FENCE();
    if (valid) store_acc(ge_out + (size_t)row * L, Z);
  }
#undef PDG_GEMM_2
#undef PDG_GEMM_C
}

extern "C" int pdg_edge_bwd(int n_edges, const int* dst, const float* gaggr, const float* ge_next,
                            const float* a2m, const float* a1m, const float* a2e, const float* a1e,
                            const pdg_ln_stat* st_m, const pdg_ln_stat* st_e, const pdg_ln_bwd* lb_m,
                            const pdg_ln_bwd* lb_e, const float* ln_g, const float* W2T, const float* WcT,
                            float* gz2m, float* gz1m, float* gz2e, float* gz1e, float* gC, float* ge_out,
                            const double* pairs_m, int npairs_m, const double* pairs_e, int npairs_e,
                            void* stream) {
  PDG_CHECK_ARG(n_edges > 0, "pdg_edge_bwd: n_edges must be > 0");
  PDG_CHECK_ARG(lb_m || pairs_m, "pdg_edge_bwd: need lb_m or pairs_m");
  // null outputs are refused here rather than written through on the device (a host-side mix-up of the
  // fused and unfused paths once passed gz2m == NULL and faulted the GPU)
  PDG_CHECK_ARG(dst && gaggr && a2m && a1m && st_m && ln_g && W2T && WcT && gz2m && gz1m && gC && ge_out,
                "pdg_edge_bwd: null argument");
  PDG_CHECK_ARG(!ge_next || (a2e && a1e && gz2e && gz1e), "pdg_edge_bwd: null edge-update argument");
  PDG_CHECK_ARG(PDG_ALIGNED(gaggr) && PDG_ALIGNED(a2m) && PDG_ALIGNED(a1m) && PDG_ALIGNED(gz2m) &&
                    PDG_ALIGNED(gz1m) && PDG_ALIGNED(gC) && PDG_ALIGNED(ge_out),
                "pdg_edge_bwd: misaligned pointer");
  PDG_CHECK_ARG(!ge_next || (PDG_ALIGNED(ge_next) && PDG_ALIGNED(a2e) && PDG_ALIGNED(a1e) && PDG_ALIGNED(gz2e) &&
                             PDG_ALIGNED(gz1e) && st_e && (lb_e || pairs_e)),
                "pdg_edge_bwd: edge-update arguments missing or misaligned");
  PDG_CHECK_ARG(ge_out != ge_next, "pdg_edge_bwd: ge_out must not alias ge_next");
  const int grid = persistent_grid(n_edges, EB_WAVES, 1);
  const size_t shm = (size_t)EDGE_LDS_BYTES;
  if (ge_next)
    hipLaunchKernelGGL(edge_bwd_kernel<true>, dim3(grid), dim3(64 * EB_WAVES), shm, (hipStream_t)stream,
                       n_edges, dst, gaggr, ge_next, a2m, a1m, a2e, a1e, st_m, st_e, lb_m, lb_e, ln_g, W2T, WcT, gz2m,
                       gz1m, gz2e, gz1e, gC, ge_out, pairs_m, npairs_m, pairs_e, npairs_e);
  else
    hipLaunchKernelGGL(edge_bwd_kernel<false>, dim3(grid), dim3(64 * EB_WAVES), shm, (hipStream_t)stream,
                       n_edges, dst, gaggr, ge_next, a2m, a1m, a2e, a1e, st_m, st_m, lb_m, lb_m, ln_g, W2T, WcT, gz2m,
                       gz1m, gz2e, gz1e, gC, ge_out, pairs_m, npairs_m, pairs_m, npairs_m);
  PDG_CHECK_LAUNCH("pdg_edge_bwd");
  return PDG_OK;
}

// ============================================================================ P/Q gather backward
constexpr int PQ_U = 8;   // rows of each half in flight per node (6: 3 % slower; 12: spills)
#ifndef PQ_CHUNK
#define PQ_CHUNK 512
#endif

// Half-wave (32 lanes x 16 B) per node.  Both halves' first PQ_U rows of a node are in flight
// together (row pointers -> destination rows and source permutation -> source rows: 3 dependent
// round trips per node instead of 5), which also brings a node's destination-side and source-side
// rows into the XCD's L2 at the same time: 405 -> 324 MB per launch at config 2 (algorithmic
// 288 MB), 67.7 -> 62.2 us.  Loads past a segment's end re-read row / entry 0 and are not
// accumulated, so every sum is formed row by row in segment order (destination rows, then source
// rows) as a serial loop would.
// SUMC: the second array holds gC = gz1m + gz1e (what pdg_edge_bwd_w2 writes for the Wc pass) and each
// row's gz1e is formed as gC - gz1m (one fp32 subtraction: within one rounding of |gC| of the stored
// gz1e), so the edge backward writes one E-row array fewer (gz1e is never materialised).
template <bool SUMC>
__global__ __launch_bounds__(256) void pq_scatter_bwd_kernel(int N, int chunk, const int* __restrict__ rpd,
                                                             const int* __restrict__ rps,
                                                             const int* __restrict__ perm_s,
                                                             const float* __restrict__ gz1m,
                                                             const float* __restrict__ gz1e,
                                                             float* __restrict__ gP, float* __restrict__ gQ) {
  const int hw = threadIdx.x >> 5, j = threadIdx.x & 31;
  const int nhw = blockDim.x >> 5;
  // node order: chunks of `chunk` consecutive nodes dealt round-robin over the 8 XCDs (block b
  // runs on XCD b & 7), so the source-side rows of a node (in its mesh neighbours' destination
  // segments) are mostly read by the same XCD at about the same time
  // (the launcher makes the grid a multiple of 8; node_of grows with i, so the first v >= N ends)
  const int x = blockIdx.x & 7, m = blockIdx.x >> 3, step = (gridDim.x >> 3) * nhw;
  auto node_of = [&](int i) { return ((i / chunk) * 8 + x) * chunk + i % chunk; };
  int i = m * nhw + hw;
  int v = node_of(i);
  if (v >= N) return;
  int d0 = rpd[v], d1 = rpd[v + 1], s0 = rps[v], s1 = rps[v + 1];
  int ks[PQ_U];
#pragma unroll
  for (int u = 0; u < PQ_U; ++u) ks[u] = perm_s[s0 + u < s1 ? s0 + u : 0];
  for (;;) {
    const int vn = node_of(i + step);
    const bool more = vn < N;
    f32x4 xm[PQ_U], xe[PQ_U], ym[PQ_U], ye[PQ_U];
#pragma unroll
    for (int u = 0; u < PQ_U; ++u) {
      const size_t kk = (size_t)(d0 + u < d1 ? d0 + u : 0) * L;
      xm[u] = reinterpret_cast<const f32x4*>(gz1m + kk)[j];
      if (gz1e) xe[u] = reinterpret_cast<const f32x4*>(gz1e + kk)[j];
    }
#pragma unroll
    for (int u = 0; u < PQ_U; ++u) {
      const size_t kk = (size_t)ks[u] * L;
      ym[u] = reinterpret_cast<const f32x4*>(gz1m + kk)[j];
      if (gz1e) ye[u] = reinterpret_cast<const f32x4*>(gz1e + kk)[j];
    }
    f32x4 p = {0.f, 0.f, 0.f, 0.f}, q = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < PQ_U; ++u) {
      if (d0 + u >= d1) break;
      p += xm[u];
      if (gz1e) q += SUMC ? xe[u] - xm[u] : xe[u];
    }
    for (int k = d0 + PQ_U; k < d1; ++k) {   // destination segments longer than PQ_U
      const f32x4 a = reinterpret_cast<const f32x4*>(gz1m + (size_t)k * L)[j];
      p += a;
      if (gz1e) {
        const f32x4 b = reinterpret_cast<const f32x4*>(gz1e + (size_t)k * L)[j];
        q += SUMC ? b - a : b;
      }
    }
#pragma unroll
    for (int u = 0; u < PQ_U; ++u) {
      if (s0 + u >= s1) break;
      q += ym[u];
      if (gz1e) p += SUMC ? ye[u] - ym[u] : ye[u];
    }
    for (int k = s0 + PQ_U; k < s1; ++k) {   // source segments longer than PQ_U
      const size_t kk = (size_t)perm_s[k] * L;
      const f32x4 a = reinterpret_cast<const f32x4*>(gz1m + kk)[j];
      q += a;
      if (gz1e) {
        const f32x4 b = reinterpret_cast<const f32x4*>(gz1e + kk)[j];
        p += SUMC ? b - a : b;
      }
    }
    stg4(gP + (size_t)v * L + 4 * j, p);
    stg4(gQ + (size_t)v * L + 4 * j, q);
    if (!more) break;
    i += step;
    v = vn;
    d0 = rpd[v]; d1 = rpd[v + 1]; s0 = rps[v]; s1 = rps[v + 1];
#pragma unroll
    for (int u = 0; u < PQ_U; ++u) ks[u] = perm_s[s0 + u < s1 ? s0 + u : 0];
  }
}

extern "C" int pdg_pq_scatter_bwd(int n_nodes, const int* rowptr_dst, const int* rowptr_src, const int* perm_src,
                                  const float* gz1m, const float* gz1e, int e_is_sum, float* gP, float* gQ,
                                  void* stream) {
  PDG_CHECK_ARG(n_nodes > 0, "pdg_pq_scatter_bwd: n_nodes must be > 0");
  PDG_CHECK_ARG(rowptr_dst && rowptr_src && perm_src && gz1m && gP && gQ, "pdg_pq_scatter_bwd: null argument");
  PDG_CHECK_ARG(!e_is_sum || gz1e, "pdg_pq_scatter_bwd: e_is_sum needs the gC rows");
  PDG_CHECK_ARG(PDG_ALIGNED(gz1m) && (!gz1e || PDG_ALIGNED(gz1e)) && PDG_ALIGNED(gP) && PDG_ALIGNED(gQ),
                "pdg_pq_scatter_bwd: misaligned pointer");
  long want = (n_nodes + 7) / 8;
  long cap = (long)device_cus() * 8;
  const int grid = (int)(((want < cap ? want : cap) + 7) / 8 * 8);   // a multiple of 8 (node order)
  // 512-node chunks: contiguous per-XCD ranges (0) and 128 / 2,048 measured slower
  const int chunk = PQ_CHUNK > 0 ? PQ_CHUNK : (n_nodes + 7) / 8;
  hipLaunchKernelGGL(e_is_sum && gz1e ? pq_scatter_bwd_kernel<true> : pq_scatter_bwd_kernel<false>, dim3(grid),
                     dim3(256), 0, (hipStream_t)stream, n_nodes, chunk, rowptr_dst, rowptr_src, perm_src, gz1m, gz1e,
                     gP, gQ);
  PDG_CHECK_LAUNCH("pdg_pq_scatter_bwd");
  return PDG_OK;
}
