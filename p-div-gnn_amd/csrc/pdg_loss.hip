// Loss kernels: per-graph normalised MSE (scripts/gnn_train.py:41-57) and the
// divergence penalty (scripts/gnn_train.py:60-92), segmented by the batch's
// node offsets `ptr` instead of the reference's Python loop over Batch[i]
// (gnn_local_stress/data_utils.py:25-33).  One workgroup per graph, fp64
// accumulation, fixed summation order (deterministic).
//
// The divergence operator is applied sparsely (CSR, ~14 nnz per row) instead
// of the reference's dense `to_dense()[:, :2N]` (8*N^2 bytes per graph).
#include "pdg_common.hpp"
#include "pdg_runtime.hpp"

using namespace pdg;

__device__ __forceinline__ double block_sum(double x, double* red) {
  x = wave_sum(x);
  const int w = wave_id(), nw = blockDim.x >> 6;
  __syncthreads();
  if (lane_id() == 0) red[w] = x;
  __syncthreads();
  double s = 0;
  for (int i = 0; i < nw; ++i) s += red[i];
  return s;  // valid in every thread
}

// ============================================================================ NMSE
// K doubles summed over the block at once (one LDS round instead of K); valid in every thread.
template <int K>
__device__ __forceinline__ void block_sum_k(double (&x)[K], double* red) {
#pragma unroll
  for (int k = 0; k < K; ++k) x[k] = wave_sum(x[k]);
  const int w = wave_id(), nw = blockDim.x >> 6;
  __syncthreads();
  if (lane_id() == 0)
#pragma unroll
    for (int k = 0; k < K; ++k) red[k * 16 + w] = x[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k) {
    double s = 0;
    for (int i = 0; i < nw; ++i) s += red[k * 16 + i];
    x[k] = s;
  }
}

// One block of 1024 threads per graph; the three channels in one pass over the graph's nodes
// (loads of NF_U nodes issued together): a 256-thread block with one channel per pass and a
// reduction per channel ran 31 us for 8 graphs of 5,041 nodes (latency-bound).  The first NF_C
// loop iterations (NF_C NF_U 1024 = 8,192 nodes) keep their gt / pred values in registers, so for
// such graphs the mean, the sums and the gradient rows take one round trip of loads instead of
// three; larger graphs re-read the rest.  Same sums in the same order as the three-pass form.
constexpr int NF_U = 4;
constexpr int NF_C = 2;

__global__ __launch_bounds__(1024) void nmse_fwd_kernel(const int* __restrict__ ptr, const float* __restrict__ gt,
                                                        const float* __restrict__ pred, float* __restrict__ loss,
                                                        float* __restrict__ den_out, const float* __restrict__ scale,
                                                        int accumulate, float* __restrict__ gp) {
  __shared__ double red[6 * 16];
  const int g = blockIdx.x;
  const int n0 = ptr[g], n1 = ptr[g + 1];
  const double n = (double)(n1 - n0);
  const int T = blockDim.x;
  // node of iteration k, slot u: n0 + t + (k NF_U + u) T (the loops below step NF_U T per iteration)
  float tc[NF_C][NF_U][3], pc[NF_C][NF_U][3];
#pragma unroll
  for (int k = 0; k < NF_C; ++k)
#pragma unroll
    for (int u = 0; u < NF_U; ++u)
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int i = n0 + (int)threadIdx.x + (k * NF_U + u) * T;
        const bool ok = i < n1;
        tc[k][u][c] = ok ? gt[(size_t)i * 3 + c] : 0.f;
        pc[k][u][c] = ok ? pred[(size_t)i * 3 + c] : 0.f;
      }
  const int rest = n0 + (int)threadIdx.x + NF_C * NF_U * T;   // the first iteration past the cached ones
  double m[3] = {0, 0, 0};
  // cached iterations past the graph's end add exact zeros (the loop form skips them: the same sums)
#pragma unroll
  for (int k = 0; k < NF_C; ++k)
#pragma unroll
    for (int u = 0; u < NF_U; ++u)
#pragma unroll
      for (int c = 0; c < 3; ++c) m[c] += (double)tc[k][u][c];
  for (int i = rest; i < n1; i += NF_U * T) {
    float t[NF_U][3];
#pragma unroll
    for (int u = 0; u < NF_U; ++u)
#pragma unroll
      for (int c = 0; c < 3; ++c) t[u][c] = i + u * T < n1 ? gt[(size_t)(i + u * T) * 3 + c] : 0.f;
#pragma unroll
    for (int u = 0; u < NF_U; ++u)
#pragma unroll
      for (int c = 0; c < 3; ++c) m[c] += (double)t[u][c];
  }
  block_sum_k<3>(m, red);
  float mean[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) mean[c] = (float)(m[c] / n);   // gt.mean(axis=0)
  double sd[6] = {0, 0, 0, 0, 0, 0};   // se[3], sd[3]
#pragma unroll
  for (int k = 0; k < NF_C; ++k)
#pragma unroll
    for (int u = 0; u < NF_U; ++u)
      if (n0 + (int)threadIdx.x + (k * NF_U + u) * T < n1)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const float d = tc[k][u][c] - pc[k][u][c];
          const float mm = tc[k][u][c] - mean[c];
          sd[c] += (double)(d * d);
          sd[3 + c] += (double)(mm * mm);
        }
  for (int i = rest; i < n1; i += NF_U * T) {
    float t[NF_U][3], p[NF_U][3];
#pragma unroll
    for (int u = 0; u < NF_U; ++u)
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const bool ok = i + u * T < n1;
        t[u][c] = ok ? gt[(size_t)(i + u * T) * 3 + c] : 0.f;
        p[u][c] = ok ? pred[(size_t)(i + u * T) * 3 + c] : 0.f;
      }
#pragma unroll
    for (int u = 0; u < NF_U; ++u)
      if (i + u * T < n1)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const float d = t[u][c] - p[u][c];
          const float mm = t[u][c] - mean[c];
          sd[c] += (double)(d * d);
          sd[3 + c] += (double)(mm * mm);
        }
  }
  block_sum_k<6>(sd, red);
  float ratio[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float mse = (float)sd[c];
    const float den = (float)sd[3 + c];
    ratio[c] = mse / den;
    if (threadIdx.x == 0) den_out[g * 3 + c] = den;
  }
  if (threadIdx.x == 0) loss[g] = (ratio[0] + ratio[1] + ratio[2]) / 3.0f;
  if (gp == nullptr) return;
  // pdg_nmse_fwd_bwd: the graph's gradient rows with nmse_bwd_kernel's arithmetic (bitwise), den from the
  // block's own sums
  const float sc = scale[0];
  auto grad = [&](int i, int c, float t, float p) {
    const float den = (float)sd[3 + c];
    const float d = t - p;
    const float v = sc * ((-2.0f * d) / den) / 3.0f;
    const size_t e = (size_t)i * 3 + c;
    gp[e] = accumulate ? gp[e] + v : v;
  };
#pragma unroll
  for (int k = 0; k < NF_C; ++k)
#pragma unroll
    for (int u = 0; u < NF_U; ++u) {
      const int i = n0 + (int)threadIdx.x + (k * NF_U + u) * T;
      if (i < n1)
#pragma unroll
        for (int c = 0; c < 3; ++c) grad(i, c, tc[k][u][c], pc[k][u][c]);
    }
  for (int i = rest; i < n1; i += T)
#pragma unroll
    for (int c = 0; c < 3; ++c) grad(i, c, gt[(size_t)i * 3 + c], pred[(size_t)i * 3 + c]);
}

extern "C" int pdg_nmse_fwd(int n_graphs, const int* ptr, const float* gt, const float* pred, float* loss,
                            float* den, void* stream) {
  PDG_CHECK_ARG(n_graphs > 0, "pdg_nmse_fwd: n_graphs must be > 0");
  hipLaunchKernelGGL(nmse_fwd_kernel, dim3(n_graphs), dim3(1024), 0, (hipStream_t)stream, ptr, gt, pred, loss, den,
                     nullptr, 0, nullptr);
  PDG_CHECK_LAUNCH("pdg_nmse_fwd");
  return PDG_OK;
}

extern "C" int pdg_nmse_fwd_bwd(int n_graphs, const int* ptr, const float* gt, const float* pred, float* loss,
                                float* den, const float* scale, int accumulate, float* g_pred, void* stream) {
  PDG_CHECK_ARG(n_graphs > 0 && scale && g_pred, "pdg_nmse_fwd_bwd: bad arguments");
  hipLaunchKernelGGL(nmse_fwd_kernel, dim3(n_graphs), dim3(1024), 0, (hipStream_t)stream, ptr, gt, pred, loss, den,
                     scale, accumulate, g_pred);
  PDG_CHECK_LAUNCH("pdg_nmse_fwd_bwd");
  return PDG_OK;
}

__device__ __forceinline__ int graph_of(const int* __restrict__ ptr, int B, int node) {
  int lo = 0, hi = B;  // ptr[lo] <= node < ptr[hi]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (ptr[mid] <= node) lo = mid; else hi = mid;
  }
  return lo;
}

// d loss_g / d pred[n][c] = (1/3) * (-2) (gt - pred) / den_c ; times the upstream scale.
__global__ void nmse_bwd_kernel(int B, const int* __restrict__ ptr, int N, const float* __restrict__ gt,
                                const float* __restrict__ pred, const float* __restrict__ den,
                                const float* __restrict__ scale, int accumulate, float* __restrict__ gp) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= N * 3) return;
  const int n = e / 3, c = e % 3;
  const int g = graph_of(ptr, B, n);
  const float sc = scale[0];
  const float d = gt[e] - pred[e];
  const float v = sc * ((-2.0f * d) / den[g * 3 + c]) / 3.0f;
  gp[e] = accumulate ? gp[e] + v : v;
}

extern "C" int pdg_nmse_bwd(int n_graphs, const int* ptr, int n_nodes, const float* gt, const float* pred,
                            const float* den, const float* scale, int accumulate, float* g_pred, void* stream) {
  PDG_CHECK_ARG(n_graphs > 0 && n_nodes > 0, "pdg_nmse_bwd: empty");
  const long tot = (long)n_nodes * 3;
  hipLaunchKernelGGL(nmse_bwd_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     n_graphs, ptr, n_nodes, gt, pred, den, scale, accumulate, g_pred);
  PDG_CHECK_LAUNCH("pdg_nmse_bwd");
  return PDG_OK;
}

// ============================================================================ divergence
// div[v][0] = sum_j a_j * (col_j < n ? sxx : sxy)[off + col_j mod n]
// div[v][1] = sum_j a_j * (col_j < n ? sxy : syy)[off + col_j mod n]
// One block of 1024 threads per graph (4x the 256-thread form's node parallelism: each node walks its
// CSR row of the divergence operator with dependent loads).
__global__ __launch_bounds__(1024) void div_fwd_kernel(const int* __restrict__ ptr, const int* __restrict__ arp,
                                                      const int* __restrict__ acol, const float* __restrict__ aval,
                                                      const int64_t* __restrict__ types,
                                                      const float* __restrict__ sig, int rabs,
                                                      float* __restrict__ div, float* __restrict__ loss) {
  __shared__ double red[16];
  const int g = blockIdx.x;
  const int n0 = ptr[g], n1 = ptr[g + 1];
  const int n = n1 - n0;
  double s0 = 0, s1 = 0;
  for (int v = n0 + threadIdx.x; v < n1; v += blockDim.x) {
    float d0 = 0.f, d1 = 0.f;
    const long t = types[v];
    if (t != 1 && t != -1) {   // NodeType.EXTERNAL_BOUNDARY / INTERNAL_BOUNDARY rows zeroed
      for (int j = arp[v]; j < arp[v + 1]; ++j) {
        const int c = acol[j];
        const float a = aval[j];
        if (c < n) {
          const float* sv = sig + (size_t)(n0 + c) * 3;
          d0 = fmaf(a, sv[0], d0);   // sxx
          d1 = fmaf(a, sv[2], d1);   // sxy
        } else if (c < 2 * n) {
          const float* sv = sig + (size_t)(n0 + c - n) * 3;
          d0 = fmaf(a, sv[2], d0);   // sxy
          d1 = fmaf(a, sv[1], d1);   // syy
        }
      }
    }
    div[(size_t)v * 2] = d0;
    div[(size_t)v * 2 + 1] = d1;
    s0 += rabs ? (double)fabsf(d0) : (double)(d0 * d0);
    s1 += rabs ? (double)fabsf(d1) : (double)(d1 * d1);
  }
  const float m0 = (float)(block_sum(s0, red) / n);
  const float m1 = (float)(block_sum(s1, red) / n);
  if (threadIdx.x == 0) loss[g] = m0 + m1;
}

extern "C" int pdg_div_fwd(int n_graphs, const int* ptr, const int* a_rowptr, const int* a_col, const float* a_val,
                           const int64_t* node_types, const float* sigma, int reduce_abs, float* div, float* loss,
                           void* stream) {
  PDG_CHECK_ARG(n_graphs > 0, "pdg_div_fwd: n_graphs must be > 0");
  hipLaunchKernelGGL(div_fwd_kernel, dim3(n_graphs), dim3(1024), 0, (hipStream_t)stream, ptr, a_rowptr, a_col, a_val,
                     node_types, sigma, reduce_abs, div, loss);
  PDG_CHECK_LAUNCH("pdg_div_fwd");
  return PDG_OK;
}

// g_div[v][c] = scale * 2 div[v][c] / n_g  (abs: scale * sign(div) / n_g); g_sigma[m] = sum over A^T entries.
__device__ __forceinline__ float dsign(float x) { return x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f); }

__global__ void div_bwd_kernel(int B, const int* __restrict__ ptr, int N, const int* __restrict__ atp,
                               const int* __restrict__ atrow, const int* __restrict__ atcomp,
                               const float* __restrict__ atval, const float* __restrict__ div,
                               const float* __restrict__ scale, int rabs, int accumulate, float* __restrict__ gs) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= N) return;
  const int g = graph_of(ptr, B, m);
  const float f = (rabs ? 1.0f : 2.0f) * scale[0] / (float)(ptr[g + 1] - ptr[g]);
  float gxx = 0.f, gyy = 0.f, gxy = 0.f;
  for (int j = atp[m]; j < atp[m + 1]; ++j) {
    const int v = atrow[j];
    const float a = atval[j];
    const float d0 = div[(size_t)v * 2], d1 = div[(size_t)v * 2 + 1];
    const float g0 = f * (rabs ? dsign(d0) : d0), g1 = f * (rabs ? dsign(d1) : d1);
    if (atcomp[j] == 0) {
      gxx = fmaf(a, g0, gxx);
      gxy = fmaf(a, g1, gxy);
    } else {
      gxy = fmaf(a, g0, gxy);
      gyy = fmaf(a, g1, gyy);
    }
  }
  float* o = gs + (size_t)m * 3;
  if (accumulate) { o[0] += gxx; o[1] += gyy; o[2] += gxy; }
  else { o[0] = gxx; o[1] = gyy; o[2] = gxy; }
}

extern "C" int pdg_div_bwd(int n_graphs, const int* ptr, int n_nodes, const int* at_rowptr, const int* at_row,
                           const int* at_comp, const float* at_val, const float* div, const float* scale,
                           int reduce_abs, int accumulate, float* g_sigma, void* stream) {
  PDG_CHECK_ARG(n_graphs > 0 && n_nodes > 0, "pdg_div_bwd: empty");
  hipLaunchKernelGGL(div_bwd_kernel, dim3((n_nodes + 255) / 256), dim3(256), 0, (hipStream_t)stream, n_graphs, ptr,
                     n_nodes, at_rowptr, at_row, at_comp, at_val, div, scale, reduce_abs, accumulate, g_sigma);
  PDG_CHECK_LAUNCH("pdg_div_bwd");
  return PDG_OK;
}

// ============================================================================ utilities
__global__ void transpose_kernel(int R, int C, int ld, const float* __restrict__ in, float* __restrict__ out) {
  __shared__ float tile[32][33];
  const int bx = blockIdx.x * 32, by = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;   // 32 x 8
  for (int y = ty; y < 32; y += 8) {
    const int r = by + y, c = bx + tx;
    if (r < R && c < C) tile[y][tx] = in[(size_t)r * ld + c];
  }
  __syncthreads();
  for (int y = ty; y < 32; y += 8) {
    const int c = bx + y, r = by + tx;
    if (r < R && c < C) out[(size_t)c * R + r] = tile[tx][y];
  }
}

extern "C" int pdg_transpose(int rows, int cols, int ld, const float* in, float* out, void* stream) {
  PDG_CHECK_ARG(rows > 0 && cols > 0 && ld >= cols && in != out, "pdg_transpose: bad args");
  hipLaunchKernelGGL(transpose_kernel, dim3((cols + 31) / 32, (rows + 31) / 32), dim3(256), 0, (hipStream_t)stream,
                     rows, cols, ld, in, out);
  PDG_CHECK_LAUNCH("pdg_transpose");
  return PDG_OK;
}

// Up to 16 transposes of 128 x 128 blocks in one launch (the backward's W^T copies).
struct TransposeJobs {
  const float* in[16];
  float* out[16];
  int ld[16];
};

__global__ void transpose128_batch_kernel(TransposeJobs jobs) {
  __shared__ float tile[32][33];
  const int j = blockIdx.z;
  const float* __restrict__ in = jobs.in[j];
  float* __restrict__ out = jobs.out[j];
  const int ld = jobs.ld[j];
  const int bx = blockIdx.x * 32, by = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;   // 32 x 8
  for (int y = ty; y < 32; y += 8) tile[y][tx] = in[(size_t)(by + y) * ld + bx + tx];
  __syncthreads();
  for (int y = ty; y < 32; y += 8) out[(size_t)(bx + y) * 128 + by + tx] = tile[tx][y];
}

extern "C" int pdg_transpose128_batch(int n, const float* const* in_ptrs, const int* lds, float* const* out_ptrs,
                                      void* stream) {
  PDG_CHECK_ARG(n > 0 && n <= 16 && in_ptrs && lds && out_ptrs, "pdg_transpose128_batch: 1..16 jobs");
  TransposeJobs jobs;
  for (int i = 0; i < n; ++i) {
    PDG_CHECK_ARG(in_ptrs[i] && out_ptrs[i] && lds[i] >= 128 && in_ptrs[i] != out_ptrs[i],
                  "pdg_transpose128_batch: bad job");
    jobs.in[i] = in_ptrs[i];
    jobs.out[i] = out_ptrs[i];
    jobs.ld[i] = lds[i];
  }
  hipLaunchKernelGGL(transpose128_batch_kernel, dim3(4, 4, n), dim3(256), 0, (hipStream_t)stream, jobs);
  PDG_CHECK_LAUNCH("pdg_transpose128_batch");
  return PDG_OK;
}

// The step's non-finite test and the zero-mean-stress skip in one launch, with no memset: flags[2] is
// double-buffered by call parity (as Adam's step count): every block ORs into flags[parity], block 0
// clears flags[parity ^ 1] for the next call (which runs after this one on the stream).  *zero_flag (a
// float, nullable) of 0 forces the skip: the zero-mean-stress guard of models.py:294-299.
__global__ void nonfinite2_kernel(const float* __restrict__ x, long n, const float* __restrict__ nz,
                                  int* __restrict__ flags, int parity) {
  int bad = 0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    bad |= !isfinite(x[i]);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    flags[parity ^ 1] = 0;
    if (nz && *nz == 0.f) bad = 1;
  }
  if (__any(bad) && lane_id() == 0) atomicOr(flags + parity, 1);
}

extern "C" int pdg_nonfinite2(const float* x, int64_t n, const float* zero_flag, int* flags, int parity,
                              void* stream) {
  PDG_CHECK_ARG(n >= 0 && flags != nullptr && (parity == 0 || parity == 1), "pdg_nonfinite2: bad args");
  long blocks = (n + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(nonfinite2_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, x, (long)n,
                     zero_flag, flags, parity);
  PDG_CHECK_LAUNCH("pdg_nonfinite2");
  return PDG_OK;
}

// The step's loss scalars (gnn_train.py:189-197) in one launch: out[0] = *zero_flag (or 1 when NULL),
// out[1] = scale_nmse * sum_g loss_nmse[g], out[2] = scale_div * sum_g loss_div[g] (0 when NULL),
// out[3] = out[1] + out[2].  Sums in fp64, graph order, rounded once.
__global__ void loss_reduce_kernel(int B, const float* __restrict__ ln, const float* __restrict__ ld, float sn,
                                   float sd, const float* __restrict__ nz, float* __restrict__ out) {
  __shared__ double red[2 * 16];
  double a = 0, b = 0;
  for (int g = threadIdx.x; g < B; g += blockDim.x) {
    a += (double)ln[g];
    if (ld) b += (double)ld[g];
  }
  double v[2] = {a, b};
  block_sum_k<2>(v, red);
  if (threadIdx.x == 0) {
    const float fn = (float)v[0] * sn;
    const float fd = ld ? (float)v[1] * sd : 0.f;
    out[0] = nz ? *nz : 1.f;
    out[1] = fn;
    out[2] = fd;
    out[3] = fn + fd;
  }
}

extern "C" int pdg_loss_reduce(int n_graphs, const float* loss_nmse, const float* loss_div, float scale_nmse,
                               float scale_div, const float* zero_flag, float* out, void* stream) {
  PDG_CHECK_ARG(n_graphs > 0 && loss_nmse != nullptr && out != nullptr, "pdg_loss_reduce: bad args");
  hipLaunchKernelGGL(loss_reduce_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, n_graphs, loss_nmse, loss_div,
                     scale_nmse, scale_div, zero_flag, out);
  PDG_CHECK_LAUNCH("pdg_loss_reduce");
  return PDG_OK;
}

// torch.optim.Adam._single_tensor_adam (amsgrad=False, weight_decay=0, maximize=False) driven by
// GradScaler.step (gnn_train.py:111,118,204-207): a skipped step (non-finite gradient) leaves the
// parameters, both moments AND Adam's step count untouched.  The step count therefore lives on the
// device, double-buffered by call parity: the kernel reads count[parity] (optimizer steps taken so
// far), uses table entry count[parity] (the host-computed float32 images of torch's double-precision
// step_size = lr / (1 - beta1^t) and sqrt(1 - beta2^t) for t = count + 1) and block 0 writes
// count[parity ^ 1] = count + (skipped ? 0 : 1).  No host sync, no extra launch.
__global__ void adam_kernel(long n, float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, const float2* __restrict__ tab, float w1, float b2, float w2,
                            float eps, const int* __restrict__ skip, int* __restrict__ count, int parity, int tab_len) {
  const int c = count[parity];
  const int sk = skip ? *skip : 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) count[parity ^ 1] = c + (sk ? 0 : 1);
  if (sk) return;
  // {step_size, bias_correction2_sqrt} of step c + 1; the host keeps tab_len > its call count >= c
  const float2 t = tab[c < tab_len ? c : tab_len - 1];
  // Explicitly rounded operations in torch's CPU kernel order (no contraction beyond what it does):
  //   lerp_vec:  fmadd(w1, g - m, m)                 (weight < 0.5)
  //   mul_ then addcmul_: fmadd(w2 * g, g, v * b2)   (checked against torch's CPU kernels)
  //   denom:     sqrt(v) / bc2_sqrt + eps
  //   addcdiv_:  p + ((-step_size) * m) / denom
  const float nstep = -t.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float gi = g[i];
    const float mi = __fmaf_rn(w1, __fsub_rn(gi, m[i]), m[i]);
    const float vi = __fmaf_rn(__fmul_rn(w2, gi), gi, __fmul_rn(v[i], b2));
    m[i] = mi;
    v[i] = vi;
    const float denom = __fadd_rn(__fdiv_rn(__fsqrt_rn(vi), t.y), eps);
    p[i] = __fadd_rn(p[i], __fdiv_rn(__fmul_rn(nstep, mi), denom));
  }
}

extern "C" int pdg_adam(int64_t n, float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                        const float* table, int table_len, float w1, float beta2, float w2, float eps,
                        const int* skip_flag, int* step_count, int parity, void* stream) {
  PDG_CHECK_ARG(n >= 0 && table != nullptr && table_len >= 1 && step_count != nullptr && (parity == 0 || parity == 1),
                "pdg_adam: bad args");
  long blocks = (n + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;             // block 0 always advances the step count
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, (long)n, param, grad,
                     exp_avg, exp_avg_sq, (const float2*)table, w1, beta2, w2, eps, skip_flag, step_count, parity, table_len);
  PDG_CHECK_LAUNCH("pdg_adam");
  return PDG_OK;
}
