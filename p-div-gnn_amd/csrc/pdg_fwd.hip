// Forward kernels of the P-DivGNN hot path (EncodeProcessDecode.forward,
// gnn_local_stress/models.py:288-326) for gfx950.
//
// Layout and wave-tile conventions: pdg_common.hpp.  Every kernel that ends in a
// graph-LayerNorm writes per-block (sum, sum of squares) partials in fp64; the
// statistics are reduced by pdg_ln_finalize and applied by the *consumer* of the
// normalised tensor (LN is graph-global, so it cannot be applied in the producer).
#include <stdarg.h>
#include <stdio.h>

#include "pdg_common.hpp"
#include "pdg_runtime.hpp"

using namespace pdg;

namespace pdg {

static thread_local char g_err[512];

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int device_cus() {
  static int cached[64] = {0};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 64) dev = 0;
  if (!cached[dev]) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
    cached[dev] = cus;
  }
  return cached[dev];
}

}  // namespace pdg

// ============================================================================ input formatting
__global__ void format_inputs_kernel(int N, int E, const float* __restrict__ pos,
                                     const float* __restrict__ ms, const int64_t* __restrict__ types,
                                     const float* __restrict__ ea, const int* __restrict__ perm,
                                     const float* __restrict__ st8, int scale, float* __restrict__ x_in,
                                     float* __restrict__ e_in) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  float mp = 0.f, sp = 1.f, mm = 0.f, sm = 1.f, me = 0.f, se = 1.f;
  if (scale) { mp = st8[0]; sp = st8[1]; mm = st8[2]; sm = st8[3]; me = st8[6]; se = st8[7]; }
  if (i < N) {
    float* o = x_in + i * 6;
    // models.py:147-151: hstack[(mean_stress - mu)/s, (pos - mu)/s, node_type]
    for (int c = 0; c < 3; ++c) { float v = ms[i * 3 + c]; o[c] = scale ? (v - mm) / sm : v; }
    for (int c = 0; c < 2; ++c) { float v = pos[i * 2 + c]; o[3 + c] = scale ? (v - mp) / sp : v; }
    o[5] = (float)types[i];
  }
  if (i < E) {
    const float v = ea[perm[i]];
    e_in[i] = scale ? (v - me) / se : v;
  }
}

extern "C" int pdg_format_inputs(int n_nodes, int n_edges, const float* pos, const float* mean_stress,
                                 const int64_t* node_types, const float* edge_attr, const int* perm,
                                 const float* stats8, int scale_input, float* x_in, float* e_in,
                                 void* stream) {
  PDG_CHECK_ARG(n_nodes >= 0 && n_edges >= 0, "pdg_format_inputs: negative size");
  const long n = n_nodes > n_edges ? n_nodes : n_edges;
  if (n == 0) return PDG_OK;
  PDG_CHECK_ARG(stats8 != nullptr || !scale_input, "pdg_format_inputs: stats8 is NULL");
  const int threads = 256;
  const long blocks = (n + threads - 1) / threads;
  hipLaunchKernelGGL(format_inputs_kernel, dim3((unsigned)blocks), dim3(threads), 0, (hipStream_t)stream,
                     n_nodes, n_edges, pos, mean_stress, node_types, edge_attr, perm, stats8, scale_input,
                     x_in, e_in);
  PDG_CHECK_LAUNCH("pdg_format_inputs");
  return PDG_OK;
}

// ============================================================================ tile helpers
// Persistent tile loop: wave w of block b takes tiles b*nw + w, then strides by
// gridDim*nw; a tile is 16 rows, lane row = tile*16 + (lane & 15).
__device__ __forceinline__ void accum_stats(const float (&v)[FRAG], bool valid, double& s1, double& s2) {
  if (!valid) return;
  // 32 values of one quarter row: fp32 partials per 16, fp64 across
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) { const float x = v[16 * q + j]; a += x; b += x * x; }
    s1 += (double)a;
    s2 += (double)b;
  }
}

__device__ __forceinline__ void write_partials(double s1, double s2, double* part) {
  __shared__ double red[2 * 16];
  block_sum2(s1, s2, red);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = s1;
    part[2 * blockIdx.x + 1] = s2;
  }
}

// v = LN(a2 row) [+ residual row], four fenced chunks of 8 floats.
template <bool RES>
__device__ __forceinline__ void ln_res_frag(float (&v)[FRAG], const float* __restrict__ a2row,
                                            const float* __restrict__ resrow, const LNStat& st,
                                            const float* __restrict__ g, const float* __restrict__ b) {
  const int lc = lane_col();
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    f32x4 x[2], r[2], gg[2], bb[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      x[t] = ld4(a2row + lc, 2 * q + t);
      if (RES) r[t] = ld4(resrow + lc, 2 * q + t);
      gg[t] = ld4(g + lc, 2 * q + t);
      bb[t] = ld4(b + lc, 2 * q + t);
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float y = div_den(x[t][j] - st.mean, st.den, st.rstd) * gg[t][j] + bb[t][j];
        if (RES) y += r[t][j];
        v[8 * q + 4 * t + j] = y;
      }
    PDG_FENCE();
  }
}

// v[s] = relu(acc[s] + bias[feature of s]).
__device__ __forceinline__ void bias_relu(float (&v)[FRAG], const Acc& acc, const float* __restrict__ bias) {
  const float* bp = bias + lane_col();
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const f32x4 bb = ld4(bp, t);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[4 * t + j] = fmaxf(acc.b[t][j] + bb[j], 0.f);
  }
}

// ============================================================================ encoder
// models.py:260-274.  W2 in LDS (A-image); W0 (128 x IN) and b0 appended.
template <int IN>
__global__ __launch_bounds__(384, 3) void encoder_kernel(int M, const float* __restrict__ x_in,
                                                          const float* __restrict__ W0,
                                                          const float* __restrict__ b0,
                                                          const float* __restrict__ W2,
                                                          const float* __restrict__ b2,
                                                          float* __restrict__ a1, float* __restrict__ a2,
                                                          double* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* w0l = lds + WBLK;           // [128][IN]
  float* b0l = w0l + 128 * IN;       // [128]
  load_wblock(lds, W2, 128, 0);
  for (int i = threadIdx.x; i < 128 * IN; i += blockDim.x) w0l[i] = W0[i];
  for (int i = threadIdx.x; i < 128; i += blockDim.x) b0l[i] = b0[i];
  __syncthreads();
  const int l = lane_id();
  double s1 = 0, s2 = 0;
  PDG_TILE_LOOP(M) {
    const int row = tile * TILE + (l & 15);
    const bool valid = row < M;
    const int rc = valid ? row : M - 1;
    float xi[IN];
#pragma unroll
    for (int i = 0; i < IN; ++i) xi[i] = x_in[(size_t)rc * IN + i];
    float v[FRAG];
    const int lc = lane_col();
#pragma unroll
    for (int q = 0; q < 2; ++q) {
#pragma unroll
      for (int s = 16 * q; s < 16 * q + 16; ++s) {
        const int o = lc + 16 * (s >> 2) + (s & 3);
        float d = 0.f;
#pragma unroll
        for (int i = 0; i < IN; ++i) d = fmaf(w0l[o * IN + i], xi[i], d);
        v[s] = fmaxf(d + b0l[o], 0.f);
      }
      PDG_FENCE();
    }
    if (valid && a1) store_frag(a1 + (size_t)row * L, v);   // a1 == NULL: recomputed by the backward
    Acc acc;
    zero_acc(acc);
    gemm128(acc, lds, v);
    bias_relu(v, acc, b2);
    if (valid) store_frag(a2 + (size_t)row * L, v);
    accum_stats(v, valid, s1, s2);
  }
  write_partials(s1, s2, part);
}

extern "C" int pdg_encoder_fwd(int rows, int in_features, const float* x_in, const float* W0,
                               const float* b0, const float* W2, const float* b2, float* a1, float* a2,
                               double* partials, int* nparts, void* stream) {
  PDG_CHECK_ARG(rows > 0, "pdg_encoder_fwd: rows must be > 0");
  PDG_CHECK_ARG(in_features == 1 || in_features == 6, "pdg_encoder_fwd: in_features must be 1 or 6");
  PDG_CHECK_ARG(PDG_ALIGNED(a1) && PDG_ALIGNED(a2) && PDG_ALIGNED(W2) && PDG_ALIGNED(b2),
                "pdg_encoder_fwd: misaligned pointer");
  const int grid = persistent_grid(rows, 6, 2);
  const size_t shm = (size_t)(WBLK + 128 * in_features + 128) * sizeof(float);
  if (in_features == 6)
    hipLaunchKernelGGL(encoder_kernel<6>, dim3(grid), dim3(384), shm, (hipStream_t)stream, rows, x_in, W0,
                       b0, W2, b2, a1, a2, partials);
  else
    hipLaunchKernelGGL(encoder_kernel<1>, dim3(grid), dim3(384), shm, (hipStream_t)stream, rows, x_in, W0,
                       b0, W2, b2, a1, a2, partials);
  PDG_CHECK_LAUNCH("pdg_encoder_fwd");
  if (nparts) *nparts = grid;
  return PDG_OK;
}

// ============================================================================ LN finalize
__device__ __forceinline__ void ln_finalize_block(const double* __restrict__ part, int n, double count,
                                                  pdg_ln_stat* __restrict__ out) {
  __shared__ double red[2 * 16];
  ln_stat_from_partials(part, n, count, out, red);
}

__global__ void ln_finalize_kernel(const double* __restrict__ part, int n, double count,
                                   pdg_ln_stat* __restrict__ out) {
  ln_finalize_block(part, n, count, out);
}

// two independent statistics in one launch (one block each, the same per-block arithmetic as
// ln_finalize_kernel, so the results are bit-identical to two separate launches)
__global__ void ln_finalize2_kernel(const double* __restrict__ part_a, const double* __restrict__ part_b, int n,
                                    double count, pdg_ln_stat* __restrict__ out_a, pdg_ln_stat* __restrict__ out_b) {
  if (blockIdx.x == 0)
    ln_finalize_block(part_a, n, count, out_a);
  else
    ln_finalize_block(part_b, n, count, out_b);
}

extern "C" int pdg_ln_finalize2(const double* part_a, const double* part_b, int nparts, double count,
                                pdg_ln_stat* out_a, pdg_ln_stat* out_b, void* stream) {
  PDG_CHECK_ARG(nparts > 0 && count > 0, "pdg_ln_finalize2: empty");
  PDG_CHECK_ARG(part_a && part_b && out_a && out_b && out_a != out_b, "pdg_ln_finalize2: bad pointers");
  hipLaunchKernelGGL(ln_finalize2_kernel, dim3(2), dim3(256), 0, (hipStream_t)stream, part_a, part_b, nparts, count,
                     out_a, out_b);
  PDG_CHECK_LAUNCH("pdg_ln_finalize2");
  return PDG_OK;
}

extern "C" int pdg_ln_finalize(const double* partials, int nparts, double count, pdg_ln_stat* out,
                               void* stream) {
  PDG_CHECK_ARG(nparts > 0 && count > 0, "pdg_ln_finalize: empty");
  hipLaunchKernelGGL(ln_finalize_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, partials, nparts, count,
                     out);
  PDG_CHECK_LAUNCH("pdg_ln_finalize");
  return PDG_OK;
}

// Exact data-parallel LayerNorm ("sync" mode): each rank reduces its
// per-block partials to one (sum, sumsq) pair, the pairs are all-reduced over the
// process group, and pdg_ln_finalize(pair, 1, global_count) yields the statistics of
// the whole minibatch, as the reference computes them on one device (models.py:42-55).
__global__ void ln_partials_sum_kernel(const double* __restrict__ part, int n, double* __restrict__ out2) {
  __shared__ double red[2 * 16];
  double a = 0, b = 0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) { a += part[2 * i]; b += part[2 * i + 1]; }
  block_sum2(a, b, red);
  if (threadIdx.x == 0) { out2[0] = a; out2[1] = b; }
}

extern "C" int pdg_ln_partials_sum(const double* partials, int nparts, double* out2, void* stream) {
  PDG_CHECK_ARG(nparts > 0 && out2, "pdg_ln_partials_sum: empty");
  hipLaunchKernelGGL(ln_partials_sum_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, partials, nparts, out2);
  PDG_CHECK_LAUNCH("pdg_ln_partials_sum");
  return PDG_OK;
}

// ============================================================================ node P/Q pre-pass
template <bool RES>
__global__ __launch_bounds__(768, 3) void node_pq_kernel(int N, const float* __restrict__ a2p,
                                                          const pdg_ln_stat* __restrict__ stp,
                                                          const float* __restrict__ lg,
                                                          const float* __restrict__ lb,
                                                          const float* __restrict__ xres,
                                                          float* __restrict__ xout,
                                                          const float* __restrict__ W1,
                                                          float* __restrict__ P, float* __restrict__ Q) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  load_wblock(lds, W1, 3 * L, 0);           // W_a: input block x_i (target)
  load_wblock(lds + WBLK, W1, 3 * L, L);    // W_b: input block x_j (source)
  __syncthreads();
  const LNStat st = *reinterpret_cast<const LNStat*>(stp);
  const int l = lane_id();
  PDG_TILE_LOOP(N) {
    const int row = tile * TILE + (l & 15);
    const bool valid = row < N;
    const int rc = valid ? row : N - 1;
    float v[FRAG];
    ln_res_frag<RES>(v, a2p + (size_t)rc * L, RES ? xres + (size_t)rc * L : nullptr, st, lg, lb);
    if (valid) store_frag(xout + (size_t)row * L, v);
    Acc acc;
    zero_acc(acc);
    gemm128(acc, lds, v);
    if (valid) store_acc(P + (size_t)row * L, acc);
    zero_acc(acc);
    gemm128(acc, lds + WBLK, v);
    if (valid) store_acc(Q + (size_t)row * L, acc);
  }
}

extern "C" int pdg_node_pq(int n_nodes, const float* a2_prev, const pdg_ln_stat* st, const float* ln_g,
                           const float* ln_b, const float* x_res, float* x_out, const float* W1, float* P,
                           float* Q, void* stream) {
  PDG_CHECK_ARG(n_nodes > 0, "pdg_node_pq: n_nodes must be > 0");
  PDG_CHECK_ARG(PDG_ALIGNED(a2_prev) && PDG_ALIGNED(x_out) && PDG_ALIGNED(P) && PDG_ALIGNED(Q) &&
                    PDG_ALIGNED(W1) && (!x_res || PDG_ALIGNED(x_res)),
                "pdg_node_pq: misaligned pointer");
  const int grid = persistent_grid(n_nodes, 12, 1);
  if (x_res)
    hipLaunchKernelGGL(node_pq_kernel<true>, dim3(grid), dim3(768), 2 * WBLK * sizeof(float), (hipStream_t)stream,
                       n_nodes, a2_prev, st, ln_g, ln_b, x_res, x_out, W1, P, Q);
  else
    hipLaunchKernelGGL(node_pq_kernel<false>, dim3(grid), dim3(768), 2 * WBLK * sizeof(float), (hipStream_t)stream,
                       n_nodes, a2_prev, st, ln_g, ln_b, x_res, x_out, W1, P, Q);
  PDG_CHECK_LAUNCH("pdg_node_pq");
  return PDG_OK;
}

// ============================================================================ fused edge pass
// First layer of both edge_net evaluations from the shared C = W_c e + b1, in
// four chunks of 8 features (each accumulator block pair dies as its chunk is
// consumed):
//   edge update: relu(C + P[src] + Q[dst]) -> ve (kept for layer 2)
//   message:     relu(C + P[dst] + Q[src]) -> v
// Chunk 0's gathers are issued before the W_c GEMM so their latency hides behind
// it; chunk q+1's are in flight while chunk q is computed.
//
// Memory-order discipline of the tile loop: vmcnt counts loads and stores together
// and in issue order, so a load issued after a store cannot be waited for without
// also waiting for the store.  Every per-tile load is therefore issued before the
// stores it would otherwise queue behind: the next tile's rows and indices before
// this tile's last store, the gathers before a1m / a1e are stored, and the
// loop-invariant vectors (b1, b2, LayerNorm weight and bias) never touch vector
// memory inside the loop (FeatVec, ds_bpermute).
#ifndef PDG_EDGE_FWD_WAVES
#define PDG_EDGE_FWD_WAVES 8   // 2 waves per SIMD, 256 VGPRs: room for the prefetches (measured)
#endif
constexpr int EF_WAVES = PDG_EDGE_FWD_WAVES;
struct Gather8 {
  f32x4 xs[2], yd[2], xd[2], ys[2];
};

template <bool EU>
__device__ __forceinline__ void gather_chunk(Gather8& g, int q, const float* __restrict__ ps,
                                             const float* __restrict__ qd, const float* __restrict__ pd,
                                             const float* __restrict__ qs) {
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    if (EU) {
      g.xs[t] = ld4(ps, 2 * q + t);
      g.yd[t] = ld4(qd, 2 * q + t);
    }
    g.xd[t] = ld4(pd, 2 * q + t);
    g.ys[t] = ld4(qs, 2 * q + t);
  }
}

// ps/qd/pd/qs already offset by lane_col(); g0 holds chunk 0, already issued.
template <bool EU>
__device__ __forceinline__ void first_layers(float (&v)[FRAG], float (&ve)[FRAG], const Acc& C, Gather8 g0,
                                             const float* __restrict__ ps, const float* __restrict__ qd,
                                             const float* __restrict__ pd, const float* __restrict__ qs) {
  Gather8 cur = g0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    Gather8 nxt;
    if (q < 3) gather_chunk<EU>(nxt, q + 1, ps, qd, pd, qs);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float c = C.b[2 * q + t][j];
        if (EU) ve[8 * q + 4 * t + j] = fmaxf((c + cur.xs[t][j]) + cur.yd[t][j], 0.f);
        v[8 * q + 4 * t + j] = fmaxf((c + cur.xd[t][j]) + cur.ys[t][j], 0.f);
      }
    }
    if (q < 3) cur = nxt;
    PDG_FENCE();
  }
}

// v = LN(x) [+ r] from rows already in registers (models.py:225 residual).
template <bool RES>
__device__ __forceinline__ void ln_apply(float (&v)[FRAG], const float (&x)[FRAG], const float (&r)[FRAG],
                                         const LNStat& st, const FeatVec& g, const FeatVec& b) {
#pragma unroll
  for (int T = 0; T < 8; ++T) {
    const f32x4 gg = featvec_chunk(g, T), bb = featvec_chunk(b, T);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float y = div_den(x[4 * T + j] - st.mean, st.den, st.rstd) * gg[j] + bb[j];
      if (RES) y += r[4 * T + j];
      v[4 * T + j] = y;
    }
  }
}

// v = relu(acc + bias); the bias is added after the GEMM so that the accumulator
// starts as the MFMA's inline zero and occupies no registers before the GEMM.
__device__ __forceinline__ void bias_relu_fv(float (&v)[FRAG], const Acc& acc, const FeatVec& b) {
#pragma unroll
  for (int T = 0; T < 8; ++T) {
    const f32x4 bb = featvec_chunk(b, T);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[4 * T + j] = fmaxf(acc.b[T][j] + bb[j], 0.f);
  }
}

template <bool RES, bool EU>
__global__ __launch_bounds__(64 * EF_WAVES, EF_WAVES / 4) void edge_fwd_kernel(
    int E, const float* __restrict__ a2p, const pdg_ln_stat* __restrict__ stp, const float* __restrict__ lg,
    const float* __restrict__ lb, const float* __restrict__ eres, float* __restrict__ eout,
    const int* __restrict__ src, const int* __restrict__ dst, const float* __restrict__ P,
    const float* __restrict__ Q, const float* __restrict__ W1, const float* __restrict__ b1,
    const float* __restrict__ W2, const float* __restrict__ b2, float* __restrict__ a1m,
    float* __restrict__ a2m, float* __restrict__ a1e, float* __restrict__ a2e, double* __restrict__ part_m,
    double* __restrict__ part_e) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  load_wblock_swz(lds, W1, 3 * L, 2 * L);   // W_c (fp32): edge-feature block
  unsigned char* w2p = reinterpret_cast<unsigned char*>(lds + 128 * 128);
  load_wplanes(w2p, W2, L, 0);             // W2 as three bf16 term planes
#define PDG_GEMM_C(acc, v) gemm128_swz(acc, lds, v)
#define PDG_GEMM_2(acc, v) gemm128_x6(acc, w2p, v)
  const FeatVec fg = load_featvec(lg), fb = load_featvec(lb), fb1 = load_featvec(b1), fb2 = load_featvec(b2);
  __syncthreads();
  const LNStat st = *reinterpret_cast<const LNStat*>(stp);
  const int l = lane_id();
  const int lc = lane_col();
  double sm1 = 0, sm2 = 0, se1 = 0, se2 = 0;
  const int nw = blockDim.x >> 6, ntiles = tiles_of(E), stride = gridDim.x * nw;
  int tile = xcd_block() * nw + wave_id();
  // raw inputs of the current tile: LayerNorm input row, residual row, endpoints
  float xa[FRAG], xr[FRAG];
  int s_node = 0, d_node = 0;
  auto issue = [&](int t) {
    const int r = t * TILE + (l & 15);
    const int rc = r < E ? r : E - 1;
    s_node = src[rc];
    d_node = dst[rc];
    load_frag(xa, a2p + (size_t)rc * L);
    if (RES) load_frag(xr, eres + (size_t)rc * L);
  };
  issue(tile);   // unconditional (rows clamped), so the buffers are not live across the whole loop
  for (; tile < ntiles; tile += stride) {
    const int row = tile * TILE + (l & 15);
    const bool valid = row < E;
    const float* ps = P + (size_t)s_node * L + lc;
    const float* qd = Q + (size_t)d_node * L + lc;
    const float* pd = P + (size_t)d_node * L + lc;
    const float* qs = Q + (size_t)s_node * L + lc;
    Gather8 g0;
    gather_chunk<EU>(g0, 0, ps, qd, pd, qs);
    float v[FRAG];
    // e_t = LN(a2_prev) + e_res   (models.py:225 residual of the previous step)
    ln_apply<RES>(v, xa, xr, st, fg, fb);
    // C = W_c e_t + b1 (shared by both edge_net evaluations)
    Acc C;
    zero_acc(C);
    if (valid) store_frag(eout + (size_t)row * L, v);
    PDG_GEMM_C(C, v);
#pragma unroll
    for (int T = 0; T < 8; ++T) C.b[T] += featvec_chunk(fb1, T);
    // layer 1 of the edge update (models.py:219-222, x[row] = x[src], x[col] = x[dst]) and of
    // the message (models.py:233-238, x_i = x[dst], x_j = x[src])
    float ve[FRAG];
    first_layers<EU>(v, ve, C, g0, ps, qd, pd, qs);
    Acc Z;
    zero_acc(Z);
    if (valid && a1m) store_frag(a1m + (size_t)row * L, v);   // a1m / a1e: kept for the backward only
    if (EU && valid && a1e) store_frag(a1e + (size_t)row * L, ve);
    PDG_GEMM_2(Z, v);
    bias_relu_fv(v, Z, fb2);
    accum_stats(v, valid, sm1, sm2);
    if (EU) {
      // edge-update layer 2
      zero_acc(Z);
      if (valid) store_frag(a2m + (size_t)row * L, v);
      PDG_GEMM_2(Z, ve);
      bias_relu_fv(v, Z, fb2);
      accum_stats(v, valid, se1, se2);
    }
    issue(tile + stride);   // before this tile's last store
    PDG_FENCE();
    if (valid) store_frag((EU ? a2e : a2m) + (size_t)row * L, v);
  }
#undef PDG_GEMM_C
#undef PDG_GEMM_2
  // the weight images are dead once every wave has passed block_sum2's first barrier
  double* red = reinterpret_cast<double*>(lds);
  block_sum2(sm1, sm2, red);
  if (threadIdx.x == 0) {
    part_m[2 * blockIdx.x] = sm1;
    part_m[2 * blockIdx.x + 1] = sm2;
  }
  if (EU) {
    block_sum2(se1, se2, red + 32);
    if (threadIdx.x == 0) {
      part_e[2 * blockIdx.x] = se1;
      part_e[2 * blockIdx.x + 1] = se2;
    }
  }
}

extern "C" int pdg_edge_fwd(int n_edges, const float* a2_prev, const pdg_ln_stat* st, const float* ln_g,
                            const float* ln_b, const float* e_res, float* e_out, const int* src, const int* dst,
                            const float* P, const float* Q, const float* W1, const float* b1, const float* W2,
                            const float* b2, float* a1m, float* a2m, float* a1e, float* a2e, double* part_m,
                            double* part_e, int with_edge_update, int* nparts, void* stream) {
  PDG_CHECK_ARG(n_edges > 0, "pdg_edge_fwd: n_edges must be > 0");
  PDG_CHECK_ARG(a2_prev && st && ln_g && ln_b && e_out && src && dst && P && Q && W1 && b1 && W2 && b2 && a2m &&
                    part_m && nparts,
                "pdg_edge_fwd: null argument");
  PDG_CHECK_ARG(PDG_ALIGNED(a2_prev) && PDG_ALIGNED(e_out) && PDG_ALIGNED(P) && PDG_ALIGNED(Q) &&
                    PDG_ALIGNED(a1m) && PDG_ALIGNED(a2m) && (!e_res || PDG_ALIGNED(e_res)),
                "pdg_edge_fwd: misaligned pointer");
  PDG_CHECK_ARG(!with_edge_update || (a2e && part_e && PDG_ALIGNED(a1e) && PDG_ALIGNED(a2e)),
                "pdg_edge_fwd: edge-update outputs missing or misaligned");
  const int grid = persistent_grid(n_edges, EF_WAVES, 1);
  const size_t shm = (size_t)EDGE_LDS_BYTES;
  hipStream_t s = (hipStream_t)stream;
#define PDG_EDGE_FWD(R, U)                                                                                     \
  hipLaunchKernelGGL((edge_fwd_kernel<R, U>), dim3(grid), dim3(64 * EF_WAVES), shm, s, n_edges, a2_prev, st, ln_g, ln_b, \
                     e_res, e_out, src, dst, P, Q, W1, b1, W2, b2, a1m, a2m, a1e, a2e, part_m, part_e)
  if (e_res) {
    if (with_edge_update) PDG_EDGE_FWD(true, true); else PDG_EDGE_FWD(true, false);
  } else {
    if (with_edge_update) PDG_EDGE_FWD(false, true); else PDG_EDGE_FWD(false, false);
  }
#undef PDG_EDGE_FWD
  PDG_CHECK_LAUNCH("pdg_edge_fwd");
  if (nparts) *nparts = grid;
  return PDG_OK;
}

// ============================================================================ segment sum
// Half-wave (32 lanes x 16 B) per destination node; rows of a segment are
// contiguous in the dst-sorted edge order, summed sequentially from zero in
// segment order (= PyG scatter_add_ order for a coalesced edge_index).
constexpr int SEG_U = 8;

// part_a (pdg_segment_sum_fin): the message LayerNorm's statistics are reduced here from the edge
// forward's per-block partials (ln_stat_from_partials: bitwise pdg_ln_finalize) instead of by a
// finalize launch; block 0 stores them to st_a (read by the backward) and, from part_b, the
// edge-update LayerNorm's to st_b (read by the next step's edge forward).
__global__ __launch_bounds__(256) void segment_sum_kernel(int N, const int* __restrict__ rowptr,
                                                          const float* __restrict__ rows,
                                                          const pdg_ln_stat* __restrict__ stp,
                                                          const float* __restrict__ lg,
                                                          const float* __restrict__ lb,
                                                          float* __restrict__ out, float* __restrict__ xsum,
                                                          const double* __restrict__ part_a,
                                                          const double* __restrict__ part_b, int nparts, double count,
                                                          pdg_ln_stat* __restrict__ st_a, pdg_ln_stat* __restrict__ st_b) {
  const int hw = threadIdx.x >> 5, j = threadIdx.x & 31;
  const int nhw = blockDim.x >> 5;
  float mean = 0.f, den = 1.f, rstd = 1.f;
  f32x4 g = {1.f, 1.f, 1.f, 1.f}, b = {0.f, 0.f, 0.f, 0.f};
  __shared__ pdg_ln_stat st_sh;
  __shared__ double red[8];
  if (part_a) {
    if (blockIdx.x == 0 && part_b) {
      ln_stat_from_partials(part_b, nparts, count, st_b, red);
      __syncthreads();
    }
    ln_stat_from_partials(part_a, nparts, count, &st_sh, red);
    __syncthreads();
    if (blockIdx.x == 0 && threadIdx.x == 0) *st_a = st_sh;
    stp = &st_sh;
  }
  const bool ln = stp != nullptr;
  if (ln) {
    mean = stp->mean;
    den = stp->den;
    rstd = stp->rstd;
    g = reinterpret_cast<const f32x4*>(lg)[j];
    b = reinterpret_cast<const f32x4*>(lb)[j];
  }
  for (int v = blockIdx.x * nhw + hw; v < N; v += gridDim.x * nhw) {
    const int k0 = rowptr[v], k1 = rowptr[v + 1];
    f32x4 acc = {0.f, 0.f, 0.f, 0.f}, xs = {0.f, 0.f, 0.f, 0.f};
    // SEG_U rows in flight per round trip (the in-degree of a triangulated mesh is ~6): loads past
    // the segment end re-read its last row (an L1/L2 hit) and are not accumulated, so the sums
    // are formed row by row in CSR order exactly as a one-row-at-a-time loop would
    for (int k = k0; k < k1; k += SEG_U) {
      f32x4 x[SEG_U];
#pragma unroll
      for (int u = 0; u < SEG_U; ++u) {
        const int kk = k + u < k1 ? k + u : k1 - 1;
        x[u] = reinterpret_cast<const f32x4*>(rows + (size_t)kk * L)[j];
      }
#pragma unroll
      for (int u = 0; u < SEG_U; ++u) {
        if (k + u >= k1) break;
        if (ln) {
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const float h = div_den(x[u][c] - mean, den, rstd);
            xs[c] += h;
            x[u][c] = h * g[c] + b[c];
          }
        }
        acc += x[u];
      }
    }
    stg4(out + (size_t)v * L + 4 * j, acc);
    if (xsum) stg4(xsum + (size_t)v * L + 4 * j, xs);
  }
}

extern "C" int pdg_segment_sum(int n_nodes, const int* rowptr, const float* rows, const pdg_ln_stat* st,
                               const float* ln_g, const float* ln_b, float* out, float* xhat_sum, void* stream) {
  PDG_CHECK_ARG(!xhat_sum || (st && PDG_ALIGNED(xhat_sum)), "pdg_segment_sum: xhat_sum needs st, 16-B alignment");
  PDG_CHECK_ARG(n_nodes > 0, "pdg_segment_sum: n_nodes must be > 0");
  PDG_CHECK_ARG(PDG_ALIGNED(rows) && PDG_ALIGNED(out), "pdg_segment_sum: misaligned pointer");
  long want = (n_nodes + 7) / 8;
  long cap = (long)device_cus() * 8;
  const int grid = (int)(want < cap ? want : cap);
  hipLaunchKernelGGL(segment_sum_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, n_nodes, rowptr, rows,
                     st, ln_g, ln_b, out, xhat_sum, nullptr, nullptr, 0, 0.0, nullptr, nullptr);
  PDG_CHECK_LAUNCH("pdg_segment_sum");
  return PDG_OK;
}

extern "C" int pdg_segment_sum_fin(int n_nodes, const int* rowptr, const float* rows, const double* part_a,
                                   const double* part_b, int nparts, double count, pdg_ln_stat* st_a,
                                   pdg_ln_stat* st_b, const float* ln_g, const float* ln_b, float* out,
                                   float* xhat_sum, void* stream) {
  PDG_CHECK_ARG(n_nodes > 0, "pdg_segment_sum_fin: n_nodes must be > 0");
  PDG_CHECK_ARG(part_a && st_a && ln_g && ln_b && nparts > 0 && nparts <= MAX_BLOCKS && count > 0 &&
                    (!part_b || st_b),
                "pdg_segment_sum_fin: bad statistics arguments");
  PDG_CHECK_ARG(PDG_ALIGNED(rows) && PDG_ALIGNED(out) && (!xhat_sum || PDG_ALIGNED(xhat_sum)),
                "pdg_segment_sum_fin: misaligned pointer");
  long want = (n_nodes + 7) / 8;
  long cap = (long)device_cus() * 8;
  const int grid = (int)(want < cap ? want : cap);
  hipLaunchKernelGGL(segment_sum_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, n_nodes, rowptr, rows,
                     nullptr, ln_g, ln_b, out, xhat_sum, part_a, part_b, nparts, count, st_a, st_b);
  PDG_CHECK_LAUNCH("pdg_segment_sum_fin");
  return PDG_OK;
}

// ============================================================================ node MLP layer 1
__global__ __launch_bounds__(768, 3) void node_mlp1_kernel(int N, const float* __restrict__ aggr,
                                                            const float* __restrict__ x,
                                                            const float* __restrict__ Wn1,
                                                            const float* __restrict__ bn1,
                                                            float* __restrict__ a1n) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  load_wblock(lds, Wn1, 2 * L, 0);          // aggr block (models.py:241 cat order)
  load_wblock(lds + WBLK, Wn1, 2 * L, L);   // x block
  __syncthreads();
  const int l = lane_id();
  PDG_TILE_LOOP(N) {
    const int row = tile * TILE + (l & 15);
    const bool valid = row < N;
    const int rc = valid ? row : N - 1;
    float v[FRAG];
    Acc acc;
    zero_acc(acc);
    load_frag(v, aggr + (size_t)rc * L);
    gemm128(acc, lds, v);
    load_frag(v, x + (size_t)rc * L);
    gemm128(acc, lds + WBLK, v);
    bias_relu(v, acc, bn1);
    if (valid) store_frag(a1n + (size_t)row * L, v);
  }
}

extern "C" int pdg_node_mlp1(int n_nodes, const float* aggr, const float* x, const float* Wn1,
                             const float* bn1, float* a1n, void* stream) {
  PDG_CHECK_ARG(n_nodes > 0, "pdg_node_mlp1: n_nodes must be > 0");
  PDG_CHECK_ARG(PDG_ALIGNED(aggr) && PDG_ALIGNED(x) && PDG_ALIGNED(a1n) && PDG_ALIGNED(Wn1),
                "pdg_node_mlp1: misaligned pointer");
  const int grid = persistent_grid(n_nodes, 12, 1);
  hipLaunchKernelGGL(node_mlp1_kernel, dim3(grid), dim3(768), 2 * WBLK * sizeof(float), (hipStream_t)stream,
                     n_nodes, aggr, x, Wn1, bn1, a1n);
  PDG_CHECK_LAUNCH("pdg_node_mlp1");
  return PDG_OK;
}

// ============================================================================ MLP layer 2 (+ LN partials)
__global__ __launch_bounds__(384, 3) void mlp2_fwd_kernel(int M, const float* __restrict__ a1,
                                                           const float* __restrict__ W2,
                                                           const float* __restrict__ b2,
                                                           float* __restrict__ a2, double* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  load_wblock(lds, W2, L, 0);
  __syncthreads();
  const int l = lane_id();
  double s1 = 0, s2 = 0;
  PDG_TILE_LOOP(M) {
    const int row = tile * TILE + (l & 15);
    const bool valid = row < M;
    const int rc = valid ? row : M - 1;
    float v[FRAG];
    load_frag(v, a1 + (size_t)rc * L);
    Acc acc;
    zero_acc(acc);
    gemm128(acc, lds, v);
    bias_relu(v, acc, b2);
    if (valid) store_frag(a2 + (size_t)row * L, v);
    accum_stats(v, valid, s1, s2);
  }
  write_partials(s1, s2, part);
}

extern "C" int pdg_mlp2_fwd(int rows, const float* a1, const float* W2, const float* b2, float* a2,
                            double* partials, int* nparts, void* stream) {
  PDG_CHECK_ARG(rows > 0, "pdg_mlp2_fwd: rows must be > 0");
  PDG_CHECK_ARG(PDG_ALIGNED(a1) && PDG_ALIGNED(a2) && PDG_ALIGNED(W2), "pdg_mlp2_fwd: misaligned pointer");
  const int grid = persistent_grid(rows, 6, 2);
  hipLaunchKernelGGL(mlp2_fwd_kernel, dim3(grid), dim3(384), WBLK * sizeof(float), (hipStream_t)stream, rows,
                     a1, W2, b2, a2, partials);
  PDG_CHECK_LAUNCH("pdg_mlp2_fwd");
  if (nparts) *nparts = grid;
  return PDG_OK;
}

// ============================================================================ decoder
__global__ __launch_bounds__(384, 3) void decoder_kernel(int N, const float* __restrict__ a2p,
                                                          const pdg_ln_stat* __restrict__ stp,
                                                          const float* __restrict__ lg,
                                                          const float* __restrict__ lb,
                                                          const float* __restrict__ xres,
                                                          float* __restrict__ xout,
                                                          const float* __restrict__ Wd1,
                                                          const float* __restrict__ bd1,
                                                          float* __restrict__ a1d,
                                                          const float* __restrict__ Wd2,
                                                          const float* __restrict__ bd2,
                                                          const float* __restrict__ st8, int scale,
                                                          float* __restrict__ y, const double* __restrict__ part,
                                                          int nparts, double count, pdg_ln_stat* __restrict__ st_out) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* w2l = lds + WBLK;   // Wd2 (3 x 128)
  __shared__ LNStat st_sh;
  __shared__ double red_fin[2 * 384 / 64];
  if (part) {   // the last node LayerNorm's statistics folded in (pdg_decoder_fwd_fin; pdg_ln_finalize's order)
    ln_stat_from_partials(part, nparts, count, &st_sh, red_fin);
    __syncthreads();
    if (blockIdx.x == 0 && threadIdx.x == 0) *st_out = st_sh;
  }
  load_wblock(lds, Wd1, L, 0);
  for (int i = threadIdx.x; i < 3 * L; i += blockDim.x) w2l[i] = Wd2[i];
  __syncthreads();
  const LNStat st = part ? st_sh : *reinterpret_cast<const LNStat*>(stp);
  const int l = lane_id(), q = l >> 4;
  PDG_TILE_LOOP(N) {
    const int row = tile * TILE + (l & 15);
    const bool valid = row < N;
    const int rc = valid ? row : N - 1;
    float v[FRAG];
    ln_res_frag<true>(v, a2p + (size_t)rc * L, xres + (size_t)rc * L, st, lg, lb);
    if (valid) store_frag(xout + (size_t)row * L, v);
    Acc acc;
    zero_acc(acc);
    gemm128(acc, lds, v);
    bias_relu(v, acc, bd1);
    if (valid) store_frag(a1d + (size_t)row * L, v);
    // Linear(128 -> 3): quarter-row partial dots, combined across the four lane quarters
    float o3[3];
#pragma unroll
    for (int o = 0; o < 3; ++o) {
      const float* wp = w2l + o * L + lane_col();
      float d = 0.f;
#pragma unroll
      for (int s = 0; s < FRAG; ++s) d = fmaf(wp[16 * (s >> 2) + (s & 3)], v[s], d);
      o3[o] = d;
      PDG_FENCE();
    }
#pragma unroll
    for (int o = 0; o < 3; ++o) {
      // fixed combination order (q0 + q1) + (q2 + q3) in every lane
      const float x1 = __shfl_xor(o3[o], 16);
      const float lo = (q & 1) ? x1 + o3[o] : o3[o] + x1;     // pair (0,1) or (2,3)
      const float x2 = __shfl_xor(lo, 32);
      float r = (q & 2) ? x2 + lo : lo + x2;
      r = r + bd2[o];
      if (scale) r = r * st8[5] + st8[4];
      o3[o] = r;
    }
    if (valid && q == 0) {
      y[(size_t)row * 3 + 0] = o3[0];
      y[(size_t)row * 3 + 1] = o3[1];
      y[(size_t)row * 3 + 2] = o3[2];
    }
  }
}

static int decoder_fwd_launch(int n_nodes, const float* a2_prev, const pdg_ln_stat* st, const float* ln_g,
                              const float* ln_b, const float* x_res, float* x_out, const float* Wd1, const float* bd1,
                              float* a1d, const float* Wd2, const float* bd2, const float* stats8, int scale_output,
                              float* y, const double* partials, int nparts, double count, pdg_ln_stat* st_out,
                              void* stream) {
  PDG_CHECK_ARG(n_nodes > 0, "pdg_decoder_fwd: n_nodes must be > 0");
  PDG_CHECK_ARG(x_res != nullptr, "pdg_decoder_fwd: x_res is NULL");
  PDG_CHECK_ARG(!scale_output || stats8 != nullptr, "pdg_decoder_fwd: stats8 is NULL");
  PDG_CHECK_ARG(PDG_ALIGNED(a2_prev) && PDG_ALIGNED(x_res) && PDG_ALIGNED(x_out) && PDG_ALIGNED(a1d) &&
                    PDG_ALIGNED(Wd1) && PDG_ALIGNED(Wd2),
                "pdg_decoder_fwd: misaligned pointer");
  PDG_CHECK_ARG(partials ? (nparts > 0 && count > 0 && st_out != nullptr) : st != nullptr,
                "pdg_decoder_fwd: statistics arguments");
  const int grid = persistent_grid(n_nodes, 6, 2);
  hipLaunchKernelGGL(decoder_kernel, dim3(grid), dim3(384), (WBLK + 3 * L) * sizeof(float), (hipStream_t)stream,
                     n_nodes, a2_prev, st, ln_g, ln_b, x_res, x_out, Wd1, bd1, a1d, Wd2, bd2, stats8, scale_output, y,
                     partials, nparts, count, st_out);
  PDG_CHECK_LAUNCH("pdg_decoder_fwd");
  return PDG_OK;
}

extern "C" int pdg_decoder_fwd(int n_nodes, const float* a2_prev, const pdg_ln_stat* st, const float* ln_g,
                               const float* ln_b, const float* x_res, float* x_out, const float* Wd1,
                               const float* bd1, float* a1d, const float* Wd2, const float* bd2,
                               const float* stats8, int scale_output, float* y, void* stream) {
  return decoder_fwd_launch(n_nodes, a2_prev, st, ln_g, ln_b, x_res, x_out, Wd1, bd1, a1d, Wd2, bd2, stats8,
                            scale_output, y, nullptr, 0, 0.0, nullptr, stream);
}

extern "C" int pdg_decoder_fwd_fin(int n_nodes, const float* a2_prev, const double* partials, int nparts, double count,
                                   pdg_ln_stat* st_out, const float* ln_g, const float* ln_b, const float* x_res,
                                   float* x_out, const float* Wd1, const float* bd1, float* a1d, const float* Wd2,
                                   const float* bd2, const float* stats8, int scale_output, float* y, void* stream) {
  PDG_CHECK_ARG(partials != nullptr, "pdg_decoder_fwd_fin: partials are required");
  return decoder_fwd_launch(n_nodes, a2_prev, nullptr, ln_g, ln_b, x_res, x_out, Wd1, bd1, a1d, Wd2, bd2, stats8,
                            scale_output, y, partials, nparts, count, st_out, stream);
}

// ============================================================================ any-nonzero guard
// The flag is cleared by a one-thread kernel, not hipMemsetAsync: captured into a HIP graph
// (pdg/serve.py), a 4-byte memset node was replayed on the test box with a garbage byte value (the flag
// read 0x7c7c7c7c on one replay, 0 on the next; tests/test_gpu_published.py), kernel nodes are exact.
__global__ void flag_clear_kernel(int* __restrict__ flag) { *flag = 0; }

__global__ void any_nonzero_kernel(const float* __restrict__ x, long n, int* __restrict__ flag) {
  int found = 0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    found |= (x[i] != 0.f);
  if (__any(found) && lane_id() == 0) atomicOr(flag, 1);
}

extern "C" int pdg_any_nonzero(const float* x, int64_t n, int* flag, void* stream) {
  PDG_CHECK_ARG(n >= 0 && flag != nullptr, "pdg_any_nonzero: bad args");
  hipLaunchKernelGGL(flag_clear_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, flag);
  PDG_CHECK_LAUNCH("pdg_any_nonzero");
  if (n == 0) return PDG_OK;
  long blocks = (n + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(any_nonzero_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, x, (long)n,
                     flag);
  PDG_CHECK_LAUNCH("pdg_any_nonzero");
  return PDG_OK;
}

__global__ void zero_unless_kernel(const int* __restrict__ flag, float* __restrict__ y, long n) {
  if (*flag) return;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) y[i] = 0.f;
}

extern "C" int pdg_zero_unless(const int* flag, float* y, int64_t n, void* stream) {
  PDG_CHECK_ARG(n >= 0 && flag != nullptr && (n == 0 || y != nullptr), "pdg_zero_unless: bad args");
  if (n == 0) return PDG_OK;
  long blocks = (n + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(zero_unless_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, flag, y, (long)n);
  PDG_CHECK_LAUNCH("pdg_zero_unless");
  return PDG_OK;
}

// ============================================================================ library info
extern "C" const char* pdg_last_error(void) { return pdg::g_err; }
extern "C" int pdg_version(void) { return 1; }
extern "C" int pdg_max_blocks(void) { return MAX_BLOCKS; }
