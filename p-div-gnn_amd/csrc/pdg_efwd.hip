// Forward kernels in the block-cooperative layout (pdg_coop.hpp): the edge forward (training and inference
// forms), the edge and node encoders and the decoder (models.py:194-200, 219-238, 260-286).  Split from
// pdg_ebw.hip in round 6 (the same code; per-kernel ISA unchanged, tools/isa_diff.py).
#include "pdg_coop.hpp"

using namespace pdg;

// ============================================================================ edge forward, cooperative
// pdg_edge_fwd in the block-cooperative layout of the edge backward (one block of 8 waves per CU,
// contiguous row ranges, 32-row rounds): wave w owns output features [16w, 16w + 16) of both
// products with Wc and W2 stationary in registers as bf16 terms, the operands are 32-row bf16x6
// images in LDS, and every HBM row access is whole-row (outputs through fp32 row tiles).  Per round:
//   stage    e_t = LN(a2_prev) [+ e_res] (whole rows) -> HBM and the e image
//   | barrier | next round's rows issued
//   product  C = Wc e + b1; message a1m = relu(C + P[dst] + Q[src]), edge update
//            a1e = relu(C + P[src] + Q[dst]) (P / Q rows gathered at the wave's 16 features)
//            -> a1 images and row tiles
//   | barrier | a1 rows stored (training)
//   product  a2 = relu(W2 a1 + b2) -> LayerNorm partials, row tiles
//   | barrier | a2 rows stored; the next round's stage
// C = Wc e is an UNBIASED bf16x6 product (gemm_x6f from an e image; Wc as bf16 terms, the lo terms of
// its first two K chunks in LDS), round 5.  Rounds 2-4 kept C an exact fp32 product (v_mfma_f32_16x16x4_f32):
// C in the BIASED bf16x6 chain had shifted the LayerNorm statistics the
// way bf16x6 node_net did (parameter gradients 2e-4 from fp64 instead of 2.5e-6), a bias gemm_x6f does not
// have (rms error 3.6x below the fp32 MFMA chain's).  The fp32 C was half of this kernel's matrix time.


// Deferred a2 stores: a2 goes into two tiles of its own
// and its rows are stored after the NEXT round's first barrier, behind that round's gathers and row
// loads, so a round has two barriers instead of four (the barrier that freed the a1 tiles for a2 and
// the one that completed the a2 tiles go: the loop-top barrier completes both the e tile and the
// previous round's a2 tiles), and the C product's wait for its gathers no longer covers the previous
// round's a2 stores.  Bitwise the same outputs as storing each round's a2 at once; 32 KB more LDS (131 KB;
// 216 -> 210.5 us per config-2 call with X, the step -0.05 ms, in two same-box A/B pairs, round 3).
//
// X (XCD-interleaved rounds): the blocks that share an XCD's L2 (b and b + 8; the grid
// a multiple of 8) sweep one contiguous eighth of the rows together, taking its 32-row rounds
// round-robin, instead of each block owning a contiguous range.  The P / Q rows an edge gathers are
// reused by the edges of the mesh neighbours of its nodes, about +-13 rounds away in dst order: with
// per-block ranges every block of an XCD keeps such a window live (32 x ~280 KB, over the 4 MiB L2, so
// the reuse was served by the Infinity Cache), with interleaved rounds the XCD has one window.
template <bool RES, bool EU, bool X = false>
__global__ __launch_bounds__(EBW_THREADS, 1) void edge_fwd_coop_kernel(
    int E, const float* __restrict__ a2p, const pdg_ln_stat* __restrict__ stp, const float* __restrict__ lg,
    const float* __restrict__ lb, const float* __restrict__ eres, float* __restrict__ eout,
    const int* __restrict__ src, const int* __restrict__ dst, const float* __restrict__ P,
    const float* __restrict__ Q, const float* __restrict__ W1, const float* __restrict__ b1,
    const float* __restrict__ W2, const float* __restrict__ b2, float* __restrict__ a1m, float* __restrict__ a2m,
    float* __restrict__ a1e, float* __restrict__ a2e, double* __restrict__ part_m, double* __restrict__ part_e) {
  extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
  unsigned char* img_m = sm;                                   // a1m
  unsigned char* img_x = sm + EBW_IMG;                         // a1e (EU)
  float* t_m = reinterpret_cast<float*>(sm + 2 * EBW_IMG);     // fp32 row tiles: a1m / a2m
  float* t_x = t_m + EFC_TILE;                                 //                 a1e / a2e
  float* t_e = t_x + EFC_TILE;                                 //                 e_t
  // e as a bf16x6 image (24 KB)
  unsigned char* img_e = reinterpret_cast<unsigned char*>(t_e);
  constexpr int E_BYTES = EBW_IMG;
  float* t_am = reinterpret_cast<float*>(img_e + E_BYTES);     // deferred a2m / a2e tiles
  float* t_ae = t_am + EFC_TILE;
  // the lo bf16 terms of Wc's K chunks 0 and 1 in LDS, after every region (with all 12 terms
  // in registers the main instantiation spilled 5 VGPRs and was no faster than fp32 MFMAs)
  unsigned char* wlo = reinterpret_cast<unsigned char*>(t_am) + 2 * EFC_TILE * 4;
  const int l = lane_id(), w = wave_id();
  const int cg = threadIdx.x & 31, rg = threadIdx.x >> 5;
  const int oc = 16 * w + 4 * (l >> 4);
  // rows: [r0, r1) is the range the block's buffer resources span and its loads clamp to; the block's
  // rounds start at `first` and are `stride` rows apart (X: the XCD's range, every (G/8)-th round)
  int r0, r1, first, stride;
  row_schedule(X, E, r0, r1, first, stride);
  // the weights as A operands, rows = output features 16w .. 16w + 15 (W is out x in, row-major):
  // Wc = W1[:, 256:384] (row stride 384), W2
  WSlice wsc;     // Wc as bf16 terms (gemm_x6f's A operand)
  WSlice ws2;     // both loaded after the first round's row loads (the round trips overlap)
  const LNStat st = *reinterpret_cast<const LNStat*>(stp);
  const f32x4 g4 = *reinterpret_cast<const f32x4*>(lg + 4 * cg), bb4 = *reinterpret_cast<const f32x4*>(lb + 4 * cg);
  const f32x4 b1o = *reinterpret_cast<const f32x4*>(b1 + oc), b2o = *reinterpret_cast<const f32x4*>(b2 + oc);
  double sm1 = 0, sm2 = 0, se1 = 0, se2 = 0;
  f32x4 xa[2], xr[2];
  int dq[2], sq[2];
  // the row outputs through range-checked buffer stores: no memory operation of the loop is
  // conditional, so the compiler's vmcnt counts stay exact (a store skipped on some path made them
  // collapse).  An omitted output (a1m / a1e in inference, a2m beside the inference sums) gets an
  // empty range: its stores are issued and dropped.
  const __amdgpu_buffer_rsrc_t rs_e = rows_rsrc(eout, r0, r1);
  const __amdgpu_buffer_rsrc_t rs_a1m = rows_rsrc(a1m, r0, r1);
  const __amdgpu_buffer_rsrc_t rs_a1e = rows_rsrc(EU ? a1e : nullptr, r0, r1);
  const __amdgpu_buffer_rsrc_t rs_a2m = rows_rsrc(a2m, r0, r1);
  const __amdgpu_buffer_rsrc_t rs_a2e = rows_rsrc(EU ? a2e : nullptr, r0, r1);
  auto issue = [&](int base) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const size_t rc = (size_t)clamp_row(base + rg + 16 * u, r1) * L + 4 * cg;
      xa[u] = *reinterpret_cast<const f32x4*>(a2p + rc);
      if (RES) xr[u] = *reinterpret_cast<const f32x4*>(eres + rc);
      const int pr = clamp_row(base + 16 * u + (l & 15), r1);   // this lane's product rows
      dq[u] = dst[pr];
      sq[u] = src[pr];
    }
  };
  auto stage = [&](int base) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int r = rg + 16 * u;
      const bool ok = base + r < r1;
      f32x4 e;
#pragma unroll
      for (int j = 0; j < 4; ++j) {   // ln_apply (pdg_fwd.hip), element by element
        float y = div_den(xa[u][j] - st.mean, st.den, st.rstd) * g4[j] + bb4[j];
        if (RES) y += xr[u][j];
        e[j] = y;
      }
      rows_store4_nt(rs_e, base + r - r0, 4 * cg, e);
      img_store4(img_e, r, cg, ok ? e : f32x4{0.f, 0.f, 0.f, 0.f});
    }
  };
  issue(first);   // E > 0: an empty block (first = r1 = E) reads row E - 1
  load_wslice(wsc, W1 + 2 * L, w, 3 * L);
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) *reinterpret_cast<bf16x8*>(wlo + ((2 * w + ks) * 64 + l) * 16) = wsc.a[ks][2];
  load_wslice(ws2, W2, w);
  // the loop-invariant weights and biases are in registers before the loop (an empty asm using them
  // here): left to the compiler, their loads were sunk to the loop's preheader, still in flight at
  // the loop head, and the count merged there made every round's C product wait for the previous
  // round's stores (vmcnt 23 .. 16)
#pragma unroll
  for (int ks = 0; ks < 4; ++ks)
#pragma unroll
    for (int p = 0; p < 3; ++p)
      if (p < 2 || ks >= 2) pin_vgpr(wsc.a[ks][p]);
#pragma unroll
  for (int ks = 0; ks < 4; ++ks)
#pragma unroll
    for (int p = 0; p < 3; ++p) pin_vgpr(ws2.a[ks][p]);
  pin_vgpr(b1o);
  pin_vgpr(b2o);
  // and the first round's gather indices (pending at the loop head, they made every round wait for
  // the previous round's a1 / a2 stores, vmcnt(2))
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    pin_vgpr(dq[u]);
    pin_vgpr(sq[u]);
  }
  stage(first);
  for (int base = first; base < r1; base += stride) {
    __syncthreads();   // e tile complete
    int dc[2] = {dq[0], dq[1]}, sc[2] = {sq[0], sq[1]};
    // ---- this round's P / Q rows first, then the next round's rows (pinned by sched_barrier): the
    // gathers are waited for in the C product below, and with the next round's HBM loads issued
    // ahead of them (vmcnt counts in issue order) every round waited for those too
    f32x4 gpd[2], gqs[2], gps[2], gqd[2];
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      gpd[nb] = *reinterpret_cast<const f32x4*>(P + (size_t)dc[nb] * PQ_LD + pq_col(oc));
      gqs[nb] = *reinterpret_cast<const f32x4*>(Q + (size_t)sc[nb] * PQ_LD + pq_col(oc));
      if (EU) {
        gps[nb] = *reinterpret_cast<const f32x4*>(P + (size_t)sc[nb] * PQ_LD + pq_col(oc));
        gqd[nb] = *reinterpret_cast<const f32x4*>(Q + (size_t)dc[nb] * PQ_LD + pq_col(oc));
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    issue(base + stride);   // clamped past r1: unconditional
    __builtin_amdgcn_sched_barrier(0);
    {   // the previous round's a2 rows (tiles completed by the barrier above; none before the first
               // round: base - stride lies below the range and its stores are dropped)
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int r = rg + 16 * u;
        rows_store4_nt(rs_a2m, base - stride + r - r0, 4 * cg, *reinterpret_cast<const f32x4*>(t_am + r * OT_STRIDE + 4 * cg));
        if (EU) rows_store4_nt(rs_a2e, base - stride + r - r0, 4 * cg, *reinterpret_cast<const f32x4*>(t_ae + r * OT_STRIDE + 4 * cg));
      }
    }
    // ---- C = Wc e + b1 and the two first layers at this wave's 16 features
    f32x4 d[2];
    d[0] = d[1] = f32x4{0.f, 0.f, 0.f, 0.f};
    {
      WSlice wc = wsc;   // the lo terms of K chunks 0-1 from LDS
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) wc.a[ks][2] = *reinterpret_cast<const bf16x8*>(wlo + ((2 * w + ks) * 64 + l) * 16);
      gemm_x6f<2, X6_TERM, true>(d, wc, img_e);
    }
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      const int r = 16 * nb + (l & 15);
      f32x4 am, ae;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float c = d[nb][j] + b1o[j];
        am[j] = fmaxf((c + gpd[nb][j]) + gqs[nb][j], 0.f);
        if (EU) ae[j] = fmaxf((c + gps[nb][j]) + gqd[nb][j], 0.f);
      }
      img_store4(img_m, r, 4 * w + (l >> 4), am);
      if (a1m) *reinterpret_cast<f32x4*>(t_m + r * OT_STRIDE + oc) = am;
      if (EU) {
        img_store4(img_x, r, 4 * w + (l >> 4), ae);
        if (a1e) *reinterpret_cast<f32x4*>(t_x + r * OT_STRIDE + oc) = ae;
      }
    }
    __syncthreads();   // a1 images and tiles complete
#pragma unroll
    for (int u = 0; u < 2; ++u) {   // (dropped without a1m / a1e: the tiles are then not written)
      const int r = rg + 16 * u;
      rows_store4_nt(rs_a1m, base + r - r0, 4 * cg, *reinterpret_cast<const f32x4*>(t_m + r * OT_STRIDE + 4 * cg));
      if (EU) rows_store4_nt(rs_a1e, base + r - r0, 4 * cg, *reinterpret_cast<const f32x4*>(t_x + r * OT_STRIDE + 4 * cg));
    }
    // ---- a2 = relu(W2 a1 + b2) for both evaluations
    float* t_a2 = t_am;
    float* t_a2e = t_ae;
    constexpr int NI = EU ? 2 : 1;
    f32x4 d2[NI][2];
    const unsigned char* ia[NI];
    ia[0] = img_m;
    if (EU) ia[NI - 1] = img_x;
    gemm_round<NI>(d2, ws2, ia);
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      const int r = 16 * nb + (l & 15);
      const bool ok = base + r < r1;
#pragma unroll
      for (int u = 0; u < NI; ++u) {
        f32x4 a;
#pragma unroll
        for (int j = 0; j < 4; ++j) a[j] = fmaxf(d2[u][nb][j] + b2o[j], 0.f);
        *reinterpret_cast<f32x4*>((u ? t_a2e : t_a2) + r * OT_STRIDE + oc) = a;
        if (ok) {
          const double p1 = (double)((a[0] + a[1]) + (a[2] + a[3]));
          const double p2 = (double)((a[0] * a[0] + a[1] * a[1]) + (a[2] * a[2] + a[3] * a[3]));
          if (u) { se1 += p1; se2 += p2; } else { sm1 += p1; sm2 += p2; }
        }
      }
    }
    stage(base + stride);   // past r1: stores dropped, the tile unused; the e tile was last read before the second barrier
  }
  {   // the last round's a2 rows
    __syncthreads();
    const int last = first < r1 ? first + (r1 - 1 - first) / stride * stride : first;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int r = rg + 16 * u;
      rows_store4_nt(rs_a2m, last + r - r0, 4 * cg, *reinterpret_cast<const f32x4*>(t_am + r * OT_STRIDE + 4 * cg));
      if (EU) rows_store4_nt(rs_a2e, last + r - r0, 4 * cg, *reinterpret_cast<const f32x4*>(t_ae + r * OT_STRIDE + 4 * cg));
    }
  }
  double* red = reinterpret_cast<double*>(sm);
  __syncthreads();
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

// ============================================================================ edge forward, inference
// pdg_edge_fwd_coop's work without the layer-1 outputs (inference: nothing reads them) in 16-row rounds
// with ONE barrier per round, the rounds' two product phases
// overlapped (the layout of pdg_edge_bwd_w2: two register sets of row loads by round parity, double-
// buffered images).  After the barrier that completes round k's e image and round k-1's a1 images, a wave
// runs, for its 16 features:
//   C_k = Wc e_k (unbiased bf16x6, gemm_x6f) and the two W2 products of round k-1 (gemm_round): three
//   independent MFMA chains in one phase, where pdg_edge_fwd_coop runs them in two phases with a
//   barrier between; then a2_{k-1} (+ LayerNorm partials) into its row tiles; a1_k = relu(C_k + b1 +
//   gathered P / Q rows) into round k's a1 images (the gathers were issued one round earlier, so the
//   products of the whole phase cover their latency); round k+1's gathers; the stage of round k+1 (its
//   rows loaded two rounds earlier: LayerNorm + residual, e_{k+1} stored and imaged, the set re-issued for
//   round k+3); the stores of a2_{k-2} from its tiles (written before the barrier).
// Per output element the MFMA chains are those of pdg_edge_fwd_coop (bitwise the same e_t, a2); the
// LayerNorm partial sums visit the rows in another order.  LDS: e images 2 x 12 KB, a1 images 4 x 12 KB,
// a2 tiles 4 x 8.25 KB, Wc lo terms 16 KB = 121 KB.  Inference edge forward 494 -> 446 us (edge update)
// and 344 -> 312 us (message only) per 614k-edge call; in training (the a1 rows stored through tiles as
// well) it measured no faster than pdg_edge_fwd_coop (EXPERIMENTS §5), which stays the training kernel.
constexpr int EP_TILE = R16 * OT_STRIDE;          // floats per 16-row fp32 tile
template <bool RES, bool EU, bool X>
__global__ __launch_bounds__(EBW_THREADS, 1) void edge_fwd_infer_kernel(
    int E, const float* __restrict__ a2p, const pdg_ln_stat* __restrict__ stp, const float* __restrict__ lg,
    const float* __restrict__ lb, const float* __restrict__ eres, float* __restrict__ eout,
    const int* __restrict__ src, const int* __restrict__ dst, const float* __restrict__ P,
    const float* __restrict__ Q, const float* __restrict__ W1, const float* __restrict__ b1,
    const float* __restrict__ W2, const float* __restrict__ b2, float* __restrict__ a2m, float* __restrict__ a2e,
    double* __restrict__ part_m, double* __restrict__ part_e) {
  extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
  unsigned char* img_e = sm;                                    // [2] e images (round parity)
  unsigned char* img_a = sm + 2 * IMG16;                        // [2][2] a1 images: [parity][m, e]
  float* t_a2 = reinterpret_cast<float*>(sm + 6 * IMG16);       // [2][2] a2 tiles: [parity][m, e]
  unsigned char* wlo = reinterpret_cast<unsigned char*>(t_a2 + 4 * EP_TILE);
  const int l = lane_id(), w = wave_id();
  const int cg = threadIdx.x & 31, rg = threadIdx.x >> 5;      // the thread's staged row rg (0..15)
  const int oc = 16 * w + 4 * (l >> 4), pr = l & 15;            // this lane's product features and row
  int r0, r1, first, stride;   // 32-row units (rounds base and base + 16), the next unit `stride` rows on
  row_schedule(X, E, r0, r1, first, stride);
  const int units = first < r1 ? (r1 - 1 - first) / stride + 1 : 0;
  const int K = 2 * units;                                       // rounds of this block
  auto rbase = [&](int k) { return first + (k >> 1) * stride + R16 * (k & 1); };
  WSlice wsc, ws2;
  const LNStat st = *reinterpret_cast<const LNStat*>(stp);
  const f32x4 g4 = *reinterpret_cast<const f32x4*>(lg + 4 * cg), bb4 = *reinterpret_cast<const f32x4*>(lb + 4 * cg);
  const f32x4 b1o = *reinterpret_cast<const f32x4*>(b1 + oc), b2o = *reinterpret_cast<const f32x4*>(b2 + oc);
  double sm1 = 0, sm2 = 0, se1 = 0, se2 = 0;
  // row outputs through range-checked buffer stores (no conditional memory operation in the loop)
  const __amdgpu_buffer_rsrc_t rs_e = rows_rsrc(eout, r0, r1);
  const __amdgpu_buffer_rsrc_t rs_a2m = rows_rsrc(a2m, r0, r1);
  const __amdgpu_buffer_rsrc_t rs_a2e = rows_rsrc(EU ? a2e : nullptr, r0, r1);
  // two register sets of prefetched rows (round parity): the staged row's a2_prev / e_prev chunk and the
  // product row's dst / src
  f32x4 xa[2], xr[2];
  int dq[2], sq[2];
  auto issue = [&](int s, int k) {
    const int base = rbase(k);
    const size_t rc = (size_t)clamp_row(base + rg, r1) * L + 4 * cg;
    xa[s] = *reinterpret_cast<const f32x4*>(a2p + rc);
    if (RES) xr[s] = *reinterpret_cast<const f32x4*>(eres + rc);
    const int q = clamp_row(base + pr, r1);
    dq[s] = dst[q];
    sq[s] = src[q];
  };
  f32x4 gpd, gqs, gps, gqd;   // the next round's gathered P / Q rows at this lane's features
  auto gather = [&](int s) {
    gpd = *reinterpret_cast<const f32x4*>(P + (size_t)dq[s] * PQ_LD + pq_col(oc));
    gqs = *reinterpret_cast<const f32x4*>(Q + (size_t)sq[s] * PQ_LD + pq_col(oc));
    if (EU) {
      gps = *reinterpret_cast<const f32x4*>(P + (size_t)sq[s] * PQ_LD + pq_col(oc));
      gqd = *reinterpret_cast<const f32x4*>(Q + (size_t)dq[s] * PQ_LD + pq_col(oc));
    }
  };
  auto stage = [&](int s, int k) {   // round k's e rows from set s into e image s; the set re-issued for k + 2
    const int base = rbase(k);
    const bool ok = base + rg < r1;
    f32x4 e;
#pragma unroll
    for (int j = 0; j < 4; ++j) {   // ln_apply (pdg_fwd.hip), element by element
      float y = div_den(xa[s][j] - st.mean, st.den, st.rstd) * g4[j] + bb4[j];
      if (RES) y += xr[s][j];
      e[j] = y;
    }
    rows_store4_nt(rs_e, base + rg - r0, 4 * cg, e);
    img_store4<T16>(img_e + s * IMG16, rg, cg, ok ? e : f32x4{0.f, 0.f, 0.f, 0.f});
    issue(s, k + 2);
  };
  // the a1 images of "round -1" (read by the first phase's W2 products, whose rows are all dropped) zeroed
  for (int i = threadIdx.x; i < 4 * IMG16 / 16; i += EBW_THREADS)
    reinterpret_cast<f32x4*>(img_a)[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  issue(0, 0);
  __builtin_amdgcn_sched_barrier(0);
  issue(1, 1);
  __builtin_amdgcn_sched_barrier(0);
  load_wslice(wsc, W1 + 2 * L, w, 3 * L);
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) *reinterpret_cast<bf16x8*>(wlo + ((2 * w + ks) * 64 + l) * 16) = wsc.a[ks][2];
  load_wslice(ws2, W2, w);
#pragma unroll
  for (int ks = 0; ks < 4; ++ks)
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      if (p < 2 || ks >= 2) pin_vgpr(wsc.a[ks][p]);
      pin_vgpr(ws2.a[ks][p]);
    }
  pin_vgpr(b1o);
  pin_vgpr(b2o);
  gather(0);
  __builtin_amdgcn_sched_barrier(0);
  stage(0, 0);
  // one round; its parity S is a compile-time constant (the loop runs rounds in pairs): register sets indexed
  // by a run-time parity became selects that waited for both sets' loads (vmcnt(0)) every round
  auto round = [&](auto S, const int k) {
    constexpr int s = decltype(S)::value, sp = s ^ 1;   // round k's buffers / set, round k +- 1's
    const int basep = rbase(k - 1);
    __syncthreads();   // e image k, a1 images k - 1, the a2 / a1 tiles of rounds k - 2 / k - 1 complete
    // ---- C_k = Wc e_k and W2 a1_{k-1} for both evaluations: three independent MFMA chains
    f32x4 dc[1] = {{0.f, 0.f, 0.f, 0.f}};
    {
      WSlice wc = wsc;   // the lo terms of K chunks 0-1 from LDS
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) wc.a[ks][2] = *reinterpret_cast<const bf16x8*>(wlo + ((2 * w + ks) * 64 + l) * 16);
      gemm_x6f<1, T16, true>(dc, wc, img_e + s * IMG16);
    }
    constexpr int NI = EU ? 2 : 1;
    f32x4 d2[NI][1];
    const unsigned char* ia[NI];
    ia[0] = img_a + (2 * sp) * IMG16;
    if (EU) ia[NI - 1] = img_a + (2 * sp + 1) * IMG16;
    gemm_round<NI, 1, T16>(d2, ws2, ia);
    // ---- a2_{k-1} into its tiles (parity sp) and the LayerNorm partials of its valid rows
    {
      const bool ok = k > 0 && basep + pr < r1;
#pragma unroll
      for (int u = 0; u < NI; ++u) {
        f32x4 a;
#pragma unroll
        for (int j = 0; j < 4; ++j) a[j] = fmaxf(d2[u][0][j] + b2o[j], 0.f);
        *reinterpret_cast<f32x4*>(t_a2 + (2 * sp + u) * EP_TILE + pr * OT_STRIDE + oc) = a;
        if (ok) {
          const double p1 = (double)((a[0] + a[1]) + (a[2] + a[3]));
          const double p2 = (double)((a[0] * a[0] + a[1] * a[1]) + (a[2] * a[2] + a[3] * a[3]));
          if (u) { se1 += p1; se2 += p2; } else { sm1 += p1; sm2 += p2; }
        }
      }
    }
    // ---- a1_k = relu(C_k + b1 + gathered rows) into round k's a1 images
    {
      f32x4 am, ae;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float c = dc[0][j] + b1o[j];
        am[j] = fmaxf((c + gpd[j]) + gqs[j], 0.f);
        if (EU) ae[j] = fmaxf((c + gps[j]) + gqd[j], 0.f);
      }
      img_store4<T16>(img_a + (2 * s) * IMG16, pr, 4 * w + (l >> 4), am);
      if (EU) img_store4<T16>(img_a + (2 * s + 1) * IMG16, pr, 4 * w + (l >> 4), ae);
    }
    // ---- round k + 1: its gathers (indices in set sp, before the stage re-issues the set), its stage
    __builtin_amdgcn_sched_barrier(0);
    gather(sp);
    __builtin_amdgcn_sched_barrier(0);
    stage(sp, k + 1);
    // ---- the stores of a2_{k-2} (tiles of parity s), every tile read first
    {
      const int base2 = rbase(k - 2);
      f32x4 v[2];
      v[0] = *reinterpret_cast<const f32x4*>(t_a2 + (2 * s) * EP_TILE + rg * OT_STRIDE + 4 * cg);
      if (EU) v[1] = *reinterpret_cast<const f32x4*>(t_a2 + (2 * s + 1) * EP_TILE + rg * OT_STRIDE + 4 * cg);
      // rounds before the first (k < 2) lie below r0: their stores are dropped
      rows_store4_nt(rs_a2m, (k >= 2 ? base2 : r0 - R16) + rg - r0, 4 * cg, v[0]);
      if (EU) rows_store4_nt(rs_a2e, (k >= 2 ? base2 : r0 - R16) + rg - r0, 4 * cg, v[1]);
    }
  };
  for (int k = 0; k < K; k += 2) {   // K = 2 x units is even
    round(std::integral_constant<int, 0>{}, k);
    round(std::integral_constant<int, 1>{}, k + 1);
  }
  round(std::integral_constant<int, 0>{}, K);   // the last round's products, stores of the last two rounds
  {   // the last round's a2 rows (round K - 1, tiles of parity (K - 1) & 1)
    __syncthreads();
    constexpr int sl = 1;   // round K - 1 (K even)
    f32x4 v0 = *reinterpret_cast<const f32x4*>(t_a2 + (2 * sl) * EP_TILE + rg * OT_STRIDE + 4 * cg), v1;
    if (EU) v1 = *reinterpret_cast<const f32x4*>(t_a2 + (2 * sl + 1) * EP_TILE + rg * OT_STRIDE + 4 * cg);
    const int bl = K > 0 ? rbase(K - 1) : r0 - R16;
    rows_store4_nt(rs_a2m, bl + rg - r0, 4 * cg, v0);
    if (EU) rows_store4_nt(rs_a2e, bl + rg - r0, 4 * cg, v1);
  }
  double* red = reinterpret_cast<double*>(sm);
  __syncthreads();
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

// ============================================================================ edge encoder forward
// The edge encoder (models.py:264-275, input 1 -> 128 -> 128 + the LayerNorm partials of the
// output) in the cooperative layout: a1 = relu(w0 e + b0) formed per element (encoder_kernel's
// formula, bitwise), W2 a1 as a bf16x6 product with W2 stationary in registers (the W2 products
// of the edge forward), a2 rows stored whole through an fp32 row tile.  Replaces the fp32-MFMA
// encoder_kernel<1> (LDS weights), which the W2 product's matrix time bounded.  a1 is not stored
// (pdg_edge_enc_bwd recomputes it).
__global__ __launch_bounds__(EBW_THREADS, 1) void edge_enc_fwd_kernel(
    int E, const float* __restrict__ e_in, const float* __restrict__ w0, const float* __restrict__ b0,
    const float* __restrict__ W2, const float* __restrict__ b2, float* __restrict__ a2,
    double* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
  unsigned char* img = sm;                                     // a1 (bf16x6)
  float* t_a = reinterpret_cast<float*>(sm + EBW_IMG);         // a2 row tile
  const int l = lane_id(), w = wave_id();
  const int cg = threadIdx.x & 31, rg = threadIdx.x >> 5;
  const int oc = 16 * w + 4 * (l >> 4);
  int r0, r1;
  block_rows(E, r0, r1);
  WSlice ws2;
  load_wslice(ws2, W2, w);
  const f32x4 w04 = *reinterpret_cast<const f32x4*>(w0 + 4 * cg);
  const f32x4 b04 = *reinterpret_cast<const f32x4*>(b0 + 4 * cg);
  const f32x4 b2o = *reinterpret_cast<const f32x4*>(b2 + oc);
  double s1 = 0, s2 = 0;
  float pe[2];
  auto issue = [&](int base) {
#pragma unroll
    for (int u = 0; u < 2; ++u) pe[u] = e_in[clamp_row(base + rg + 16 * u, r1)];
  };
  // every memory operation of the loop unconditional (clamped loads, range-checked stores: a store
  // skipped on some path made the stage wait for the previous round's stores), the next round's
  // inputs issued before the barrier, the first round's and the weights complete before the loop
  const __amdgpu_buffer_rsrc_t rs_a2 = rows_rsrc(a2, r0, r1);
  issue(r0);   // E > 0: an empty block (r0 = r1 = E) reads row E - 1
#pragma unroll
  for (int u = 0; u < 2; ++u) pin_vgpr(pe[u]);
#pragma unroll
  for (int ks = 0; ks < 4; ++ks)
#pragma unroll
    for (int q = 0; q < 3; ++q) pin_vgpr(ws2.a[ks][q]);
  pin_vgpr(b2o);
  // the first round peeled off (unconditional: an empty block runs it with every store dropped), so
  // the loop is entered in its steady state: next round's loads, then this round's stores
  auto round = [&](const int base) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int r = rg + 16 * u;
      f32x4 a;
#pragma unroll
      for (int j = 0; j < 4; ++j) a[j] = fmaxf(fmaf(w04[j], pe[u], 0.f) + b04[j], 0.f);
      img_store4(img, r, cg, base + r < r1 ? a : f32x4{0.f, 0.f, 0.f, 0.f});
    }
    issue(base + X6_ROWS);
    __syncthreads();   // the a1 image is complete
    f32x4 d[1][2];
    const unsigned char* imgs[1] = {img};
    gemm_round<1>(d, ws2, imgs);
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      const int r = 16 * nb + (l & 15);
      f32x4 a;
#pragma unroll
      for (int j = 0; j < 4; ++j) a[j] = fmaxf(d[0][nb][j] + b2o[j], 0.f);
      *reinterpret_cast<f32x4*>(t_a + r * OT_STRIDE + oc) = a;
      if (base + r < r1) {
        s1 += (double)((a[0] + a[1]) + (a[2] + a[3]));
        s2 += (double)((a[0] * a[0] + a[1] * a[1]) + (a[2] * a[2] + a[3] * a[3]));
      }
    }
    __syncthreads();   // the a2 tile is complete; the image is free
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int r = rg + 16 * u;
      rows_store4_nt(rs_a2, base + r - r0, 4 * cg, *reinterpret_cast<const f32x4*>(t_a + r * OT_STRIDE + 4 * cg));
    }
  };
  round(r0);
  for (int base = r0 + X6_ROWS; base < r1; base += X6_ROWS) round(base);
  double* red = reinterpret_cast<double*>(sm);
  __syncthreads();
  block_sum2(s1, s2, red);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = s1;
    part[2 * blockIdx.x + 1] = s2;
  }
}

// ============================================================================ node encoder forward
// The node encoder (models.py:260-274, 6 inputs -> 128 -> 128 + the LayerNorm partials of the output) in
// the layout of edge_enc_fwd_kernel: a1 = relu(W0 x + b0) per element in encoder_kernel's order (bitwise
// its a1, stored for the backward), W2 a1 as an UNBIASED bf16x6 product (gemm_x6f; the fp32-MFMA
// encoder_kernel<6> was bound by its matrix time and its LDS weight copy), a2 rows stored whole.
__global__ __launch_bounds__(EBW_THREADS, 1) void node_enc_fwd_kernel(
    int N, const float* __restrict__ x_in, const float* __restrict__ w0, const float* __restrict__ b0,
    const float* __restrict__ W2, const float* __restrict__ b2, float* __restrict__ a1, float* __restrict__ a2,
    double* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
  unsigned char* img = sm;                                     // a1 (bf16x6)
  float* t_a = reinterpret_cast<float*>(sm + EBW_IMG);         // a2 row tile
  const int l = lane_id(), w = wave_id();
  const int cg = threadIdx.x & 31, rg = threadIdx.x >> 5;
  const int oc = 16 * w + 4 * (l >> 4);
  int r0, r1;
  block_rows(N, r0, r1);
  WSlice ws2;
  load_wslice(ws2, W2, w);
  f32x4 w0v[6];   // rows 4 cg .. 4 cg + 3 of W0 (128 x 6, row-major): 24 consecutive floats
#pragma unroll
  for (int k = 0; k < 6; ++k) w0v[k] = *reinterpret_cast<const f32x4*>(w0 + 24 * cg + 4 * k);
  const f32x4 b04 = *reinterpret_cast<const f32x4*>(b0 + 4 * cg);
  const f32x4 b2o = *reinterpret_cast<const f32x4*>(b2 + oc);
  double s1 = 0, s2 = 0;
  float px[2][6];
  auto issue = [&](int base) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const float* xr = x_in + (size_t)clamp_row(base + rg + 16 * u, r1) * 6;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const f32x2 v = *reinterpret_cast<const f32x2*>(xr + 2 * k);
        px[u][2 * k] = v[0];
        px[u][2 * k + 1] = v[1];
      }
    }
  };
  const __amdgpu_buffer_rsrc_t rs_a1 = rows_rsrc(a1, r0, r1);
  const __amdgpu_buffer_rsrc_t rs_a2 = rows_rsrc(a2, r0, r1);
  issue(r0);   // N > 0: an empty block (r0 = r1 = N) reads row N - 1
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int k = 0; k < 6; ++k) pin_vgpr(px[u][k]);
#pragma unroll
  for (int ks = 0; ks < 4; ++ks)
#pragma unroll
    for (int q = 0; q < 3; ++q) pin_vgpr(ws2.a[ks][q]);
  pin_vgpr(b2o);
  auto round = [&](const int base) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int r = rg + 16 * u;
      f32x4 a;
#pragma unroll
      for (int j = 0; j < 4; ++j) {   // encoder_kernel's a1: fma over the 6 inputs in order, then + b0
        float d = 0.f;   // W0 row 4 cg + j: the thread's floats 6 j .. 6 j + 5
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          const int f = 6 * j + i;   // float index within the thread's 24
          d = fmaf(w0v[f >> 2][f & 3], px[u][i], d);
        }
        a[j] = fmaxf(d + b04[j], 0.f);
      }
      const bool ok = base + r < r1;
      rows_store4_nt(rs_a1, base + r - r0, 4 * cg, a);
      img_store4(img, r, cg, ok ? a : f32x4{0.f, 0.f, 0.f, 0.f});
    }
    issue(base + X6_ROWS);
    __syncthreads();   // the a1 image is complete
    f32x4 d[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    gemm_x6f<2, X6_TERM, true>(d, ws2, img);
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      const int r = 16 * nb + (l & 15);
      f32x4 a;
#pragma unroll
      for (int j = 0; j < 4; ++j) a[j] = fmaxf(d[nb][j] + b2o[j], 0.f);
      *reinterpret_cast<f32x4*>(t_a + r * OT_STRIDE + oc) = a;
      if (base + r < r1) {
        s1 += (double)((a[0] + a[1]) + (a[2] + a[3]));
        s2 += (double)((a[0] * a[0] + a[1] * a[1]) + (a[2] * a[2] + a[3] * a[3]));
      }
    }
    __syncthreads();   // the a2 tile is complete; the image is free
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int r = rg + 16 * u;
      rows_store4_nt(rs_a2, base + r - r0, 4 * cg, *reinterpret_cast<const f32x4*>(t_a + r * OT_STRIDE + 4 * cg));
    }
  };
  round(r0);
  for (int base = r0 + X6_ROWS; base < r1; base += X6_ROWS) round(base);
  double* red = reinterpret_cast<double*>(sm);
  __syncthreads();
  block_sum2(s1, s2, red);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = s1;
    part[2 * blockIdx.x + 1] = s2;
  }
}

// ============================================================================ decoder forward
// The node decoder (models.py:316-321: x_S = LN(a2_prev) + x_prev, a1d = relu(Wd1 x_S + bd1),
// y = Wd2 a1d + bd2, unscaled when asked) in the layout of node_enc_fwd_kernel: x_S element by element as
// ln_res_frag forms it (bitwise), Wd1 x_S as an unbiased bf16x6 product from registers (decoder_kernel: fp32
// MFMAs from an LDS weight copy), a1d rows through an fp32 tile, the 3 outputs of a row as fp32 dot products
// over the tile (96 threads, features in order).  part != NULL: the last node LayerNorm's statistics reduced
// in every block from the partials (pdg_ln_finalize's order), block 0 stores them to st_out.
__global__ __launch_bounds__(EBW_THREADS, 1) void decoder_coop_kernel(
    int N, const float* __restrict__ a2p, const pdg_ln_stat* __restrict__ stp, const float* __restrict__ lg,
    const float* __restrict__ lb, const float* __restrict__ xres, float* __restrict__ xout,
    const float* __restrict__ Wd1, const float* __restrict__ bd1, float* __restrict__ a1d,
    const float* __restrict__ Wd2, const float* __restrict__ bd2, const float* __restrict__ st8, int scale,
    float* __restrict__ y, const double* __restrict__ part, int nparts, double count, pdg_ln_stat* __restrict__ st_out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
  unsigned char* img = sm;                                     // x_S (bf16x6)
  float* t_a = reinterpret_cast<float*>(sm + EBW_IMG);         // a1d row tile
  float* w2l = t_a + EFC_TILE;                                 // Wd2 (3 x 128)
  __shared__ LNStat st_sh;
  __shared__ double red_fin[2 * EBW_WAVES];
  if (part) {
    ln_stat_from_partials(part, nparts, count, &st_sh, red_fin);
    __syncthreads();
    if (blockIdx.x == 0 && threadIdx.x == 0) *st_out = st_sh;
  }
  const LNStat st = part ? st_sh : *reinterpret_cast<const LNStat*>(stp);
  const int l = lane_id(), w = wave_id();
  const int cg = threadIdx.x & 31, rg = threadIdx.x >> 5;
  const int oc = 16 * w + 4 * (l >> 4);
  int r0, r1;
  block_rows(N, r0, r1);
  for (int i = threadIdx.x; i < 3 * L; i += blockDim.x) w2l[i] = Wd2[i];
  const f32x4 gg = *reinterpret_cast<const f32x4*>(lg + 4 * cg), bb = *reinterpret_cast<const f32x4*>(lb + 4 * cg);
  const f32x4 b1o = *reinterpret_cast<const f32x4*>(bd1 + oc);
  f32x4 xa[2], xr[2];
  auto issue = [&](int base) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const size_t rc = (size_t)clamp_row(base + rg + 16 * u, r1) * L + 4 * cg;
      xa[u] = *reinterpret_cast<const f32x4*>(a2p + rc);
      xr[u] = *reinterpret_cast<const f32x4*>(xres + rc);
    }
  };
  const __amdgpu_buffer_rsrc_t rs_x = rows_rsrc(xout, r0, r1);
  const __amdgpu_buffer_rsrc_t rs_a = rows_rsrc(a1d, r0, r1);
  issue(r0);   // N > 0: an empty block reads row N - 1
  WSlice ws;   // after the first rows' loads: the round trips overlap
  load_wslice(ws, Wd1, w);
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    pin_vgpr(xa[u]);
    pin_vgpr(xr[u]);
  }
#pragma unroll
  for (int ks = 0; ks < 4; ++ks)
#pragma unroll
    for (int q = 0; q < 3; ++q) pin_vgpr(ws.a[ks][q]);
  pin_vgpr(b1o);
  const int yo = threadIdx.x % 3, yr = threadIdx.x / 3;   // threads 0 .. 95: output yo of tile row yr
  const float yb = bd2[yo];
  const float ys = scale ? st8[5] : 1.f, yt = scale ? st8[4] : 0.f;
  const __amdgpu_buffer_rsrc_t rs_y = __builtin_amdgcn_make_buffer_rsrc(y + (size_t)r0 * 3, (short)0, (r1 - r0) * 3 * 4,
                                                                        0x00020000);
  auto round = [&](const int base) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int r = rg + 16 * u;
      f32x4 x;
#pragma unroll
      for (int j = 0; j < 4; ++j) {   // ln_res_frag, element by element
        float v = div_den(xa[u][j] - st.mean, st.den, st.rstd) * gg[j] + bb[j];
        v += xr[u][j];
        x[j] = v;
      }
      const bool ok = base + r < r1;
      rows_store4_nt(rs_x, base + r - r0, 4 * cg, x);
      img_store4(img, r, cg, ok ? x : f32x4{0.f, 0.f, 0.f, 0.f});
    }
    issue(base + X6_ROWS);
    __syncthreads();   // the x_S image is complete
    f32x4 d[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    gemm_x6f<2, X6_TERM, true>(d, ws, img);
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      const int r = 16 * nb + (l & 15);
      f32x4 a;
#pragma unroll
      for (int j = 0; j < 4; ++j) a[j] = fmaxf(d[nb][j] + b1o[j], 0.f);
      *reinterpret_cast<f32x4*>(t_a + r * OT_STRIDE + oc) = a;
    }
    __syncthreads();   // the a1d tile is complete; the image is free
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int r = rg + 16 * u;
      rows_store4_nt(rs_a, base + r - r0, 4 * cg, *reinterpret_cast<const f32x4*>(t_a + r * OT_STRIDE + 4 * cg));
    }
    {   // y = Wd2 a1d + bd2 (features in order): threads 0 .. 95; the others compute a clamped row and their
        // store falls outside the buffer range (every thread stores: no memory operation is conditional)
      const float* ar = t_a + min(yr, X6_ROWS - 1) * OT_STRIDE;
      const float* wr = w2l + yo * L;
      float acc = 0.f;
#pragma unroll 2
      for (int k = 0; k < L; k += 4) {
        const f32x4 av = *reinterpret_cast<const f32x4*>(ar + k), wv = *reinterpret_cast<const f32x4*>(wr + k);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc = fmaf(wv[j], av[j], acc);
      }
      float out = acc + yb;
      if (scale) out = out * ys + yt;
      const int off = threadIdx.x < 3 * X6_ROWS ? ((base + yr - r0) * 3 + yo) * 4 : 0x7ffffff0;
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, out), rs_y, off, 0, 0);
    }
    // (the next round writes the tile after its first barrier, which every thread reaches after these reads)
  };
  for (int base = r0; base < r1; base += X6_ROWS) round(base);
}

extern "C" int pdg_decoder_fwd_coop(int n_nodes, const float* a2_prev, const pdg_ln_stat* st, const double* partials,
                                    int nparts, double count, pdg_ln_stat* st_out, const float* ln_g,
                                    const float* ln_b, const float* x_res, float* x_out, const float* Wd1,
                                    const float* bd1, float* a1d, const float* Wd2, const float* bd2,
                                    const float* stats8, int scale_output, float* y, int nblocks, void* stream) {
  PDG_CHECK_ARG(n_nodes > 0 && nblocks > 0 && nblocks <= MAX_BLOCKS, "pdg_decoder_fwd_coop: bad sizes");
  PDG_CHECK_ARG(a2_prev && x_res && x_out && a1d && Wd1 && bd1 && Wd2 && bd2 && y && ln_g && ln_b,
                "pdg_decoder_fwd_coop: null argument");
  PDG_CHECK_ARG(!scale_output || stats8 != nullptr, "pdg_decoder_fwd_coop: stats8 is NULL");
  PDG_CHECK_ARG(PDG_ALIGNED(a2_prev) && PDG_ALIGNED(x_res) && PDG_ALIGNED(x_out) && PDG_ALIGNED(a1d) &&
                    PDG_ALIGNED(Wd1) && PDG_ALIGNED(bd1) && PDG_ALIGNED(ln_g) && PDG_ALIGNED(ln_b),
                "pdg_decoder_fwd_coop: misaligned pointer");
  PDG_CHECK_ARG(partials ? (nparts > 0 && count > 0 && st_out != nullptr) : st != nullptr,
                "pdg_decoder_fwd_coop: statistics arguments");
  const size_t shm = EBW_IMG + (size_t)(EFC_TILE + 3 * L) * sizeof(float);
  hipLaunchKernelGGL(decoder_coop_kernel, dim3(nblocks), dim3(EBW_THREADS), shm, (hipStream_t)stream, n_nodes,
                     a2_prev, st, ln_g, ln_b, x_res, x_out, Wd1, bd1, a1d, Wd2, bd2, stats8, scale_output, y,
                     partials, nparts, count, st_out);
  PDG_CHECK_LAUNCH("pdg_decoder_fwd_coop");
  return PDG_OK;
}




// the P / Q layout this library was built for (pdg_common.hpp PDG_PQ_BLOCKED): 0 = two N x 128 arrays,
// 1 = one N x 256 array of interleaved 16-feature blocks (Q = P + 16 floats)
extern "C" int pdg_pq_layout(void) { return PDG_PQ_BLOCKED; }

extern "C" int pdg_edge_fwd_coop(int n_edges, const float* a2_prev, const pdg_ln_stat* st, const float* ln_g,
                                 const float* ln_b, const float* e_res, float* e_out, const int* src, const int* dst,
                                 const float* P, const float* Q, const float* W1, const float* b1, const float* W2,
                                 const float* b2, float* a1m, float* a2m, float* a1e, float* a2e, double* part_m,
                                 double* part_e, int with_edge_update, int nblocks, void* stream) {
  PDG_CHECK_ARG(n_edges > 0, "pdg_edge_fwd_coop: n_edges must be > 0");
  PDG_CHECK_ARG(nblocks > 0 && nblocks <= MAX_BLOCKS, "pdg_edge_fwd_coop: bad nblocks");
  PDG_CHECK_ARG(PDG_ALIGNED(a2_prev) && PDG_ALIGNED(e_out) && PDG_ALIGNED(P) && PDG_ALIGNED(Q) &&
                    PDG_ALIGNED(a1m) && PDG_ALIGNED(a2m) && PDG_ALIGNED(W1) && PDG_ALIGNED(W2) &&
                    PDG_ALIGNED(b1) && PDG_ALIGNED(b2) && PDG_ALIGNED(ln_g) && PDG_ALIGNED(ln_b) &&
                    (!e_res || PDG_ALIGNED(e_res)),
                "pdg_edge_fwd_coop: misaligned pointer");
  PDG_CHECK_ARG(!with_edge_update || (a2e && part_e && PDG_ALIGNED(a1e) && PDG_ALIGNED(a2e)),
                "pdg_edge_fwd_coop: edge-update outputs missing or misaligned");
  // every required input and output refused when null (a null output would be dropped by its buffer
  // resource, silently leaving the caller's array unwritten): e_res (first step) and a1m / a1e (inference)
  // are the optional ones
  PDG_CHECK_ARG(a2_prev && st && ln_g && ln_b && e_out && src && dst && P && Q && W1 && b1 && W2 && b2 && a2m &&
                    part_m,
                "pdg_edge_fwd_coop: null argument");
  // the XCD-interleaved rounds are compiled for the 256-block grid; any other grid (tests, other parts)
  // walks contiguous block ranges
  const bool xcd = nblocks == XCD_GRID;
  const size_t shm = 2 * EBW_IMG + 2 * EFC_TILE * sizeof(float) + EBW_IMG + 2 * EFC_TILE * sizeof(float) +
                     2 * EBW_WAVES * 64 * 16;
  hipStream_t s = (hipStream_t)stream;
#define PDG_EFC_X(R, U, X)                                                                                    \
  hipLaunchKernelGGL((edge_fwd_coop_kernel<R, U, X>), dim3(nblocks), dim3(EBW_THREADS), shm, s,               \
                     n_edges, a2_prev, st, ln_g, ln_b, e_res, e_out, src, dst, P, Q, W1, b1, W2, b2, a1m, a2m, a1e,   \
                     a2e, part_m, part_e)
#define PDG_EFC(R, U)            \
  do {                           \
    if (xcd) {                   \
      PDG_EFC_X(R, U, true);     \
    } else {                     \
      PDG_EFC_X(R, U, false);    \
    }                            \
  } while (0)
  if (e_res) {
    if (with_edge_update) PDG_EFC(true, true); else PDG_EFC(true, false);
  } else {
    if (with_edge_update) PDG_EFC(false, true); else PDG_EFC(false, false);
  }
#undef PDG_EFC
#undef PDG_EFC_X
  PDG_CHECK_LAUNCH("pdg_edge_fwd_coop");
  return PDG_OK;
}

extern "C" int pdg_edge_fwd_infer(int n_edges, const float* a2_prev, const pdg_ln_stat* st, const float* ln_g,
                                  const float* ln_b, const float* e_res, float* e_out, const int* src, const int* dst,
                                  const float* P, const float* Q, const float* W1, const float* b1, const float* W2,
                                  const float* b2, float* a2m, float* a2e, double* part_m, double* part_e,
                                  int with_edge_update, int nblocks, void* stream) {
  PDG_CHECK_ARG(n_edges > 0, "pdg_edge_fwd_infer: n_edges must be > 0");
  PDG_CHECK_ARG(nblocks > 0 && nblocks <= MAX_BLOCKS, "pdg_edge_fwd_infer: bad nblocks");
  PDG_CHECK_ARG(a2_prev && st && ln_g && ln_b && e_out && src && dst && P && Q && W1 && b1 && W2 && b2 && a2m &&
                    part_m,
                "pdg_edge_fwd_infer: null argument");
  PDG_CHECK_ARG(PDG_ALIGNED(a2_prev) && PDG_ALIGNED(e_out) && PDG_ALIGNED(P) && PDG_ALIGNED(Q) &&
                    PDG_ALIGNED(a2m) && PDG_ALIGNED(W1) && PDG_ALIGNED(W2) && PDG_ALIGNED(b1) && PDG_ALIGNED(b2) &&
                    PDG_ALIGNED(ln_g) && PDG_ALIGNED(ln_b) && (!e_res || PDG_ALIGNED(e_res)),
                "pdg_edge_fwd_infer: misaligned pointer");
  PDG_CHECK_ARG(!with_edge_update || (a2e && part_e && PDG_ALIGNED(a2e)),
                "pdg_edge_fwd_infer: edge-update outputs missing or misaligned");
  const bool xcd = nblocks == XCD_GRID;
  const size_t shm = 6 * IMG16 + 4 * EP_TILE * sizeof(float) + 2 * EBW_WAVES * 64 * 16;
  hipStream_t s = (hipStream_t)stream;
#define PDG_EI_X(R, U, X)                                                                                     \
  hipLaunchKernelGGL((edge_fwd_infer_kernel<R, U, X>), dim3(nblocks), dim3(EBW_THREADS), shm, s, n_edges, a2_prev, \
                     st, ln_g, ln_b, e_res, e_out, src, dst, P, Q, W1, b1, W2, b2, a2m, a2e, part_m, part_e)
#define PDG_EI(R, U)             \
  do {                           \
    if (xcd) {                   \
      PDG_EI_X(R, U, true);      \
    } else {                     \
      PDG_EI_X(R, U, false);     \
    }                            \
  } while (0)
  if (e_res) {
    if (with_edge_update) PDG_EI(true, true); else PDG_EI(true, false);
  } else {
    if (with_edge_update) PDG_EI(false, true); else PDG_EI(false, false);
  }
#undef PDG_EI
#undef PDG_EI_X
  PDG_CHECK_LAUNCH("pdg_edge_fwd_infer");
  return PDG_OK;
}

extern "C" int pdg_node_enc_fwd(int n_nodes, const float* x_in, const float* w0, const float* b0, const float* W2,
                                const float* b2, float* a1, float* a2, double* partials, int nblocks, void* stream) {
  PDG_CHECK_ARG(n_nodes > 0 && nblocks > 0 && nblocks <= MAX_BLOCKS, "pdg_node_enc_fwd: bad sizes");
  PDG_CHECK_ARG(x_in && w0 && b0 && W2 && b2 && a2 && partials, "pdg_node_enc_fwd: null argument");
  PDG_CHECK_ARG(((uintptr_t)x_in & 7) == 0 && PDG_ALIGNED(w0) && PDG_ALIGNED(b0) && PDG_ALIGNED(W2) &&
                    PDG_ALIGNED(b2) && PDG_ALIGNED(a2) && (!a1 || PDG_ALIGNED(a1)),
                "pdg_node_enc_fwd: misaligned pointer");
  const size_t shm = EBW_IMG + (size_t)EFC_TILE * sizeof(float);
  hipLaunchKernelGGL(node_enc_fwd_kernel, dim3(nblocks), dim3(EBW_THREADS), shm, (hipStream_t)stream, n_nodes, x_in,
                     w0, b0, W2, b2, a1, a2, partials);
  PDG_CHECK_LAUNCH("pdg_node_enc_fwd");
  return PDG_OK;
}

extern "C" int pdg_edge_enc_fwd(int n_edges, const float* e_in, const float* w0, const float* b0, const float* W2,
                                const float* b2, float* a2, double* partials, int nblocks, void* stream) {
  PDG_CHECK_ARG(n_edges > 0 && nblocks > 0 && nblocks <= MAX_BLOCKS, "pdg_edge_enc_fwd: bad sizes");
  PDG_CHECK_ARG(e_in && w0 && b0 && W2 && b2 && a2 && partials, "pdg_edge_enc_fwd: null argument");
  PDG_CHECK_ARG(PDG_ALIGNED(w0) && PDG_ALIGNED(b0) && PDG_ALIGNED(W2) && PDG_ALIGNED(b2) && PDG_ALIGNED(a2),
                "pdg_edge_enc_fwd: misaligned pointer");
  const size_t shm = EBW_IMG + (size_t)EFC_TILE * sizeof(float);
  hipLaunchKernelGGL(edge_enc_fwd_kernel, dim3(nblocks), dim3(EBW_THREADS), shm, (hipStream_t)stream, n_edges, e_in,
                     w0, b0, W2, b2, a2, partials);
  PDG_CHECK_LAUNCH("pdg_edge_enc_fwd");
  return PDG_OK;
}

