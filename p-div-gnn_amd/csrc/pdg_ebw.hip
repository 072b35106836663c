// Edge backward with the shared-weight gradients fused in (models.py:194-208 edge_net,
// backward of one message-passing step; SURVEY §8 rows a5/a6 and the weight gradients).
//
// The plain edge backward (pdg_edge_bwd, pdg_bwd.hip) keeps W2^T and Wc^T in LDS, so
// the weight gradients dW2 = sum gz2^T a1 and dWc = sum gC^T e need a second pass
// (pdg_wgrad_segments) that re-reads gz2 / a1 / gC / e from HBM.  Here the weights
// are STATIONARY IN REGISTERS (wave w of 8 owns output features [16w, 16w + 16) of
// the product, 48 VGPRs of bf16 terms) and LDS holds the 32-row images of the
// operands instead: the same images feed the activation GEMM (straight 16-B reads)
// and the weight-gradient MFMAs (transposed reads), so the gradients cost no HBM
// traffic and gz2m / gz2e are never written.  Two kernels, one per weight:
//
//   pdg_edge_bwd_w2:  gz2 = LN_bwd(gy) [a2 > 0] for the message (gy = gaggr[dst]) and the
//                     edge update (gy = ge_next); gz1 = (W2^T gz2) [a1 > 0]; gC = gz1m + gz1e;
//                     slab += gz2m^T a1m + gz2e^T a1e (and the b2 sums).
//   pdg_edge_gout_wc: ge_out = ge_next + Wc^T gC; slab += gC^T e (and the b1 sums).
//
// All products are bf16x6 (fp32-accurate).  Rows are split into one contiguous range per
// block (one block of 8 waves per CU); a block's 128x128 (+128) fp32 slab is
// read-modified-written once at the end, so slabs accumulate over the steps of a
// backward pass and are reduced once by pdg_wgrad_reduce (deterministic).
//
// Per round: stage (loads -> LN backward / split -> images) | loads of a later round issued |
// barrier | weight-gradient MFMAs | activation MFMAs | stores.  Every load of a round is issued
// before the previous round's stores (vmcnt counts loads and stores together, in issue order).
#include "pdg_coop.hpp"

using namespace pdg;


// ============================================================================ W2 path
// 16-row rounds with TWO rounds of row loads in flight, in the registers one 32-row round used to
// take (two sets of one row per thread): set s is consumed by the stage of round n and re-issued for
// round n + 2 at once, so a CU always has rows landing while it computes.  (The round-2 kernel staged
// 32-row rounds and issued the next round's loads after the stage's barrier, with no loads in flight
// between their arrival and the next issue: 219-221 -> 190-196 us per config-2 call, 1,039 MB of DRAM
// traffic at 5.4 instead of 4.7 TB/s, same box.)  The images and masks are double-buffered by round
// parity, which leaves one barrier per round.  No memory operation is conditional (rows past the
// block's end are clamped on load and range-dropped on store): a load or store skipped on some path
// made the compiler's loop-carried count collapse to vmcnt(0) in the stage, a wait for both sets.
// gz1m / gz1e / gC are bitwise those of the 32-row kernel; dW2 sums the same products in another
// order (message and edge-update rows of a round interleave per 16 rows instead of per 32).
// (A form recomputing a1m / a1e from the forward's C = Wc e + b1 and the step's gathered P / Q rows,
// one E-row array read and written fewer, measured slower and was removed: DESIGN §4 round 3.)
template <bool EU>
__global__ __launch_bounds__(EBW_THREADS, 1) void edge_bwd_w2_kernel(
    const int* __restrict__ dst, const float* __restrict__ gaggr, const float* __restrict__ ge_next,
    const float* __restrict__ a2m, const float* __restrict__ a1m, const float* __restrict__ a2e,
    const float* __restrict__ a1e, const pdg_ln_stat* __restrict__ stm_p, const pdg_ln_stat* __restrict__ ste_p,
    const pdg_ln_bwd* __restrict__ lbm_p, const pdg_ln_bwd* __restrict__ lbe_p, const float* __restrict__ lg,
    const float* __restrict__ W2T, float* __restrict__ gz1m, float* __restrict__ gz1e, float* __restrict__ gC,
    float* __restrict__ slabs, int E, const double* __restrict__ pm, int npm, const double* __restrict__ pe,
    int npe, int slab_init) {
  extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
  constexpr int NIMG = EU ? 4 : 2, NMSK = EU ? 2 : 1;
  constexpr int BUF = NIMG * IMG16 + NMSK * MSK16;           // one round's images + masks
  const int l = lane_id(), w = wave_id();
  const int cg = threadIdx.x & 31, rg = threadIdx.x >> 5;    // the thread's staged row: rg (0..15)
  const int oc = 16 * w + 4 * (l >> 4);
  int r0, r1, first, stride;   // 32-row units: rounds base and base + 16, the next unit stride rows on
  row_schedule(0, E, r0, r1, first, stride);
  WSlice ws;
  const f32x4 g4 = *reinterpret_cast<const f32x4*>(lg + 4 * cg);
  const LNStat stm = *reinterpret_cast<const LNStat*>(stm_p);
  const LNStat ste = *reinterpret_cast<const LNStat*>(EU ? ste_p : stm_p);
  f32x16 acc[2];
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[b][r] = 0.f;
  f32x4 bsum = f32x4{0.f, 0.f, 0.f, 0.f};
  // two register sets of prefetched rows (round parity), and the dst id each set gathers next
  f32x4 pg[2], pa2[2], pa1[2], pge[2], pa2e[2], pa1e[2];
  int dn[2];
  auto issue = [&](int s, int base) {
    const size_t rc = (size_t)clamp_row(base + rg, r1) * L + 4 * cg;
    pg[s] = *reinterpret_cast<const f32x4*>(gaggr + (size_t)dn[s] * L + 4 * cg);
    pa2[s] = *reinterpret_cast<const f32x4*>(a2m + rc);
    pa1[s] = *reinterpret_cast<const f32x4*>(a1m + rc);
    if (EU) {
      pge[s] = *reinterpret_cast<const f32x4*>(ge_next + rc);
      pa2e[s] = *reinterpret_cast<const f32x4*>(a2e + rc);
      pa1e[s] = *reinterpret_cast<const f32x4*>(a1e + rc);
    }
  };
  // no memory operation below is conditional (rows past the block's end are clamped on load and
  // dropped by the buffer range check on store), so the compiler can count the loads in flight: a
  // skipped store or load on some path made it wait for all of them (vmcnt(0)) in the stage
  // without the edge update gC = gz1m: a caller passing gC == gz1m gets it written once (an empty range
  // drops the second store)
  const __amdgpu_buffer_rsrc_t out_m = rows_rsrc(gz1m, r0, r1);
  const __amdgpu_buffer_rsrc_t out_c = rows_rsrc(EU || gC != gz1m ? gC : nullptr, r0, r1);
  // gz1e == nullptr (the edge update without a gz1e array): its stores dropped the same way
  const __amdgpu_buffer_rsrc_t out_e = rows_rsrc(EU ? gz1e : gz1m, r0, r1);
  dn[0] = dst[clamp_row(first + rg, r1)];   // E > 0: an empty block (first = r1 = E) reads row E - 1
  dn[1] = dst[clamp_row(first + R16 + rg, r1)];
  // each set's loads strictly before the next set's (sched_barrier), in the order the loop re-issues
  // them: the loop waits for one set by count, and an interleaved prologue lowers that count
  issue(0, first);
  dn[0] = dst[clamp_row(first + stride + rg, r1)];
  __builtin_amdgcn_sched_barrier(0);
  issue(1, first + R16);
  dn[1] = dst[clamp_row(first + stride + R16 + rg, r1)];
  __builtin_amdgcn_sched_barrier(0);
  // the weights and the LayerNorm scalars after the first rounds' row loads: the round trips overlap
  load_wslice(ws, W2T, w);
  const pdg_ln_bwd lbm = lnb_resolve(lbm_p, pm, npm, stm_p);
  const pdg_ln_bwd lbe = EU ? lnb_resolve(lbe_p, pe, npe, ste_p) : lbm;
  auto stage = [&](const int s, const int base) {
    unsigned char* img_gm = sm + s * BUF;                      // gz2m
    unsigned char* img_am = img_gm + IMG16;                    // a1m
    unsigned char* img_ge = img_gm + 2 * IMG16;                // gz2e (EU)
    unsigned char* img_ae = img_gm + 3 * IMG16;                // a1e (EU)
    unsigned char* msk_m = img_gm + NIMG * IMG16;              // [a1m > 0]
    unsigned char* msk_e = msk_m + MSK16;                      // [a1e > 0] (EU)
    // ---- gz2 (LN + relu backward), a1 and its relu mask into this round's images
    {
      const bool ok = base + rg < r1;
      const f32x4 a1mv = pa1[s], a1ev = pa1e[s];
      // a row past r1 has gz2 = 0, which zeroes its products whatever its (finite, clamped-row) a1:
      // no select on a1.  (gz2 computed for every row and selected, branch-free as in pdg_edge_enc_bwd:
      // 256 -> 226 VGPRs but 3-4 us slower per call, gpurun_out/r04s)
      const f32x4 zero = f32x4{0.f, 0.f, 0.f, 0.f};
      const f32x4 zm = ok ? ln_relu_bwd4(pg[s], pa2[s], stm, lbm, g4) : zero;
      const f32x4 am = a1mv;
      bsum += zm;
      img_store4<T16>(img_gm, rg, cg, zm);
      img_store4<T16>(img_am, rg, cg, am);
      *reinterpret_cast<unsigned*>(msk_m + rg * MSK_STRIDE + 4 * cg) = relu_mask4(am);
      if (EU) {
        const f32x4 ze = ok ? ln_relu_bwd4(pge[s], pa2e[s], ste, lbe, g4) : zero;
        const f32x4 ae = a1ev;
        bsum += ze;
        img_store4<T16>(img_ge, rg, cg, ze);
        img_store4<T16>(img_ae, rg, cg, ae);
        *reinterpret_cast<unsigned*>(msk_e + rg * MSK_STRIDE + 4 * cg) = relu_mask4(ae);
      }
    }
    // ---- the set is free: its rows of the round after next (the same half of the next unit), then
    // the dst ids of the one after that
    issue(s, base + stride);
    dn[s] = dst[clamp_row(base + 2 * stride + rg, r1)];
  };
  auto compute = [&](const int s, const int base) {
    const unsigned char* img_gm = sm + s * BUF;
    const unsigned char* img_am = img_gm + IMG16;
    const unsigned char* img_ge = img_gm + 2 * IMG16;
    const unsigned char* img_ae = img_gm + 3 * IMG16;
    const unsigned char* msk_m = img_gm + NIMG * IMG16;
    const unsigned char* msk_e = msk_m + MSK16;
    // ---- dW2 += gz2m^T a1m (+ gz2e^T a1e)
    wgrad_round<1, T16>(acc, img_gm, img_am);
    if (EU) wgrad_round<1, T16>(acc, img_ge, img_ae);
    // ---- gz1 = (W2^T gz2) [a1 > 0], gC = gz1m + gz1e
    constexpr int NI = EU ? 2 : 1;
    f32x4 d[NI][1];
    const unsigned char* imgs[NI];
    imgs[0] = img_gm;
    if (EU) imgs[NI - 1] = img_ge;
    gemm_round<NI, 1, T16>(d, ws, imgs);
    const int r = l & 15;
    const int row = base + r;
    const unsigned mm = *reinterpret_cast<const unsigned*>(msk_m + r * MSK_STRIDE + oc);
    f32x4 zm;
#pragma unroll
    for (int j = 0; j < 4; ++j) zm[j] = (mm >> (8 * j)) & 1u ? d[0][0][j] : 0.f;
    f32x4 c = zm;
    if (EU) {
      const unsigned me = *reinterpret_cast<const unsigned*>(msk_e + r * MSK_STRIDE + oc);
      f32x4 ze;
#pragma unroll
      for (int j = 0; j < 4; ++j) ze[j] = (me >> (8 * j)) & 1u ? d[NI - 1][0][j] : 0.f;
      c = zm + ze;
      rows_store4(out_e, row - r0, oc, ze);
    }
    rows_store4(out_m, row - r0, oc, zm);
    rows_store4(out_c, row - r0, oc, c);
  };
  // both rounds of a 32-row step always run: a round past r1 stages zero rows (adding exact zeros to
  // the weight gradient) and stores nothing
  // (the software-pipelined form of pdg_edge_enc_bwd, products of round k beside the stage of round k + 1,
  // did not interleave here: the compiler kept the 72 products of a round together even with scheduling
  // groups)
  for (int base = first; base < r1; base += stride) {
    stage(0, base);
    __syncthreads();   // this round's images complete (the other buffer is the previous round's)
    compute(0, base);
    stage(1, base + R16);
    __syncthreads();
    compute(1, base + R16);
  }
  __syncthreads();   // the last rounds' image reads precede the LDS reuse below
  slab_accumulate(slabs + (size_t)blockIdx.x * WSLAB, acc, bsum, reinterpret_cast<float*>(sm), slab_init);
}

// ============================================================================ Wc path
// ge_out = [ge_next +] Wc^T gC, dWc += gC^T e (+ b1 sums) and the column sums of the LayerNorm that
// produced e, in pdg_edge_bwd_w2's layout: 16-row rounds, two rounds of row loads in flight
// (register sets by round parity, each re-issued for the round after next as soon as its stage has
// consumed it), double-buffered images, ONE barrier per round.  The products of round k go to an fp32 row
// tile (parity k & 1) and its whole-row epilogue (ge_out = ge_next + Wc^T gC, the LayerNorm column sums)
// runs after the NEXT round's barrier, so no second barrier waits for the tile.  The round's residual and
// xhat rows are held from its stage to that epilogue.  Bitwise the outputs of the round-5 form (32-row
// rounds, the next round's loads issued after the first of two barriers; removed): the same product chain
// per element, dWc / b1 sums and the fp32 / fp64 column-sum steps in the same order (a 32-row unit's two
// epilogues add into one fp32 sum before it is folded into the fp64 one); 125.7 -> 122.0 us per config-2
// call (same box, EXPERIMENTS §5).
constexpr int GO_TILE = R16 * OT_STRIDE;   // floats per 16-row output tile
template <bool RES, bool LN>
__global__ __launch_bounds__(EBW_THREADS, 1) void edge_gout_wc_kernel(
    const float* __restrict__ gC, const float* __restrict__ e, const float* __restrict__ ge_next,
    const float* __restrict__ WcT, float* __restrict__ ge_out, float* __restrict__ slabs,
    const float* __restrict__ a2ln, const pdg_ln_stat* __restrict__ stln_p, double* __restrict__ part, int E,
    const float* __restrict__ ln_g, double* __restrict__ pairs, int accumulate, int slab_init) {
  extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
  unsigned char* img = sm;                                           // [parity][gC, e] 16-row images
  float* tile = reinterpret_cast<float*>(sm + 4 * IMG16);            // [parity] Wc^T gC rows
  LNStat stln;
  if (LN) stln = *reinterpret_cast<const LNStat*>(stln_p);
  const int l = lane_id(), w = wave_id();
  const int cg = threadIdx.x & 31, rg = threadIdx.x >> 5;
  const int oc = 16 * w + 4 * (l >> 4);
  int r0, r1, first, stride;
  row_schedule(0, E, r0, r1, first, stride);
  WSlice ws;
  f32x16 acc[2];
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[b][r] = 0.f;
  f32x4 bsum = f32x4{0.f, 0.f, 0.f, 0.f};
  const f32x4 zero = f32x4{0.f, 0.f, 0.f, 0.f};
  double cs_g[4] = {0, 0, 0, 0}, cs_x[4] = {0, 0, 0, 0};
  f32x4 sg = zero, sx = zero;   // the current 32-row unit's column sums (fp32, as edge_gout_wc_kernel's)
  const __amdgpu_buffer_rsrc_t rs_out = rows_rsrc(ge_out, r0, r1);
  f32x4 pc[2], pe[2], pres[2], pa2[2];   // rows in flight, by round parity
  f32x4 hres[2], hx[2];                  // a staged round's residual and xhat, held to its epilogue
  auto issue = [&](int s, int base) {
    const size_t rc = (size_t)clamp_row(base + rg, r1) * L + 4 * cg;
    pc[s] = *reinterpret_cast<const f32x4*>(gC + rc);
    pe[s] = *reinterpret_cast<const f32x4*>(e + rc);
    if (RES) pres[s] = *reinterpret_cast<const f32x4*>(ge_next + rc);
    if (LN) pa2[s] = *reinterpret_cast<const f32x4*>(a2ln + rc);
  };
  auto stage = [&](const int s, const int base) {
    const bool ok = base + rg < r1;
    const f32x4 c = ok ? pc[s] : zero;
    bsum += c;
    img_store4<T16>(img + (2 * s) * IMG16, rg, cg, c);
    img_store4<T16>(img + (2 * s + 1) * IMG16, rg, cg, ok ? pe[s] : zero);
    hres[s] = RES ? pres[s] : zero;
    if (LN) {
#pragma unroll
      for (int j = 0; j < 4; ++j) hx[s][j] = div_den(pa2[s][j] - stln.mean, stln.den, stln.rstd);
    }
    issue(s, base + stride);
  };
  auto compute = [&](const int s) {
    wgrad_round<1, T16>(acc, img + (2 * s) * IMG16, img + (2 * s + 1) * IMG16);
    f32x4 d[1][1];
    const unsigned char* imgs[1] = {img + (2 * s) * IMG16};
    gemm_round<1, 1, T16>(d, ws, imgs);
    *reinterpret_cast<f32x4*>(tile + s * GO_TILE + (l & 15) * OT_STRIDE + oc) = d[0][0];
  };
  auto epilogue = [&](const int s, const int base) {   // round `base` (parity s), staged and computed before
    const int row = base + rg;
    const f32x4 dv = *reinterpret_cast<const f32x4*>(tile + s * GO_TILE + rg * OT_STRIDE + 4 * cg);
    const f32x4 go = RES ? hres[s] + dv : dv;
    rows_store4(rs_out, row - r0, 4 * cg, go);   // rows outside [r0, r1) dropped by the range
    if (LN && row >= r0 && row < r1) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        sg[j] += go[j];
        sx[j] += go[j] * hx[s][j];
      }
    }
  };
  auto fold = [&]() {   // a unit's two epilogues done
    if (LN) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        cs_g[j] += (double)sg[j];
        cs_x[j] += (double)sx[j];
      }
      sg = zero;
      sx = zero;
    }
  };
  // each set's loads strictly before the next set's, in the loop's re-issue order
  issue(0, first);
  __builtin_amdgcn_sched_barrier(0);
  issue(1, first + R16);
  __builtin_amdgcn_sched_barrier(0);
  load_wslice(ws, WcT, w);   // after the first rounds' row loads: the round trips overlap
  int last = first - stride;   // the last unit's base (none: its rows lie below r0, every store dropped)
  for (int base = first; base < r1; base += stride) {
    stage(0, base);
    __syncthreads();   // round base's images; the previous unit's second tile
    compute(0);
    epilogue(1, base - stride + R16);
    fold();
    stage(1, base + R16);
    __syncthreads();
    compute(1);
    epilogue(0, base);
    last = base;
  }
  __syncthreads();   // the last round's tile
  epilogue(1, last + R16);
  fold();
  __syncthreads();   // the last tile reads precede the LDS reuse below
  slab_accumulate(slabs + (size_t)blockIdx.x * WSLAB, acc, bsum, reinterpret_cast<float*>(sm), slab_init);
  if (LN) {
    // block partial = the 16 row groups' column sums, reduced in order through LDS (after slab_accumulate's 8 KB)
    double* red = reinterpret_cast<double*>(sm + 16384);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      red[rg * 2 * L + 4 * cg + j] = cs_g[j];
      red[rg * 2 * L + L + 4 * cg + j] = cs_x[j];
    }
    __syncthreads();
    double* row = red + EBW_THREADS / 32 * 2 * L;
    for (int i = threadIdx.x; i < 2 * L; i += blockDim.x) {
      double v = 0;
      for (int g = 0; g < EBW_THREADS / 32; ++g) v += red[g * 2 * L + i];
      row[i] = v;
    }
    __syncthreads();
    lnb_emit(row, ln_g, part, accumulate, pairs, row + 2 * L);
  }
}

// ============================================================================ edge encoder narrow reduction
// grad_w0 += sum over blocks of the dw0 sums, grad_b0 += the db0 sums.  Block c (of 2) owns columns
// 128 c .. 128 c + 127; its 4 thread groups sum every 4th slab row with 4 loads in flight each, then
// the 4 partial sums are added in group order (deterministic).
__global__ __launch_bounds__(512) void enc_narrow_reduce_kernel(const double* __restrict__ nsums, int nb,
                                                                float* __restrict__ gw0, float* __restrict__ gb0) {
  __shared__ double part[4][L];
  const int col = threadIdx.x & (L - 1), grp = threadIdx.x >> 7, e = L * blockIdx.x + col;
  double s0 = 0, s1 = 0, s2 = 0, s3 = 0;
  int b = grp;
  for (; b + 12 < nb; b += 16) {
    s0 += nsums[(size_t)b * 2 * L + e];
    s1 += nsums[(size_t)(b + 4) * 2 * L + e];
    s2 += nsums[(size_t)(b + 8) * 2 * L + e];
    s3 += nsums[(size_t)(b + 12) * 2 * L + e];
  }
  for (; b < nb; b += 4) s0 += nsums[(size_t)b * 2 * L + e];
  part[grp][col] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (grp == 0) {
    const double t = ((part[0][col] + part[1][col]) + part[2][col]) + part[3][col];
    if (blockIdx.x == 0) gw0[col] += (float)t;
    else gb0[col] += (float)t;
  }
}

// ============================================================================ node input gradient
// pdg_gemm_sum2_rw in the cooperative layout: out = W0T in0 + W1T in1 + res (the input gradient of
// x_t through P = Wa x, Q = Wb x plus the node_net path: in0 = gP, in1 = gQ, W0T = Wa^T, W1T = Wb^T)
// with both weights stationary in registers as bf16 terms and the two products in bf16x6 (the
// edge backward's W^T products), 32-row rounds, whole-row HBM access; COLS: the column partials of
// the backward of the LayerNorm LN(ln_a2) whose upstream gradient is `out` (as gemm_sum2_rw).  The
// fp32-MFMA kernel was bound by its matrix time (about half the fp32 MFMA rate at 12 waves / 168
// VGPRs); this one does 2.7x less matrix work.
template <int NB = 2, int TERM = X6_TERM>
__device__ __forceinline__ void gemm_sum2_round(f32x4 (&d)[NB], const WSlice& ws0, const unsigned char* img0,
                                                const WSlice& ws1, const unsigned char* img1) {
  const int l = lane_id(), n = l & 15, kg = l >> 4;
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) d[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 4; ++ks)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const int off = x6_addr(16 * nb + n, 64 * ks + 16 * kg);
      bf16x8 B[3], C[3];
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        B[p] = *reinterpret_cast<const bf16x8*>(img0 + p * TERM + off);
        C[p] = *reinterpret_cast<const bf16x8*>(img1 + p * TERM + off);
      }
      f32x4 t = d[nb];
      t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ws0.a[ks][2], B[0], t, 0, 0, 0);
      t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ws0.a[ks][1], B[1], t, 0, 0, 0);
      t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ws0.a[ks][0], B[2], t, 0, 0, 0);
      t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ws1.a[ks][2], C[0], t, 0, 0, 0);
      t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ws1.a[ks][1], C[1], t, 0, 0, 0);
      t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ws1.a[ks][0], C[2], t, 0, 0, 0);
      t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ws0.a[ks][1], B[0], t, 0, 0, 0);
      t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ws0.a[ks][0], B[1], t, 0, 0, 0);
      t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ws1.a[ks][1], C[0], t, 0, 0, 0);
      t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ws1.a[ks][0], C[1], t, 0, 0, 0);
      t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ws0.a[ks][0], B[0], t, 0, 0, 0);
      d[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ws1.a[ks][0], C[0], t, 0, 0, 0);
    }
}

// In 16-row rounds with two rounds of row loads in flight and one barrier per round, each round's output rows
// stored from an fp32 tile after the next round's barrier (pdg_edge_gout_wc's structure, round 6): bitwise the
// outputs, column partials and pairs of the 32-row two-barrier form it replaced (the same fp32 / fp64 summation
// steps per 32-row unit), 31.0 -> 30.0 us per config-2 call (EXPERIMENTS §5).
template <bool COLS, bool RES>
__global__ __launch_bounds__(EBW_THREADS, 1) void gemm_sum2_coop_kernel(
    int N, const float* __restrict__ in0, const float* __restrict__ in1, const float* __restrict__ W0T,
    const float* __restrict__ W1T, const float* __restrict__ res, float* __restrict__ out,
    const float* __restrict__ ln_a2, const pdg_ln_stat* __restrict__ ln_st, double* __restrict__ part,
    const float* __restrict__ ln_g, double* __restrict__ pairs, int accumulate) {
  extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
  unsigned char* img = sm;                                        // [parity][in0, in1] 16-row images
  float* tile = reinterpret_cast<float*>(sm + 4 * IMG16);         // [parity] output rows
  constexpr int TL = R16 * OT_STRIDE;
  LNStat stln;
  if (COLS) stln = *reinterpret_cast<const LNStat*>(ln_st);
  const int l = lane_id(), w = wave_id();
  const int cg = threadIdx.x & 31, rg = threadIdx.x >> 5;
  const int oc = 16 * w + 4 * (l >> 4);
  int r0, r1;
  block_rows(N, r0, r1);
  WSlice ws0, ws1;
  const f32x4 zero = f32x4{0.f, 0.f, 0.f, 0.f};
  double cs_g[4] = {0, 0, 0, 0}, cs_x[4] = {0, 0, 0, 0};
  f32x4 sg = zero, sx = zero;
  const __amdgpu_buffer_rsrc_t rs_out = rows_rsrc(out, r0, r1);
  f32x4 p0[2], p1[2], pres[2], pa2[2], hres[2], hx[2];
  auto issue = [&](int s, int base) {
    const size_t rc = (size_t)clamp_row(base + rg, r1) * L + 4 * cg;
    p0[s] = *reinterpret_cast<const f32x4*>(in0 + rc);
    p1[s] = *reinterpret_cast<const f32x4*>(in1 + rc);
    if (RES) pres[s] = *reinterpret_cast<const f32x4*>(res + rc);
    if (COLS) pa2[s] = *reinterpret_cast<const f32x4*>(ln_a2 + rc);
  };
  auto stage = [&](const int s, const int base) {
    const bool ok = base + rg < r1;
    img_store4<T16>(img + (2 * s) * IMG16, rg, cg, ok ? p0[s] : zero);
    img_store4<T16>(img + (2 * s + 1) * IMG16, rg, cg, ok ? p1[s] : zero);
    hres[s] = RES ? pres[s] : zero;
    if (COLS) {
#pragma unroll
      for (int j = 0; j < 4; ++j) hx[s][j] = div_den(pa2[s][j] - stln.mean, stln.den, stln.rstd);
    }
    issue(s, base + X6_ROWS);
  };
  auto compute = [&](const int s) {
    f32x4 d[1];
    gemm_sum2_round<1, T16>(d, ws0, img + (2 * s) * IMG16, ws1, img + (2 * s + 1) * IMG16);
    *reinterpret_cast<f32x4*>(tile + s * TL + (l & 15) * OT_STRIDE + oc) = d[0];
  };
  auto epilogue = [&](const int s, const int base) {
    const int row = base + rg;
    const f32x4 o = *reinterpret_cast<const f32x4*>(tile + s * TL + rg * OT_STRIDE + 4 * cg) + hres[s];
    rows_store4(rs_out, row - r0, 4 * cg, o);
    if (COLS && row >= r0 && row < r1) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        sg[j] += o[j];
        sx[j] += o[j] * hx[s][j];
      }
    }
  };
  auto fold = [&]() {
    if (COLS) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        cs_g[j] += (double)sg[j];
        cs_x[j] += (double)sx[j];
      }
      sg = zero;
      sx = zero;
    }
  };
  issue(0, r0);   // N > 0: an empty block (r0 = r1 = N) reads row N - 1
  __builtin_amdgcn_sched_barrier(0);
  issue(1, r0 + R16);
  __builtin_amdgcn_sched_barrier(0);
  load_wslice(ws0, W0T, w);
  load_wslice(ws1, W1T, w);
  int last = r0 - X6_ROWS;
  for (int base = r0; base < r1; base += X6_ROWS) {
    stage(0, base);
    __syncthreads();
    compute(0);
    epilogue(1, base - R16);
    fold();
    stage(1, base + R16);
    __syncthreads();
    compute(1);
    epilogue(0, base);
    last = base;
  }
  __syncthreads();
  epilogue(1, last + R16);
  fold();
  if (COLS) {
    double* red = reinterpret_cast<double*>(sm);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      red[rg * 2 * L + 4 * cg + j] = cs_g[j];
      red[rg * 2 * L + L + 4 * cg + j] = cs_x[j];
    }
    __syncthreads();
    double* row = red + EBW_THREADS / 32 * 2 * L;
    for (int i = threadIdx.x; i < 2 * L; i += blockDim.x) {
      double v = 0;
      for (int g = 0; g < EBW_THREADS / 32; ++g) v += red[g * 2 * L + i];
      row[i] = v;
    }
    __syncthreads();
    lnb_emit(row, ln_g, part, accumulate, pairs, row + 2 * L);
  }
}

// ============================================================================ node_net backward
// pdg_node_bwd in the cooperative layout (models.py:240-243 backward; gy = d loss / d x_{t+1}):
//   gz2 = LN_bwd(gy) [a2 > 0]                      (whole rows -> HBM and a bf16x6 image)
//   gz1 = (W2^T gz2) [a1 > 0]                      (image -> product -> masked -> second image)
//   gaggr = W1a^T gz1,  gx_part = W1b^T gz1 + gy   (one image, two weight slices)
// with the three 128x128 weights stationary in registers as bf16 terms and the products in
// bf16x6 (the edge backward's W^T products); outputs stored whole-row through fp32 row tiles.
__device__ __forceinline__ void gemm_round_2w(f32x4 (&da)[2], f32x4 (&db)[2], const WSlice& wa, const WSlice& wb,
                                              const unsigned char* img) {
  const int l = lane_id(), n = l & 15, kg = l >> 4;
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) da[nb] = db[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 4; ++ks)
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      const int off = x6_addr(16 * nb + n, 64 * ks + 16 * kg);
      bf16x8 B[3];
#pragma unroll
      for (int p = 0; p < 3; ++p) B[p] = *reinterpret_cast<const bf16x8*>(img + p * X6_TERM + off);
      f32x4 t = da[nb], u = db[nb];
      t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa.a[ks][2], B[0], t, 0, 0, 0);
      u = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb.a[ks][2], B[0], u, 0, 0, 0);
      t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa.a[ks][1], B[1], t, 0, 0, 0);
      u = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb.a[ks][1], B[1], u, 0, 0, 0);
      t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa.a[ks][0], B[2], t, 0, 0, 0);
      u = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb.a[ks][0], B[2], u, 0, 0, 0);
      t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa.a[ks][1], B[0], t, 0, 0, 0);
      u = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb.a[ks][1], B[0], u, 0, 0, 0);
      t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa.a[ks][0], B[1], t, 0, 0, 0);
      u = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb.a[ks][0], B[1], u, 0, 0, 0);
      da[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa.a[ks][0], B[0], t, 0, 0, 0);
      db[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb.a[ks][0], B[0], u, 0, 0, 0);
    }
}

__global__ __launch_bounds__(EBW_THREADS, 1) void node_bwd_coop_kernel(
    int N, const float* __restrict__ gy, const float* __restrict__ a2, const float* __restrict__ a1,
    const pdg_ln_stat* __restrict__ stp, const pdg_ln_bwd* __restrict__ lbp, const double* __restrict__ lb_pairs,
    int lb_npairs, const float* __restrict__ lg, const float* __restrict__ W2T, const float* __restrict__ W1aT,
    const float* __restrict__ W1bT, float* __restrict__ gz2_out, float* __restrict__ gz1_out,
    float* __restrict__ gaggr, float* __restrict__ gx_part) {
  extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
  unsigned char* img2 = sm;                                    // gz2
  unsigned char* img1 = sm + EBW_IMG;                          // gz1
  unsigned char* msk = sm + 2 * EBW_IMG;                       // [a1 > 0]
  float* t_z = reinterpret_cast<float*>(msk + EBW_MASK);       // gz1 rows
  float* t_a = t_z + EFC_TILE;                                 // W1a^T gz1
  float* t_b = t_a + EFC_TILE;                                 // W1b^T gz1
  float* t_g = t_b + EFC_TILE;                                 // gy rows (the residual; no registers)
  const int l = lane_id(), w = wave_id();
  const int cg = threadIdx.x & 31, rg = threadIdx.x >> 5;
  const int oc = 16 * w + 4 * (l >> 4);
  int r0, r1;
  block_rows(N, r0, r1);
  WSlice w2, wa, wb;
  load_wslice(w2, W2T, w);
  load_wslice(wa, W1aT, w);
  load_wslice(wb, W1bT, w);
  const LNStat st = *reinterpret_cast<const LNStat*>(stp);
  const pdg_ln_bwd lb = lnb_resolve(lbp, lb_pairs, lb_npairs, stp);
  const f32x4 g4 = *reinterpret_cast<const f32x4*>(lg + 4 * cg);
  f32x4 pg[2], pa2[2], pa1[2];
  auto issue = [&](int base) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const size_t rc = (size_t)clamp_row(base + rg + 16 * u, r1) * L + 4 * cg;
      pg[u] = *reinterpret_cast<const f32x4*>(gy + rc);
      pa2[u] = *reinterpret_cast<const f32x4*>(a2 + rc);
      pa1[u] = *reinterpret_cast<const f32x4*>(a1 + rc);
    }
  };
  if (r0 < r1) issue(r0);
  for (int base = r0; base < r1; base += X6_ROWS) {
    const f32x4 zero = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int r = rg + 16 * u;
      const bool ok = base + r < r1;
      const f32x4 z2 = ok ? ln_relu_bwd4(pg[u], pa2[u], st, lb, g4) : zero;
      if (ok) stnt4(gz2_out + (size_t)(base + r) * L + 4 * cg, z2);
      img_store4(img2, r, cg, z2);
      *reinterpret_cast<unsigned*>(msk + r * MSK_STRIDE + 4 * cg) = relu_mask4(pa1[u]);
      *reinterpret_cast<f32x4*>(t_g + r * OT_STRIDE + 4 * cg) = pg[u];
    }
    __syncthreads();   // gz2 image and the a1 mask complete
    if (base + X6_ROWS < r1) issue(base + X6_ROWS);
    {
      f32x4 d[1][2];
      const unsigned char* imgs[1] = {img2};
      gemm_round<1>(d, w2, imgs);
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        const int r = 16 * nb + (l & 15);
        const unsigned mm = *reinterpret_cast<const unsigned*>(msk + r * MSK_STRIDE + oc);
        f32x4 z1;
#pragma unroll
        for (int j = 0; j < 4; ++j) z1[j] = (mm >> (8 * j)) & 1u ? d[0][nb][j] : 0.f;   // relu_mask_acc
        img_store4(img1, r, 4 * w + (l >> 4), z1);
        *reinterpret_cast<f32x4*>(t_z + r * OT_STRIDE + oc) = z1;
      }
    }
    __syncthreads();   // gz1 image complete
    {
      f32x4 da[2], db[2];
      gemm_round_2w(da, db, wa, wb, img1);
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        const int r = 16 * nb + (l & 15);
        *reinterpret_cast<f32x4*>(t_a + r * OT_STRIDE + oc) = da[nb];
        *reinterpret_cast<f32x4*>(t_b + r * OT_STRIDE + oc) = db[nb];
      }
    }
    __syncthreads();   // tiles complete; images and mask free for the next round
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int r = rg + 16 * u;
      const int row = base + r;
      if (row < r1) {
        const size_t o = (size_t)row * L + 4 * cg;
        stnt4(gz1_out + o, *reinterpret_cast<const f32x4*>(t_z + r * OT_STRIDE + 4 * cg));
        stg4(gaggr + o, *reinterpret_cast<const f32x4*>(t_a + r * OT_STRIDE + 4 * cg));
        stg4(gx_part + o, *reinterpret_cast<const f32x4*>(t_b + r * OT_STRIDE + 4 * cg) +
                              *reinterpret_cast<const f32x4*>(t_g + r * OT_STRIDE + 4 * cg));
      }
    }
  }
}

// ============================================================================ narrow weight gradients
// The block partial of a narrow weight gradient T[c][i] = sum_rows wide[c] narrow[i] (c < 128, i < K) in
// wgrad_narrow_kernel's layout [T (128 K) | wide sums (128) | narrow sums (K)], reduced by
// pdg_wgrad_narrow_finalize.  Thread (rg, cg) holds the fp64 sums of columns 4cg .. 4cg + 3 over the rows
// it visited (t[4 K + 4 + K]: products, wide sums, narrow sums — the narrow sums counted by the cg = 0
// threads only); the 16 row groups are added in order through LDS (`red`: 16 x tot doubles).
template <int K>
__device__ __forceinline__ void narrow_emit(const double (&t)[4 * K + 4 + K], double* red, double* __restrict__ out) {
  constexpr int tot = L * K + L + K;
  const int cg = threadIdx.x & 31, rg = threadIdx.x >> 5;
  __syncthreads();   // the caller's LDS is free
  double* mine = red + rg * tot;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
#pragma unroll
    for (int i = 0; i < K; ++i) mine[(4 * cg + c) * K + i] = t[c * K + i];
    mine[L * K + 4 * cg + c] = t[4 * K + c];
  }
  if (cg == 0)
#pragma unroll
    for (int i = 0; i < K; ++i) mine[L * K + L + i] = t[4 * K + 4 + i];
  __syncthreads();
  for (int e = threadIdx.x; e < tot; e += blockDim.x) {
    double v = 0;
    for (int g = 0; g < EBW_THREADS / 32; ++g) v += red[g * tot + e];
    out[(size_t)blockIdx.x * tot + e] = v;
  }
}

// ============================================================================ encoder backward
// pdg_mlp2_bwd in the cooperative layout (the node encoder's backward, models.py:264-275 for the
// 6-input encoder): gz2 = LN_bwd(gy) [a2 > 0] (whole rows -> HBM and a bf16x6 image),
// gz1 = (W2^T gz2) [a1 > 0] (the product in bf16x6 with W2^T in registers) -> row tile -> HBM.
// node_bwd_coop_kernel's first half.
__global__ __launch_bounds__(EBW_THREADS, 1) void mlp2_bwd_coop_kernel(
    int N, const float* __restrict__ gy, const float* __restrict__ a2, const float* __restrict__ a1,
    const pdg_ln_stat* __restrict__ stp, const pdg_ln_bwd* __restrict__ lbp, const double* __restrict__ lb_pairs,
    int lb_npairs, const float* __restrict__ lg, const float* __restrict__ W2T, float* __restrict__ gz2_out,
    float* __restrict__ gz1_out, const float* __restrict__ xn, double* __restrict__ npart) {
  extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
  unsigned char* img2 = sm;                                    // gz2
  unsigned char* msk = sm + EBW_IMG;                           // [a1 > 0]
  float* t_z = reinterpret_cast<float*>(msk + EBW_MASK);       // gz1 rows
  const int l = lane_id(), w = wave_id();
  const int cg = threadIdx.x & 31, rg = threadIdx.x >> 5;
  const int oc = 16 * w + 4 * (l >> 4);
  int r0, r1;
  block_rows(N, r0, r1);
  WSlice w2;
  load_wslice(w2, W2T, w);
  const LNStat st = *reinterpret_cast<const LNStat*>(stp);
  const pdg_ln_bwd lb = lnb_resolve(lbp, lb_pairs, lb_npairs, stp);
  const f32x4 g4 = *reinterpret_cast<const f32x4*>(lg + 4 * cg);
  // xn != NULL: the first layer's weight gradient from the gz1 rows of the epilogue (wgrad_narrow_kernel<6>'s
  // products and order per row, wide = gz1, narrow = xn = the encoder input), gz1 itself not needed
  constexpr int NK = 6, NT = 4 * NK + 4 + NK;
  double nt[NT];
#pragma unroll
  for (int p = 0; p < NT; ++p) nt[p] = 0;
  f32x4 pg[2], pa2[2], pa1[2];
  float px[2][NK], xv[2][NK];
  auto issue = [&](int base) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int rr = clamp_row(base + rg + 16 * u, r1);
      const size_t rc = (size_t)rr * L + 4 * cg;
      pg[u] = *reinterpret_cast<const f32x4*>(gy + rc);
      pa2[u] = *reinterpret_cast<const f32x4*>(a2 + rc);
      pa1[u] = *reinterpret_cast<const f32x4*>(a1 + rc);
      if (xn)
#pragma unroll
        for (int i = 0; i < NK; ++i) px[u][i] = xn[(size_t)rr * NK + i];
    }
  };
  if (r0 < r1) issue(r0);
  for (int base = r0; base < r1; base += X6_ROWS) {
    const f32x4 zero = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int r = rg + 16 * u;
      const bool ok = base + r < r1;
      const f32x4 z2 = ok ? ln_relu_bwd4(pg[u], pa2[u], st, lb, g4) : zero;
      if (ok) stnt4(gz2_out + (size_t)(base + r) * L + 4 * cg, z2);
      img_store4(img2, r, cg, z2);
      *reinterpret_cast<unsigned*>(msk + r * MSK_STRIDE + 4 * cg) = relu_mask4(pa1[u]);
#pragma unroll
      for (int i = 0; i < NK; ++i) xv[u][i] = px[u][i];
    }
    __syncthreads();   // gz2 image and the a1 mask complete
    if (base + X6_ROWS < r1) issue(base + X6_ROWS);
    f32x4 d[1][2];
    const unsigned char* imgs[1] = {img2};
    gemm_round<1>(d, w2, imgs);
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      const int r = 16 * nb + (l & 15);
      const unsigned mm = *reinterpret_cast<const unsigned*>(msk + r * MSK_STRIDE + oc);
      f32x4 z1;
#pragma unroll
      for (int j = 0; j < 4; ++j) z1[j] = (mm >> (8 * j)) & 1u ? d[0][nb][j] : 0.f;   // relu_mask_acc
      *reinterpret_cast<f32x4*>(t_z + r * OT_STRIDE + oc) = z1;
    }
    __syncthreads();   // the gz1 tile is complete; image and mask free for the next round
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int r = rg + 16 * u;
      if (base + r < r1) {
        const f32x4 z1 = *reinterpret_cast<const f32x4*>(t_z + r * OT_STRIDE + 4 * cg);
        if (gz1_out) stnt4(gz1_out + (size_t)(base + r) * L + 4 * cg, z1);
        if (xn) {
#pragma unroll
          for (int c = 0; c < 4; ++c) {
#pragma unroll
            for (int i = 0; i < NK; ++i) nt[c * NK + i] += (double)(z1[c] * xv[u][i]);
            nt[4 * NK + c] += (double)z1[c];
          }
#pragma unroll
          for (int i = 0; i < NK; ++i) nt[4 * NK + 4 + i] += (double)xv[u][i];
        }
      }
    }
  }
  if (xn) narrow_emit<NK>(nt, reinterpret_cast<double*>(sm), npart);
}

// ============================================================================ decoder backward
// pdg_decoder_bwd in the cooperative layout (models.py:316-321 backward; gy = d loss / d y, 3 wide):
//   gz1d = (gy Wd2) [a1d > 0]   (the 3-wide product in fp32 FMAs, pdg_decoder_bwd's order)
//   gx   = Wd1^T gz1d           (bf16x6, Wd1^T stationary in registers)
// COLS: gx is the upstream gradient of the last node LayerNorm; its pdg_ln_colsum column sums /
// (S1, S2) pairs are formed from the row tile (gemm_sum2_coop_kernel's reduction).
template <bool COLS>
__global__ __launch_bounds__(EBW_THREADS, 1) void decoder_bwd_coop_kernel(
    int N, const float* __restrict__ gy, const float* __restrict__ a1d, const float* __restrict__ Wd2,
    const float* __restrict__ Wd1T, float* __restrict__ gz1d, float* __restrict__ gx,
    const float* __restrict__ ln_a2, const pdg_ln_stat* __restrict__ ln_st, double* __restrict__ part,
    const float* __restrict__ ln_g, double* __restrict__ pairs, int accumulate, double* __restrict__ npart) {
  extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
  unsigned char* img = sm;
  float* t_o = reinterpret_cast<float*>(sm + EBW_IMG);
  // npart != NULL: node_decoder.2's weight gradient from the staged rows (wgrad_narrow_kernel<3>'s products
  // per row, wide = a1d, narrow = gy)
  constexpr int NK = 3, NT = 4 * NK + 4 + NK;
  double nt[NT];
#pragma unroll
  for (int p = 0; p < NT; ++p) nt[p] = 0;
  LNStat stln;
  if (COLS) stln = *reinterpret_cast<const LNStat*>(ln_st);
  const int l = lane_id(), w = wave_id();
  const int cg = threadIdx.x & 31, rg = threadIdx.x >> 5;
  const int oc = 16 * w + 4 * (l >> 4);
  int r0, r1;
  block_rows(N, r0, r1);
  WSlice ws;
  load_wslice(ws, Wd1T, w);
  f32x4 wd[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) wd[k] = *reinterpret_cast<const f32x4*>(Wd2 + k * L + 4 * cg);
  double cs_g[4] = {0, 0, 0, 0}, cs_x[4] = {0, 0, 0, 0};
  f32x4 pa1[2], pa2[2];
  float pg[2][3];
  auto issue = [&](int base) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int rc = clamp_row(base + rg + 16 * u, r1);
#pragma unroll
      for (int k = 0; k < 3; ++k) pg[u][k] = gy[(size_t)rc * 3 + k];
      pa1[u] = *reinterpret_cast<const f32x4*>(a1d + (size_t)rc * L + 4 * cg);
      if (COLS) pa2[u] = *reinterpret_cast<const f32x4*>(ln_a2 + (size_t)rc * L + 4 * cg);
    }
  };
  if (r0 < r1) issue(r0);
  for (int base = r0; base < r1; base += X6_ROWS) {
    const f32x4 zero = f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 av[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int r = rg + 16 * u;
      const bool ok = base + r < r1;
      f32x4 z;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float ga = fmaf(pg[u][2], wd[2][j], fmaf(pg[u][1], wd[1][j], pg[u][0] * wd[0][j]));
        z[j] = ok && pa1[u][j] > 0.f ? ga : 0.f;
      }
      if (ok) stnt4(gz1d + (size_t)(base + r) * L + 4 * cg, z);
      img_store4(img, r, cg, z);
      av[u] = COLS ? pa2[u] : zero;
      if (npart && ok) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
#pragma unroll
          for (int i = 0; i < NK; ++i) nt[c * NK + i] += (double)(pa1[u][c] * pg[u][i]);
          nt[4 * NK + c] += (double)pa1[u][c];
        }
#pragma unroll
        for (int i = 0; i < NK; ++i) nt[4 * NK + 4 + i] += (double)pg[u][i];
      }
    }
    __syncthreads();   // image complete
    if (base + X6_ROWS < r1) issue(base + X6_ROWS);
    f32x4 d[1][2];
    const unsigned char* imgs[1] = {img};
    gemm_round<1>(d, ws, imgs);
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) *reinterpret_cast<f32x4*>(t_o + (16 * nb + (l & 15)) * OT_STRIDE + oc) = d[0][nb];
    __syncthreads();   // tile complete; the image is free for the next round
    f32x4 sg = zero, sx = zero;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int r = rg + 16 * u;
      const int row = base + r;
      if (row < r1) {
        const f32x4 o = *reinterpret_cast<const f32x4*>(t_o + r * OT_STRIDE + 4 * cg);
        stg4(gx + (size_t)row * L + 4 * cg, o);
        if (COLS) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {   // the pdg_ln_colsum formulas
            sg[j] += o[j];
            sx[j] += o[j] * div_den(av[u][j] - stln.mean, stln.den, stln.rstd);
          }
        }
      }
    }
    if (COLS) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        cs_g[j] += (double)sg[j];
        cs_x[j] += (double)sx[j];
      }
    }
  }
  if (COLS) {
    double* red = reinterpret_cast<double*>(sm);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      red[rg * 2 * L + 4 * cg + j] = cs_g[j];
      red[rg * 2 * L + L + 4 * cg + j] = cs_x[j];
    }
    __syncthreads();
    double* row = red + EBW_THREADS / 32 * 2 * L;
    for (int i = threadIdx.x; i < 2 * L; i += blockDim.x) {
      double v = 0;
      for (int g = 0; g < EBW_THREADS / 32; ++g) v += red[g * 2 * L + i];
      row[i] = v;
    }
    __syncthreads();
    lnb_emit(row, ln_g, part, accumulate, pairs, row + 2 * L);
  }
  if (npart) narrow_emit<NK>(nt, reinterpret_cast<double*>(sm), npart);
}

// ============================================================================ C ABI
extern "C" int pdg_edge_bwd_w2(int n_edges, const int* dst, const float* gaggr, const float* ge_next,
                               const float* a2m, const float* a1m, const float* a2e, const float* a1e,
                               const pdg_ln_stat* st_m, const pdg_ln_stat* st_e, const pdg_ln_bwd* lb_m,
                               const pdg_ln_bwd* lb_e, const float* ln_g, const float* W2T, float* gz1m,
                               float* gz1e, float* gC, float* slabs, int nslabs, const double* pairs_m, int npairs_m,
                               const double* pairs_e, int npairs_e, int slab_init, void* stream) {
  PDG_CHECK_ARG(n_edges > 0, "pdg_edge_bwd_w2: n_edges must be > 0");
  PDG_CHECK_ARG(nslabs > 0 && nslabs <= MAX_BLOCKS && slabs, "pdg_edge_bwd_w2: bad slabs");
  PDG_CHECK_ARG(dst && gaggr && a2m && a1m && st_m && (lb_m || pairs_m) && ln_g && W2T && gz1m && gC,
                "pdg_edge_bwd_w2: null argument");
  PDG_CHECK_ARG(PDG_ALIGNED(gaggr) && PDG_ALIGNED(a2m) && PDG_ALIGNED(a1m) && PDG_ALIGNED(ln_g) &&
                    PDG_ALIGNED(W2T) && PDG_ALIGNED(gz1m) && PDG_ALIGNED(gC) && PDG_ALIGNED(slabs),
                "pdg_edge_bwd_w2: misaligned pointer");
  const bool eu = ge_next != nullptr;
  PDG_CHECK_ARG(!eu || gC != gz1m, "pdg_edge_bwd_w2: gC may alias gz1m only without the edge update");
  // gz1e may be NULL with the edge update: not stored (an empty range drops its stores);
  // pdg_pq_scatter_bwd(e_is_sum) then forms it from gC - gz1m
  PDG_CHECK_ARG(!eu || (PDG_ALIGNED(ge_next) && a2e && a1e && st_e && (lb_e || pairs_e) &&
                        PDG_ALIGNED(a2e) && PDG_ALIGNED(a1e) && (!gz1e || PDG_ALIGNED(gz1e))),
                "pdg_edge_bwd_w2: edge-update arguments missing or misaligned");
  // 16-row rounds, two rounds of loads in flight (edge_bwd_w2_kernel): two buffers of images + masks
  const size_t shm = eu ? 2 * (4 * IMG16 + 2 * MSK16) : 2 * (2 * IMG16 + MSK16);
  hipStream_t s = (hipStream_t)stream;
  if (eu)
    hipLaunchKernelGGL(edge_bwd_w2_kernel<true>, dim3(nslabs), dim3(EBW_THREADS), shm, s, dst, gaggr, ge_next, a2m,
                       a1m, a2e, a1e, st_m, st_e, lb_m, lb_e, ln_g, W2T, gz1m, gz1e, gC, slabs, n_edges, pairs_m,
                       npairs_m, pairs_e, npairs_e, slab_init);
  else
    hipLaunchKernelGGL(edge_bwd_w2_kernel<false>, dim3(nslabs), dim3(EBW_THREADS), shm, s, dst, gaggr, ge_next, a2m,
                       a1m, a2e, a1e, st_m, st_m, lb_m, lb_m, ln_g, W2T, gz1m, gz1e, gC, slabs, n_edges, pairs_m,
                       npairs_m, pairs_m, npairs_m, slab_init);
  PDG_CHECK_LAUNCH("pdg_edge_bwd_w2");
  return PDG_OK;
}

extern "C" int pdg_edge_gout_wc(int n_edges, const float* gC, const float* e, const float* ge_next, const float* WcT,
                                float* ge_out, float* slabs, int nslabs, const float* a2ln, const pdg_ln_stat* st_ln,
                                double* ln_partials, const float* ln_g, double* pairs, int accumulate, int slab_init,
                                void* stream) {
  PDG_CHECK_ARG(n_edges > 0, "pdg_edge_gout_wc: n_edges must be > 0");
  PDG_CHECK_ARG(nslabs > 0 && nslabs <= MAX_BLOCKS && slabs, "pdg_edge_gout_wc: bad slabs");
  PDG_CHECK_ARG(gC && e && WcT && ge_out, "pdg_edge_gout_wc: null argument");
  PDG_CHECK_ARG(PDG_ALIGNED(gC) && PDG_ALIGNED(e) && PDG_ALIGNED(WcT) && PDG_ALIGNED(ge_out) &&
                    PDG_ALIGNED(slabs) && (!ge_next || PDG_ALIGNED(ge_next)),
                "pdg_edge_gout_wc: misaligned pointer");
  PDG_CHECK_ARG(ge_out != ge_next, "pdg_edge_gout_wc: ge_out must not alias ge_next");
  PDG_CHECK_ARG(!a2ln || (PDG_ALIGNED(a2ln) && st_ln && ln_partials), "pdg_edge_gout_wc: LayerNorm column-sum arguments");
  PDG_CHECK_ARG(!pairs || (a2ln && ln_g), "pdg_edge_gout_wc: pairs need a2ln and ln_g");
  // LDS: two rounds' images (gC, e) + two output tiles; afterwards the slab reduction (8 KB) and the
  // LayerNorm column sums (row groups + one row + its scratch) from 16 KB on
  const size_t shm_pipe = 4 * IMG16 + 2 * GO_TILE * sizeof(float);
  const size_t shm_ln = 16384 + ((size_t)EBW_THREADS / 32 + 2) * 2 * L * sizeof(double);
  const size_t shm = shm_pipe > shm_ln ? shm_pipe : shm_ln;
  hipStream_t s = (hipStream_t)stream;
#define PDG_GO2(R, LNF)                                                                                       \
  hipLaunchKernelGGL((edge_gout_wc_kernel<R, LNF>), dim3(nslabs), dim3(EBW_THREADS), shm, s, gC, e, ge_next,   \
                     WcT, ge_out, slabs, a2ln, st_ln, ln_partials, n_edges, ln_g, pairs, accumulate, slab_init)
  if (ge_next) {
    if (a2ln) PDG_GO2(true, true); else PDG_GO2(true, false);
  } else {
    if (a2ln) PDG_GO2(false, true); else PDG_GO2(false, false);
  }
#undef PDG_GO2
  PDG_CHECK_LAUNCH("pdg_edge_gout_wc");
  return PDG_OK;
}

// ============================================================================ edge encoder backward
// Backward of edge_encoder = Lin(1 -> 128) ReLU Lin(128 -> 128) ReLU LN (models.py:268-274) over the E scalar
// inputs e_in, upstream gradient gy = d loss / d e_0 (ge_out of the first step), gz2 = LN_bwd(gy) [a2 > 0],
// without the W2^T product: the layer-1 input is one scalar e per edge,
// so a1 = mask . (w0 e + b0) with mask = [a1 > 0], and every gradient of the encoder's first two layers is a
// linear function of two products over the rows with the BINARY mask as operand:
//   M = (gz2 . e)^T mask,  N = gz2^T mask       (128 x 128 each, per block, K = rows)
//   dW2[j][k] = w0[k] M[j][k] + b0[k] N[j][k],  dw0[k] = sum_j W2[j][k] M[j][k],  db0[k] = sum_j W2[j][k] N[j][k]
// (the same sums regrouped; a1 enters exactly instead of rounded to fp32).  The mask is exact in ONE bf16 term,
// so each product costs 3 MFMAs per K step instead of bf16x6's 6, and the per-row W2^T product of the
// two-deep kernel (another 6 per step, with its weight slice in registers) is gone: half the matrix time.
// 16-row rounds with two rounds of row loads in flight (edge_bwd_w2_kernel's form); the block's slab gets its
// dW2 and its narrow-sum row its dw0 / db0 partials, so pdg_bwd_epilogue reduces them.  a1 is recomputed from
// the scalar input (the forward keeps no a1), gz2 / gz1 are never written.  (Round 5, A/B on one box: 89.5 /
// 88.9 -> 75.1 / 76.0 us per config-2 call against the earlier W2^T-product kernels, since removed; gradients
// within 7e-8 of theirs.)
constexpr int EEB3_BUF = 2 * IMG16 + T16;   // one round's gz2 and gz2.e images and the mask image
// NS register sets of row loads: set s holds round n's rows (n = s mod NS) from its issue NS - 1 stages ahead
// until its stage; the two LDS buffers alternate by round parity.  Four sets (64 KB of loads in flight per CU)
// measured the same as two (69.7 / 70.4 vs 70.3 / 69.0 us per config-2 call): the kernel is not waiting on rows.
#ifndef PDG_EEB_SETS
#define PDG_EEB_SETS 2
#endif
template <int NS>
__global__ __launch_bounds__(EBW_THREADS, 1) void edge_enc_bwd3_kernel(
    const float* __restrict__ gy, const float* __restrict__ a2, const float* __restrict__ e_in,
    const float* __restrict__ w0, const float* __restrict__ b0, const pdg_ln_stat* __restrict__ st_p,
    const pdg_ln_bwd* __restrict__ lb_p, const double* __restrict__ pairs, int npairs,
    const float* __restrict__ lg, const float* __restrict__ W2T, float* __restrict__ slabs,
    double* __restrict__ nsums, int E, int slab_init) {
  extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
  const int l = lane_id(), w = wave_id(), h = l >> 5, c = l & 31;
  const int cg = threadIdx.x & 31, rg = threadIdx.x >> 5;    // the thread's staged row: rg (0..15)
  const int ob = 32 * (w & 3), ib = 64 * (w >> 2);
  const int lrow = 8 * h + ((l & 15) >> 2);
  const int lcolb = 2 * (16 * ((l >> 4) & 1) + 4 * (l & 3));
  int r0, r1;
  block_rows(E, r0, r1);
  f32x16 accM[2], accN[2];
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int r = 0; r < 16; ++r) accM[b][r] = accN[b][r] = 0.f;
  f32x4 bsum = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 pg[NS], pa2[NS];
  float pe[NS];
  auto issue = [&](const int s, int base) {   // clamped: E > 0 (an empty block reads row E - 1)
    const int rc = clamp_row(base + rg, r1);
    pg[s] = *reinterpret_cast<const f32x4*>(gy + (size_t)rc * L + 4 * cg);
    pa2[s] = *reinterpret_cast<const f32x4*>(a2 + (size_t)rc * L + 4 * cg);
    pe[s] = e_in[rc];
  };
  const f32x4 g4 = *reinterpret_cast<const f32x4*>(lg + 4 * cg);
  const f32x4 w04 = *reinterpret_cast<const f32x4*>(w0 + 4 * cg);
  const f32x4 b04 = *reinterpret_cast<const f32x4*>(b0 + 4 * cg);
  const LNStat st = *reinterpret_cast<const LNStat*>(st_p);
#pragma unroll
  for (int q = 0; q < NS; ++q) {
    issue(q, r0 + q * R16);
    __builtin_amdgcn_sched_barrier(0);
  }
  const pdg_ln_bwd lb = lnb_resolve(lb_p, pairs, npairs, st_p);
  pin_vgpr(g4);
  pin_vgpr(w04);
  pin_vgpr(b04);
  auto stage = [&](const int s, const int base) {   // set s into LDS buffer s & 1
    unsigned char* img_g = sm + (s & 1) * EEB3_BUF;            // gz2
    unsigned char* img_e = img_g + IMG16;                      // gz2 . e
    unsigned char* img_m = img_g + 2 * IMG16;                  // [a1 > 0] as bf16 0 / 1 (one term)
    const f32x4 zero = f32x4{0.f, 0.f, 0.f, 0.f};
    const bool ok = base + rg < r1;
    const f32x4 zr = ln_relu_bwd4(pg[s], pa2[s], st, lb, g4);
    f32x4 zg, ze;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      zg[j] = ok ? zr[j] : 0.f;
      ze[j] = zg[j] * pe[s];
    }
    bsum += zg;
    img_store4<T16>(img_g, rg, cg, zg);
    img_store4<T16>(img_e, rg, cg, ze);
    unsigned mb[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {   // encoder_kernel's a1 sign: fma(w0, e, 0) + b0 > 0
      const float a = fmaf(w04[j], pe[s], 0.f) + b04[j];
      mb[j] = (ok && a > 0.f) ? 0x3F80u : 0u;
    }
    *reinterpret_cast<u32x2*>(img_m + x6_addr(rg, 8 * cg)) = u32x2{mb[0] | (mb[1] << 16), mb[2] | (mb[3] << 16)};
    issue(s, base + NS * R16);   // the set is free: NS rounds on
  };
  auto compute = [&](const int s) {
    const unsigned char* img_g = sm + s * EEB3_BUF;
    const unsigned char* img_e = img_g + IMG16;
    const unsigned char* img_m = img_g + 2 * IMG16;
    bf16x8 Ag[3], Ae[3], Bm[2];
    const int g0 = x6_addr(lrow, lcolb + 2 * ob), g1 = x6_addr(lrow + 4, lcolb + 2 * ob);
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      Ag[p] = x6_operand(img_g + p * T16, g0, g1);
      Ae[p] = x6_operand(img_e + p * T16, g0, g1);
    }
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int x0 = x6_addr(lrow, lcolb + 2 * (ib + 32 * b)), x1 = x6_addr(lrow + 4, lcolb + 2 * (ib + 32 * b));
      Bm[b] = x6_operand(img_m, x0, x1);
    }
#pragma unroll
    for (int b = 0; b < 2; ++b) {   // the small terms first, as wgrad_round chains them
      f32x16 t = accM[b];
      t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(Ae[2], Bm[b], t, 0, 0, 0);
      t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(Ae[1], Bm[b], t, 0, 0, 0);
      accM[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(Ae[0], Bm[b], t, 0, 0, 0);
      f32x16 u = accN[b];
      u = __builtin_amdgcn_mfma_f32_32x32x16_bf16(Ag[2], Bm[b], u, 0, 0, 0);
      u = __builtin_amdgcn_mfma_f32_32x32x16_bf16(Ag[1], Bm[b], u, 0, 0, 0);
      accN[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(Ag[0], Bm[b], u, 0, 0, 0);
    }
  };
  stage(0, r0);
  __syncthreads();
  for (int base = r0; base < r1; base += NS * R16) {
#pragma unroll
    for (int q = 0; q < NS; ++q) {
      compute(q & 1);
      if (q + 1 < NS && base + (q + 1) * R16 >= r1) break;   // block-uniform
      stage((q + 1) % NS, base + (q + 1) * R16);   // past r1 on the last step: zero rows nobody reads
      __syncthreads();
    }
  }
  __syncthreads();   // the last rounds' image reads precede the LDS reuse below
  // dW2 into the block's slab; dw0 / db0 partials: per thread over its 16 rows o of each column i, then the
  // two lane halves (h), then the four waves sharing ib, in order through LDS
  f32x16 accD[2];
  double dm[2], dn[2];
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const int i = ib + 32 * b + c;
    const float wi = w0[i], bi = b0[i];
    dm[b] = dn[b] = 0.;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int o = ob + (r & 3) + 8 * (r >> 2) + 4 * h;
      accD[b][r] = wi * accM[b][r] + bi * accN[b][r];
      const double wt = (double)W2T[(size_t)i * L + o];
      dm[b] += wt * (double)accM[b][r];
      dn[b] += wt * (double)accN[b][r];
    }
    dm[b] += __shfl_xor(dm[b], 32);
    dn[b] += __shfl_xor(dn[b], 32);
  }
  slab_accumulate(slabs + (size_t)blockIdx.x * WSLAB, accD, bsum, reinterpret_cast<float*>(sm), slab_init);
  double* red = reinterpret_cast<double*>(sm + 16 * L * 4);   // after slab_accumulate's 8 KB
  if (h == 0) {
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int i = ib + 32 * b + c;
      red[(w & 3) * 2 * L + i] = dm[b];
      red[(w & 3) * 2 * L + L + i] = dn[b];
    }
  }
  __syncthreads();
  if (threadIdx.x < 2 * L) {
    const int e = threadIdx.x;
    const double v = ((red[e] + red[2 * L + e]) + red[4 * L + e]) + red[6 * L + e];
    nsums[(size_t)blockIdx.x * 2 * L + e] = v;
  }
}

extern "C" int pdg_edge_enc_bwd(int n_edges, const float* gy, const float* a2, const float* e_in, const float* w0,
                                const float* b0, const pdg_ln_stat* st, const pdg_ln_bwd* lb, const double* lb_pairs,
                                int lb_npairs, const float* ln_g, const float* W2T, float* slabs, double* narrow_sums,
                                int nslabs, int slab_init, void* stream) {
  PDG_CHECK_ARG(n_edges > 0, "pdg_edge_enc_bwd: n_edges must be > 0");
  PDG_CHECK_ARG(nslabs > 0 && nslabs <= MAX_BLOCKS && slabs && narrow_sums, "pdg_edge_enc_bwd: bad slabs");
  PDG_CHECK_ARG(gy && a2 && e_in && w0 && b0 && st && (lb || lb_pairs) && ln_g && W2T,
                "pdg_edge_enc_bwd: null argument");
  PDG_CHECK_ARG(PDG_ALIGNED(gy) && PDG_ALIGNED(a2) && PDG_ALIGNED(w0) && PDG_ALIGNED(b0) && PDG_ALIGNED(ln_g) &&
                    PDG_ALIGNED(W2T) && PDG_ALIGNED(slabs),
                "pdg_edge_enc_bwd: misaligned pointer");
  const size_t shm = 2 * EEB3_BUF > 16 * L * 4 + 8 * L * 8 ? 2 * EEB3_BUF : 16 * L * 4 + 8 * L * 8;
  hipLaunchKernelGGL(edge_enc_bwd3_kernel<PDG_EEB_SETS>, dim3(nslabs), dim3(EBW_THREADS), shm, (hipStream_t)stream, gy,
                     a2, e_in, w0, b0, st, lb, lb_pairs, lb_npairs, ln_g, W2T, slabs, narrow_sums, n_edges, slab_init);
  PDG_CHECK_LAUNCH("pdg_edge_enc_bwd");
  return PDG_OK;
}

extern "C" int pdg_enc_narrow_reduce(const double* narrow_sums, int nslabs, float* grad_w0, float* grad_b0,
                                     void* stream) {
  PDG_CHECK_ARG(nslabs > 0 && narrow_sums && grad_w0 && grad_b0, "pdg_enc_narrow_reduce: bad arguments");
  hipLaunchKernelGGL(enc_narrow_reduce_kernel, dim3(2), dim3(4 * L), 0, (hipStream_t)stream, narrow_sums, nslabs,
                     grad_w0, grad_b0);
  PDG_CHECK_LAUNCH("pdg_enc_narrow_reduce");
  return PDG_OK;
}

extern "C" int pdg_gemm_sum2_coop(int rows, const float* in0, const float* in1, const float* W0T, const float* W1T,
                                  const float* res, float* out, const float* ln_a2, const pdg_ln_stat* ln_st,
                                  double* partials, const float* ln_g, double* pairs, int accumulate, int nblocks,
                                  void* stream) {
  PDG_CHECK_ARG(rows > 0 && nblocks > 0 && nblocks <= MAX_BLOCKS, "pdg_gemm_sum2_coop: bad sizes");
  PDG_CHECK_ARG(in0 && in1 && W0T && W1T && out, "pdg_gemm_sum2_coop: null argument");
  PDG_CHECK_ARG(PDG_ALIGNED(in0) && PDG_ALIGNED(in1) && PDG_ALIGNED(out) && PDG_ALIGNED(W0T) && PDG_ALIGNED(W1T) &&
                    PDG_ALIGNED(res),
                "pdg_gemm_sum2_coop: misaligned pointer");
  // LDS: two rounds' images + two output tiles; afterwards (COLS) the row groups' sums + one row + its scratch
  const size_t pipe = 4 * IMG16 + (size_t)2 * R16 * OT_STRIDE * sizeof(float);
  const size_t cols = ((size_t)EBW_THREADS / 32 + 2) * 2 * L * sizeof(double);
  hipStream_t s = (hipStream_t)stream;
#define PDG_GS2(C, R)                                                                                          \
  hipLaunchKernelGGL((gemm_sum2_coop_kernel<C, R>), dim3(nblocks), dim3(EBW_THREADS), C ? (pipe > cols ? pipe : cols) \
                     : pipe, s, rows, in0, in1, W0T, W1T, res, out, ln_a2, ln_st, partials, ln_g, pairs, accumulate)
  if (partials) {
    PDG_CHECK_ARG(ln_a2 && ln_st && PDG_ALIGNED(ln_a2) && (!pairs || ln_g),
                  "pdg_gemm_sum2_coop: column partials need an aligned ln_a2, ln_st (and ln_g for pairs)");
    if (res) PDG_GS2(true, true); else PDG_GS2(true, false);
  } else {
    if (res) PDG_GS2(false, true); else PDG_GS2(false, false);
  }
#undef PDG_GS2
  PDG_CHECK_LAUNCH("pdg_gemm_sum2_coop");
  return PDG_OK;
}

extern "C" int pdg_node_bwd_coop(int n_nodes, const float* gy, const float* a2n, const float* a1n,
                                 const pdg_ln_stat* st, const pdg_ln_bwd* lb, const float* ln_g, const float* Wn2T,
                                 const float* Wn1aT, const float* Wn1bT, float* gz2, float* gz1, float* gaggr,
                                 float* gx_part, const double* lb_pairs, int lb_npairs, int nblocks, void* stream) {
  PDG_CHECK_ARG(n_nodes > 0 && nblocks > 0 && nblocks <= MAX_BLOCKS, "pdg_node_bwd_coop: bad sizes");
  PDG_CHECK_ARG(gy && a2n && a1n && st && (lb || lb_pairs) && ln_g && Wn2T && Wn1aT && Wn1bT && gz2 && gz1 && gaggr &&
                    gx_part,
                "pdg_node_bwd_coop: null argument");
  PDG_CHECK_ARG(PDG_ALIGNED(gy) && PDG_ALIGNED(a2n) && PDG_ALIGNED(a1n) && PDG_ALIGNED(Wn2T) &&
                    PDG_ALIGNED(Wn1aT) && PDG_ALIGNED(Wn1bT) && PDG_ALIGNED(gz2) && PDG_ALIGNED(gz1) &&
                    PDG_ALIGNED(gaggr) && PDG_ALIGNED(gx_part) && PDG_ALIGNED(ln_g),
                "pdg_node_bwd_coop: misaligned pointer");
  const size_t shm = 2 * EBW_IMG + EBW_MASK + (size_t)4 * EFC_TILE * sizeof(float);
  hipLaunchKernelGGL(node_bwd_coop_kernel, dim3(nblocks), dim3(EBW_THREADS), shm, (hipStream_t)stream, n_nodes, gy,
                     a2n, a1n, st, lb, lb_pairs, lb_npairs, ln_g, Wn2T, Wn1aT, Wn1bT, gz2, gz1, gaggr, gx_part);
  PDG_CHECK_LAUNCH("pdg_node_bwd_coop");
  return PDG_OK;
}

// LDS of a narrow weight gradient's block reduction (narrow_emit): 16 row groups x tot doubles
static constexpr size_t narrow_lds(int K) { return (size_t)(EBW_THREADS / 32) * (L * K + L + K) * sizeof(double); }

extern "C" int pdg_mlp2_bwd_coop(int rows, const float* gy, const float* a2, const float* a1, const pdg_ln_stat* st,
                                 const pdg_ln_bwd* lb, const float* ln_g, const float* W2T, float* gz2, float* gz1,
                                 const double* lb_pairs, int lb_npairs, const float* x_narrow, double* narrow_partials,
                                 int nblocks, void* stream) {
  PDG_CHECK_ARG(rows > 0 && nblocks > 0 && nblocks <= MAX_BLOCKS, "pdg_mlp2_bwd_coop: bad sizes");
  PDG_CHECK_ARG(gy && a2 && a1 && st && (lb || lb_pairs) && ln_g && W2T && gz2 && (gz1 || x_narrow),
                "pdg_mlp2_bwd_coop: null argument");
  PDG_CHECK_ARG(PDG_ALIGNED(gy) && PDG_ALIGNED(a2) && PDG_ALIGNED(a1) && PDG_ALIGNED(W2T) && PDG_ALIGNED(gz2) &&
                    (!gz1 || PDG_ALIGNED(gz1)) && PDG_ALIGNED(ln_g),
                "pdg_mlp2_bwd_coop: misaligned pointer");
  PDG_CHECK_ARG(!x_narrow == !narrow_partials, "pdg_mlp2_bwd_coop: x_narrow and narrow_partials go together");
  size_t shm = EBW_IMG + EBW_MASK + (size_t)EFC_TILE * sizeof(float);
  if (x_narrow && narrow_lds(6) > shm) shm = narrow_lds(6);
  hipLaunchKernelGGL(mlp2_bwd_coop_kernel, dim3(nblocks), dim3(EBW_THREADS), shm, (hipStream_t)stream, rows, gy, a2,
                     a1, st, lb, lb_pairs, lb_npairs, ln_g, W2T, gz2, gz1, x_narrow, narrow_partials);
  PDG_CHECK_LAUNCH("pdg_mlp2_bwd_coop");
  return PDG_OK;
}

extern "C" int pdg_decoder_bwd_coop(int rows, const float* gy, const float* a1d, const float* Wd2, const float* Wd1T,
                                    float* gz1d, float* gx, const float* ln_a2, const pdg_ln_stat* ln_st,
                                    double* partials, const float* ln_g, double* pairs, int accumulate,
                                    double* narrow_partials, int nblocks, void* stream) {
  PDG_CHECK_ARG(rows > 0 && nblocks > 0 && nblocks <= MAX_BLOCKS, "pdg_decoder_bwd_coop: bad sizes");
  PDG_CHECK_ARG(gy && a1d && Wd2 && Wd1T && gz1d && gx, "pdg_decoder_bwd_coop: null argument");
  PDG_CHECK_ARG(PDG_ALIGNED(a1d) && PDG_ALIGNED(Wd2) && PDG_ALIGNED(Wd1T) && PDG_ALIGNED(gz1d) && PDG_ALIGNED(gx),
                "pdg_decoder_bwd_coop: misaligned pointer");
  const size_t tile = (size_t)EFC_TILE * sizeof(float);
  const size_t cols = ((size_t)EBW_THREADS / 32 + 2) * 2 * L * sizeof(double);
  size_t shm = EBW_IMG + tile;
  if (partials && cols > shm) shm = cols;
  if (narrow_partials && narrow_lds(3) > shm) shm = narrow_lds(3);
  if (partials) {
    PDG_CHECK_ARG(ln_a2 && ln_st && PDG_ALIGNED(ln_a2) && (!pairs || ln_g),
                  "pdg_decoder_bwd_coop: column partials need an aligned ln_a2, ln_st (and ln_g for pairs)");
    hipLaunchKernelGGL(decoder_bwd_coop_kernel<true>, dim3(nblocks), dim3(EBW_THREADS), shm, (hipStream_t)stream,
                       rows, gy, a1d, Wd2, Wd1T, gz1d, gx, ln_a2, ln_st, partials, ln_g, pairs, accumulate,
                       narrow_partials);
  } else {
    hipLaunchKernelGGL(decoder_bwd_coop_kernel<false>, dim3(nblocks), dim3(EBW_THREADS), shm, (hipStream_t)stream,
                       rows, gy, a1d, Wd2, Wd1T, gz1d, gx, nullptr, nullptr, nullptr, nullptr, nullptr, 0,
                       narrow_partials);
  }
  PDG_CHECK_LAUNCH("pdg_decoder_bwd_coop");
  return PDG_OK;
}
