/*
 * pdivgnn.h — C ABI of libpdivgnn_hip.so, the MI355X (gfx950) implementation of
 * the P-DivGNN hot path: EncodeProcessDecode forward/backward
 * (gnn_local_stress/models.py:98-326) and the divergence-regularised loss
 * (scripts/gnn_train.py:41-92).
 *
 * The reference is pure Python over PyTorch ATen + torch_geometric; it has no
 * FFI of its own.  Each entry point below replaces the group of ATen/PyG ops
 * named in its comment (file:line of the reference call site).  The Python
 * mirror (p-div-gnn_amd/gnn_local_stress) binds them with ctypes; INTEGRATION.md
 * shows the binding a maintainer would add to the reference.
 *
 * Conventions (all entry points):
 *   - device pointers to fp32 / int32 arrays; latent tensors are row-major
 *     (rows x 128) fp32, natural feature order, 16-byte aligned;
 *   - `stream` is a hipStream_t passed as void* (0 = null stream);
 *   - kernels never allocate; partial-sum buffers are caller-provided, sized
 *     by pdg_max_blocks();
 *   - return 0 on success, otherwise a nonzero code; pdg_last_error() gives
 *     the message of the last failure on the calling thread;
 *   - edges are in dst-sorted order (CSR over edge_index[1]); `src`/`dst` are
 *     the endpoints of each dst-sorted edge, `rowptr` the dst-CSR offsets.
 */
#ifndef PDIVGNN_H
#define PDIVGNN_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PDG_LATENT 128
#define PDG_OK 0
#define PDG_ERR_ARG 1
#define PDG_ERR_HIP 2

/* Graph-LayerNorm statistics of one call (torch_geometric LayerNorm, mode="graph", batch=None). */
typedef struct pdg_ln_stat {
  float mean;   /* mean over all rows x channels of the call */
  float den;    /* std_pop + eps (the forward divides by it) */
  float rstd;   /* 1 / den */
  float std_;   /* population std */
  double mean_d, std_d, count; /* fp64 copies and the element count M */
} pdg_ln_stat;

/* Backward scalars of one graph-LayerNorm call. */
typedef struct pdg_ln_bwd {
  float c1, c2;
  double S1, S2;
} pdg_ln_bwd;

/* ---------------------------------------------------------------- library */
const char* pdg_last_error(void);
int pdg_version(void);
/* Hash of the sources the library was built from (16 hex digits; build.py). */
const char* pdg_source_hash(void);
/* Upper bound on the number of per-block partials any launcher writes. */
int pdg_max_blocks(void);
/* Layout of the node pre-pass outputs P, Q (pdg_node_pq_rw[_fin] writes it, pdg_edge_fwd_coop reads it):
 * 0 = two N x 128 row-major arrays; 1 = one N x 256 array whose rows hold, per 16-feature block b,
 * P[16b..16b+15] then Q[16b..16b+15], passed as P = base, Q = base + 16 floats. */
int pdg_pq_layout(void);

/* ---------------------------------------------------------------- forward */

/* models.py:140-152 (format_node_features) + :154-162, :303-307 (format_edge_features):
 * x_in[n] = [(mean_stress-mu)/s (3), (pos-mu)/s (2), node_type (1)]; e_in[k] = (edge_attr[perm[k]]-mu)/s.
 * stats8 = {mean_pos, std_pos, mean_mean_stress, std_mean_stress, mean_local_stress,
 *           std_local_stress, mean_edge_weight, std_edge_weight} (device, fp32). */
int pdg_format_inputs(int n_nodes, int n_edges, const float* pos, const float* mean_stress,
                      const int64_t* node_types, const float* edge_attr, const int* perm,
                      const float* stats8, int scale_input, float* x_in, float* e_in, void* stream);

/* The node encoder (models.py:260-274, 6 inputs) in the cooperative layout: a1 = relu(W0 x + b0) bitwise
 * pdg_encoder_fwd's (stored when a1 != NULL), a2 = relu(W2 a1 + b2) as an unbiased bf16x6 product from
 * registers, nblocks blocks of 512 threads (partials: nblocks (sum, sumsq) pairs).  x_in 8-byte aligned. */
int pdg_node_enc_fwd(int n_nodes, const float* x_in, const float* w0, const float* b0, const float* W2,
                     const float* b2, float* a1, float* a2, double* partials, int nblocks, void* stream);
/* Encoder MLP (models.py:260-274): a1 = relu(W0 x + b0) (K = in_features in {1..8}),
 * a2 = relu(W2 a1 + b2); writes a1, a2 and per-block LayerNorm partials (sum, sumsq). */
int pdg_encoder_fwd(int rows, int in_features, const float* x_in, const float* W0, const float* b0,
                    const float* W2, const float* b2, float* a1, float* a2,
                    double* partials, int* nparts, void* stream);
/* (a1 == NULL: the layer-1 output is not stored; pdg_edge_enc_bwd recomputes it.) */

/* Reduce LayerNorm partials -> statistics (mean, std_pop + eps). */
int pdg_ln_finalize(const double* partials, int nparts, double count, pdg_ln_stat* out, void* stream);
/* Two pdg_ln_finalize calls with the same nparts and count in one launch (the message and
 * edge-update LayerNorms after pdg_edge_fwd); bit-identical to the two calls.  New in this
 * build: the reference has no separate statistics step (models.py:42-55 computes them inline). */
int pdg_ln_finalize2(const double* part_a, const double* part_b, int nparts, double count,
                     pdg_ln_stat* out_a, pdg_ln_stat* out_b, void* stream);
/* Exact data-parallel LayerNorm (optional "sync" DP mode): reduce the
 * per-block partials to out2 = {sum, sumsq} (device, 2 doubles) for an all-reduce over
 * ranks, then pdg_ln_finalize(out2, 1, global_count, ...).  New in this build: the
 * reference LayerNorm (models.py:42-55) runs on one device and needs no exchange. */
int pdg_ln_partials_sum(const double* partials, int nparts, double* out2, void* stream);

/* Processor node pre-pass (models.py:221/236 re-associated): x_t = LN(a2_prev) [+ x_res];
 * P = W1[:, 0:128] x_t, Q = W1[:, 128:256] x_t  (W1 = processor.edge_net.0.weight, 128 x 384). */
int pdg_node_pq(int n_nodes, const float* a2_prev, const pdg_ln_stat* st, const float* ln_g,
                const float* ln_b, const float* x_res, float* x_out, const float* W1,
                float* P, float* Q, void* stream);
/* Same result as pdg_node_pq (bitwise), with Wa/Wb held in registers by 8 compute waves and
 * the LN + residual rows staged by 4 loader waves (better for node-sized row counts). */
int pdg_node_pq_rw(int n_nodes, const float* a2_prev, const pdg_ln_stat* st, const float* ln_g,
                   const float* ln_b, const float* x_res, float* x_out, const float* W1, float* P,
                   float* Q, void* stream);
/* pdg_node_pq_rw with the node LayerNorm statistics of a2_prev folded in: every block reduces the
 * (sum, sumsq) partials of pdg_node_net itself in the pdg_ln_finalize order (bit-identical) and
 * block 0 stores them to st_out for the backward, replacing a separate pdg_ln_finalize launch.
 * New in this build (the reference computes the statistics inline, models.py:42-55). */
int pdg_node_pq_rw_fin(int n_nodes, const float* a2_prev, const double* partials, int nparts, double count,
                       pdg_ln_stat* st_out, const float* ln_g, const float* ln_b, const float* x_res,
                       float* x_out, const float* W1, float* P, float* Q, void* stream);

/* Fused edge pass of one message-passing step (models.py:215-222, :233-238).
 * with_edge_update == 0 skips the edge-update branch (the last step's e_S is never consumed,
 * models.py:316): a1e/a2e/part_e unused and may be NULL.
 * e_t = LN(a2_prev) [+ e_res]; C = W1[:, 256:384] e_t + b1;
 * message:  a1m = relu(C + P[dst] + Q[src]), a2m = relu(W2 a1m + b2)
 * edge upd: a1e = relu(C + P[src] + Q[dst]), a2e = relu(W2 a1e + b2)
 * writes e_t, a1m, a2m, a1e, a2e and LayerNorm partials of a2m and a2e.  a1m and a1e are only
 * needed by the backward: NULL skips storing them (inference). */
int pdg_edge_fwd(int n_edges, const float* a2_prev, const pdg_ln_stat* st, const float* ln_g,
                 const float* ln_b, const float* e_res, float* e_out, const int* src, const int* dst,
                 const float* P, const float* Q, const float* W1, const float* b1,
                 const float* W2, const float* b2, float* a1m, float* a2m, float* a1e, float* a2e,
                 double* part_m, double* part_e, int with_edge_update, int* nparts, void* stream);

/* PyG "add" aggregation (scatter_add_ at edge_index[1]) of LN-normalised rows:
 * out[v] = sum_{k in rowptr[v]..rowptr[v+1]} LN(rows[k]); st == NULL -> raw rows.
 * xhat_sum (nullable): sum_k (rows[k] - mean)/(std + eps), kept for the LayerNorm backward. */
int pdg_segment_sum(int n_nodes, const int* rowptr, const float* rows, const pdg_ln_stat* st,
                    const float* ln_g, const float* ln_b, float* out, float* xhat_sum, void* stream);
/* pdg_segment_sum with the message LayerNorm's statistics reduced in the kernel from the edge
 * forward's per-block (sum, sumsq) partials part_a (nparts pairs, count = rows x 128 elements), bitwise
 * pdg_ln_finalize's, stored to st_a; with part_b also the edge-update LayerNorm's, stored to st_b.
 * Replaces pdg_ln_finalize2 + pdg_segment_sum (one launch fewer per message-passing step). */
int pdg_segment_sum_fin(int n_nodes, const int* rowptr, const float* rows, const double* part_a,
                        const double* part_b, int nparts, double count, pdg_ln_stat* st_a, pdg_ln_stat* st_b,
                        const float* ln_g, const float* ln_b, float* out, float* xhat_sum, void* stream);

/* Processor.update first layer (models.py:240-243, :202-204):
 * a1n = relu(Wn1[:, 0:128] aggr + Wn1[:, 128:256] x + bn1). */
int pdg_node_mlp1(int n_nodes, const float* aggr, const float* x, const float* Wn1,
                  const float* bn1, float* a1n, void* stream);

/* Second MLP layer with LN partials: a2 = relu(W2 a1 + b2). */
int pdg_mlp2_fwd(int rows, const float* a1, const float* W2, const float* b2, float* a2,
                 double* partials, int* nparts, void* stream);

/* Fused node_net of one step (models.py:240-243): a1n = relu(Wn1 [aggr | x] + bn1),
 * a2n = relu(Wn2 a1n + bn2) and LayerNorm partials of a2n, in one pass with the weights held
 * in registers.  Bitwise the same a1n / a2n as pdg_node_mlp1 + pdg_mlp2_fwd.  a1n is only
 * needed by the backward and may be NULL. */
int pdg_node_net(int n_nodes, const float* aggr, const float* x, const float* Wn1, const float* bn1,
                 const float* Wn2, const float* bn2, float* a1n, float* a2n, double* partials,
                 int* nparts, void* stream);
/* Decoder (models.py:282-286, :316-321): x_S = LN(a2_prev) + x_res; a1d = relu(Wd1 x_S + bd1);
 * y = Wd2 a1d + bd2 (3 outputs); if scale_output: y = y * std_local_stress + mean_local_stress. */
int pdg_decoder_fwd(int n_nodes, const float* a2_prev, const pdg_ln_stat* st, const float* ln_g,
                    const float* ln_b, const float* x_res, float* x_out, const float* Wd1,
                    const float* bd1, float* a1d, const float* Wd2, const float* bd2,
                    const float* stats8, int scale_output, float* y, void* stream);
/* pdg_decoder_fwd with the last node LayerNorm's statistics folded in: every block reduces the
 * (sum, sumsq) partials of pdg_node_net in pdg_ln_finalize's order (bit-identical) and block 0
 * stores them to st_out for the backward, replacing a separate pdg_ln_finalize launch (as
 * pdg_node_pq_rw_fin does for the earlier steps). */
int pdg_decoder_fwd_fin(int n_nodes, const float* a2_prev, const double* partials, int nparts, double count,
                        pdg_ln_stat* st_out, const float* ln_g, const float* ln_b, const float* x_res,
                        float* x_out, const float* Wd1, const float* bd1, float* a1d, const float* Wd2,
                        const float* bd2, const float* stats8, int scale_output, float* y, void* stream);
/* The decoder in the cooperative layout (pdg_efwd.hip): x_out bitwise pdg_decoder_fwd's, Wd1 x_S as an
 * unbiased bf16x6 product from registers, a1d and y to fp32 rounding; partials != NULL: the statistics
 * reduced in-kernel as pdg_decoder_fwd_fin does (st unused), else st.  nblocks blocks of 512 threads. */
int pdg_decoder_fwd_coop(int n_nodes, const float* a2_prev, const pdg_ln_stat* st, const double* partials,
                         int nparts, double count, pdg_ln_stat* st_out, const float* ln_g, const float* ln_b,
                         const float* x_res, float* x_out, const float* Wd1, const float* bd1, float* a1d,
                         const float* Wd2, const float* bd2, const float* stats8, int scale_output, float* y,
                         int nblocks, void* stream);

/* torch.any(x != 0) into *flag (int, device). models.py:294 */
int pdg_any_nonzero(const float* x, int64_t n, int* flag, void* stream);

/* y[i] = 0 for every i < n unless *flag (device int) is set: the zero-stress guard of models.py:294-299
 * ("return zeros_like(mean_stress)") decided on the device, for a forward replayed from a HIP graph
 * (pdg/serve.py) where the reference's host-side torch.any would cost a synchronisation per call. */
int pdg_zero_unless(const int* flag, float* y, int64_t n, void* stream);

/* ---------------------------------------------------------------- backward */

/* Decoder backward: gz1d = (Wd2^T gy) * [a1d > 0]; gx = Wd1^T gz1d. */
int pdg_decoder_bwd(int n_nodes, const float* gy, const float* a1d, const float* Wd2,
                    const float* Wd1T, float* gz1d, float* gx, void* stream);

/* LayerNorm backward without finalize launches (every column-sum producer below): block b of a
 * producer emits its row of per-channel partials, partials[b] = [sum gy (128) | sum gy*xhat (128)]
 * (accumulate != 0: added to the row, so one buffer spans all message-passing steps and
 * pdg_ln_param_grads turns it into the LayerNorm weight / bias gradients once), and, when
 * pairs != NULL, pairs[2b..2b+1] = (sum_c g_c row_c, sum_c g_c row_{128+c}) with g = ln_g.  The
 * consumer kernels (pdg_node_bwd, pdg_edge_bwd(_w2), pdg_mlp2_bwd) take these pairs in place of
 * a finalized pdg_ln_bwd and reduce them themselves (S1, S2, c1 = S1/M, c2 = S2/(M std)).
 * New in this build: the reference's autograd computes these sums inside the LayerNorm backward
 * (models.py:199,207,265,273). */
/* Per-channel LayerNorm backward sums over rows: sum gy, sum gy*xhat (xhat from a2 and st);
 * gy row k = gy_rows[gidx ? gidx[k] : k]. Writes per-block partials (2 x 128 doubles each). */
int pdg_ln_colsum(int rows, const float* gy_rows, const int* gidx, const float* a2,
                  const pdg_ln_stat* st, double* partials, int* nparts, const float* ln_g,
                  double* pairs, int accumulate, void* stream);

/* Node-level form of pdg_ln_colsum for the message LayerNorm, whose upstream gradient is the
 * gathered gaggr[dst]: sum_k gy = sum_v deg_v gaggr[v], sum_k gy*xhat = sum_v gaggr[v]*xhat_sum[v]
 * (deg from rowptr, xhat_sum from pdg_segment_sum).  Same partial layout as pdg_ln_colsum. */
int pdg_ln_colsum_nodes(int n_nodes, const float* gaggr, const int* rowptr, const float* xhat_sum,
                        double* partials, int* nparts, const float* ln_g, double* pairs, int accumulate,
                        void* stream);

/* Reduce colsum partials: grad_b += sum gy, grad_g += sum gy*xhat, and the call's
 * backward scalars (S1 = sum g*gy, S2 = sum g*gy*xhat): the column sums of the LayerNorm
 * backward (PyG LayerNorm graph mode, models.py:199,207,265,273; autograd of its weight/bias).
 * One launch (a single 1024-thread block, fixed-order fp64 sums). */
int pdg_ln_colsum_finalize(const double* partials, int nparts, const float* ln_g,
                           const pdg_ln_stat* st, float* grad_g, float* grad_b, pdg_ln_bwd* out,
                           void* stream);
/* LayerNorm weight / bias gradients from producer accumulators (accumulate mode above): for
 * group i, grad_b[i][c] += sum over rows r < rows[i] of acc[i][r][c], grad_g[i][c] += ... [128 + c];
 * fixed order; ngroups <= 4 (node_net, edge_net, node encoder, edge encoder LayerNorms).
 * acc/rows/grad_g/grad_b are HOST arrays of device pointers. */
int pdg_ln_param_grads(int ngroups, const double* const* acc, const int* rows, float* const* grad_g,
                       float* const* grad_b, void* stream);

/* MLP tail backward (LN -> relu -> Linear2 -> relu): ga2 = LNbwd(gy); gz2 = ga2 * [a2 > 0];
 * gz1 = (W2^T gz2) * [a1 > 0].  gy row k = gy_rows[gidx ? gidx[k] : k]. */
int pdg_mlp2_bwd(int rows, const float* gy_rows, const int* gidx, const float* a2, const float* a1,
                 const pdg_ln_stat* st, const pdg_ln_bwd* lb, const float* ln_g, const float* W2T,
                 float* gz2, float* gz1, const double* lb_pairs, int lb_npairs, void* stream);

/* pdg_decoder_bwd in the block-cooperative layout (the Wd1^T product in bf16x6). With partials != NULL
 * it also forms pdg_ln_colsum's column partials / (S1, S2) pairs of gx for the LayerNorm with output
 * statistics ln_st over ln_a2 (one partial per block: *nparts = nblocks), as pdg_gemm_sum2_coop.
 * narrow_partials != NULL: also node_decoder.2's weight / bias gradient (models.py:316-321 backward,
 * pdg_wgrad_narrow(rows, a1d, gy, 3, ...)'s block partials, nblocks of them) for
 * pdg_wgrad_narrow_finalize(narrow_partials, nblocks, 3, 1, ...): one pass over a1d / gy fewer. */
int pdg_decoder_bwd_coop(int rows, const float* gy, const float* a1d, const float* Wd2, const float* Wd1T,
                         float* gz1d, float* gx, const float* ln_a2, const pdg_ln_stat* ln_st, double* partials,
                         const float* ln_g, double* pairs, int accumulate, double* narrow_partials, int nblocks,
                         void* stream);

/* pdg_mlp2_bwd (gidx = NULL) in the block-cooperative layout: the W2^T product in bf16x6 with W2^T
 * stationary in registers, whole-row access (the node encoder's backward).  x_narrow != NULL (rows x 6,
 * the encoder input): also the first layer's weight / bias gradient from gz1, as the block partials of
 * pdg_wgrad_narrow(rows, gz1, x_narrow, 6, ...) in narrow_partials (nblocks of them, for
 * pdg_wgrad_narrow_finalize(narrow_partials, nblocks, 6, 0, ...)); gz1 may then be NULL (not stored). */
int pdg_mlp2_bwd_coop(int rows, const float* gy, const float* a2, const float* a1, const pdg_ln_stat* st,
                      const pdg_ln_bwd* lb, const float* ln_g, const float* W2T, float* gz2, float* gz1,
                      const double* lb_pairs, int lb_npairs, const float* x_narrow, double* narrow_partials,
                      int nblocks, void* stream);

/* Fused node_net backward of one step (the work of pdg_mlp2_bwd + pdg_gemm_dual with
 * res0 = NULL, res1 = gy): gz2 = LN_bwd(gy) * [a2n > 0]; gz1 = (Wn2^T gz2) * [a1n > 0];
 * gaggr = Wn1a^T gz1; gx_part = Wn1b^T gz1 + gy.  Weights held in registers; bitwise the
 * results of the separate kernels. */
int pdg_node_bwd(int n_nodes, const float* gy, const float* a2n, const float* a1n, const pdg_ln_stat* st,
                 const pdg_ln_bwd* lb, const float* ln_g, const float* Wn2T, const float* Wn1aT,
                 const float* Wn1bT, float* gz2, float* gz1, float* gaggr, float* gx_part,
                 const double* lb_pairs, int lb_npairs, void* stream);
/* lb_pairs != NULL: the LayerNorm backward scalars come from a producer's pairs (see
 * pdg_ln_colsum) and lb is ignored. */

/* out0 = W0T in [+ res0]; out1 = W1T in [+ res1]  (two 128x128 products of one input). */
int pdg_gemm_dual(int rows, const float* in, const float* W0T, const float* W1T,
                  const float* res0, const float* res1, float* out0, float* out1, void* stream);

/* out = res + W0T in0 + W1T in1. */
int pdg_gemm_sum2(int rows, const float* in0, const float* in1, const float* W0T, const float* W1T,
                  const float* res, float* out, void* stream);
/* Same result as pdg_gemm_sum2 (bitwise), weights held in registers.  partials != NULL: also
 * the pdg_ln_colsum partials of the LayerNorm backward with upstream gradient `out` and input
 * ln_a2 / statistics ln_st (the node LayerNorm of the previous message-passing step, whose
 * output x_t = LN(a2n) + x_{t-1} receives this gradient), *nparts rows of 256 doubles. */
int pdg_gemm_sum2_rw(int rows, const float* in0, const float* in1, const float* W0T, const float* W1T,
                     const float* res, float* out, const float* ln_a2, const pdg_ln_stat* ln_st,
                     double* partials, int* nparts, const float* ln_g, double* pairs, int accumulate,
                     void* stream);

/* Fused edge backward of one step: both edge_net evaluations' LN/relu/Linear2 backward
 * (message: gy = gaggr[dst]; edge update: gy = ge_next), gC = gz1m + gz1e,
 * ge_out = ge_next + WcT gC.  Writes gz2m, gz1m, gz2e, gz1e, gC, ge_out.
 * ge_next == NULL: the edge-update branch had no consumer (last step): gz2e/gz1e are not
 * written, gC = gz1m, ge_out = WcT gC. */
/* Edge encoder forward (models.py:264-275, 1 -> 128 -> 128) in the block-cooperative layout: a2 =
 * relu(W2 relu(w0 e_in + b0) + b2) with the W2 product in bf16x6 (as pdg_edge_fwd's), and the
 * LayerNorm partials of a2 (nblocks pairs).  a1 is not stored (pdg_edge_enc_bwd recomputes it). */
int pdg_edge_enc_fwd(int n_edges, const float* e_in, const float* w0, const float* b0, const float* W2,
                     const float* b2, float* a2, double* partials, int nblocks, void* stream);
/* pdg_gemm_sum2_rw in the block-cooperative layout (nblocks blocks of 512 threads, contiguous row
 * ranges): out = W0T in0 + W1T in1 [+ res], both products in bf16x6 with the weights stationary in
 * registers; partials != NULL: the LayerNorm column partials and pairs as pdg_gemm_sum2_rw (nblocks
 * rows of 256 doubles). */
int pdg_gemm_sum2_coop(int rows, const float* in0, const float* in1, const float* W0T, const float* W1T,
                       const float* res, float* out, const float* ln_a2, const pdg_ln_stat* ln_st,
                       double* partials, const float* ln_g, double* pairs, int accumulate, int nblocks,
                       void* stream);
/* pdg_node_bwd in the block-cooperative layout (nblocks blocks of 512 threads): the same outputs with
 * the three W^T products in bf16x6, weights stationary in registers. */
int pdg_node_bwd_coop(int n_nodes, const float* gy, const float* a2n, const float* a1n, const pdg_ln_stat* st,
                      const pdg_ln_bwd* lb, const float* ln_g, const float* Wn2T, const float* Wn1aT,
                      const float* Wn1bT, float* gz2, float* gz1, float* gaggr, float* gx_part,
                      const double* lb_pairs, int lb_npairs, int nblocks, void* stream);
/* pdg_edge_fwd in the block-cooperative layout (pdg_efwd.hip): nblocks blocks of 512 threads, one
 * contiguous row range each, Wc and W2 stationary in registers as bf16 terms, whole-row HBM access.
 * Same outputs to fp32 rounding (e_t bitwise; C = Wc e and the W2 products as unbiased bf16x6
 * products); part_m / part_e get nblocks partials.  P and Q in the pdg_pq_layout() layout (what
 * pdg_node_pq_rw[_fin] writes; pdg_edge_fwd takes two N x 128 arrays). */
int pdg_edge_fwd_coop(int n_edges, const float* a2_prev, const pdg_ln_stat* st, const float* ln_g,
                      const float* ln_b, const float* e_res, float* e_out, const int* src, const int* dst,
                      const float* P, const float* Q, const float* W1, const float* b1, const float* W2,
                      const float* b2, float* a1m, float* a2m, float* a1e, float* a2e, double* part_m,
                      double* part_e, int with_edge_update, int nblocks, void* stream);
/* Inference edge forward (no layer-1 outputs: nothing reads them without a backward): pdg_edge_fwd_coop's
 * e_out, a2m, a2e (bitwise) and LayerNorm partials (the rows added in another order) from 16-row rounds with
 * one barrier per round -- the C product of round k beside the two W2 products of round k - 1, the gathers
 * one round ahead, two register sets of row loads (pdg_efwd.hip).  Arguments as pdg_edge_fwd_coop's without
 * a1m / a1e. */
int pdg_edge_fwd_infer(int n_edges, const float* a2_prev, const pdg_ln_stat* st, const float* ln_g,
                       const float* ln_b, const float* e_res, float* e_out, const int* src, const int* dst,
                       const float* P, const float* Q, const float* W1, const float* b1, const float* W2,
                       const float* b2, float* a2m, float* a2e, double* part_m, double* part_e,
                       int with_edge_update, int nblocks, void* stream);
int pdg_edge_bwd(int n_edges, const int* dst, const float* gaggr, const float* ge_next,
                 const float* a2m, const float* a1m, const float* a2e, const float* a1e,
                 const pdg_ln_stat* st_m, const pdg_ln_stat* st_e, const pdg_ln_bwd* lb_m,
                 const pdg_ln_bwd* lb_e, const float* ln_g, const float* W2T, const float* WcT,
                 float* gz2m, float* gz1m, float* gz2e, float* gz1e, float* gC, float* ge_out,
                 const double* pairs_m, int npairs_m, const double* pairs_e, int npairs_e, void* stream);

/* Edge backward with the shared-weight gradients fused (pdg_ebw.hip), replacing
 * pdg_edge_bwd + the W2 / Wc passes of pdg_wgrad_segments (gnn_local_stress/models.py:194-208,
 * backward).  Weights stationary in registers, 32-row operand images in LDS; one block per
 * slab, `nslabs` blocks (the same value for every call of a backward pass: the block ->
 * slab map is fixed and the slabs accumulate, reduced once by pdg_wgrad_reduce).
 *   pdg_edge_bwd_w2:  gz1m/gz1e/gC as pdg_edge_bwd; slabs += gz2m^T a1m + gz2e^T a1e and the
 *                     b2 column sums (slab_init != 0: slabs = ..., the first call of a backward,
 *                     so the slabs need no zero fill; the same for pdg_edge_gout_wc and
 *                     pdg_edge_enc_bwd); gz2m/gz2e are not
 *                     materialised.  ge_next == NULL: message branch only, gC = gz1m (gC may
 *                     then be the gz1m pointer itself: written once).  gz1e may be NULL with
 *                     the edge update: it is then not stored (pdg_pq_scatter_bwd with
 *                     e_is_sum forms it from gC - gz1m).
 *   pdg_edge_gout_wc: ge_out = [ge_next +] WcT gC; slabs += gC^T e and the b1 column sums.
 *                     a2ln != NULL: also the column sums of the backward of the LayerNorm that
 *                     produced e (input a2ln, statistics st_ln, upstream gradient ge_out), as
 *                     pdg_ln_colsum partials: nslabs rows of 256 doubles in ln_partials (one
 *                     spare row after them for pdg_ln_colsum_finalize). */
int pdg_edge_bwd_w2(int n_edges, const int* dst, const float* gaggr, const float* ge_next,
                    const float* a2m, const float* a1m, const float* a2e, const float* a1e,
                    const pdg_ln_stat* st_m, const pdg_ln_stat* st_e, const pdg_ln_bwd* lb_m,
                    const pdg_ln_bwd* lb_e, const float* ln_g, const float* W2T, float* gz1m,
                    float* gz1e, float* gC, float* slabs, int nslabs, const double* pairs_m, int npairs_m,
                    const double* pairs_e, int npairs_e, int slab_init, void* stream);
/* Edge encoder backward (models.py:268-274), fused: gz2 = LN_bwd(gy) [a2 > 0], slabs (zeroed
 * before, pdg_wgrad_reduce layout) += gz2^T a1 and the b2 sums, gz1 = (W2T gz2) [a1 > 0], and per
 * block narrow_sums[b] = (sum gz1 e_in, sum gz1) as 2 x 128 doubles; a1 = relu(w0 e_in + b0) is
 * recomputed (pdg_encoder_fwd may skip storing it).  Replaces pdg_mlp2_bwd + the edge encoder's
 * pdg_wgrad_segments and pdg_wgrad_narrow passes.  lb / lb_pairs as pdg_mlp2_bwd.  Computed (default)
 * as M = (gz2 e)^T mask and N = gz2^T mask with mask = [a1 > 0]: slab += w0 M + b0 N,
 * narrow_sums = (sum_j W2[j][k] M[j][k], sum_j W2[j][k] N[j][k]) -- the same sums regrouped. */
int pdg_edge_enc_bwd(int n_edges, const float* gy, const float* a2, const float* e_in, const float* w0,
                     const float* b0, const pdg_ln_stat* st, const pdg_ln_bwd* lb, const double* lb_pairs,
                     int lb_npairs, const float* ln_g, const float* W2T, float* slabs, double* narrow_sums,
                     int nslabs, int slab_init, void* stream);
/* grad_w0 += sum_b narrow_sums[b][0:128], grad_b0 += sum_b narrow_sums[b][128:256] (block order). */
int pdg_enc_narrow_reduce(const double* narrow_sums, int nslabs, float* grad_w0, float* grad_b0, void* stream);
int pdg_edge_gout_wc(int n_edges, const float* gC, const float* e, const float* ge_next,
                     const float* WcT, float* ge_out, float* slabs, int nslabs, const float* a2ln,
                     const pdg_ln_stat* st_ln, double* ln_partials, const float* ln_g, double* pairs,
                     int accumulate, int slab_init, void* stream);

/* Mesh graph on the device (pdg_graph.hip): FaceToEdge of a triangle
 * mesh (convert_utils.py:47-60), edge lengths (datasets.py:182-188) and, when `periodic`,
 * compute_periodic_graph (datasets.py:39-119), coalesced (rows ascending, columns ascending
 * within a row; attribute = the length for a mesh edge, 0 for a periodic-only pair).
 * points: (n_nodes, dim) fp32, dim 2 or 3 (sides from the first two coordinates); faces:
 * (n_faces, 3) int64.  Outputs edge_rows / edge_cols (int64) / edge_attr (fp32) of
 * `capacity` >= 6 n_faces (+ 4 PDG_SIDE_MAX + 4 when periodic) entries; *n_edges (device
 * int) receives the edge count, or -1 for invalid periodic geometry (opposite sides of
 * different lengths, a corner that is not exactly one node, a side longer than
 * PDG_SIDE_MAX = 4096).  scratch: pdg_mesh_graph_scratch_bytes(n_nodes, n_faces) bytes. */
long pdg_mesh_graph_scratch_bytes(int n_nodes, int n_faces);
int pdg_mesh_graph(int n_nodes, const float* points, int dim, int n_faces, const int64_t* faces,
                   int periodic, int64_t* edge_rows, int64_t* edge_cols, float* edge_attr,
                   long capacity, int* n_edges, void* scratch, long scratch_bytes, void* stream);

/* Backward of the P/Q gathers: gP[v] = sum_{dst-seg(v)} gz1m + sum_{src-seg(v)} gz1e,
 * gQ[v] = sum_{src-seg(v)} gz1m + sum_{dst-seg(v)} gz1e.  src-seg uses rowptr_src and
 * perm_src (positions of the dst-sorted edges grouped by src).  gz1e may be NULL (no
 * edge-update branch).  e_is_sum != 0: the gz1e argument holds gC = gz1m + gz1e instead and
 * each row's gz1e is formed as gC - gz1m in fp32 (the edge backward then stores no gz1e). */
int pdg_pq_scatter_bwd(int n_nodes, const int* rowptr_dst, const int* rowptr_src,
                       const int* perm_src, const float* gz1m, const float* gz1e, int e_is_sum,
                       float* gP, float* gQ, void* stream);

/* Weight gradient of a 128x128 Linear: per-block partial of sum_k G[k]^T X[k] (+ a second
 * pair G2/X2) and of sum_k G[k] (+G2); accumulated (+=) into slab[block] (128*128 + 128 floats),
 * so repeated calls over message-passing steps sum in a fixed order. */
int pdg_wgrad_accum(int rows, const float* G, const float* X, const float* G2, const float* X2,
                    float* slabs, int nslabs, void* stream);
/* grad_W[o*ld + col0 + i] += sum over slabs; grad_b[o] += (if grad_b) sum over slabs.
 * Two fixed-order passes; the slabs are scratch and are overwritten. */
int pdg_wgrad_reduce(float* slabs, int nslabs, float* grad_W, int ld, int col0,
                     float* grad_b, void* stream);
/* Weight gradient of a 128x128 Linear over a list of row segments (all message-passing steps
 * and both edge_net evaluations in one pass): slab[b] = per-block partial of
 * sum_seg sum_k G_seg[k]^T X_seg[k] and of sum G_seg[k] (written, not accumulated);
 * reduce with pdg_wgrad_reduce.  g_ptrs/x_ptrs/rows are HOST arrays of nseg <= PDG_MAX_SEGS entries. */
#define PDG_MAX_SEGS 32
/* Blocks per CU that pdg_wgrad_segments is built for (its nslabs should be this x the CU count). */
int pdg_wgrad_slabs_per_cu(void);
int pdg_wgrad_segments(int nseg, const float* const* g_ptrs, const float* const* x_ptrs, const int* rows,
                       float* slabs, int nslabs, void* stream);
/* Two weight gradients sharing an operand in one pass over nseg row segments (the shared array is
 * read once): shared_x != 0: slabs0 += A0^T A2, slabs1 += A1^T A2 (bias rows: column sums of A0 /
 * A1); shared_x == 0: slabs0 += A0^T A1, slabs1 += A0^T A2 (bias rows: column sums of A0).  The
 * slabs are written (not accumulated), nslabs each, reduced with pdg_wgrad_reduce.  Pointer and
 * row arrays are HOST arrays of nseg <= PDG_MAX_SEGS entries. */
int pdg_wgrad_pairs(int nseg, const float* const* a0_ptrs, const float* const* a1_ptrs, const float* const* a2_ptrs,
                    const int* rows, int shared_x, float* slabs0, float* slabs1, int nslabs, void* stream);
/* Narrow weight gradient: T[c][i] = sum_k Wide[k][c] Narrow[k][i] (c < 128, i < k_narrow <= 8),
 * sums sum_k Wide[k][c] and sum_k Narrow[k][i]; added into grad arrays:
 * transpose == 0: grad_W[c*k_narrow + i] (shape 128 x k), else grad_W[i*128 + c] (k x 128);
 * grad_b_wide[c] += ..., grad_b_narrow[i] += ... (each nullable). */
int pdg_wgrad_narrow(int rows, const float* wide, const float* narrow, int k_narrow, int transpose,
                     double* partials, float* grad_W, float* grad_b_wide, float* grad_b_narrow,
                     void* stream);
/* The finalize step of pdg_wgrad_narrow alone (grad_W / grad_b_* += the reduced block partials, in
 * pdg_wgrad_narrow's order), for partials formed inside pdg_mlp2_bwd_coop / pdg_decoder_bwd_coop. */
int pdg_wgrad_narrow_finalize(const double* partials, int nparts, int k_narrow, int transpose, float* grad_W,
                              float* grad_b_wide, float* grad_b_narrow, void* stream);
/* Every end-of-backward reduction in one launch: n_reduce slab reductions as pdg_wgrad_reduce_batch
 * (<= 16), n_ln LayerNorm groups as pdg_ln_param_grads (<= 4), n_narrow (<= 2) narrow finalizes as
 * pdg_wgrad_narrow_finalize, and (enc_sums != NULL) the edge encoder's first-layer sums as
 * pdg_enc_narrow_reduce.  Bitwise the separate launches' gradients except the encoder sums, which add
 * their rows in another fixed order.  New in this build (the reference's autograd accumulates the
 * parameter gradients in place, gnn_train.py:160-161). */
int pdg_bwd_epilogue(int n_reduce, const float* const* slabs, const int* nslabs, float* const* grad_W,
                     const int* ld, const int* col0, float* const* grad_b, int n_ln, const double* const* ln_acc,
                     const int* ln_rows, float* const* ln_grad_g, float* const* ln_grad_b, int n_narrow,
                     const double* const* narrow_partials, const int* narrow_nparts, const int* narrow_k,
                     const int* narrow_transpose, float* const* narrow_gW, float* const* narrow_gb_wide,
                     float* const* narrow_gb_narrow, const double* enc_sums, int enc_nslabs, float* enc_grad_w0,
                     float* enc_grad_b0, void* stream);

/* ---------------------------------------------------------------- losses */

/* Per-graph normalised MSE (gnn_train.py:41-57) over node segments ptr[0..B]:
 * loss_g = mean_c sum_n (gt-pred)^2 / sum_n (gt - mean gt)^2.  Writes loss[g] and den[g*3+c]. */
int pdg_nmse_fwd(int n_graphs, const int* ptr, const float* gt, const float* pred,
                 float* loss, float* den, void* stream);
/* g_pred[n][c] (+)= scale * (-2/3) (gt-pred)/den_c. */
int pdg_nmse_bwd(int n_graphs, const int* ptr, int n_nodes, const float* gt, const float* pred,
                 const float* den, const float* scale, int accumulate, float* g_pred, void* stream);
/* pdg_nmse_fwd + pdg_nmse_bwd in one launch (bitwise the two): each graph's block also writes its
 * gradient rows from the denominators it just formed. */
int pdg_nmse_fwd_bwd(int n_graphs, const int* ptr, const float* gt, const float* pred, float* loss, float* den,
                     const float* scale, int accumulate, float* g_pred, void* stream);

/* Divergence penalty (gnn_train.py:60-92) with the operator in CSR over global rows and
 * graph-local columns (col < n_i: x-derivative, else y-derivative), ptr = node offsets:
 * div[v] = A_v . [[sxx;sxy],[sxy;syy]], rows with node_type +-1 zeroed, loss_g = mean_v |div|^2. */
int pdg_div_fwd(int n_graphs, const int* ptr, const int* a_rowptr, const int* a_col,
                const float* a_val, const int64_t* node_types, const float* sigma, int reduce_abs,
                float* div, float* loss, void* stream);
/* g_sigma (+)= A^T-weighted grads: uses A^T in CSR (at_rowptr over global nodes, at_row = source
 * row v, at_comp = 0/1 (x/y column block), at_val).  d loss_g / d div = 2 div / n_g ("square")
 * or sign(div) / n_g ("abs"), times *scale. */
int pdg_div_bwd(int n_graphs, const int* ptr, int n_nodes, const int* at_rowptr, const int* at_row,
                const int* at_comp, const float* at_val, const float* div, const float* scale,
                int reduce_abs, int accumulate, float* g_sigma, void* stream);

/* ---------------------------------------------------------------- utilities */
/* out (cols x rows, contiguous) = in^T for a (rows x cols) row-major matrix with row stride ld. */
int pdg_transpose(int rows, int cols, int ld, const float* in, float* out, void* stream);
/* n <= 16 transposes of 128 x 128 blocks in one launch: out_ptrs[i] (128 x 128, row-major) =
 * in_ptrs[i]^T, in_ptrs[i] with row stride lds[i]; host arrays. */
/* Up to 3 pdg_wgrad_segments passes in one launch: job j has nseg[j] segments (its entries of g_ptrs /
 * x_ptrs / rows follow job j-1's) and its own slab set slabs[j] (nslabs slabs each). */
int pdg_wgrad_segments_batch(int njobs, const int* nseg, const float* const* g_ptrs, const float* const* x_ptrs,
                             const int* rows, float* const* slabs, int nslabs, void* stream);
/* Several pdg_wgrad_reduce calls in one launch (njobs <= 16): job i adds the sum of its nslabs[i]
 * slabs into grad_W[i] (row stride ld[i], column offset col0[i]) and, when grad_b[i] != NULL,
 * the bias sums into grad_b[i].  Slab sets must be distinct buffers. */
int pdg_wgrad_reduce_batch(int njobs, const float* const* slabs, const int* nslabs, float* const* grad_W,
                           const int* ld, const int* col0, float* const* grad_b, void* stream);
int pdg_transpose128_batch(int n, const float* const* in_ptrs, const int* lds, float* const* out_ptrs, void* stream);
/* pdg_nonfinite + the zero-mean-stress skip in one launch, no memset: flags[2] double-buffered by call
 * parity; flags[parity] = any non-finite x[i] || (zero_flag && *zero_flag == 0), and flags[parity ^ 1] is
 * cleared for the next call (replaces GradScaler's inf check, gnn_train.py:205-207, and the guard of
 * models.py:294-299; pdg_adam then reads flags + parity as its skip flag). */
int pdg_nonfinite2(const float* x, int64_t n, const float* zero_flag, int* flags, int parity, void* stream);
/* The step's loss scalars (gnn_train.py:189-197) in one launch: out[0] = *zero_flag (1 when NULL),
 * out[1] = scale_nmse * sum_g loss_nmse[g], out[2] = scale_div * sum_g loss_div[g] (0 when loss_div is
 * NULL), out[3] = out[1] + out[2]; fp64 sums in graph order, rounded once. */
int pdg_loss_reduce(int n_graphs, const float* loss_nmse, const float* loss_div, float scale_nmse,
                    float scale_div, const float* zero_flag, float* out, void* stream);
/* Adam as torch.optim.Adam (amsgrad=False, weight_decay=0) stepped by GradScaler.step
 * (gnn_train.py:111,118,204-207) on a flat parameter buffer.  Adam's step count lives on the
 * device: step_count[parity] = optimizer steps taken so far (c); the update uses
 * table[2c] = (float) lr / (1 - beta1^(c+1)) and table[2c+1] = (float) sqrt(1 - beta2^(c+1)), both
 * computed in double on the host as torch does, and writes step_count[parity ^ 1] = c + !skip.
 * When *skip_flag (nullable, device) is set nothing else changes: parameters, moments and the
 * step count stay as they were (GradScaler skips optimizer.step()).  w1 = (float)(1 - beta1),
 * w2 = (float)(1 - beta2) rounded from double.  Requires table_len > c. */
int pdg_adam(int64_t n, float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
             const float* table, int table_len, float w1, float beta2, float w2, float eps,
             const int* skip_flag, int* step_count, int parity, void* stream);

/* ---------------------------------------------------------------- device-side collate (§8f row 1) */
/* One copy job: dst[i] = src[i] (+ add for the integer kinds), i < count.  `src`/`dst` are
 * device pointers; the job table itself lives in device memory (40 bytes per job). */
enum { PDG_COPY_F32 = 0, PDG_COPY_B32 = 1, PDG_COPY_B64 = 2 };
typedef struct pdg_copy_job {
  const void* src;
  void* dst;
  int64_t count;
  int64_t add;
  int32_t kind;
  int32_t pad_;
} pdg_copy_job;
/* Assemble a minibatch from HBM-resident graphs (PyG collate, gnn_train.py:387-394): runs all
 * jobs (njobs <= 65535, the largest count max_count) in one launch. */
int pdg_collate(const pdg_copy_job* jobs, int njobs, long max_count, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* PDIVGNN_H */
