/*
 * eelg.h -- C ABI of the MI355X-native EnergyEquivGNN message-passing hot path.
 *
 * Every entry point takes plain device pointers (fp32 data, int32 indices),
 * sizes and a HIP stream (hipStream_t passed as void*), launches asynchronously
 * on that stream and returns 0 on success or a negative code; the message of
 * the last failure on the calling thread is in eelg_last_error().  Nothing here
 * allocates, frees or synchronises, so every call can be captured in a hipGraph.
 *
 * Layout conventions (reference: gnn/datasets.py:256-269, e3nn mul-major rows):
 *   node features   [N, sum_l mul*(2l+1)]   block (mul, l) laid out [mul][2l+1]
 *   edge SH         [E, (lmax+1)^2] in rows padded to a multiple of 4 floats (row stride
 *                   nshp = round_up((lmax+1)^2, 4): 28 for lmax 4, 16 for lmax 3)
 *   TP weights      [E, npaths*mul]          index = path*mul + channel
 *   edges           receiver-sorted; rowptr[N+1] is the receiver CSR,
 *                   sperm/srowptr the sender CSR over the same edge order.
 *
 * Which reference interface each entry point replaces is given per function.
 */
#ifndef EELG_H
#define EELG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Library / error handling ------------------------------------------------ */
const char* eelg_version(void);
const char* eelg_last_error(void);

/* Config discovery: the irreps-specialised kernels are looked up by name
 * ("tpA_l4" = 32x0e node irreps, "tpB_l4" = 32x0e+..+32x4e, "sc_l4_c3" ...).
 * info receives {din, dmid, weight_numel, nsh, ngroups, npaths, lmax};
 * sig is a structural hash the host re-derives to detect a stale build. */
int eelg_tp_find(const char* name);
int eelg_tp_info(int cfg, int* info7, uint64_t* sig);
/* info receives {D, x_row, out_row, nterms, n_term_groups, D_out, coef_chunk, coef_ld}
 * (D: coupling components per channel of the input, D_out: of the output; they differ when the
 * product maps the SH-lmax interaction irreps onto wider hidden irreps; coef_chunk: the node
 * chunk of eelg_sc_bwd_coef; coef_ld: the row stride of the coefficient matrix, nterms rounded
 * up to a multiple of 16, so every channel row starts on a 64-byte line) */
int eelg_sc_find(const char* name);
int eelg_sc_info(int cfg, int* info8, uint64_t* sig);

/* Edge geometry + embeddings.
 * Replaces get_edge_vectors_and_lengths (gnn/mace.py:338-352),
 * soft_one_hot_linspace x2 + cat (gnn/model.py:146-156) and
 * o3.SphericalHarmonics(lmax, normalize=True, 'component') (gnn/model.py:126-129,157).
 * sh[E, nshp] (padded rows, pad zeroed), feats[E, 2*nb] =
 * [gauss(len; 0..len_end) | gauss(radius; 0..rad_end)]. */
int eelg_edge_embed(const float* pos, const int* sender, const int* receiver, const float* shifts,
                    const float* radius, int n_edges, int lmax, int nb, float len_end,
                    float rad_end, float* sh, float* feats, void* stream);

/* Fused interaction: agg[n] = inv_norm * sum_{e: recv(e)=n} TP_uvu(x[sender(e)], sh[e], w[e]).
 * Replaces conv_tp(node_feats[sender], edge_attrs, tp_weights) followed by
 * scatter(..., reduce='sum') / agg_norm_const (gnn/blocks.py:591-597).
 * x, sh and w must be 16-byte aligned (the rows travel by LDS-DMA in 16-B pieces); -2 otherwise. */
int eelg_tp_fwd(int cfg, const float* x, const float* sh, const float* w, const int* sender,
                const int* rowptr, int n_nodes, float inv_norm, float* agg, void* stream);

/* Backward of eelg_tp_fwd: grad_w[E, weight_numel] and per-edge grad of
 * x[sender] gxe[E, din] (to be summed per sender with eelg_segment_sum_csr). */
int eelg_tp_bwd(int cfg, const float* x, const float* sh, const float* w, const int* sender,
                const int* receiver, int n_edges, const float* grad_agg, float inv_norm,
                float* grad_w, float* gxe, void* stream);

/* BASELINE config 5 (bf16 storage, fp32 arithmetic): eelg_tp_fwd / eelg_tp_bwd with the
 * edge-sized tensors w, grad_w [E, weight_numel] and gxe [E, din] held as bf16 bit patterns
 * (uint16, round-to-nearest-even on store).  Same reference call sites
 * (gnn/blocks.py:590-597).  eelg_tp_fwd_bf16 moves rows by LDS-DMA like eelg_tp_fwd: x, sh
 * and w must be 16-byte aligned; -2 otherwise. */
int eelg_tp_fwd_bf16(int cfg, const float* x, const float* sh, const void* w, const int* sender,
                     const int* rowptr, int n_nodes, float inv_norm, float* agg, void* stream);
int eelg_tp_bwd_bf16(int cfg, const float* x, const float* sh, const void* w, const int* sender,
                     const int* receiver, int n_edges, const float* grad_agg, float inv_norm,
                     void* grad_w, void* gxe, void* stream);

/* eelg_tp_bwd / eelg_tp_bwd_bf16 with gxe written in sender order: the gxe row of edge e
 * is spos[e] (spos = inverse of the sender-CSR permutation sperm), so the sender sum
 * (eelg_segment_sum_csr with idx = NULL over srowptr) reads gxe contiguously.  Same
 * reference call sites (gnn/blocks.py:591-597). */
int eelg_tp_bwd_sorted(int cfg, const float* x, const float* sh, const float* w, const int* sender,
                       const int* receiver, const int* spos, int n_edges, const float* grad_agg,
                       float inv_norm, float* grad_w, float* gxe, void* stream);
int eelg_tp_bwd_sorted_bf16(int cfg, const float* x, const float* sh, const void* w,
                            const int* sender, const int* receiver, const int* spos, int n_edges,
                            const float* grad_agg, float inv_norm, void* grad_w, void* gxe,
                            void* stream);

/* Backward of eelg_tp_fwd in sender order: one pass over the sender CSR (srowptr [N+1],
 * sperm [E] = edge ids sorted by sender) that writes grad_w[E, weight_numel] at each edge's
 * row and grad_x[N, din] summed per sender in registers -- eelg_tp_bwd + the sender
 * eelg_segment_sum_csr in one launch, without the gxe [E, din] intermediate.  Same
 * reference call sites (gnn/blocks.py:591-597, the autograd of conv_tp + scatter).
 * _bf16: w / grad_w as bf16 bit patterns; grad_x is fp32 either way. */
int eelg_tp_bwd_sender(int cfg, const float* x, const float* sh, const float* w, const int* sperm,
                       const int* srowptr, const int* receiver, int n_nodes,
                       const float* grad_agg, float inv_norm, float* grad_w, float* grad_x,
                       void* stream);
int eelg_tp_bwd_sender_bf16(int cfg, const float* x, const float* sh, const void* w,
                            const int* sperm, const int* srowptr, const int* receiver,
                            int n_nodes, const float* grad_agg, float inv_norm, void* grad_w,
                            float* grad_x, void* stream);

/* Fused backward of linear(tp_interaction(x, sh, w)) -- the interaction's output o3.Linear
 * (7360 -> 800 at lmax 4) and the fused TP + scatter -- w.r.t. x and w, from the linear's output
 * gradient gy [n_nodes, target dim] and its flat weight lin_w (16-B aligned).  Replaces the
 * linear's grad-x followed by eelg_tp_bwd (gnn/blocks.py:591-604 autograd): grad_agg is computed
 * per receiver tile into LDS and never written to HBM.  Writes grad_w [E, wn] and the per-edge
 * grad_x rows gxe [E, din] in receiver-sorted edge order, as eelg_tp_bwd; rowptr is the receiver
 * CSR (int32 [n_nodes + 1]) and receiver the sorted edges' receivers (int32 [E]).  Generated for mul 32; returns -2 for other configs.  The linear
 * is o3.Linear(irreps_mid.simplify(), target): eelg_tp_bwf_slot returns, per TP slot, the
 * weight offset of its 32 x 32 block, its alpha and its gy offset, for the caller to check
 * against its own linear before using this path. */
int eelg_tp_bwd_fused(int cfg, const float* x, const float* sh, const float* w, const int* sender,
                      const int* receiver,
                      const int* rowptr, int n_nodes, const float* gy, const float* lin_w,
                      float inv_norm, float* grad_w, float* gxe, void* stream);
int eelg_tp_bwd_fused_bf16(int cfg, const float* x, const float* sh, const void* w,
                           const int* sender, const int* receiver, const int* rowptr,
                           int n_nodes, const float* gy,
                           const float* lin_w, float inv_norm, void* grad_w, void* gxe,
                           void* stream);
int eelg_tp_bwf_slot(int cfg, int slot, int* w_off, float* alpha, int* gy_off);

/* CSR segmented sum (deterministic, no atomics):
 * out[r, :] = scale * row_scale[r] * sum_{j in [rowptr[r], rowptr[r+1])} src[idx ? idx[j] : j, :].
 * Replaces torch_scatter.scatter(..., reduce='sum'|'mean') (gnn/blocks.py:595-597,
 * gnn/model.py:100-106) on sorted segments; row_scale may be NULL. */
int eelg_segment_sum_csr(const float* src, const int* rowptr, const int* idx,
                         const float* row_scale, float scale, int n_rows, int width, float* out,
                         void* stream);

/* eelg_segment_sum_csr over bf16 source rows (bit patterns), fp32 accumulation and output:
 * the sender sums of the bf16 per-edge gradient gxe (config 5). */
int eelg_segment_sum_csr_bf16(const void* src, const int* rowptr, const int* idx,
                              const float* row_scale, float scale, int n_rows, int width,
                              float* out, void* stream);

/* Few long segments (per-graph pooling): each segment is cut into n_split pieces summed
 * separately into work[n_rows, n_split, width], then combined in a fixed order:
 * out[r, :] = scale * row_scale[r] * sum_pieces.  Same result contract as
 * eelg_segment_sum_csr (gnn/model.py:100-106 global mean pool), without the
 * one-wave-per-segment serialisation. */
/* Gate nonlinearity of the readout (e3nn nn.Gate, gnn/blocks.py:268-273): rows
 * x = [scalars | gates | gated blocks], y = [cst*silu(scalars) | gated block b channel u
 * times cst*silu(gate of (b, u))], cst = normalize2mom(silu).  blk_mul / blk_dim: the gated
 * blocks (mul copies of a (2l+1)-dim irrep, in row order); n_gates = sum of blk_mul.
 * eelg_gate_bwd writes grad_x for grad_y (one fused pass instead of the split / mul / cat and
 * their backward in torch). */
#define EELG_GATE_MAXBLK 8
#define EELG_GATE_MAXGATED 2048   /* gated elements per row (the kernels' LDS lookup tables) */
#define EELG_GATE_MAXGATES 512
typedef struct { int n_scal, n_gates, n_blk, pad; int blk_mul[EELG_GATE_MAXBLK]; int blk_dim[EELG_GATE_MAXBLK]; } eelg_gate_desc;
int eelg_gate_fwd(const float* x, int n_nodes, const eelg_gate_desc* desc, float cst, float* y,
                  void* stream);
int eelg_gate_bwd(const float* x, const float* grad_y, int n_nodes, const eelg_gate_desc* desc,
                  float cst, float* grad_x, void* stream);

int eelg_segment_sum_split(const float* src, const int* rowptr, const int* idx,
                           const float* row_scale, float scale, int n_rows, int width, int n_split,
                           float* work, float* out, void* stream);

/* torch_scatter's order reductions over CSR segments of src rows (rows rowptr[r]..rowptr[r+1]):
 * op 0 = max, 1 = min, 2 = mul.  Replaces scatter(..., reduce='max'|'min'|'mul') for
 * interaction_reduction (gnn/blocks.py:595-597, on the per-edge messages in receiver order)
 * and global_reduction (gnn/model.py:100-106, on the readout rows in graph order).
 * out[r, c]: the segment's first maximum / minimum (strict compare, so ties keep the earliest
 * row, torch_scatter's CPU arg) or its product; an empty segment gives 0 (max / min) or 1 (mul).
 * arg[r, c] (max / min only, required): the row of the kept element, -1 for an empty segment. */
int eelg_segment_order(const float* src, const int* rowptr, int n_rows, int width, int op,
                       float* out, int* arg, void* stream);
/* Backward: grad_src for every row of every segment (rows outside all segments are not
 * written): max / min -> grad_out at arg, 0 elsewhere (the whole gradient to one element, as
 * torch_scatter's scatter_max / scatter_min); mul -> grad_out times the product of the
 * segment's other entries (prefix x suffix products, exact at zeros).
 * Deliberate differences from torch_scatter on CUDA (parity unpinned, the oracle's torch.prod /
 * torch.max agree with these kernels): scatter_mul's backward divides the product by src, so
 * an entry that is exactly 0 gives NaN/inf there and a finite gradient here; scatter_max /
 * scatter_min on CUDA pick the arg of a tie by an atomic race, here it is always the first. */
int eelg_segment_order_bwd(const float* src, const int* rowptr, const int* arg, const float* grad_out,
                           int n_rows, int width, int op, float* grad_src, void* stream);

/* Crystal-graph edge convolution (CGC/mCGC benchmark models): replaces
 *   c = cat([x[sender], x[receiver], edge_ft]); msg = softplus(fc_values(c)) * sigmoid(fc_multip(c));
 *   scatter(msg, receiver, reduce)          (scripts/benchmark_models/cgc_modified.py:20-25,
 *                                            cgc_vanilla.py:20-25, gnn/blocks.py:960-966)
 * with the linear split by input block: ps = x W_s^T, pr = x W_r^T + b ([N, 2D], values
 * then multipliers), ep = edge_ft W_e^T ([E, 2D], receiver-sorted edge order).
 * agg[n] = row_scale[n] * sum_e softplus(zv) sigmoid(zm)  (row_scale NULL -> 'sum').
 * Built for D <= EELG_CGC_MAXD (the benchmark models use 128 and 64); -2 otherwise. */
#define EELG_CGC_MAXD 256   /* node_dim of the built CGC kernels (one lane per 64 channels, <= 4) */
int eelg_cgc_fwd(const float* ps, const float* pr, const float* ep, const int* sender,
                 const int* rowptr, const float* row_scale, int n_nodes, int D, float* agg,
                 void* stream);
/* Backward: dz[E, 2D] = d agg / d z per edge and grad_pr[N, 2D] = receiver sums of dz;
 * the sender sums are eelg_segment_sum_csr(dz, srowptr, sperm).  D <= EELG_CGC_MAXD as the forward. */
int eelg_cgc_bwd(const float* ps, const float* pr, const float* ep, const int* sender,
                 const int* rowptr, const float* row_scale, int n_nodes, int D,
                 const float* grad_agg, float* dz, float* grad_pr, void* stream);
/* The same edge convolution with factored edge features (both reference models embed the 5
 * per-edge inputs with one Linear, cgc_modified.py:71-74 / cgc_vanilla.py:60-63, so
 * Ep = [e5 | 1] A): ef[E, 8] = [e5 | 1 | 0 | 0] in CSR edge order and ea[8, 2D] (rows 0..5:
 * A = [W5^T W_e^T ; b5 W_e^T], rows 6..7 unused) replace ep[E, 2D]; the kernels form Ep in
 * registers.  Same outputs as eelg_cgc_fwd / eelg_cgc_bwd on Ep = ef[:, :6] @ ea[:6].
 * receiver[E] (the CSR's receiver of each sorted edge; may be NULL) enables the receiver-
 * streaming kernels: a wave walks the edges of 8 consecutive receivers in batches of 8, the
 * next batch's loads in flight (EELG_CGC_STREAM bit 0 forward, bit 1 backward; default 2). */
int eelg_cgc_fwd_ef(const float* ps, const float* pr, const float* ef, const float* ea,
                    const int* sender, const int* receiver, const int* rowptr,
                    const float* row_scale, int n_nodes, int D, float* agg, void* stream);
/* The factored forward with the layer residual added in the store (round 5):
 * agg[n] = row_scale[n] sum_e msg_e + res[n] (res [N, D], the layer input h of
 * h + conv(h), cgc_modified.py:77 / cgc_vanilla.py:69; NULL: no residual). */
int eelg_cgc_fwd_ef_res(const float* ps, const float* pr, const float* ef, const float* ea,
                        const int* sender, const int* rowptr, const float* row_scale, int n_nodes,
                        int D, const float* res, float* agg, void* stream);
int eelg_cgc_bwd_ef(const float* ps, const float* pr, const float* ef, const float* ea,
                    const int* sender, const int* receiver, const int* rowptr,
                    const float* row_scale, int n_nodes, int D, const float* grad_agg, float* dz,
                    float* grad_pr, float* dea_part, void* stream);
/* dea_part (may be NULL; needs receiver): per-workgroup partials [eelg_cgc_bwd_ef_parts(n), 6, 2D]
 * of d ea[0..5] = ef[:, :6]^T dz, summed by the caller (deterministic); a workgroup covers
 * 4 * EELG_CGC_RPW receivers. */
#define EELG_CGC_RPW 8
int eelg_cgc_bwd_ef_parts(int n_nodes);

/* Sparse (CSR) x dense with strided operands:
 * out[r*ldo_r + c*ldo_c] = sum_{j in row r} val[j] * B[col[j]*ldb_r + c*ldb_c].
 * Builds the symmetric-contraction coefficients coef = U_sym . W and their weight
 * gradient U_sym^T . g (U_sym 1.6 % dense; replaces the dense U.W contraction of
 * gnn/mace.py:242-277 at the weight level). */
int eelg_csr_spmm(const int* rowptr, const int* col, const float* val, int n_rows, const float* B,
                  int ldb_r, int ldb_c, int n_cols, float* out, int ldo_r, int ldo_c, void* stream);

/* Symmetric contraction (correlation 3) as a sparse polynomial per (node, channel).
 * Replaces SymmetricContraction.forward (gnn/mace.py:173-177, 242-277).
 * x, out: [N, mul*D] mul-major rows; coef: [mul, coef_ld] (info[7]; entries past nterms are
 * read but unused), 16-byte aligned: each wave streams its channel's row into LDS by LDS-DMA in
 * 16-B pieces.  The row tensors (x, out, grad_out, grad_x) must be 16-byte aligned (float4 row
 * access); a misaligned pointer returns -2. */
int eelg_sc_fwd(int cfg, const float* x, const float* coef, int n_nodes, int mul, float* out,
                void* stream);
int eelg_sc_bwd_x(int cfg, const float* x, const float* coef, const float* grad_out, int n_nodes,
                  int mul, float* grad_x, void* stream);
/* eelg_sc_bwd_x that also writes the channel-major copies xt[(c*D + a)*N + n] of x and
 * gt[(c*D_out + q)*N + n] of grad_out (the operands of eelg_sc_bwd_coef) from the tiles it
 * stages anyway, replacing two eelg_sc_cmajor passes; xt / gt may be NULL. */
int eelg_sc_bwd_x_cm(int cfg, const float* x, const float* coef, const float* grad_out,
                     int n_nodes, int mul, float* grad_x, float* xt, float* gt, void* stream);
/* Channel-major copy xt[(c*D + a)*N + n] of a mul-major row tensor (feeds sc_bwd_coef);
 * which = 0: input (coupling) layout, 1: output layout. */
int eelg_sc_cmajor(int cfg, int which, const float* x, int n_nodes, int mul, float* xt,
                   void* stream);
/* Coefficient gradient (replaces the weight gradient through the U.W contraction of
 * gnn/mace.py:242-277) from the channel-major copies xt[(c*D + a)*N + n] / gt of x and
 * grad_out (eelg_sc_bwd_x_cm or eelg_sc_cmajor).  partial[n_parts, mul, coef_ld] (the
 * entries past nterms of each row are not written), n_parts = eelg_sc_bwd_coef_parts(cfg,
 * n_nodes, mul): one partial per node range (streaming kernel: ranges of whole coef_chunk-node
 * chunks, about 1024 / (mul x term-group sets) of them and at least 2048 nodes each; round-5
 * chunk kernel: one per coef_chunk nodes).  chunk must be the
 * config's coef_chunk (info[6]).  The caller sums over the partials (deterministic).
 * Non-overlapping xt / gt; 16-byte aligned rows (n_nodes % 4 == 0) take the LDS-DMA path. */
int eelg_sc_bwd_coef(int cfg, const float* xt, const float* gt, int n_nodes,
                     int mul, int chunk, float* partial, void* stream);
/* The number of partial rows eelg_sc_bwd_coef writes for n_nodes (-1: unknown config). */
int eelg_sc_bwd_coef_parts(int cfg, int n_nodes, int mul);

/* Symmetric contraction from a term table (correlation 4: U_matrix_real with filter_ir_mid,
 * gnn/mace.py:435-477; the contraction itself gnn/mace.py:242-277).  Replaces
 * SymmetricContraction.forward for the structures without generated kernels.
 * terms[t]: four 8-bit component indices (slot k at bits 8k; an unused slot = D, a constant 1),
 * sorted by output component, desc.orow[q] .. orow[q+1]-1 the terms of output q.  Component a of
 * channel c of node n: x[n*ldx + xb[a] + c*xs[a]]; outputs likewise (ob, os, ldo).
 * coef [mul, ldc], ldc a multiple of 64 >= nterms.  eelg_scg_bwd_coef writes deterministic
 * partials [ceil(n_nodes / EELG_SCG_CHUNK), mul, ldc] (term_out[t]: output of term t; padding
 * terms t >= nterms need indices D and output Dout: they produce 0); the caller sums them. */
#define EELG_SCG_MAXD 25
#define EELG_SCG_CHUNK 256
typedef struct {
  int D, Dout, mul, nterms;
  int xb[EELG_SCG_MAXD], xs[EELG_SCG_MAXD];
  int ob[EELG_SCG_MAXD], os[EELG_SCG_MAXD];
  int orow[EELG_SCG_MAXD + 1];
} eelg_scg_desc;
int eelg_scg_fwd(const eelg_scg_desc* d, const unsigned* terms, const float* x, int ldx, const float* coef,
                 int ldc, int n_nodes, float* out, int ldo, void* stream);
int eelg_scg_bwd_x(const eelg_scg_desc* d, const unsigned* terms, const float* x, int ldx, const float* coef,
                   int ldc, const float* grad_out, int ldg, int n_nodes, float* grad_x, void* stream);
int eelg_scg_bwd_coef(const eelg_scg_desc* d, const unsigned* terms, const int* term_out, int ldc, const float* x,
                      int ldx, const float* grad_out, int ldg, int n_nodes, float* partial, void* stream);

/* Channel-mixing linear on mul-major irreps rows (o3.Linear, gnn/blocks.py:516-521,
 * 553-559,471-476; gnn/model.py:82-86), fp32 MFMA.  A descriptor lists output
 * slots; each slot sums alpha * x_block @ W over its sources, W element
 * B[k][j] = w[w_off + k*ldk + j*ldj] (ldk = n_out, ldj = 1 forward; swapped for
 * grad-x), plus bias[bias_off + j] on scalar slots (bias_off < 0: none). */
#define EELG_LIN_MAXSRC 4
#define EELG_LIN_MAXSLOT 8
typedef struct { int x_off, k, w_off, ldk, ldj; float alpha; } eelg_lin_src;
typedef struct { int y_off, n_out, d, bias_off, n_src; eelg_lin_src src[EELG_LIN_MAXSRC]; } eelg_lin_slot;
typedef struct { int n_slots, max_jt, max_rows, pad; eelg_lin_slot slot[EELG_LIN_MAXSLOT]; } eelg_lin_desc;
int eelg_linear_fwd(const float* x, int x_row, const float* w, const float* bias, int n_nodes,
                    float* y, int y_row, const eelg_lin_desc* desc, void* stream);
/* eelg_linear_fwd plus a residual res (y's layout, may be NULL) added in the epilogue:
 * y = linear(x) + res, the layer residual h + layer_i(h) of gnn/model.py:92-96 with the
 * product block's o3.Linear (gnn/blocks.py:486) producing layer_i(h). */
int eelg_linear_fwd_res(const float* x, int x_row, const float* w, const float* bias,
                        const float* res, int n_nodes, float* y, int y_row,
                        const eelg_lin_desc* desc, void* stream);

/* The same linear on bf16 MFMA with fp32-accurate split operands (three exact bf16 parts of
 * every fp32 operand, six part products accumulated in fp32).  The weights come
 * pre-split by eelg_linear_pack for this descriptor: pack = bf16 [3][P], P =
 * eelg_linear_pack_size(desc) = sum over slots of n_out * (summed source K), entry
 * [p][off_slot + j*K_slot + k] = part p of alpha * W[k][j] (ldk / ldj of the descriptor, so a
 * grad-x descriptor packs W^T).  The packed path needs every slot to have whole 32-wide K
 * chunks and column tiles, d in {1,3,5,7,9} and 16-byte aligned rows / pack / res; else -2.
 * Replaces the same o3.Linear calls as eelg_linear_fwd_res. */
long long eelg_linear_pack_size(const eelg_lin_desc* desc);
int eelg_linear_pack(const float* w, const eelg_lin_desc* desc, void* pack, void* stream);
int eelg_linear_fwd_pk(const float* x, int x_row, const void* pack, const float* bias,
                       const float* res, int n_nodes, float* y, int y_row,
                       const eelg_lin_desc* desc, void* stream);

/* grad of the weights: partial[p, w_off + u*n_out + j] over node slices p of
 * nodes_per_slice nodes (sum over p on the caller side; deterministic).
 * n_partial must be >= ceil(n_nodes / nodes_per_slice). */
#define EELG_LINW_MAXINS 8
typedef struct { int x_off, k, g_off, n_out, d, w_off; float alpha; } eelg_linw_ins;
typedef struct { int n_ins, max_jt, max_ut, max_rows; eelg_linw_ins ins[EELG_LINW_MAXINS]; } eelg_linw_desc;
int eelg_linear_bwd_w(const float* x, int x_row, const float* g, int g_row, int n_nodes,
                      int nodes_per_slice, float* partial, int n_partial, int w_total,
                      const eelg_linw_desc* desc, void* stream);
/* Dense weight gradient (a Linear y = x W^T, x [n_rows, k] row stride ldx, g = dL/dy [n_rows,
 * n_out] row stride ldg) on bf16 MFMA with fp32-accurate split operands (round 5; the weight
 * gradients of the CGC models' Linear layers, cgc_modified.py:11-25):
 * partial[s, j, kk] = sum over the rows r of split s (tiles_per_split 32-row tiles) of
 * g[r, j] x[r, kk], s < ceil(ceil(n_rows / 32) / tiles_per_split); the caller sums over s
 * (eelg_sum_rows) to grad W [n_out, k] in torch layout.  k in {32, 64, 96, 128}; -2 otherwise. */
int eelg_linear_bwd_w_x6(const float* g, int ldg, const float* x, int ldx, int n_rows, int n_out,
                         int k, int tiles_per_split, float* partial, void* stream);

/* Radial MLP of the interaction block, fused (gnn/blocks.py:537-549, applied at :590):
 *   [Linear(n_feat -> hidden) + SiLU] + ([Linear(hidden -> hidden) + SiLU]) * (n_hidden - 1)
 *   + Linear(hidden -> n_out, no bias)
 * on edge features feats[E, n_feat].  The hidden layers run on fp32 MFMA; the output layer and
 * its gradients on bf16 MFMA with fp32-accurate operand splitting (each fp32 operand = three
 * bf16 parts exactly, six part products accumulated in fp32; eelg_split_bf16x3).  Built for
 * hidden 32 / 64, n_hidden 1..3, n_feat <= 32, n_out a multiple of 8 (the reference default is
 * 12 -> 64 -> 64 -> weight_numel).  w / b: the hidden Linear weights [hidden, in] and biases
 * [hidden] in torch layout.  Forward: out[E, n_out] (fp32, or bf16 bit patterns when out_bf16)
 * and the pre-activations zsave[n_hidden, E, hidden] (the backward's operand); wo_parts =
 * eelg_split_bf16x3 of W_o [n_out, hidden] (bf16 [3][n_out][hidden], 16-byte aligned). */
#define EELG_RADIAL_MAXH 3
typedef struct {
  int n_feat, hidden, n_hidden, n_out;
  const float* w[EELG_RADIAL_MAXH];
  const float* b[EELG_RADIAL_MAXH];
} eelg_radial_desc;
int eelg_radial_fwd(const float* feats, int n_edges, const eelg_radial_desc* d, const void* wo_parts,
                    int out_bf16, float* zsave, void* out, void* stream);
/* parts[p*n + i] (bf16 bit patterns, p = 0..2): src[i] = parts[i] + parts[n+i] + parts[2n+i]
 * exactly (truncation split: the top 8 significant bits, the next 8, the rest). */
int eelg_split_bf16x3(const float* src, long long n, void* parts, void* stream);
/* Partial-buffer sizes of eelg_radial_bwd for E edges: part_h has n_part rows of
 * hidden*n_feat + hidden + (n_hidden-1)*(hidden^2 + hidden) floats (grad W_0, grad b_0, grad W_1,
 * ... in torch layout); part_wo is [n_split, n_out, hidden]. */
int eelg_radial_plan(int n_edges, int n_out, int* n_part, int* n_split);
/* Backward from grad_w[E, n_out] (fp32, or bf16 when grad_bf16; 16-byte aligned); wot_parts =
 * eelg_split_bf16x3 of W_o^T [hidden, n_out] (bf16 [3][hidden][n_out]):
 * per-wave / per-split partials of every weight and bias gradient; the caller sums part_h
 * and part_wo over their first axis (deterministic).  grad_h[E, hidden] is workspace (it
 * receives grad_w W_o).  No gradient w.r.t. feats (the reference's edge features carry
 * none). */
int eelg_radial_bwd(const void* grad_w, int grad_bf16, int n_edges, const eelg_radial_desc* d,
                    const void* wot_parts, const float* zsave, const float* feats, float* grad_h,
                    float* part_h, float* part_wo, void* stream);
/* The same backward with the hidden-layer weight and bias gradients left to the caller (hidden
 * 64): grad_h as above; gz[n_hidden, E, 64] = grad of the pre-activations z_n; hin[n_hidden - 1,
 * E, 64] = the inputs SiLU(z_{n-1}) of the hidden layers n >= 1; part_wo as above.  The caller
 * forms grad W_n = gz_n^T hin_n (n >= 1), grad W_0 = gz_0^T feats and grad b_n = column sums of
 * gz_n (eelg_linear_bwd_w / eelg_sum_rows). */
int eelg_radial_bwd_chain(const void* grad_w, int grad_bf16, int n_edges, const eelg_radial_desc* d,
                          const void* wot_parts, const float* zsave, float* grad_h, float* gz,
                          float* hin, float* part_wo, void* stream);

/* Deterministic sum over the leading dimension of partial results (the partial buffers of
 * eelg_linear_bwd_w, eelg_radial_bwd and eelg_sc_bwd_coef, and the bias gradients = column
 * sums of grad_out; replaces the reference's implicit autograd reductions, gnn/blocks.py and
 * e3nn o3.Linear biases): out[c] = scale * sum_{r < rows} part[r*ld + c] for c < cols, rows
 * summed in a fixed order.  rows > 256 needs a workspace of eelg_sum_rows_work(rows, cols)
 * floats (0 otherwise).  16-byte aligned part / out with ld, cols multiples of 4 take the
 * float4 path.  -2 on bad sizes. */
long long eelg_sum_rows_work(int rows, long long cols);
int eelg_sum_rows(const float* part, long long ld, int rows, long long cols, float scale, float* out,
                  float* work, long long work_len, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* EELG_H */
