/* C2DSR MI355X (gfx950) kernel library — C ABI.
 *
 * Drop-in boundary for the C2DSR per-step training path.  The
 * reference (crystal22/C2DSR) is pure PyTorch: its "operator interface" is the
 * ATen calls made from models/C2DSR.py, models/encoders.py and trainer.py.  Each
 * entry point below replaces the ATen work of one reference site (cited per
 * function); the host-side mirror of the reference's module API
 * (c2dsr_amd/models/C2DSR.py, c2dsr_amd/models/encoders.py, c2dsr_amd/trainer.py)
 * reaches them through the PyTorch-ROCm operator library libc2dsr_torch.so (TORCH_LIBRARY c2dsr / c2dsr_raw,
 * c2dsr_amd/csrc_torch/).  See INTEGRATION.md.
 *
 * Conventions: plain device pointers (fp32 unless stated, int64 index tensors as
 * the reference's LongTensors), row-major, sizes as ints; `stream` is a
 * hipStream_t passed as void*.  Every function is asynchronous on `stream` and
 * returns 0 or a hipError_t code (hipErrorInvalidValue = 1 for bad shapes).
 * Dropout (where a `p` appears) uses the stateless counter hash
 * h(q) = lowbias32(lowbias32(lo(q)^k0) ^ hi(q) ^ k1) for the element pair q = idx >> 1 and
 * keep(idx) = ((h(q) >> 16·(idx & 1)) & 0xffff) >= floor(p·2^16), scale 1/(1-p); (k0,k1) come from
 * (seed, step, site) — see c2dsr_amd/dropout.py.
 */
#ifndef C2DSR_H
#define C2DSR_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* K1 GCN propagation, CSR SpMM with fused dropout / mean.
 * Replaces models/encoders.py:42-48 (F.dropout, torch.spmm, torch.stack(...).mean) as
 * called by models/C2DSR.py:59-62, and its backward (CSR of Aᵀ, mask_on_output=1).
 *   P[i] = Σ_e val[e]·(Mask⊙X)[col[e]];  Y[i] = alpha·P[i] + (beta + (i!=pad_row ? delta : 0))·Z[i] + gamma·Y[i];
 *   Y2[i] = P[i] (optional).
 * work: int32 [n_work][4] = {row, e_begin, e_end, slot} (slot -1: whole row); split: int32
 * [n_split][4] = {row, slot_begin, slot_end, 0} for rows cut into pieces; part: fp32 [n_slots][d]. */
int c2dsr_gcn_spmm(const int* work, int n_work, const int* split, int n_split, float* part, const int* col,
                   const float* val, int d, const float* X, uint32_t k0, uint32_t k1, float p, int mask_on_output,
                   float alpha, const float* Z, float beta, float delta, int pad_row, float gamma, float* Y, float* Y2,
                   void* stream);
/* The same on bf16 tables X, Z, Y, Y2 (fp32 arithmetic and partial slab, RNE stores): the C5 roofline run's
 * [20M, 512] tables ("bf16 tables"). */
int c2dsr_gcn_spmm_b16(const int* work, int n_work, const int* split, int n_split, float* part, const int* col,
                       const float* val, int d, const void* X, uint32_t k0, uint32_t k1, float p, int mask_on_output,
                       float alpha, const void* Z, float beta, float delta, int pad_row, float gamma, void* Y, void* Y2,
                       void* stream);

/* K2 embedding fuse.  Replaces models/C2DSR.py:65-71,81-82 + models/encoders.py:30-31:
 *   X[r] = drop((H[seq[r]] + E[seq[r]])·scale + P[pos[r]])      (Xin == NULL)
 *   X[r] = drop(Xin[r] + P[pos[r]])                              (Xin != NULL: SelfAttention.forward)
 * dropout index (idx_base + r)·d + c.
 * Index contract (F.embedding raises IndexError outside [0, N)): seq[r] must lie in [0, n_items) (H / E have
 * n_items rows; unused when Xin != NULL) and pos[r] in [0, n_pos).  An index outside sets C2DSR_IDX_ERR_ITEM /
 * C2DSR_IDX_ERR_POS in *err (atomic OR; err may be NULL) and row 0 is read instead: no load leaves the tables.
 * The caller reads the word at its next host sync and raises (c2dsr_amd/trainer.py check_index_errors). */
#define C2DSR_IDX_ERR_ITEM 1   /* an item index (seq / negative sequence) outside [0, n_items) */
#define C2DSR_IDX_ERR_POS 2    /* a position outside [0, n_pos) */
#define C2DSR_IDX_ERR_PLAN 4   /* an index-plan key outside [0, n_keys) (never followed by the segment sums) */
#define C2DSR_IDX_ERR_TARGET 8 /* a classifier target outside [0, n_items] (n_items = ignore_index) */
int c2dsr_embed_fwd(const int64_t* seq, const int64_t* pos, int n_rows, int d, const float* H, const float* E,
                    const float* Xin, const float* P, float scale, uint32_t k0, uint32_t k1, float p,
                    int64_t idx_base, float* X, int n_items, int n_pos, int* err, void* stream);
/* The gather form on chosen rows only (the row-subset encoder layer of a training pass, c2dsr::encoder_pass): output
 * row k = the row above for input row q_idx[k] (k < nq) or k_idx[k - nq] (its query rows, then its padding-key rows),
 * dropout index (idx_base + input row)·d + c; X [nq + nk, d] — the [n_rows, d] embedding is never stored.
 * Replaces the same sites as c2dsr_embed_fwd (models/C2DSR.py:65-71, encoders.py:30-31). */
int c2dsr_embed_fwd_rows(const int64_t* seq, const int64_t* pos, int n_rows, int d, const float* H, const float* E,
                         const float* P, float scale, uint32_t k0, uint32_t k1, float p, int64_t idx_base,
                         const int* q_idx, int nq, const int* k_idx, int nk, float* X, int n_items, int n_pos,
                         int* err, void* stream);
size_t c2dsr_embed_bwd_workspace(int n_rows, int d);
/* Range check of a batch's index tensor on the device (a training step whose batch has no host copy; with one,
 * the host checks it before anything is enqueued): err |= bit if any idx[r·ld + ld - cols + c] (r < rows, c < cols:
 * the last `cols` columns of each row) lies outside [0, hi).  Reference: F.embedding / nn.Embedding / F.cross_entropy
 * raise IndexError (models/C2DSR.py:65-67,81, encoders.py:30, trainer.py:143-152). */
int c2dsr_index_check(const int64_t* idx, long rows, int ld, int cols, int64_t hi, int bit, int* err, void* stream);
/* Sort plan of an index array (stable LSD radix sort; depends on the indices only, so it is built
 * on a side stream under the forward pass): plan = [keys u32 n | rows u32 n | scratch], keys
 * ascending, rows ascending within equal keys.  Replaces the sort inside embedding_dense_backward
 * (the deterministic path of F.embedding's backward, models/C2DSR.py:65). */
size_t c2dsr_index_plan_bytes(int n);
/* An index outside [0, n_keys) becomes the key n_keys (sorted last, never followed by a segment sum) and sets
 * C2DSR_IDX_ERR_PLAN in *err (err may be NULL). */
int c2dsr_index_plan(const int64_t* idx, int n, int n_keys, void* plan, size_t plan_bytes, int* err, void* stream);
/* c2dsr_index_plan of several index tensors with one launch per pass for all of them (a training step's eight
 * lookup plans: 9 launches instead of 60): desc = HOST array of count records of five int64 (idx, n, n_keys, plan,
 * plan_bytes); each plan's bytes are exactly c2dsr_index_plan's.  Same error behaviour, per record. */
int c2dsr_index_plans(const int64_t* desc, int count, int* err, void* stream);
/* c2dsr_embed_bwd on prebuilt plans of seq / pos (seq_plan needed iff G, pos_plan iff gP); the item
 * and position sums share one launch of each pass.  A plan whose keys fall outside [0, n_items) /
 * [0, n_pos) or whose split lists are inconsistent is not followed: the int at
 * plan + c2dsr_plan_err_offset(n_rows) is then nonzero (debug check). */
size_t c2dsr_embed_bwd_planned_workspace(int n_rows, int d);
size_t c2dsr_plan_err_offset(int n);
int c2dsr_embed_bwd_planned(const void* seq_plan, const void* pos_plan, int n_rows, int d, const float* gX,
                            uint32_t k0, uint32_t k1, float p, int64_t idx_base, float scale, float* G, int n_items,
                            float* gP, int n_pos, float* gXin, void* workspace, size_t ws_bytes, void* stream);
/* bf16 item tables (the C5 roofline run): the gather reads bf16 H / E rows; the item segment sums
 * read-modify-write a bf16 G (fp32 sums, RNE stores).  P, X, gX and gP stay fp32. */
int c2dsr_embed_fwd_b16(const int64_t* seq, const int64_t* pos, int n_rows, int d, const void* H, const void* E,
                        const float* P, float scale, uint32_t k0, uint32_t k1, float p, int64_t idx_base, float* X,
                        int n_items, int n_pos, int* err, void* stream);
int c2dsr_embed_bwd_planned_b16(const void* seq_plan, const void* pos_plan, int n_rows, int d, const float* gX,
                                uint32_t k0, uint32_t k1, float p, int64_t idx_base, float scale, void* G, int n_items,
                                float* gP, int n_pos, void* workspace, size_t ws_bytes, void* stream);
/* The same with gX given as two compact row sources (the row-subset attention layer's input gradient: query
 * rows + key rows, never combined into a full [n_rows, d] tensor): row r of gX = (inv_a[r] >= 0 ?
 * gXa[inv_a[r]] : 0) + (inv_b[r] >= 0 ? gXb[inv_b[r]] : 0). */
int c2dsr_embed_bwd_planned_rows(const void* seq_plan, const void* pos_plan, int n_rows, int d, const float* gXa,
                                 const int* inv_a, const float* gXb, const int* inv_b, uint32_t k0, uint32_t k1,
                                 float p, int64_t idx_base, float scale, float* G, int n_items, float* gP, int n_pos,
                                 void* workspace, size_t ws_bytes, void* stream);
/* Deterministic (radix-sort + ordered segment sum) backward of the above
 * (replaces embedding_dense_backward):  G[seq[r]] += scale·drop(gX[r]);
 * gP[pos[r]] += drop(gX[r]);  gXin[r] = drop(gX[r]).  Null outputs are skipped. */
int c2dsr_embed_bwd(const int64_t* seq, const int64_t* pos, int n_rows, int d, const float* gX, uint32_t k0,
                    uint32_t k1, float p, int64_t idx_base, float scale, float* G, int n_items, float* gP, int n_pos,
                    float* gXin, void* workspace, size_t ws_bytes, void* stream);

/* Dense GEMM on the matrix cores (nn.Linear / nn.Bilinear / classifier addmm and their
 * backward; models/encoders.py:33, trainer.py:104-108,131-140):
 *   C = alpha·op(A)·op(B) + beta·C + bias;  epilogue 1: C = drop(relu(C)), index (row_base+row)·N+col.
 * precision 0: exact fp32 MFMA (v_mfma_f32_32x32x2_f32); 1: bf16 operands, fp32 accumulate.
 * split_k 0 = automatic. */
int c2dsr_gemm(int transA, int transB, int M, int N, int K, const float* A, int lda, const float* B, int ldb,
               float* C, int ldc, float alpha, float beta, const float* bias, int epilogue, uint32_t k0, uint32_t k1,
               float p, int64_t row_base, const int* rowmap, int precision, int split_k, void* stream);
/* out[n] = beta·out[n] + alpha·Σ_m X[m·ldx + n]   (bias gradients; deterministic 2-stage) */
size_t c2dsr_colsum_workspace(int M, int N);
int c2dsr_colsum(const float* X, int M, int N, int ldx, float alpha, float beta, float* out, void* workspace,
                 void* stream);
/* out[n] = beta·out[n] + alpha·Σ_m w[m·ldw]·X[m·ldx + n]  (w null: 1; workspace: c2dsr_colsum_workspace) */
int c2dsr_wcolsum(const float* X, int M, int N, int ldx, const float* w, long ldw, float alpha, float beta, float* out,
                  void* workspace, void* stream);

/* Attention core (SDPA math path with causal + inverted key-padding mask, Q1/Q2;
 * models/encoders.py:14,33).  qkv [B,L,3d], out [B,L,d], Psave c2dsr_attn_psave_floats(B, L, d, H) floats
 * (the saved probabilities: [B,H,L,L] on the tiled paths, the wave kernels' register layout on the
 * wave path, L <= 64 and d/H % 32 == 0); L <= 128. */
size_t c2dsr_attn_psave_floats(int B, int L, int d, int H);
int c2dsr_attn_fwd(const float* qkv, const int64_t* seq, int64_t pad, int B, int L, int d, int H, uint32_t k0,
                   uint32_t k1, float p, int64_t b_base, float* out, float* Psave, void* stream);
int c2dsr_attn_bwd(const float* qkv, const int64_t* seq, int64_t pad, int B, int L, int d, int H, uint32_t k0,
                   uint32_t k1, float p, int64_t b_base, const float* Psave, const float* dout, float* dqkv,
                   void* stream);
/* The same backward writing dqkv in bf16 (wave kernels only: c2dsr_attn_bwd_b16_supported).  In bf16 mode
 * the only consumers of dqkv are the in_proj backward GEMMs, which use it as a bf16 MFMA operand anyway
 * (c2dsr_rgemm_aux_b16a, c2dsr_wgemm_b16y): half the bytes written and read back. */
int c2dsr_attn_bwd_b16_supported(int L, int d, int H);
int c2dsr_attn_bwd_b16(const float* qkv, const int64_t* seq, int64_t pad, int B, int L, int d, int H, uint32_t k0,
                       uint32_t k1, float p, int64_t b_base, const float* Psave, const float* dout, void* dqkv,
                       void* stream);
/* Row-subset attention (the last post-norm encoder layer of a training pass; wave kernels only,
 * c2dsr_attn_rows_supported): queries = the rows the loss reads, keys = the padding rows, compact per
 * sequence in position order.  q [nq, d] (row q_off[b] + i: query i of sequence b, global row
 * q_idx[q_off[b] + i] = b·L + position), kv [nk, 2d] (K | V; k_idx / k_off likewise), out [nq, d],
 * Psave B·H·4096 floats; masks and dropout indices as c2dsr_attn_fwd at those positions.  Backward:
 * dq [nq, d], dkv [nk, 2d], fp32 or (out_bf16) bf16. */
int c2dsr_attn_rows_supported(int L, int d, int H);
int c2dsr_attn_fwd_rows(const float* q, const float* kv, const int64_t* seq, int64_t pad, const int* q_idx,
                        const int* q_off, const int* k_idx, const int* k_off, int B, int L, int d, int H, uint32_t k0,
                        uint32_t k1, float p, int64_t b_base, float* out, float* Psave, void* stream);
int c2dsr_attn_bwd_rows(const float* q, const float* kv, const int64_t* seq, int64_t pad, const int* q_idx,
                        const int* q_off, const int* k_idx, const int* k_off, int B, int L, int d, int H, uint32_t k0,
                        uint32_t k1, float p, int64_t b_base, const float* Psave, const float* dout, void* dq,
                        void* dkv, int out_bf16, void* stream);

/* Residual + dropout + LayerNorm (TransformerEncoderLayer norm1/norm2, encoder.norm; eps 1e-8). */
int c2dsr_add_ln_fwd(const float* a, const float* b, int rows, int d, uint32_t k0, uint32_t k1, float p,
                     int64_t idx_base, const int* rowmap, const float* w, const float* bias, float eps, float* xsave, float* y,
                     float* mean, float* rstd, void* stream);
size_t c2dsr_ln_bwd_workspace(int d);
int c2dsr_ln_bwd(const float* x, const float* mean, const float* rstd, const float* w, const float* dy, int rows,
                 int d, float* dx, int dx_accumulate, float* db_out, uint32_t k0, uint32_t k1, float p,
                 int64_t idx_base, const int* rowmap, float* dgw, float* dgb, void* workspace, void* stream);
int c2dsr_add_dropout(const float* a, const float* b, long n, int d, uint32_t k0, uint32_t k1, float p,
                      int64_t idx_base, float* y, void* stream);
/* Two LayerNorms back to back (the last post-norm layer's norm2 and the encoder's final norm, Q16) in one pass:
 * y = LNF(LN2(a + drop(b))·w2 + b2)·wF + bF; xsave = a + drop(b); st [4][rows] = mean2, rstd2, meanF, rstdF.
 * The backward recomputes LN2's output from xsave and st: dx = ∂/∂a, db_out = dx ⊙ drop mask, and the four
 * parameter gradients accumulated (workspace c2dsr_ln2_bwd_workspace(d) bytes). */
int c2dsr_add_ln2_fwd(const float* a, const float* b, int rows, int d, uint32_t k0, uint32_t k1, float p,
                      int64_t idx_base, const int* rowmap, const float* w2, const float* b2, float eps2,
                      const float* wF, const float* bF, float epsF, float* xsave, float* y, float* st, void* stream);
size_t c2dsr_ln2_bwd_workspace(int d);
int c2dsr_ln2_bwd(const float* xsave, const float* st, const float* w2, const float* b2, const float* wF,
                  const float* dy, int rows, int d, float* dx, float* db_out, uint32_t k0, uint32_t k1, float p,
                  int64_t idx_base, const int* rowmap, float* dgw2, float* dgb2, float* dgwF, float* dgbF,
                  void* workspace, void* stream);
/* The LayerNorm parameter gradients of one post-norm encoder layer's two backwards in ONE launch: c2dsr_ln2_bwd (rows2
 * rows, workspace ws2) and c2dsr_ln_bwd (rows1, ws1) called with null parameter-gradient outputs leave their per-block
 * partials in their workspaces; this adds them onto dgw2 / dgb2 / dgwF / dgbF and dgw1 / dgb1 (null ones skipped) in
 * the fixed order of the two backwards' own reductions (the same bits). */
int c2dsr_ln_reduce2(const void* ws2, int rows2, const void* ws1, int rows1, int d, float* dgw2, float* dgb2,
                     float* dgwF, float* dgbF, float* dgw1, float* dgb1, void* stream);
/* backward of drop(relu(.)) from its output: dx = (y > 0) ? dy/(1-p) : 0 */
int c2dsr_relu_drop_bwd(const float* dy, const float* y, long n, float p, float* dx, void* stream);

/* Loss head (trainer.py:85-156). */
/* w[b,l] = gm[b,l]/Σ_l gm[b,l] (cal_mask); out[b] = Σ_l h[b,l]·w[b,l]; dh[b,l] += dout[b]·w[b,l] */
int c2dsr_pool_weights(const int64_t* gm, int B, int L, float* w, void* stream);
int c2dsr_pool_fwd(const float* h, const float* w, int B, int L, int d, float* out, void* stream);
int c2dsr_pool_bwd(const float* dout, const float* w, int B, int L, int d, float* dh, void* stream);
/* two poolings of one h in one read (rows with zero weights skipped): out1[b] = Σ_l h[b,l]·w1[b,l],
 * out2[b] = Σ_l h[b,l]·w2[b,l] (w2 may be null); and the backward in write or accumulate mode:
 * dh[b,l] = (accumulate ? dh[b,l] : 0) + d1[b]·w1[b,l] + d2[b]·w2[b,l] (d2 may be null).
 * Row subsets (an encoder pass whose last layer ran on the rows the loss reads): h row (b,l) is
 * h[hmap[b·L+l]] (hmap null: identity; every row with a nonzero weight must be mapped); the backward
 * writes the n_rows rows of a compact dh, row k being (b,l) = idx[k] (idx null: all B·L rows). */
int c2dsr_pool2_fwd(const float* h, const int* hmap, const float* w1, const float* w2, int B, int L, int d,
                    float* out1, float* out2, void* stream);
int c2dsr_pool2_bwd(const float* d1, const float* w1, const float* d2, const float* w2, int B, int L, int d,
                    const int* idx, int n_rows, int accumulate, float* dh, void* stream);
/* Stable row compaction, two launches over 1024-row tiles; ws = c2dsr_compact_workspace(M, n_sets) bytes
 * of device scratch (per-tile set sizes).
 * Valid-row compaction of a classifier head's targets (trainer.py:131-154: rows whose target is the
 * ignore_index contribute nothing to the loss or any gradient, so the fused CE runs on the valid
 * rows only): idx[k] = k-th row with t != ignore, inv[r] = compact index or -1, tc[k] = t[idx[k]],
 * counts[0..1] = valid rows in [0, split) and [split, M).  A target outside [0, ignore] (F.cross_entropy raises
 * IndexError) sets C2DSR_IDX_ERR_TARGET in *err (err may be NULL) and its row is not valid. */
size_t c2dsr_compact_workspace(int M, int n_sets);
int c2dsr_compact_valid(const int64_t* t, int M, int split, int ignore, int* idx, int* inv, int64_t* tc, int* counts,
                        int* ws, int* err, void* stream);
/* Rows of the encoder passes the loss reads (trainer.py:101-154), n_sets <= 8 at once: set q's code is
 * (bits >> 3q) & 7 — 1 / 2 = positions with gm_a / gm_b nonzero (the pass's pooling weights), 4 = the
 * last R positions (classifier heads).  idx / inv of set q at offset q·B·L: idx[k] = k-th needed row,
 * inv[r] = compact index or -1; count[q] = set size; off (may be null) [n_sets][B+1]: off[q][b] = compact
 * index of sequence b's first row (off[q][B] = count[q]). */
int c2dsr_need_rows(const int64_t* gm_a, const int64_t* gm_b, int B, int L, int R, int n_sets, int bits, int* idx,
                    int* inv, int* count, int* off, int* ws, void* stream);
/* Padding rows of n_sets <= 8 encoder passes (the attention's only admissible keys, Q1): set q = rows r of
 * seqs [n_sets][B·L] with seqs[q][r] == pad; idx / inv / count / off (required) as c2dsr_need_rows. */
int c2dsr_pad_rows(const int64_t* seqs, int64_t pad, int B, int L, int n_sets, int* idx, int* inv, int* count,
                   int* off, int* ws, void* stream);
/* dst[r] = (inv_a[r] >= 0 ? a[inv_a[r]] : 0) + (inv_b[r] >= 0 ? b[inv_b[r]] : 0), rows of d floats (d % 4 == 0):
 * the input gradient of the row-subset attention layer (query rows + key rows) */
int c2dsr_combine_rows(const float* a, const int* inv_a, const float* b, const int* inv_b, int M, int d, float* dst,
                       void* stream);
/* dst[k][:] = src[idx[k]·ld + :] (k < n);  dst[r][:] = inv[r] >= 0 ? src[inv[r]][:] : 0 (r < M) */
int c2dsr_gather_rows(const float* src, long ld, const int* idx, int n, int d, float* dst, void* stream);
int c2dsr_expand_rows(const float* src, const int* inv, int M, int d, float* dst, void* stream);
int c2dsr_rowdot(const float* x, long ldx, const float* y, long ldy, int M, int d, const float* bias, float* out,
                 long ldo, void* stream);
/* loss_mi = Σ_k Σ_b BCE(s_k[b], y_k)/B_norm, ds = (σ(s)-y)/B_norm; s = [sim_a_pos; sim_a_neg; sim_b_pos; sim_b_neg] */
/* The four discriminator scores (trainer.py:104-108: D_a(h_a, h_share_b), D_a(h_a, neg_a), D_b(...), D_b(...)) in one
 * launch: S [4][B], S[k][b] = x1_k[b]·U_k[b] + bias_k with (x1, U rows) = (x1a, Ua[0:B]), (x1a, Ua[B:2B]), (x1b, Ub[0:B]),
 * (x1b, Ub[B:2B]) (U = X2·Wᵀ of each bilinear; bias nullable) — c2dsr_rowdot's per-row sum, the same bits. */
int c2dsr_mi_scores(const float* x1a, const float* Ua, const float* ba, const float* x1b, const float* Ub, const float* bb,
                    int B, int d, float* S, void* stream);
int c2dsr_mi_loss(const float* s, int B, int B_norm, float* loss_mi, float* ds, void* stream);
int c2dsr_rec_gather(const float* hs, const int* hs_map, const float* hx, const int* hx_map, int B, int L, int d,
                     int R, float* Hcat, float* Hpad, void* stream);
/* The head's operand rows in one pass (trainer.py:122-131): Hpad as c2dsr_rec_gather, and for the Mv valid rows
 * (idx: compact → stacked row of [hs_r ; hs_r + hx_r]) Hc [Mv][d] and its MFMA image img — split hi ‖ lo [M_pad][2d]
 * (split = 1, as c2dsr_f32_split_bf16) or bf16 [M_pad][d] — rows Mv..M_pad zero.  d % 4 == 0. */
int c2dsr_rec_gather_compact(const float* hs, const int* hs_map, const float* hx, const int* hx_map, int B, int L,
                             int d, int R, const int* idx, int Mv, int M_pad, int split, float* Hpad, float* Hc,
                             void* img, void* stream);
int c2dsr_rec_targets(const int64_t* ts, const int64_t* tx, int B, int L, int R, int64_t* tcat, void* stream);
/* dhs[b,l] += dHcat[r] + dHcat[BR+r] + pad[r·pad_ld]·wpad;  dhx[b,l] += dHcat[BR+r] + pad[(BR+r)·pad_ld]·wpad
 * for the last R positions (r = b·R + l - (L-R)); pad = the pad column of the stacked dlogits (classifier_pad,
 * trainer.py:136-140), its input gradient folded in; maps as for c2dsr_rec_gather */
int c2dsr_rec_scatter(const float* dHcat, const float* pad, long pad_ld, const float* wpad, int B, int L, int d, int R,
                      float* dhs, const int* dhs_map, float* dhx, const int* dhx_map, void* stream);
int c2dsr_ce_fwd(const float* logits, long ld, int M, int ncol, const int64_t* tgt, int ignore, float* lse,
                 float* loss_row, void* stream);
int c2dsr_ce_bwd(float* logits, long ld, int M, int ncol, const int64_t* tgt, int ignore, const float* lse,
                 const float* coef, int split, const float* gscale, float lam, void* stream);
int c2dsr_outer_add(const float* a, long sa, const float* v, int M, int d, float* out, long ldo, void* stream);
/* vec[0..7] = per-head CE sums and valid counts of this rank's rows (all-reduced under DP); rowsA/rowsB
 * may be NULL (counts only: data parallel reduces the counts ahead of the forward) */
int c2dsr_loss_partials(const float* rowsA, const int64_t* tA, int n_a, const float* rowsB, const int64_t* tB, int n_b,
                        int BR, float* vec, float* workspace, void* stream);
/* floats of c2dsr_loss_partials' workspace (per-block partials; the caller allocates it on the launch stream) */
size_t c2dsr_loss_partials_workspace(int BR);
/* out3 = (loss, loss_rec, loss_mi) from vec[0..8]; coefA/B = per-row grad weights; cnt (nullable) supplies
 * the valid counts cnt[4..7] instead of vec[4..7] */
int c2dsr_loss_finalize(const float* vec, const float* cnt, int BR_global, float lam, float* out3, float* coefA,
                        float* coefB, void* stream);
/* acc3[0..2] += w·(*loss, *loss_rec, *loss_mi): run_epoch's per-epoch loss sums kept on the device (one host read per
 * epoch; reference trainer.py:50-52 accumulates loss.item()·n_batch on the host every step). */
int c2dsr_loss_accumulate(const float* loss, const float* loss_rec, const float* loss_mi, float w, float* acc3,
                          void* stream);
int c2dsr_scale_ds(float* ds, int n, const float* gscale, float f, void* stream);
int c2dsr_rowscale(const float* x, const float* s, long n, int d, float* out, int accumulate, void* stream);
/* The MI-loss backward's row-scale products of both bilinear discriminators in one launch (trainer.py:104-119 through
 * D_a / D_b; replaces eight c2dsr_rowscale calls): for j = a, b (dS [4][B]: rows 2j, 2j+1 scale the positive and
 * negative pairs): dx1_j = dS[2j] ⊙ U_j[0:B] + dS[2j+1] ⊙ U_j[B:2B] (each product rounded, then summed),
 * dU_j[0:B] = dS[2j] ⊙ x1_j, dU_j[B:2B] = dS[2j+1] ⊙ x1_j.  U_j, dU_j [2B][d]; x1_j, dx1_j [B][d]; d % 4 == 0. */
int c2dsr_bilinear_ds(const float* Ua, const float* Ub, const float* x1a, const float* x1b, const float* dS, int B, int d,
                      float* dx1a, float* dx1b, float* dUa, float* dUb, void* stream);

/* K5 fused classifier head + cross-entropy (bf16 MFMA, logits never materialised; trainer.py:131-154).
 * Hb [M][D], Wb [n][D] bf16 (D = 128 or 256); bias2 = bias·log2e padded with -inf to n_pad (multiple of
 * 128, c2dsr_ce_bias2).  Forward: lse, lse2 = lse·log2e, loss_row over the n items + the pad column
 * (padlogit); the target logit is taken from fp32 H/W/bias. */
int c2dsr_ce_supported(int D);
int c2dsr_f32_to_bf16(const float* x, long n, void* y, void* stream);
int c2dsr_ce_bias2(const float* bias, int n, int n_pad, float* bias2, void* stream);
int c2dsr_ce_fused_fwd(const void* Hb, const void* Wb, const float* bias2, int M, int n, int D, int n_split,
                       float* part_m, float* part_s, const float* padlogit, const int64_t* tgt, const float* H,
                       const float* W, const float* bias, float* lse, float* lse2, float* loss_row, void* stream);
/* The same forward plus the softmax part of the input gradient, accumulated online (flash style):
 * part_m/part_s [n_split][M] and Up [n_split][M][D] (Up[s][r] = Σ_{c∈s} 2^(v_rc − part_m[s][r])·W_c, v the
 * log2-domain logit); the backward then needs no dH sweep (c2dsr_ce_dh_from_u). */
int c2dsr_ce_fused_fwd_u(const void* Hb, const void* Wb, const float* bias2, int M, int n, int D, int n_split,
                         float* part_m, float* part_s, float* Up, const float* padlogit, const int64_t* tgt,
                         const float* H, const float* W, const float* bias, float* lse, float* lse2, float* loss_row,
                         void* stream);
/* dH[r] = rw[r]·(Σ_s 2^(part_m[s][r] − lse2[r])·Up[s][r] − (0 <= t32[r] < n ? W[t32[r]] : 0))  (fixed order) */
int c2dsr_ce_dh_from_u(const float* Up, const float* part_m, int ns, int M, int D, const float* lse2, const int* t32,
                       const float* rw, const float* W, int n, float* dH, void* stream);
/* per row r < M_pad (multiple of 64): rw = valid ? gscale·lam·coef[r >= split] : 0, t32 = target (-1 pad),
 * crow = log2(rw) - lse2 (-inf where rw = 0 and past M), dpad = exp(padlogit - lse)·rw */
int c2dsr_ce_row_weights(const int64_t* tgt, int M, int M_pad, int ignore, const float* coef, int split,
                         const float* gscale, float lam, const float* padlogit, const float* lse, float* rw, int* t32,
                         const float* lse2, float* crow, float* dpad, void* stream);
/* dHp[s][r] = Σ_{c∈split s} softmax[r][c]·rw_r·W[c]  ([n_split][M][D]; the one-hot part and the split
 * sum are applied by c2dsr_ce_dh_combine).  Wb holds ⌈n/64⌉·64 rows (zero rows past n); bias2 holds
 * n_pad + 64 values (-inf past n); crow from c2dsr_ce_row_weights. */
int c2dsr_ce_fused_dh(const void* Hb, const void* Wb, const float* bias2, int M, int n, int D, int n_split,
                      const float* crow, float* dHp, void* stream);
/* dWp[s][c] = Σ_{r∈split s} E[r][c]·H[r];  dbp[s][c] = Σ_r E[r][c]  ([n_rsplit][n][D], [n_rsplit][n]) with
 * E = softmax·rw, the softmax part of P' (the one-hot part: c2dsr_ce_onehot_dw).  Hb holds ⌈M/64⌉·64 rows
 * (zero rows past M); crow as written by c2dsr_ce_row_weights. */
/* dH[r] = Σ_s dHp[s][r] - (0 <= t32[r] < n ? rw[r]·W[t32[r]] : 0)  (W fp32 [n][D]; fixed order) */
int c2dsr_ce_dh_combine(const float* dHp, int ns, int M, int D, const int* t32, const float* rw, const float* W, int n,
                        float* dH, void* stream);
int c2dsr_ce_fused_dw(const void* Hb, const void* Wb, const float* bias2, int M, int n, int D, int n_rsplit,
                      const float* crow, float* dWp, float* dbp, void* stream);
/* one-hot part of the head's weight/bias gradient: gW[t_r] -= rw_r·H[r], gb[t_r] -= rw_r for 0 <= t_r < n
 * (t_r = n is the ignored pad target); rows radix-sorted by target, each run summed in row order
 * (deterministic).  H fp32 [M][D]; gW / gb may be null. */
size_t c2dsr_ce_onehot_workspace(int M, int n, int D);
/* the same on a prebuilt target plan (c2dsr_index_plan of tgt, n_keys = n + 1) */
size_t c2dsr_ce_onehot_planned_workspace(int M, int n, int D);
int c2dsr_ce_onehot_dw_planned(const void* plan, int M, int n, const float* H, int D, const float* rw, float* gW,
                               float* gb, void* workspace, size_t ws_bytes, void* stream);
int c2dsr_ce_onehot_dw(const int64_t* tgt, int M, int n, const float* H, int D, const float* rw, float* gW, float* gb,
                       void* workspace, size_t ws_bytes, void* stream);
/* per row: lse over the splits' (max, sum) partials and the pad column, lse2 = lse·log2e, the fp32 target
 * logit and loss_row (the row step of c2dsr_ce_fused_fwd / _fwd_u / c2dsr_ce3_fused_fwd_u) */
int c2dsr_ce_rows(const float* part_m, const float* part_s, int n_split, int M, const float* padlogit,
                  const int64_t* tgt, int n, const float* H, const float* W, const float* bias, int D, float* lse,
                  float* lse2, float* loss_row, void* stream);

/* K5 at the reference's precision (fp32 training mode; csrc/ce3.hip).  Same contract as
 * c2dsr_ce_fused_fwd_u / c2dsr_ce_fused_dw (trainer.py:131-154), but the operands are split-bf16 images
 * [rows][2·D] = hi ‖ lo (x = hi + lo to 2^-17 relative; c2dsr_f32_split_bf16) and every product runs as
 * three bf16 MFMAs (hi·hi + lo·hi + hi·lo) with fp32 accumulation.  Hx holds ⌈M/32⌉·32 rows and Wx
 * ⌈n/32⌉·32 rows (zero rows past the end); bias2 as for ce.hip; crow holds ⌈M/64⌉·64 + 64 values.
 * dw with n_rsplit == 0 (also c2dsr_ce3b_fused_dw): one split whose workgroups own their columns, added straight
 * onto dWp [n][D] / dbp [n] (the parameters' epoch-long gradients, trainer.py:42 — no partials, no sum). */
int c2dsr_ce3_supported(int D);
/* The sweep geometry of the fused-CE instantiations (split = 1: fp32 mode's split-bf16 kernels, 0: bf16 mode's):
 * what = 0 → stationary rows per workgroup (the launch grid's row block: 128 / 192), 1 → swept rows per LDS tile
 * (32 / 32); -1 for another `what`.  The host's split plans (c2dsr_amd/losshead.py) size their grids with it. */
int c2dsr_ce3_geometry(int split, int what);
int c2dsr_f32_split_bf16(const float* x, long rows, int D, long rows_out, void* out, void* stream);
int c2dsr_ce3_fused_fwd_u(const void* Hx, const void* Wx, const float* bias2, int M, int n, int D, int n_split,
                          float* part_m, float* part_s, float* Up, const float* padlogit, const int64_t* tgt,
                          const float* H, const float* W, const float* bias, float* lse, float* lse2, float* loss_row,
                          void* stream);
int c2dsr_ce3_fused_dw(const void* Hx, const void* Wx, const float* bias2, int M, int n, int D, int n_rsplit,
                       const float* crow, float* dWp, float* dbp, void* stream);
/* The bf16 mode's pair on ce3.hip's plain-bf16 instantiation (one MFMA per product, 64-row swept tiles; D = 128
 * or 256, c2dsr_ce3_supported): drop-in for c2dsr_ce_fused_fwd_u / c2dsr_ce_fused_dw — same arguments, same
 * outputs (trainer.py:131-154).  Hb holds ⌈M/64⌉·64 rows and Wb ⌈n/64⌉·64 rows (zero rows past the end); crow
 * holds ⌈M/64⌉·64 + 64 values. */
int c2dsr_ce3b_fused_fwd_u(const void* Hb, const void* Wb, const float* bias2, int M, int n, int D, int n_split,
                           float* part_m, float* part_s, float* Up, const float* padlogit, const int64_t* tgt,
                           const float* H, const float* W, const float* bias, float* lse, float* lse2,
                           float* loss_row, void* stream);
int c2dsr_ce3b_fused_dw(const void* Hb, const void* Wb, const float* bias2, int M, int n, int D, int n_rsplit,
                        const float* crow, float* dWp, float* dbp, void* stream);
/* The dW sweep as stream-K (trainer.py:131-154, the classifier's weight / bias gradients): the (128-row W block,
 * swept H tile) units are dealt to one workgroup per CU in equal contiguous ranges — one launch round, no partial
 * last round, one prologue per workgroup segment.  Row blocks swept whole by one workgroup are added straight onto
 * gW [n][D] / gb [n]; split ones leave partials in ws that a combine pass adds in workgroup order (deterministic).
 * ws: c2dsr_ce3_dw_sk_workspace(D) bytes.  Operands as c2dsr_ce3_fused_dw (split images) / c2dsr_ce3b_fused_dw. */
size_t c2dsr_ce3_dw_sk_workspace(int D);
int c2dsr_ce3_fused_dw_sk(const void* Hx, const void* Wx, const float* bias2, int M, int n, int D, const float* crow,
                          float* gW, float* gb, void* ws, size_t ws_bytes, void* stream);
int c2dsr_ce3b_fused_dw_sk(const void* Hb, const void* Wb, const float* bias2, int M, int n, int D, const float* crow,
                           float* gW, float* gb, void* ws, size_t ws_bytes, void* stream);
/* K5's dW from stored logits (fp32 mode; trainer.py:131-154, the classifier's weight / bias gradients).  The forward
 * c2dsr_ce3_fused_fwd_u_lg is c2dsr_ce3_fused_fwd_u that also writes every logit v = (h_r·w_c + b_c)·log2e of the
 * rows r < ⌈M/128⌉·128 (the image's padding rows duplicate row M−1) and columns c < ⌈n/32⌉·32 (−inf past n) into lg,
 * c2dsr_ce3_logits_floats(M, n) fp32 values: 16 × 16 blocks, column-block-major (block (c/16, r/16) at
 * ((c/16)·⌈M/128⌉·8 + r/16)·256, element (r, c) at ((r%16)/4·16 + c%16)·4 + r%4 inside it).  The dW sweeps
 * c2dsr_ce3_fused_dw_lg / _dw_lg_sk then compute E = 2^(v + crow_r) from the stored logits instead of recomputing
 * them (one split product per tile instead of two), same outputs as c2dsr_ce3_fused_dw / _dw_sk: dw_lg sweeps the
 * columns [col0, col0 + n) (col0 a multiple of 32) of the n_lg the forward wrote; n_rsplit as c2dsr_ce3_fused_dw. */
size_t c2dsr_ce3_logits_floats(int M, int n);
/* the layout's column-block grouping GRP (a build-time choice, 1 or 8): block (c/16, r/16) at
 * ((c/16 / GRP)·⌈M/128⌉·8 + r/16)·GRP + (c/16) % GRP, column blocks padded to a multiple of GRP; dw_lg's col0 then
 * a multiple of 16·max(2, GRP); what = 0 (-1 for another `what`) */
int c2dsr_ce3_logits_group(int what);
int c2dsr_ce3_fused_fwd_u_lg(const void* Hx, const void* Wx, const float* bias2, int M, int n, int D, int n_split,
                             float* part_m, float* part_s, float* Up, const float* padlogit, const int64_t* tgt,
                             const float* H, const float* W, const float* bias, float* lse, float* lse2,
                             float* loss_row, float* lg, void* stream);
int c2dsr_ce3_fused_dw_lg(const void* Hx, const float* lg, int M, int n_lg, int col0, int n, int D, int n_rsplit,
                          const float* crow, float* dWp, float* dbp, void* stream);
int c2dsr_ce3_fused_dw_lg_sk(const void* Hx, const float* lg, int M, int n, int D, const float* crow, float* gW,
                             float* gb, void* ws, size_t ws_bytes, void* stream);
/* out[i] = beta·out[i] + Σ_s part[s·n + i]  (fixed order) */
int c2dsr_sum_parts(const float* part, int nparts, long n, float beta, float* out, void* stream);
/* test hook: transposed / row fragment reads of the swizzled LDS image (int16 payload) */
int c2dsr_selftest_tr(int rr0, int kb0, short* out, void* stream);

/* K6 AdamW(amsgrad) over flat buffers, folding the fresh grad into the epoch accumulator
 * (trainer.py:21-22,42,158); accum == fresh: the backward accumulated into the epoch accumulator
 * directly (one device) and it is only read.  err (may be NULL): the step's index error word — when it is
 * nonzero the launch changes nothing (the reference raises IndexError before its optimizer step). */
int c2dsr_adamw(float* p, float* fresh, float* accum, float* m, float* v, float* vmax, long n, float lr, float wd,
                float b1, float b2, float eps, int step, const int* err, void* stream);


/* K3 projections, row-streaming bf16 MFMA (csrc/rgemm.hip).  Replaces the addmm/mm of
 * TransformerEncoderLayer in_proj/out_proj/linear1/linear2 (models/encoders.py:23-27) at
 * K ∈ {256,512,768}:  C[M,N] = alpha·A[M,K]·B[N,K]ᵀ + bias (beta must be 0; epilogue 1: relu·dropout(p),
 * index (row_base+row)·N + col).  A fp32 (lda % 4 == 0), B bf16 [N][ldb]. */
int c2dsr_rgemm_supported(int M, int N, int K);
int c2dsr_rgemm(int M, int N, int K, const float* A, int lda, const void* B, int ldb, float* C, int ldc,
                float alpha, float beta, const float* bias, int epilogue, uint32_t k0, uint32_t k1, float p,
                int64_t row_base, const int* rowmap, void* stream);
/* rowmap (GEMM epilogue 1, add_ln_fwd, ln_bwd; may be null): dropout row index = base + rowmap[row]
 * instead of base + row, so a kernel run on a compacted subset of rows drops exactly the elements the
 * full-size run would (the last encoder layer runs on the rows the loss reads). */
/* c2dsr_rgemm with an epilogue reading aux [M][ldc] at the output positions (prefetched a tile ahead):
 *   aux_mode 1: C = alpha·A·Bᵀ + bias + aux   (aux == C accumulates in place: the residual-gradient sum
 *               of a post-norm encoder layer, which autograd would otherwise add in a separate pass)
 *   aux_mode 2: C = aux > 0 ? (alpha·A·Bᵀ + bias)·aux_scale : 0   (dX of linear2 masked by the
 *               backward of drop(relu(.)) of linear1, given its output aux; models/encoders.py:23-27)
 *   aux_mode 3: C = alpha·A·Bᵀ + bias + (auxmap[r] >= 0 ? aux[auxmap[r]] : 0)   (auxmap [M]; aux holds a
 *               compacted subset of the rows — the LayerNorm gradient of the last layer's row subset)
 * epilogue must be 0 and beta 0 with an aux mode; auxmap non-null exactly for mode 3 (aux != C). */
int c2dsr_rgemm_aux(int M, int N, int K, const float* A, int lda, const void* B, int ldb, float* C, int ldc,
                    float alpha, float beta, const float* bias, int epilogue, uint32_t k0, uint32_t k1, float p,
                    int64_t row_base, const int* rowmap, int aux_mode, const float* aux, const int* auxmap,
                    float aux_scale, void* stream);
/* c2dsr_rgemm_aux with A in bf16 (the in_proj dX over the attention's bf16 gradient; no epilogue): K = 768
 * (dqkv; aux modes 0 / 1 / 3), K = 256 (the row-subset layer's dq; aux modes 0 / 1), K = 512 (its dkv;
 * aux mode 0) — the products equal the fp32-A call's, which rounds A to bf16 the same way. */
int c2dsr_rgemm_aux_b16a(int M, int N, int K, const void* A, int lda, const void* B, int ldb, float* C, int ldc,
                         float alpha, float beta, const float* bias, int aux_mode, const float* aux, const int* auxmap,
                         void* stream);
/* fp32 mode (split-bf16 products, three bf16 MFMAs per k-step, fp32 accumulation — see csrc/ce3.hip): the
 * same contract as c2dsr_rgemm_aux with B the split image [N][2K] = hi ‖ lo (ldb >= 2K), K = 256 or 512 */
int c2dsr_rgemm_x3_supported(int M, int N, int K);
int c2dsr_rgemm_x3(int M, int N, int K, const float* A, int lda, const void* B, int ldb, float* C, int ldc,
                   float alpha, float beta, const float* bias, int epilogue, uint32_t k0, uint32_t k1, float p,
                   int64_t row_base, const int* rowmap, int aux_mode, const float* aux, const int* auxmap,
                   float aux_scale, void* stream);
/* the same with B the fragment-ordered split image (c2dsr_to_split_bf16_frag_multi; no ldb): each weight load of the
 * kernel is one coalesced 1 KiB read; N % 4 == 0, ldc % 4 == 0.  Bit-identical to c2dsr_rgemm_x3 on the same W. */
int c2dsr_rgemm_x3f(int M, int N, int K, const float* A, int lda, const void* B, float* C, int ldc, float alpha,
                    float beta, const float* bias, int epilogue, uint32_t k0, uint32_t k1, float p, int64_t row_base,
                    const int* rowmap, int aux_mode, const float* aux, const int* auxmap, float aux_scale,
                    void* stream);
/* linear1 + ReLU + dropout of the fp32 mode (replaces models/encoders.py:23-27 → TransformerEncoderLayer
 * linear1 / activation / dropout): C = drop(relu(A·Wᵀ + bias)) on split-bf16 products (B = the split image of the
 * fp32 weight W [N][256], ldb >= 2K, or its fragment-ordered image, ldb = 0; K = 256, N % 4 == 0), every
 * pre-activation within the split error bound of zero (|v| ≤ 2^-15·‖a‖‖w‖) recomputed from A and W as one fp32 FMA
 * chain in k order, so the ReLU's sign decisions are those of a k-sequential fp32 product.  Dropout index
 * (row_base + (rowmap ? rowmap[r] : r))·N + c, as c2dsr_rgemm's epilogue 1.  workspace: guard_workspace bytes,
 * zero-filled before its first use (each call leaves it reusable: the flags are cleared as they are consumed).
 * wn2: the squared row norms ‖W[c]‖² [N] if the caller keeps them per weight update, or null (computed here). */
size_t c2dsr_rgemm_guard_workspace(int M, int N);
int c2dsr_rgemm_x3_relu_guard(int M, int N, int K, const float* A, int lda, const void* B, int ldb, const float* W,
                              const float* wn2, float* C, int ldc, const float* bias, uint32_t k0, uint32_t k1, float p,
                              int64_t row_base, const int* rowmap, void* workspace, size_t ws_bytes, void* stream);
/* ... and the weight-gradient products (c2dsr_wgemm / _multi contract, dY fp32) */
int c2dsr_wgemm_x3(int T, int N, int D, const float* dY, int ldy, const float* X, int ldx, float beta, float* dW,
                   float* db, void* part, void* stream);
int c2dsr_wgemm_x3_multi(const int64_t* seg, int nseg, int N, int D, float beta, float* dW, float* db, void* part,
                         void* stream);
/* split-bf16 images of a list of matrices (c2dsr_to_bf16_multi's descriptors): y = [R][2·Cc] (row = hi ‖ lo),
 * or [Cc][2·R] when trans */
int c2dsr_to_split_bf16_multi(const int64_t* desc, int count, void* stream);
/* the same values in c2dsr_rgemm_x3f's fragment order: ⌈N'/16⌉·16 rows × 2K' bf16 per matrix (N' × K' = the image's
 * rows × columns: R × Cc, or Cc × R when trans; K' = 256 or 512); element (n, k) hi / lo (hl = 0 / 1) at
 * ((⌊n/16⌋·(K'/16) + 2⌊k/32⌋ + hl)·64 + (⌊k/8⌋ mod 4)·16 + n mod 16)·8 + k mod 8; rows past N' are not written */
int c2dsr_to_split_bf16_frag_multi(const int64_t* desc, int count, void* stream);
/* bf16 images (c2dsr_to_bf16_multi's descriptors) in the bf16-mode kernel's fragment order: ⌈N'/32⌉·32 rows × K'
 * (K' = 256, 512 or 768); element (n, k) at ((⌊n/32⌋·(K'/16) + ⌊k/16⌋)·64 + (⌊k/8⌋ mod 2)·32 + n mod 32)·8 + k mod 8.
 * c2dsr_rgemm / c2dsr_rgemm_aux / c2dsr_rgemm_aux_b16a take such an image as B with ldb = 0 (every weight load one
 * coalesced 1 KiB read; results identical to the row image's). */
int c2dsr_to_bf16_frag_multi(const int64_t* desc, int count, void* stream);
/* K3 projection weight/bias gradients (csrc/rgemm.hip): dW[N][256] = beta·dW + Σ_t dY[t][N]ᵀ·X[t][256]
 * (the mm of the linear backward, N % 128 == 0) and, if db is non-null, db[N] = beta·db + Σ_t dY[t][N]
 * (fp32 column sums of the same dY chunks; replaces c2dsr_colsum there); bf16 MFMA with transposed LDS
 * reads, split over t into partials (workspace bytes from c2dsr_wgemm_workspace) combined in a fixed
 * order (deterministic).  beta ∈ {0, 1}. */
int c2dsr_wgemm_supported(int T, int N, int D);
size_t c2dsr_wgemm_workspace(int N);
int c2dsr_wgemm(int T, int N, int D, const float* dY, int ldy, const float* X, int ldx, float beta, float* dW,
                float* db, void* part, void* stream);
/* ... with dY in bf16 (the bias sums add the bf16 values) */
int c2dsr_wgemm_b16y(int T, int N, int D, const void* dY, int ldy, const float* X, int ldx, float beta, float* dW,
                     float* db, void* part, void* stream);
/* c2dsr_wgemm over up to 4 row sets in one product into the same dW (a weight several encoder passes used;
 * its gradient products deferred to the end of the backward, ops.WGradBatch): seg = HOST array of nseg
 * records of five int64 (dY, ldy, X, ldx, T); yb16: dY bf16 */
int c2dsr_wgemm_multi(const int64_t* seg, int nseg, int N, int D, int yb16, float beta, float* dW, float* db,
                      void* part, void* stream);
/* y = bf16(x), x fp32 [R][Cc] with row stride ldx; trans: y is [Cc][R] (weight copies for rgemm). */
int c2dsr_to_bf16(const float* x, int R, int Cc, int ldx, int trans, void* y, void* stream);
/* c2dsr_to_bf16 over up to 64 matrices in one launch (the projection weights' bf16 images after an optimizer
 * step): desc = HOST array of count records of six int64 (x, y, R, Cc, ldx, trans) */
int c2dsr_to_bf16_multi(const int64_t* desc, int count, void* stream);
/* Squared row norms of a list of fp32 matrices in one launch (c2dsr_to_bf16_multi's descriptors, trans = 0):
 * y[r] = Σ_c x[r·ldx + c]² (fp32 [R]; one wave per row, fixed order) — the guarded linear1's threshold
 * ‖W1[c]‖² (c2dsr_rgemm_x3_relu_guard's wn2), refreshed with the weight images after each optimizer step
 * (trainer.py:158; replaces torch.sum(W * W, 1)). */
int c2dsr_row_sqnorm_multi(const int64_t* desc, int count, void* stream);

/* Evaluation (csrc/eval.hip).  Replaces trainer.py:162-181 (evaluate_batch):
 * per row i, dom = (xory[i] == 0 ? a : b), q = h_share[i,L-1] + h_dom[i, idx_last_dom[i]],
 * s(j) = q·W_dom[j] + b_dom[j] over the candidates gt[i] and neg[i, 0..n_neg), and
 * rank[i] = 1 + #{k : s(neg[i,k]) > s(gt[i])} (ties not counted).  h_* [B,L,d]; idx_last_*, xory, gt
 * int64 [B] (the reference's [B,1] tensors); neg int64 [B][n_neg]; rank int32 [B], -1 for an index out
 * of range (the reference raises IndexError; the host binding raises). */
int c2dsr_eval_rank(const float* h_share, const float* h_a, const float* h_b, int B, int L, int d,
                    const int64_t* idx_last_a, const int64_t* idx_last_b, const int64_t* xory, const int64_t* gt,
                    const int64_t* neg, int n_neg, const float* Wa, const float* ba, int n_a, const float* Wb,
                    const float* bb, int n_b, int* rank, void* stream);
/* utils/metrics.py:4-19 (cal_metrics) as device sums: sums[0..7] += (hr5, hr20, mrr5, mrr20, ndcg5, ndcg20,
 * count, n_bad) over the rows with (xory == 0) == (dom == 0); fp64, fixed reduction order.  The metrics
 * are sums[k]/count; accumulating over all batches of an evaluation costs one host sync per epoch. */
int c2dsr_rank_metrics(const int* rank, const int64_t* xory, int B, int dom, double* sums, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* C2DSR_H */
