// One training pass of the sequence encoder as two stage operators: the embedding fuse (K2) and
// the single post-norm TransformerEncoderLayer + final LayerNorm (K3), on the rows the loss reads.
//
// Reference: models/C2DSR.py:64-85 (x = (H[seq] + E[seq])·√d), models/encoders.py:29-33 (x += pos_emb(pos),
// dropout, TransformerEncoder(n_attn = 1, post-norm) + LayerNorm) → torch TransformerEncoderLayer:
//   x1 = LN1(x + drop(out_proj(SDPA(in_proj(x)))));  y = LNF(LN2(x1 + drop(W2·drop(relu(W1 x1 + b1)) + b2)))
// Everything after the attention is row-wise and the loss reads only the rows `rs` (pooled positions, last R
// positions; trainer.py:101-154), and a query attends only to padding keys (Q1: inverted key-padding mask), so:
// Q is projected for the rs rows, K / V for the padding rows `ks` only, and the rest of the layer runs on the rs
// rows (dropout indices through the row map: the masks are the full-size run's).  The embedding is computed at
// those rows only (c2dsr_embed_fwd_rows: query rows and key rows side by side, the [B·L, d] tensor is never
// stored); the rest are the kernels of the host side's op-by-op path in its order (c2dsr_amd/ops.py: EmbedFn →
// RowsQKVAttnFn → LinearFn → AddLNFn → LinearFn ×2 → AddLN2Fn), so the results are bit-identical to it.
//
// precision 0: fp32 results, split-bf16 ×3 products (csrc/rgemm.hip rg3, linear1 guarded); 1: bf16 operands.
#include <torch/library.h>

#include "c2t.h"

namespace {

using at::Tensor;
using OptT = std::optional<Tensor>;

void want(const Tensor& t, const char* name, at::ScalarType dt, std::initializer_list<int64_t> shape) {
  TORCH_CHECK(t.defined(), "c2dsr::encoder_pass: ", name, " is undefined");
  TORCH_CHECK(t.scalar_type() == dt, "c2dsr::encoder_pass: ", name, " has dtype ", t.scalar_type(), ", expected ", dt);
  TORCH_CHECK(t.is_contiguous(), "c2dsr::encoder_pass: ", name, " must be contiguous");
  const std::vector<int64_t> s(shape);
  TORCH_CHECK(t.dim() == (int64_t)s.size(), "c2dsr::encoder_pass: ", name, " has ", t.dim(), " dims, expected ",
              s.size());
  for (size_t i = 0; i < s.size(); ++i)
    TORCH_CHECK(s[i] < 0 || t.size((int64_t)i) == s[i], "c2dsr::encoder_pass: ", name, " has shape ", t.sizes(),
                ", expected dim ", i, " = ", s[i]);
}
// after every shape check: all of the op's tensors on the HIP device
void on_device(std::initializer_list<const Tensor*> ts, const std::vector<Tensor>& more = {}) {
  for (const Tensor* t : ts)
    TORCH_CHECK(!t->defined() || t->is_cuda(), "c2dsr::encoder_pass: every tensor must be on the HIP device (no CPU "
                                                 "fallback)");
  for (const Tensor& t : more)
    TORCH_CHECK(!t.defined() || t.is_cuda(), "c2dsr::encoder_pass: every tensor must be on the HIP device (no CPU "
                                               "fallback)");
}
void* S() { return c2t::stream(); }
float* F(const Tensor& t) { return t.data_ptr<float>(); }

// weights w: W_in [3d, d], b_in, W_out [d, d], b_out, W1 [d, d], b1, W2 [d, d], b2, norm1 w / b, norm2 w / b, final w / b
enum { W_IN, B_IN, W_OUT, B_OUT, W1, B1, W2, B2, N1W, N1B, N2W, N2B, NFW, NFB, NW };
// dropout keys (k0, k1) per site: input, attention, post-attention residual, FFN middle, FFN output
enum { K_INPUT, K_ATTN, K_SA, K_FFM, K_FFO };

struct Pass {
  int64_t B, L, d, M, nq, nk;
  int prec;
  std::vector<int64_t> keys;
  uint32_t k0(int site) const { return (uint32_t)keys[2 * site]; }
  uint32_t k1(int site) const { return (uint32_t)keys[2 * site + 1]; }
};

Pass check_common(const Tensor& seq, const std::vector<Tensor>& w, const Tensor& rs_idx, const Tensor& rs_off,
                  const Tensor& ks_idx, const Tensor& ks_off, int64_t n_head, std::vector<int64_t> keys,
                  int64_t precision) {
  TORCH_CHECK(seq.dim() == 2, "c2dsr::encoder_pass: seq must be [B, L]");
  Pass ps;
  ps.B = seq.size(0);
  ps.L = seq.size(1);
  ps.M = ps.B * ps.L;
  want(seq, "seq", at::kLong, {ps.B, ps.L});
  TORCH_CHECK((int64_t)w.size() == NW, "c2dsr::encoder_pass: 14 weight tensors expected");
  ps.d = w[W_OUT].size(0);
  const int64_t d = ps.d;
  want(w[W_IN], "in_proj_weight", at::kFloat, {3 * d, d});
  want(w[B_IN], "in_proj_bias", at::kFloat, {3 * d});
  for (int i : {W_OUT, W1, W2}) want(w[i], "projection weight", at::kFloat, {d, d});
  for (int i : {B_OUT, B1, B2, N1W, N1B, N2W, N2B, NFW, NFB}) want(w[i], "bias / norm parameter", at::kFloat, {d});
  TORCH_CHECK(d == 256, "c2dsr::encoder_pass: the fused pass runs the d = 256 projection kernels");
  TORCH_CHECK(c2dsr_attn_rows_supported((int)ps.L, (int)d, (int)n_head), "c2dsr::encoder_pass: attention shape");
  TORCH_CHECK(keys.size() == 10, "c2dsr::encoder_pass: keys = 5 (k0, k1) pairs");
  TORCH_CHECK(precision == 0 || precision == 1, "c2dsr::encoder_pass: precision 0 (fp32, split) or 1 (bf16)");
  ps.prec = (int)precision;
  ps.keys = keys;
  TORCH_CHECK(rs_idx.dim() == 1 && ks_idx.dim() == 1, "c2dsr::encoder_pass: row sets are 1-D");
  ps.nq = rs_idx.size(0);
  ps.nk = ks_idx.size(0);
  want(rs_idx, "rs_idx", at::kInt, {ps.nq});
  want(ks_idx, "ks_idx", at::kInt, {ps.nk});
  want(rs_off, "rs_off", at::kInt, {ps.B + 1});
  want(ks_off, "ks_off", at::kInt, {ps.B + 1});
  TORCH_CHECK(ps.nq <= ps.M && ps.nk <= ps.M, "c2dsr::encoder_pass: row sets larger than B·L");
  return ps;
}

// weight images (ops.weight_img): fp32 mode — split-bf16 fragment images (c2dsr_rgemm_x3f), bf16 mode — bf16
// fragment images (c2dsr_rgemm*, ldb = 0); rows = the output columns of the product, k = its reduction
void check_img(const Tensor& t, const char* name, const Pass& ps, int64_t rows, int64_t k) {
  TORCH_CHECK(t.defined() && t.scalar_type() == at::kBFloat16 && t.is_contiguous(),
              "c2dsr::encoder_pass: ", name, " must be a contiguous bf16 image");
  const int64_t r_pad = ps.prec == 0 ? (rows + 15) / 16 * 16 : (rows + 31) / 32 * 32;
  const int64_t cols = ps.prec == 0 ? 2 * k : k;
  TORCH_CHECK(t.numel() >= r_pad * cols, "c2dsr::encoder_pass: ", name, " image too small (", t.numel(), " < ",
              r_pad * cols, ")");
}

// C[M, N] = A[M, K]·Wᵀ + bias  with the pass's projection kernel; epi / aux as c2dsr_rgemm_aux
void proj(const Pass& ps, int64_t M, int64_t N, int64_t K, const Tensor& A, const Tensor& img, const Tensor& C,
          const float* bias, int epi, uint32_t k0, uint32_t k1, float p, int64_t row_base, const int* rowmap,
          int aux_mode, const float* aux, float aux_scale) {
  if (M == 0) return;
  if (ps.prec == 0) {
    TORCH_CHECK(A.scalar_type() == at::kFloat, "c2dsr::encoder_pass: split products take fp32 A");
    c2t::launch("c2dsr_rgemm_x3f", &c2dsr_rgemm_x3f, (int)M, (int)N, (int)K, F(A), (int)K, (const void*)img.data_ptr(),
                F(C), (int)N, 1.f, 0.f, bias, epi, k0, k1, p, row_base, rowmap, aux_mode, aux, (const int*)nullptr,
                aux_scale, S());
  } else if (A.scalar_type() == at::kBFloat16) {  // the attention's bf16 dq / dkv (in_proj dX)
    TORCH_CHECK(epi == 0 && aux_mode != 2, "c2dsr::encoder_pass: bf16 A takes no epilogue / mask");
    c2t::launch("c2dsr_rgemm_aux_b16a", &c2dsr_rgemm_aux_b16a, (int)M, (int)N, (int)K, (const void*)A.data_ptr(),
                (int)K, (const void*)img.data_ptr(), 0, F(C), (int)N, 1.f, 0.f, bias, aux_mode, aux,
                (const int*)nullptr, S());
  } else if (aux_mode) {
    c2t::launch("c2dsr_rgemm_aux", &c2dsr_rgemm_aux, (int)M, (int)N, (int)K, F(A), (int)K,
                (const void*)img.data_ptr(), 0, F(C), (int)N, 1.f, 0.f, bias, epi, k0, k1, p, row_base, rowmap,
                aux_mode, aux, (const int*)nullptr, aux_scale, S());
  } else {
    c2t::launch("c2dsr_rgemm", &c2dsr_rgemm, (int)M, (int)N, (int)K, F(A), (int)K, (const void*)img.data_ptr(), 0,
                F(C), (int)N, 1.f, 0.f, bias, epi, k0, k1, p, row_base, rowmap, S());
  }
}

// ---------------------------------------------------------------- forward
// img: [q (W_in rows 0..d), kv (W_in rows d..3d), out_proj, linear1, linear2, ‖W1[c]‖² (fp32 mode: the guard)]
// returns [out (nq × d), then the tensors the backward reads: xc, xk, q, kv, Psave, oc, xsave1, mean1, rstd1, x1, f,
// xsave2, st]
std::vector<Tensor> encoder_pass(const Tensor& seq, const Tensor& pos, const Tensor& H, const Tensor& E,
                                 const Tensor& P, double scale, const std::vector<Tensor>& w,
                                 const std::vector<Tensor>& img, const Tensor& rs_idx, const Tensor& rs_off,
                                 const Tensor& ks_idx, const Tensor& ks_off, int64_t pad, int64_t n_head, double p_,
                                 std::vector<int64_t> keys, std::vector<double> eps, int64_t row_off,
                                 int64_t precision, const OptT& guard_ws) {
  const Pass ps = check_common(seq, w, rs_idx, rs_off, ks_idx, ks_off, n_head, keys, precision);
  const int64_t B = ps.B, L = ps.L, d = ps.d, M = ps.M, nq = ps.nq, nk = ps.nk;
  const float p = (float)p_;
  want(pos, "pos", at::kLong, {B, L});
  want(H, "H", at::kFloat, {-1, d});
  want(E, "E", at::kFloat, {H.size(0), d});
  want(P, "P", at::kFloat, {-1, d});
  TORCH_CHECK(eps.size() == 3, "c2dsr::encoder_pass: eps = (norm1, norm2, final)");
  TORCH_CHECK(img.size() == 6, "c2dsr::encoder_pass: 6 weight images expected");
  check_img(img[0], "q image", ps, d, d);
  check_img(img[1], "kv image", ps, 2 * d, d);
  for (int i : {2, 3, 4}) check_img(img[i], "projection image", ps, d, d);
  const bool guard = ps.prec == 0;
  size_t gws = 0;
  if (guard) {
    want(img[5], "‖W1‖²", at::kFloat, {d});
    gws = c2dsr_rgemm_guard_workspace((int)nq, (int)d);
    TORCH_CHECK(guard_ws.has_value() && (size_t)guard_ws->nbytes() >= gws,
                "c2dsr::encoder_pass: the guarded linear1 needs its zeroed workspace (c2dsr_rgemm_guard_workspace)");
    on_device({&*guard_ws});
  }
  on_device({&seq, &pos, &H, &E, &P, &rs_idx, &rs_off, &ks_idx, &ks_off}, w);
  on_device({}, img);
  const auto f32 = H.options();
  const int64_t rb_rows = row_off * L;
  // K2 on the rows the layer reads: xc = X[rs], xk = X[ks] with X = drop((H[seq] + E[seq])·√d + P[pos]) (never stored)
  Tensor xck = at::empty({nq + nk, d}, f32);
  c2t::launch("c2dsr_embed_fwd_rows", &c2dsr_embed_fwd_rows, seq.data_ptr<int64_t>(), pos.data_ptr<int64_t>(), (int)M,
              (int)d, F(H), F(E), F(P), (float)scale, ps.k0(K_INPUT), ps.k1(K_INPUT), p, rb_rows,
              rs_idx.data_ptr<int>(), (int)nq, ks_idx.data_ptr<int>(), (int)nk, F(xck), (int)H.size(0), (int)P.size(0),
              c2t::errp(), S());
  Tensor xc = xck.narrow(0, 0, nq), xk = xck.narrow(0, nq, nk);
  const float* bin = F(w[B_IN]);
  Tensor q = at::empty({nq, d}, f32), kv = at::empty({nk, 2 * d}, f32);
  proj(ps, nq, d, d, xc, img[0], q, bin, 0, 0, 0, 0.f, 0, nullptr, 0, nullptr, 0.f);
  proj(ps, nk, 2 * d, d, xk, img[1], kv, bin + d, 0, 0, 0, 0.f, 0, nullptr, 0, nullptr, 0.f);
  Tensor oc = at::empty({nq, d}, f32);
  Tensor Ps = at::empty({(int64_t)c2dsr_attn_psave_floats((int)B, (int)L, (int)d, (int)n_head)}, f32);
  c2t::launch("c2dsr_attn_fwd_rows", &c2dsr_attn_fwd_rows, F(q), F(kv), seq.data_ptr<int64_t>(), (int64_t)pad,
              rs_idx.data_ptr<int>(), rs_off.data_ptr<int>(), ks_idx.data_ptr<int>(), ks_off.data_ptr<int>(), (int)B,
              (int)L, (int)d, (int)n_head, ps.k0(K_ATTN), ps.k1(K_ATTN), p, (int64_t)row_off, F(oc), F(Ps), S());
  Tensor sa = at::empty({nq, d}, f32);
  proj(ps, nq, d, d, oc, img[2], sa, F(w[B_OUT]), 0, 0, 0, 0.f, 0, nullptr, 0, nullptr, 0.f);
  // x1 = LN1(xc + drop(sa))
  Tensor xsave1 = at::empty({nq, d}, f32), x1 = at::empty({nq, d}, f32);
  Tensor mean1 = at::empty({nq}, f32), rstd1 = at::empty({nq}, f32);
  if (nq)
    c2t::launch("c2dsr_add_ln_fwd", &c2dsr_add_ln_fwd, F(xc), F(sa), (int)nq, (int)d, ps.k0(K_SA), ps.k1(K_SA), p,
                rb_rows, rs_idx.data_ptr<int>(), F(w[N1W]), F(w[N1B]), (float)eps[0], F(xsave1), F(x1), F(mean1),
                F(rstd1), S());
  sa.reset();
  // f = drop(relu(x1·W1ᵀ + b1)); f2 = f·W2ᵀ + b2
  Tensor f = at::empty({nq, d}, f32), f2 = at::empty({nq, d}, f32);
  if (nq) {
    if (guard)
      c2t::launch("c2dsr_rgemm_x3_relu_guard", &c2dsr_rgemm_x3_relu_guard, (int)nq, (int)d, (int)d, F(x1), (int)d,
                  (const void*)img[3].data_ptr(), 0, F(w[W1]), F(img[5]), F(f), (int)d, F(w[B1]), ps.k0(K_FFM),
                  ps.k1(K_FFM), p, rb_rows, rs_idx.data_ptr<int>(), guard_ws->data_ptr(), (size_t)guard_ws->nbytes(),
                  S());
    else
      proj(ps, nq, d, d, x1, img[3], f, F(w[B1]), 1, ps.k0(K_FFM), ps.k1(K_FFM), p, rb_rows, rs_idx.data_ptr<int>(), 0,
           nullptr, 0.f);
  }
  proj(ps, nq, d, d, f, img[4], f2, F(w[B2]), 0, 0, 0, 0.f, 0, nullptr, 0, nullptr, 0.f);
  // out = LNF(LN2(x1 + drop(f2)))  (norm2 and the encoder's final norm in one pass, Q16)
  Tensor xsave2 = at::empty({nq, d}, f32), out = at::empty({nq, d}, f32), st = at::empty({4, nq}, f32);
  if (nq)
    c2t::launch("c2dsr_add_ln2_fwd", &c2dsr_add_ln2_fwd, F(x1), F(f2), (int)nq, (int)d, ps.k0(K_FFO), ps.k1(K_FFO), p,
                rb_rows, rs_idx.data_ptr<int>(), F(w[N2W]), F(w[N2B]), (float)eps[1], F(w[NFW]), F(w[NFB]),
                (float)eps[2], F(xsave2), F(out), F(st), S());
  return {out, xc, xk, q, kv, Ps, oc, xsave1, mean1, rstd1, x1, f, xsave2, st};
}

// ---------------------------------------------------------------- backward
// imgT: the transposed images [q, kv, out_proj, linear1, linear2] (the dX products); ln_grads: the six LayerNorm
// parameter gradients (norm1 w / b, norm2 w / b, final w / b; accumulated).  The input gradient goes straight into
// the embedding backward (its two compact parts: query rows, key rows) over the prebuilt plans: G (the GCN output's
// gradient sink) += scale·drop(·), gP += drop(·).  Returns the weight-gradient operands in the order the
// host side's op-by-op path produces them: [dY, X] of linear2, linear1, out_proj, in_proj q rows, in_proj k/v rows
// (dY bf16 for the last two in bf16 mode).
std::vector<Tensor> encoder_pass_backward(const Tensor& dout, const std::vector<Tensor>& saved, const Tensor& seq,
                                          const std::vector<Tensor>& w, const std::vector<Tensor>& imgT,
                                          const Tensor& rs_idx, const Tensor& rs_inv, const Tensor& rs_off,
                                          const Tensor& ks_idx, const Tensor& ks_inv, const Tensor& ks_off, int64_t pad,
                                          int64_t n_head, double p_, std::vector<int64_t> keys, int64_t row_off,
                                          int64_t precision, const std::vector<Tensor>& ln_grads, const OptT& seq_plan,
                                          const OptT& pos_plan, double scale, const OptT& G, const OptT& gP) {
  const Pass ps = check_common(seq, w, rs_idx, rs_off, ks_idx, ks_off, n_head, keys, precision);
  const int64_t B = ps.B, L = ps.L, d = ps.d, M = ps.M, nq = ps.nq, nk = ps.nk;
  const float p = (float)p_;
  TORCH_CHECK(saved.size() == 13, "c2dsr::encoder_pass_backward: the 13 tensors encoder_pass saved");
  const Tensor &xc = saved[0], &xk = saved[1], &q = saved[2], &kv = saved[3], &Ps = saved[4], &oc = saved[5];
  const Tensor &xsave1 = saved[6], &mean1 = saved[7], &rstd1 = saved[8], &x1 = saved[9], &f = saved[10];
  const Tensor &xsave2 = saved[11], &st = saved[12];
  want(dout, "dout", at::kFloat, {nq, d});
  for (const Tensor* t : {&xc, &oc, &xsave1, &x1, &f, &xsave2, &q}) want(*t, "saved row tensor", at::kFloat, {nq, d});
  want(xk, "xk", at::kFloat, {nk, d});
  want(kv, "kv", at::kFloat, {nk, 2 * d});
  want(mean1, "mean1", at::kFloat, {nq});
  want(rstd1, "rstd1", at::kFloat, {nq});
  want(st, "st", at::kFloat, {4, nq});
  want(Ps, "Psave", at::kFloat, {(int64_t)c2dsr_attn_psave_floats((int)B, (int)L, (int)d, (int)n_head)});
  want(rs_inv, "rs_inv", at::kInt, {M});
  want(ks_inv, "ks_inv", at::kInt, {M});
  TORCH_CHECK(imgT.size() == 5, "c2dsr::encoder_pass_backward: 5 transposed images expected");
  check_img(imgT[0], "q image (transposed)", ps, d, d);
  check_img(imgT[1], "kv image (transposed)", ps, d, 2 * d);
  for (int i : {2, 3, 4}) check_img(imgT[i], "projection image (transposed)", ps, d, d);
  TORCH_CHECK(ln_grads.size() == 6, "c2dsr::encoder_pass_backward: 6 LayerNorm gradients expected");
  for (const Tensor& g : ln_grads) want(g, "LayerNorm gradient", at::kFloat, {d});
  on_device({&dout, &seq, &rs_idx, &rs_inv, &rs_off, &ks_idx, &ks_inv, &ks_off}, saved);
  on_device({}, w);
  on_device({}, imgT);
  on_device({}, ln_grads);
  const bool hg = G.has_value() && G->defined(), hp = gP.has_value() && gP->defined();
  TORCH_CHECK((!hg || seq_plan.has_value()) && (!hp || pos_plan.has_value()),
              "c2dsr::encoder_pass_backward: a plan per embedding output");
  if (hg) want(*G, "G", at::kFloat, {-1, d});
  if (hp) want(*gP, "gP", at::kFloat, {-1, d});
  for (const OptT* pl : {&seq_plan, &pos_plan})
    if (pl->has_value() && (*pl)->defined())
      TORCH_CHECK((*pl)->scalar_type() == at::kByte && (*pl)->is_cuda() &&
                      (size_t)(*pl)->nbytes() >= c2dsr_index_plan_bytes((int)M),
                  "c2dsr::encoder_pass_backward: plan buffer too small (or not on the device)");
  if (hg) on_device({&*G});
  if (hp) on_device({&*gP});
  const auto f32 = dout.options();
  const int64_t rb_rows = row_off * L;
  const int* rmap = rs_idx.data_ptr<int>();
  // out = LNF(LN2(x1 + drop(f2))): da2 → x1's gradient (its residual branch), df2 → linear2's output gradient
  Tensor da2 = at::empty({nq, d}, f32), df2 = at::empty({nq, d}, f32);
  Tensor ws2 = at::empty({(int64_t)c2dsr_ln2_bwd_workspace((int)d)}, f32.dtype(at::kByte));
  if (nq)
    c2t::launch("c2dsr_ln2_bwd", &c2dsr_ln2_bwd, F(xsave2), F(st), F(w[N2W]), F(w[N2B]), F(w[NFW]), F(dout), (int)nq,
                (int)d, F(da2), F(df2), ps.k0(K_FFO), ps.k1(K_FFO), p, rb_rows, rmap, (float*)nullptr, (float*)nullptr,
                (float*)nullptr, (float*)nullptr, ws2.data_ptr(), S());  // (partials only: c2dsr_ln_reduce2 below)
  // linear2's dX with linear1's drop(relu) backward in its epilogue (mask = f > 0, scale 1/(1-p))
  Tensor df = at::empty({nq, d}, f32);
  proj(ps, nq, d, d, df2, imgT[4], df, nullptr, 0, 0, 0, 0.f, 0, nullptr, 2, F(f), 1.f / (1.f - p));
  // linear1's dX accumulated onto da2 in place → dx1, the gradient of x1
  proj(ps, nq, d, d, df, imgT[3], da2, nullptr, 0, 0, 0, 0.f, 0, nullptr, 1, F(da2), 0.f);
  const Tensor& dx1 = da2;
  // x1 = LN1(xc + drop(sa)): da1 → xc's gradient through the residual (parked for the q rows), dsa → out_proj
  Tensor da1 = at::empty({nq, d}, f32), dsa = at::empty({nq, d}, f32);
  Tensor ws1 = at::empty({(int64_t)c2dsr_ln_bwd_workspace((int)d)}, f32.dtype(at::kByte));
  if (nq)
    c2t::launch("c2dsr_ln_bwd", &c2dsr_ln_bwd, F(xsave1), F(mean1), F(rstd1), F(w[N1W]), F(dx1), (int)nq, (int)d,
                F(da1), 0, F(dsa), ps.k0(K_SA), ps.k1(K_SA), p, rb_rows, rmap, (float*)nullptr, (float*)nullptr,
                ws1.data_ptr(), S());
  // both LayerNorms' parameter gradients from their partials in one launch
  if (nq)
    c2t::launch("c2dsr_ln_reduce2", &c2dsr_ln_reduce2, (const void*)ws2.data_ptr(), (int)nq, (const void*)ws1.data_ptr(),
                (int)nq, (int)d, F(ln_grads[2]), F(ln_grads[3]), F(ln_grads[4]), F(ln_grads[5]), F(ln_grads[0]),
                F(ln_grads[1]), S());
  Tensor doc = at::empty({nq, d}, f32);
  proj(ps, nq, d, d, dsa, imgT[2], doc, nullptr, 0, 0, 0, 0.f, 0, nullptr, 0, nullptr, 0.f);
  // attention on the compact rows → dq [nq, d], dkv [nk, 2d] (bf16 in bf16 mode: their only consumers are the
  // in_proj products, which read them as bf16 MFMA operands)
  const bool b16 = ps.prec == 1;
  const auto gt = b16 ? f32.dtype(at::kBFloat16) : f32;
  Tensor dq = at::empty({nq, d}, gt), dkv = at::empty({nk, 2 * d}, gt);
  c2t::launch("c2dsr_attn_bwd_rows", &c2dsr_attn_bwd_rows, F(q), F(kv), seq.data_ptr<int64_t>(), (int64_t)pad,
              rs_idx.data_ptr<int>(), rs_off.data_ptr<int>(), ks_idx.data_ptr<int>(), ks_off.data_ptr<int>(), (int)B,
              (int)L, (int)d, (int)n_head, ps.k0(K_ATTN), ps.k1(K_ATTN), p, (int64_t)row_off, F(Ps), F(doc),
              dq.data_ptr(), dkv.data_ptr(), (int)b16, S());
  // in_proj dX: q rows onto the parked residual gradient (in place), k / v rows into their own part
  proj(ps, nq, d, d, dq, imgT[0], da1, nullptr, 0, 0, 0, 0.f, 0, nullptr, 1, F(da1), 0.f);
  Tensor dxk = at::empty({nk, d}, f32);
  proj(ps, nk, d, 2 * d, dkv, imgT[1], dxk, nullptr, 0, 0, 0, 0.f, 0, nullptr, 0, nullptr, 0.f);
  // the embedding backward on the two compact parts: row r = da1[rs_inv[r]] + dxk[ks_inv[r]]
  if (hg || hp) {
    Tensor ws = at::empty({(int64_t)c2dsr_embed_bwd_planned_workspace((int)M, (int)d)}, f32.dtype(at::kByte));
    c2t::launch_x("c2dsr_embed_bwd_planned_rows", std::vector<double>{(double)(nq + nk), (double)(uintptr_t)seq.data_ptr()},
                  &c2dsr_embed_bwd_planned_rows, hg ? (const void*)seq_plan->data_ptr() : nullptr,
                  hp ? (const void*)pos_plan->data_ptr() : nullptr, (int)M, (int)d, (const float*)F(da1),
                  (const int*)rs_inv.data_ptr<int>(), (const float*)F(dxk), (const int*)ks_inv.data_ptr<int>(),
                  ps.k0(K_INPUT), ps.k1(K_INPUT), p, rb_rows, (float)scale, hg ? F(*G) : nullptr,
                  hg ? (int)G->size(0) : 0, hp ? F(*gP) : nullptr, hp ? (int)gP->size(0) : 0, ws.data_ptr(),
                  (size_t)ws.nbytes(), S());
  }
  return {df2, f, df, x1, dsa, oc, dq, xc, dkv, xk};
}

}  // namespace

void register_encoder_ops(torch::Library& m) {
  m.def("encoder_pass(Tensor seq, Tensor pos, Tensor H, Tensor E, Tensor P, float scale, Tensor[] w, Tensor[] img, "
        "Tensor rs_idx, Tensor rs_off, Tensor ks_idx, Tensor ks_off, int pad, int n_head, float p, int[] keys, "
        "float[] eps, int row_off, int precision, Tensor(a!)? guard_ws) -> Tensor[]");
  m.def("encoder_pass_backward(Tensor dout, Tensor[] saved, Tensor seq, Tensor[] w, Tensor[] imgT, Tensor rs_idx, "
        "Tensor rs_inv, Tensor rs_off, Tensor ks_idx, Tensor ks_inv, Tensor ks_off, int pad, int n_head, float p, "
        "int[] keys, int row_off, int precision, Tensor(a!)[] ln_grads, Tensor? seq_plan, Tensor? pos_plan, "
        "float scale, Tensor(b!)? G, Tensor(c!)? gP) -> Tensor[]");
  m.impl("encoder_pass", c10::DispatchKey::CompositeExplicitAutograd, TORCH_FN(encoder_pass));
  m.impl("encoder_pass_backward", c10::DispatchKey::CompositeExplicitAutograd, TORCH_FN(encoder_pass_backward));
}
