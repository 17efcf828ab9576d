// The training step's loss head (trainer.py:85-156) as stage operators: the pooling +
// bilinear discriminators + BCE, each classifier head's fused linear + cross-entropy (K5; logits never materialised),
// the loss reduction, and their backward.  The kernels and their order are those of the host side's op-by-op
// path (c2dsr_amd/losshead.py: LossHeadFn), so the results are bit-identical to it; every size is derived from the
// tensors and checked before the first launch.
//   loss_disc_forward     cal_mask + pooling (:85-108, Q5 cross masks), D_a / D_b (:104-108), BCE (:113-119)
//   ce_head_forward       one classifier head: last-R rows (:122-140), [C(h) ‖ c_pad(h)] logits, CE with
//                         ignore_index = the pad column (:131-146, Q6 / Q8), forward + the softmax part of dH online
//   loss_partials / loss_finalize   the count-weighted share loss, loss_rec, loss (:147-156, Q7)
//   ce_head_backward      dH, dW, db of one head (softmax part by the recomputing sweep, one-hot part deterministic)
//   loss_disc_backward    the discriminators' and the poolings' backward, and the heads' dH scattered into the
//                         encoder outputs' gradients
// mode 0: fp32 results on split-bf16 ×3 products (csrc/ce3.hip, rgemm.hip rg3); 1: bf16 operands.
#include <torch/library.h>

#include "c2t.h"

namespace {

using at::Tensor;
using OptT = std::optional<Tensor>;

void want(const Tensor& t, const char* op, const char* name, at::ScalarType dt, std::initializer_list<int64_t> shape) {
  TORCH_CHECK(t.defined(), "c2dsr::", op, ": ", name, " is undefined");
  TORCH_CHECK(t.scalar_type() == dt, "c2dsr::", op, ": ", name, " has dtype ", t.scalar_type(), ", expected ", dt);
  TORCH_CHECK(t.is_contiguous(), "c2dsr::", op, ": ", name, " must be contiguous");
  const std::vector<int64_t> s(shape);
  TORCH_CHECK(t.dim() == (int64_t)s.size(), "c2dsr::", op, ": ", name, " has ", t.dim(), " dims, expected ", s.size());
  for (size_t i = 0; i < s.size(); ++i)
    TORCH_CHECK(s[i] < 0 || t.size((int64_t)i) == s[i], "c2dsr::", op, ": ", name, " has shape ", t.sizes(),
                ", expected dim ", i, " = ", s[i]);
}
bool has(const OptT& t) { return t.has_value() && t->defined(); }
float* F(const Tensor& t) { return t.data_ptr<float>(); }
float* FO(const OptT& t) { return has(t) ? t->data_ptr<float>() : nullptr; }
const int* IO(const OptT& t) { return has(t) ? t->data_ptr<int>() : nullptr; }
void* S() { return c2t::stream(); }
void on_device(const char* op, const std::vector<const Tensor*>& ts) {
  for (const Tensor* t : ts)
    TORCH_CHECK(!t->defined() || t->is_cuda(), "c2dsr::", op, ": every tensor must be on the HIP device (no CPU "
                                                 "fallback)");
}
void on_device(const char* op, const std::vector<OptT>& ts) {
  for (const OptT& t : ts)
    TORCH_CHECK(!has(t) || t->is_cuda(), "c2dsr::", op, ": every tensor must be on the HIP device (no CPU fallback)");
}
int64_t ceil_to(int64_t v, int64_t m) { return (v + m - 1) / m * m; }

// an encoder output: [B, L, d], or the [n, d] rows of a row subset read through map [B·L] (compact index or -1)
void check_h(const Tensor& h, const OptT& map, const char* op, const char* name, int64_t B, int64_t L, int64_t d) {
  if (has(map)) {
    want(h, op, name, at::kFloat, {-1, d});
    want(*map, op, "row map", at::kInt, {B * L});
  } else {
    TORCH_CHECK(h.numel() == B * L * d && h.is_contiguous() && h.scalar_type() == at::kFloat, "c2dsr::", op, ": ",
                name, " must be a contiguous fp32 [B, L, d]");
  }
}

// the bilinear discriminators' U = X2·Wᵀ (rows 2B) on the projection kernels: the image of W [d, d]
void check_img(const Tensor& t, const char* op, int64_t mode, int64_t rows, int64_t k) {
  TORCH_CHECK(t.defined() && t.scalar_type() == at::kBFloat16 && t.is_contiguous(), "c2dsr::", op,
              ": weight images are contiguous bf16");
  const int64_t need = mode == 0 ? ceil_to(rows, 16) * 2 * k : ceil_to(rows, 32) * k;
  TORCH_CHECK(t.numel() >= need, "c2dsr::", op, ": weight image too small (", t.numel(), " < ", need, ")");
}
void proj(int64_t mode, int64_t M, int64_t N, int64_t K, const Tensor& A, const Tensor& img, const Tensor& C) {
  if (M == 0) return;
  if (mode == 0)
    c2t::launch("c2dsr_rgemm_x3f", &c2dsr_rgemm_x3f, (int)M, (int)N, (int)K, F(A), (int)K, (const void*)img.data_ptr(),
                F(C), (int)N, 1.f, 0.f, (const float*)nullptr, 0, 0u, 0u, 0.f, (int64_t)0, (const int*)nullptr, 0,
                (const float*)nullptr, (const int*)nullptr, 0.f, S());
  else
    c2t::launch("c2dsr_rgemm", &c2dsr_rgemm, (int)M, (int)N, (int)K, F(A), (int)K, (const void*)img.data_ptr(), 0,
                F(C), (int)N, 1.f, 0.f, (const float*)nullptr, 0, 0u, 0u, 0.f, (int64_t)0, (const int*)nullptr, S());
}

void colsum(const float* X, int64_t M, int64_t N, int64_t ldx, float* out, const at::TensorOptions& o) {
  Tensor ws = at::empty({(int64_t)c2dsr_colsum_workspace((int)M, (int)N)}, o.dtype(at::kByte));
  c2t::launch("c2dsr_colsum", &c2dsr_colsum, X, (int)M, (int)N, (int)ldx, 1.f, 1.f, out, ws.data_ptr(), S());
}

// ---------------------------------------------------------------- pooling + discriminators + BCE
// h: [h_share, hx, hy, h_neg_a, h_neg_b], maps: their row maps (None: full layout); D: [Da_w [1, d, d], Da_b?,
// Db_w, Db_b?]; img: the images of Da_w, Db_w as [d, d]; writes vec[8] = loss_mi.
// Returns [wa, wb, Phx, Phy, X2a, X2b, Ua, Ub, dS] (what the backward reads).
std::vector<Tensor> loss_disc_forward(const std::vector<Tensor>& h, const std::vector<OptT>& maps, const Tensor& gm_a,
                                      const Tensor& gm_b, const std::vector<OptT>& D, const std::vector<Tensor>& img,
                                      int64_t mode, int64_t B_global, const Tensor& vec) {
  const char* op = "loss_disc_forward";
  TORCH_CHECK(h.size() == 5 && maps.size() == 5 && D.size() == 4 && img.size() == 2,
              "c2dsr::loss_disc_forward: 5 encoder outputs and maps, 4 discriminator tensors, 2 images");
  TORCH_CHECK(gm_a.dim() == 2, "c2dsr::loss_disc_forward: gm_a must be [B, L]");
  const int64_t B = gm_a.size(0), L = gm_a.size(1);
  want(gm_a, op, "gm_a", at::kLong, {B, L});
  want(gm_b, op, "gm_b", at::kLong, {B, L});
  TORCH_CHECK(has(D[0]) && has(D[2]), "c2dsr::loss_disc_forward: D_a / D_b weights");
  const int64_t d = D[0]->size(-1);
  want(*D[0], op, "D_a.weight", at::kFloat, {1, d, d});
  want(*D[2], op, "D_b.weight", at::kFloat, {1, d, d});
  if (has(D[1])) want(*D[1], op, "D_a.bias", at::kFloat, {1});
  if (has(D[3])) want(*D[3], op, "D_b.bias", at::kFloat, {1});
  for (int i = 0; i < 5; ++i) check_h(h[i], maps[i], op, "encoder output", B, L, d);
  for (const Tensor& t : img) check_img(t, op, mode, d, d);
  want(vec, op, "vec", at::kFloat, {9});
  TORCH_CHECK(mode == 0 || mode == 1, "c2dsr::loss_disc_forward: mode 0 (split) or 1 (bf16)");
  on_device(op, {&gm_a, &gm_b, &vec, &img[0], &img[1]});
  on_device(op, maps);
  on_device(op, D);
  for (const Tensor& t : h) on_device(op, {&t});
  const auto f32 = vec.options();
  Tensor wa = at::empty({B, L}, f32), wb = at::empty({B, L}, f32);
  c2t::launch("c2dsr_pool_weights", &c2dsr_pool_weights, gm_a.data_ptr<int64_t>(), (int)B, (int)L, F(wa), S());
  c2t::launch("c2dsr_pool_weights", &c2dsr_pool_weights, gm_b.data_ptr<int64_t>(), (int)B, (int)L, F(wb), S());
  Tensor Phx = at::empty({B, d}, f32), Phy = at::empty({B, d}, f32);
  Tensor X2a = at::empty({2 * B, d}, f32), X2b = at::empty({2 * B, d}, f32);  // [h_share·wb ; h_neg_a·wa], [·wa ; ·wb]
  auto pool = [&](int i, const Tensor& w1, const Tensor* w2, float* o1, float* o2) {
    c2t::launch("c2dsr_pool2_fwd", &c2dsr_pool2_fwd, (const float*)F(h[i]), IO(maps[i]), (const float*)F(w1),
                w2 ? (const float*)F(*w2) : (const float*)nullptr, (int)B, (int)L, (int)d, o1, o2, S());
  };
  pool(1, wa, nullptr, F(Phx), nullptr);
  pool(2, wb, nullptr, F(Phy), nullptr);
  pool(0, wb, &wa, F(X2a), F(X2b));  // both poolings of h_share (Q5: cross-masked)
  pool(3, wa, nullptr, F(X2a) + B * d, nullptr);
  pool(4, wb, nullptr, F(X2b) + B * d, nullptr);
  Tensor Ua = at::empty({2 * B, d}, f32), Ub = at::empty({2 * B, d}, f32);
  proj(mode, 2 * B, d, d, X2a, img[0], Ua);
  proj(mode, 2 * B, d, d, X2b, img[1], Ub);
  Tensor Sc = at::empty({4, B}, f32);
  c2t::launch("c2dsr_mi_scores", &c2dsr_mi_scores, (const float*)F(Phx), (const float*)F(Ua), (const float*)FO(D[1]),
              (const float*)F(Phy), (const float*)F(Ub), (const float*)FO(D[3]), (int)B, (int)d, F(Sc), S());
  Tensor dS = at::empty({4, B}, f32);
  c2t::launch("c2dsr_mi_loss", &c2dsr_mi_loss, (const float*)F(Sc), (int)B, (int)B_global, F(vec) + 8, F(dS), S());
  return {wa, wb, Phx, Phy, X2a, X2b, Ua, Ub, dS};
}

// ---------------------------------------------------------------- one classifier head
// hs / hd: h_share and the domain output (maps as above); W [n, d], bias [n], wpad [1, d], bpad [1]; idx / inv / tc:
// the valid-row compaction of the stacked [share; specific] targets (Trainer.prepare: c2dsr_compact_valid), Mv0 / Mv1
// its counts (host); n_split: the fwd sweep's column splits.  Returns [rows (per-row losses, 0 on ignored rows) [2BR],
// then for the backward: Hpad, Hb, Wb, padc, lse2, bias2, Hc, lse_c, Up, part_m].
std::vector<Tensor> ce_head_forward(const Tensor& hs, const OptT& hs_map, const Tensor& hd, const OptT& hd_map,
                                    int64_t B, int64_t L, int64_t R, const Tensor& W, const Tensor& bias,
                                    const Tensor& wpad, const Tensor& bpad, const Tensor& idx, const Tensor& inv,
                                    const Tensor& tc, int64_t Mv0, int64_t Mv1, int64_t n_split, int64_t mode,
                                    int64_t keep_logits) {
  const char* op = "ce_head_forward";
  TORCH_CHECK(W.dim() == 2, "c2dsr::ce_head_forward: W must be [n, d]");
  const int64_t n = W.size(0), d = W.size(1), M2 = 2 * B * R, Mv = Mv0 + Mv1;
  want(W, op, "W", at::kFloat, {n, d});
  want(bias, op, "bias", at::kFloat, {n});
  want(wpad, op, "classifier_pad.weight", at::kFloat, {1, d});
  want(bpad, op, "classifier_pad.bias", at::kFloat, {1});
  check_h(hs, hs_map, op, "h_share", B, L, d);
  check_h(hd, hd_map, op, "h_domain", B, L, d);
  want(idx, op, "idx", at::kInt, {M2});
  want(inv, op, "inv", at::kInt, {M2});
  want(tc, op, "tc", at::kLong, {M2});
  TORCH_CHECK(R <= L && Mv0 >= 0 && Mv1 >= 0 && Mv0 <= B * R && Mv1 <= B * R, "c2dsr::ce_head_forward: counts");
  TORCH_CHECK((d == 128 || d == 256) && (mode == 0 || mode == 1) && n_split >= 1 && n_split <= 64,
              "c2dsr::ce_head_forward: d ∈ {128, 256}, mode 0 / 1, 1 ≤ n_split ≤ 64");
  on_device(op, {&hs, &hd, &W, &bias, &wpad, &bpad, &idx, &inv, &tc});
  on_device(op, {hs_map, hd_map});
  const auto f32 = W.options();
  const int64_t M_pad = std::max<int64_t>(64, ceil_to(Mv, 64)), n_pad = ceil_to(n, 128) + 64;
  const auto b16 = f32.dtype(at::kBFloat16);
  // Hpad, the valid rows Hc and their MFMA image (hi ‖ lo for the fp32 mode's split products, bf16 otherwise; zero
  // rows past Mv: whole tiles) in one pass over the gathered rows
  Tensor Hpad = at::empty({M2, d}, f32), Hc = at::empty({Mv, d}, f32);
  Tensor Hb = at::empty({M_pad, (mode == 0 ? 2 : 1) * d}, b16), Wb;
  c2t::launch("c2dsr_rec_gather_compact", &c2dsr_rec_gather_compact, (const float*)F(hs), IO(hs_map),
              (const float*)F(hd), IO(hd_map), (int)B, (int)L, (int)d, (int)R, (const int*)idx.data_ptr<int>(), (int)Mv,
              (int)M_pad, (int)(mode == 0), F(Hpad), Mv ? F(Hc) : nullptr, (void*)Hb.data_ptr(), S());
  if (mode == 0) {  // hi ‖ lo images, zero rows past the end (whole 32-row tiles)
    const int64_t n32 = ceil_to(n, 32);
    Wb = at::empty({n32, 2 * d}, b16);
    c2t::launch("c2dsr_f32_split_bf16", &c2dsr_f32_split_bf16, (const float*)F(W), (long)n, (int)d, (long)n32,
                (void*)Wb.data_ptr(), S());
  } else {  // whole 64-row tiles, zero rows past the end
    const int64_t n64 = ceil_to(n, 64);
    Wb = at::empty({n64, d}, b16);
    if (n64 > n) Wb.narrow(0, n, n64 - n).zero_();
    c2t::launch("c2dsr_f32_to_bf16", &c2dsr_f32_to_bf16, (const float*)F(W), (long)W.numel(), (void*)Wb.data_ptr(), S());
  }
  Tensor bias2 = at::empty({n_pad}, f32);
  c2t::launch("c2dsr_ce_bias2", &c2dsr_ce_bias2, (const float*)F(bias), (int)n, (int)n_pad, F(bias2), S());
  Tensor padlogit = at::empty({M2}, f32);
  c2t::launch("c2dsr_rowdot", &c2dsr_rowdot, (const float*)F(Hpad), (long)d, (const float*)F(wpad), (long)0, (int)M2,
              (int)d, (const float*)F(bpad), F(padlogit), (long)1, S());
  const int64_t m1 = std::max<int64_t>(Mv, 1);
  Tensor padc = at::empty({m1}, f32);
  if (Mv)
    c2t::launch("c2dsr_gather_rows", &c2dsr_gather_rows, (const float*)F(padlogit), (long)1, idx.data_ptr<int>(),
                (int)Mv, 1, F(padc), S());
  Tensor lse_c = at::empty({m1}, f32), rows_c = at::empty({m1}, f32), lse2 = at::empty({M_pad}, f32);
  Tensor pm = at::empty({n_split, Mv}, f32), psum = at::empty({n_split, Mv}, f32), Up = at::empty({n_split, Mv, d}, f32);
  // keep_logits (fp32 mode): the forward also stores the logits for the dW sweep (c2dsr_ce3_fused_dw_lg*), which then
  // skips recomputing them; empty otherwise
  const bool lg_on = keep_logits && mode == 0 && Mv > 0;
  Tensor lg = at::empty({lg_on ? (int64_t)c2dsr_ce3_logits_floats((int)Mv, (int)n) : 0}, f32);
  if (Mv) {  // forward + the softmax part of the input gradient in one sweep (online lse, flash style)
    if (lg_on)
      c2t::launch("c2dsr_ce3_fused_fwd_u_lg", &c2dsr_ce3_fused_fwd_u_lg, (const void*)Hb.data_ptr(),
                  (const void*)Wb.data_ptr(), (const float*)F(bias2), (int)Mv, (int)n, (int)d, (int)n_split, F(pm),
                  F(psum), F(Up), (const float*)F(padc), tc.data_ptr<int64_t>(), (const float*)F(Hc),
                  (const float*)F(W), (const float*)F(bias), F(lse_c), F(lse2), F(rows_c), F(lg), S());
    else if (mode == 0)
      c2t::launch("c2dsr_ce3_fused_fwd_u", &c2dsr_ce3_fused_fwd_u, (const void*)Hb.data_ptr(), (const void*)Wb.data_ptr(),
                  (const float*)F(bias2), (int)Mv, (int)n, (int)d, (int)n_split, F(pm), F(psum), F(Up),
                  (const float*)F(padc), tc.data_ptr<int64_t>(), (const float*)F(Hc), (const float*)F(W),
                  (const float*)F(bias), F(lse_c), F(lse2), F(rows_c), S());
    else
      c2t::launch("c2dsr_ce3b_fused_fwd_u", &c2dsr_ce3b_fused_fwd_u, (const void*)Hb.data_ptr(),
                  (const void*)Wb.data_ptr(), (const float*)F(bias2), (int)Mv, (int)n, (int)d, (int)n_split, F(pm),
                  F(psum), F(Up), (const float*)F(padc), tc.data_ptr<int64_t>(), (const float*)F(Hc),
                  (const float*)F(W), (const float*)F(bias), F(lse_c), F(lse2), F(rows_c), S());
  }
  Tensor rows = at::empty({M2}, f32);
  c2t::launch("c2dsr_expand_rows", &c2dsr_expand_rows, (const float*)F(rows_c), inv.data_ptr<int>(), (int)M2, 1,
              F(rows), S());  // per-row losses, 0 on ignored rows
  return {rows, Hpad, Hb, Wb, padc, lse2, bias2, Hc, lse_c, Up, pm, lg};
}

// ---------------------------------------------------------------- loss
// vec[0..7] = the heads' CE sums and valid counts (tA / tB: the stacked targets [2BR])
void loss_partials(const Tensor& rowsA, const Tensor& tA, int64_t n_a, const Tensor& rowsB, const Tensor& tB,
                   int64_t n_b, int64_t BR, const Tensor& vec) {
  const char* op = "loss_partials";
  want(rowsA, op, "rowsA", at::kFloat, {2 * BR});
  want(rowsB, op, "rowsB", at::kFloat, {2 * BR});
  want(tA, op, "tA", at::kLong, {2 * BR});
  want(tB, op, "tB", at::kLong, {2 * BR});
  want(vec, op, "vec", at::kFloat, {9});
  on_device(op, {&rowsA, &rowsB, &tA, &tB, &vec});
  Tensor lpw = at::empty({std::max<int64_t>(1, (int64_t)c2dsr_loss_partials_workspace((int)BR))}, vec.options());
  c2t::launch("c2dsr_loss_partials", &c2dsr_loss_partials, (const float*)F(rowsA), tA.data_ptr<int64_t>(), (int)n_a,
              (const float*)F(rowsB), tB.data_ptr<int64_t>(), (int)n_b, (int)BR, F(vec), F(lpw), S());
}

// (loss, loss_rec, loss_mi) and the heads' per-row gradient coefficients; cnt: the all-reduced valid counts (DP)
std::vector<Tensor> loss_finalize(const Tensor& vec, const OptT& cnt, int64_t BR_global, double lam) {
  const char* op = "loss_finalize";
  want(vec, op, "vec", at::kFloat, {9});
  if (has(cnt)) want(*cnt, op, "cnt", at::kFloat, {9});
  on_device(op, {&vec});
  on_device(op, {cnt});
  const auto f32 = vec.options();
  Tensor out3 = at::empty({3}, f32), coefA = at::empty({2}, f32), coefB = at::empty({2}, f32);
  c2t::launch("c2dsr_loss_finalize", &c2dsr_loss_finalize, (const float*)F(vec), (const float*)FO(cnt), (int)BR_global,
              (float)lam, F(out3), F(coefA), F(coefB), S());
  return {out3, coefA, coefB};
}

// ---------------------------------------------------------------- backward of one head
// saved: ce_head_forward's outputs 1.. (Hpad, Hb, Wb, padc, lse2, bias2, Hc, lse_c, Up, part_m, logits); gW / gb / gwpad /
// gbpad: the parameters' gradients (accumulated; may be absent); tplan: the sort plan of the valid targets (the
// one-hot part's deterministic segment sums; absent: sorted here); n_rsplit: the dW sweep's row splits
// (losshead.dw_plan); dw_full: with n_rsplit < 0, the W rows of the whole rounds the plan costed (a multiple of 128
// below n — passed, not re-derived here, so the sweep splits exactly as the plan that chose it).
// Returns [dHcat [2BR, d], dpad [2BR]].
std::vector<Tensor> ce_head_backward(const std::vector<Tensor>& saved, const Tensor& W, const Tensor& inv,
                                     const Tensor& tc, int64_t Mv0, int64_t Mv1, const Tensor& coef,
                                     const Tensor& gscale, double lam, const OptT& gW, const OptT& gb,
                                     const OptT& gwpad, const OptT& gbpad, const OptT& tplan, int64_t n_rsplit,
                                     int64_t mode, int64_t dw_full) {
  const char* op = "ce_head_backward";
  TORCH_CHECK(saved.size() == 11, "c2dsr::ce_head_backward: the 11 tensors ce_head_forward saved");
  const Tensor &Hpad = saved[0], &Hb = saved[1], &Wb = saved[2], &padc = saved[3], &lse2 = saved[4];
  const Tensor &bias2 = saved[5], &Hc = saved[6], &lse_c = saved[7], &Up = saved[8], &pm = saved[9];
  const Tensor& lg = saved[10];
  TORCH_CHECK(W.dim() == 2 && Hpad.dim() == 2, "c2dsr::ce_head_backward: W [n, d], Hpad [2BR, d]");
  const int64_t n = W.size(0), d = W.size(1), M2 = Hpad.size(0), Mv = Mv0 + Mv1;
  const int64_t M_pad = std::max<int64_t>(64, ceil_to(Mv, 64)), m1 = std::max<int64_t>(Mv, 1);
  want(W, op, "W", at::kFloat, {n, d});
  want(Hpad, op, "Hpad", at::kFloat, {M2, d});
  want(inv, op, "inv", at::kInt, {M2});
  want(tc, op, "tc", at::kLong, {M2});
  want(Hc, op, "Hc", at::kFloat, {Mv, d});
  want(padc, op, "padc", at::kFloat, {m1});
  want(lse_c, op, "lse_c", at::kFloat, {m1});
  want(lse2, op, "lse2", at::kFloat, {M_pad});
  TORCH_CHECK(Up.dim() == 3 && Up.size(1) == Mv && Up.size(2) == d, "c2dsr::ce_head_backward: Up [ns, Mv, d]");
  const int64_t ns = Up.size(0);
  want(pm, op, "part_m", at::kFloat, {ns, Mv});
  want(bias2, op, "bias2", at::kFloat, {ceil_to(n, 128) + 64});
  TORCH_CHECK(Hb.scalar_type() == at::kBFloat16 && Wb.scalar_type() == at::kBFloat16 &&
                  Hb.numel() >= M_pad * (mode == 0 ? 2 : 1) * d && Wb.numel() >= n * (mode == 0 ? 2 : 1) * d,
              "c2dsr::ce_head_backward: operand images");
  want(coef, op, "coef", at::kFloat, {2});
  want(gscale, op, "gscale", at::kFloat, {1});
  if (has(gW)) want(*gW, op, "gW", at::kFloat, {n, d});
  if (has(gb)) want(*gb, op, "gb", at::kFloat, {n});
  if (has(gwpad)) want(*gwpad, op, "gwpad", at::kFloat, {1, d});
  if (has(gbpad)) want(*gbpad, op, "gbpad", at::kFloat, {1});
  if (has(tplan))
    TORCH_CHECK(tplan->scalar_type() == at::kByte && (size_t)tplan->nbytes() >= c2dsr_index_plan_bytes((int)Mv),
                "c2dsr::ce_head_backward: target plan too small");
  // stored logits (the forward's keep_logits): the dW sweeps read them instead of recomputing them
  const bool lg_on = lg.numel() > 0;
  if (lg_on)
    want(lg, op, "logits", at::kFloat, {(int64_t)c2dsr_ce3_logits_floats((int)Mv, (int)n)});
  TORCH_CHECK(!lg_on || mode == 0, "c2dsr::ce_head_backward: stored logits are the fp32 mode's");
  // n_rsplit 0: the stream-K sweep (c2dsr_ce3_fused_dw_sk); −k: whole rounds unsplit, the remainder k ways (both need
  // both gradients; losshead.dw_plan)
  TORCH_CHECK(n_rsplit >= -64 && n_rsplit <= 64 && (mode == 0 || mode == 1), "c2dsr::ce_head_backward: splits / mode");
  on_device(op, {&W, &Hpad, &inv, &tc, &Hc, &padc, &lse_c, &lse2, &Up, &pm, &bias2, &Hb, &Wb, &coef, &gscale});
  if (lg_on) on_device(op, {&lg});
  on_device(op, {gW, gb, gwpad, gbpad, tplan});
  const auto f32 = W.options();
  Tensor rw = at::empty({M_pad}, f32), t32 = at::empty({M_pad}, f32.dtype(at::kInt));
  Tensor dpad_c = at::empty({m1}, f32), crow = at::empty({M_pad + 64}, f32), dHc = at::empty({m1, d}, f32);
  if (Mv) {
    // compact rows keep their order: the first Mv0 are the shared-sequence rows (coef[0])
    c2t::launch("c2dsr_ce_row_weights", &c2dsr_ce_row_weights, tc.data_ptr<int64_t>(), (int)Mv, (int)M_pad, (int)n,
                (const float*)F(coef), (int)Mv0, (const float*)F(gscale), (float)lam, (const float*)F(padc),
                (const float*)F(lse_c), F(rw), t32.data_ptr<int>(), (const float*)F(lse2), F(crow), F(dpad_c), S());
    // dH = rw·(softmax·W − W[t]) from the forward's online partials
    c2t::launch("c2dsr_ce_dh_from_u", &c2dsr_ce_dh_from_u, (const float*)F(Up), (const float*)F(pm), (int)ns, (int)Mv,
                (int)d, (const float*)F(lse2), (const int*)t32.data_ptr<int>(), (const float*)F(rw),
                (const float*)F(W), (int)n, F(dHc), S());
    // the sweep over W rows [off, off + rows) (the stationary operand: image rows, bias2, outputs offset alike)
    auto dw_rows = [&](int nr, float* dWp, float* dbp, int64_t off, int64_t rows) {
      if (lg_on) {
        c2t::launch("c2dsr_ce3_fused_dw_lg", &c2dsr_ce3_fused_dw_lg, (const void*)Hb.data_ptr(), (const float*)F(lg),
                    (int)Mv, (int)n, (int)off, (int)rows, (int)d, nr, (const float*)F(crow), dWp, dbp, S());
        return;
      }
      const void* wimg = (const void*)((const at::BFloat16*)Wb.data_ptr() + off * (mode == 0 ? 2 : 1) * d);
      const float* b2 = (const float*)F(bias2) + off;
      if (mode == 0)
        c2t::launch("c2dsr_ce3_fused_dw", &c2dsr_ce3_fused_dw, (const void*)Hb.data_ptr(), wimg, b2, (int)Mv,
                    (int)rows, (int)d, nr, (const float*)F(crow), dWp, dbp, S());
      else
        c2t::launch("c2dsr_ce3b_fused_dw", &c2dsr_ce3b_fused_dw, (const void*)Hb.data_ptr(), wimg, b2, (int)Mv,
                    (int)rows, (int)d, nr, (const float*)F(crow), dWp, dbp, S());
    };
    auto dw = [&](int nr, float* dWp, float* dbp) { dw_rows(nr, dWp, dbp, 0, n); };
    if (n_rsplit == 0 && has(gW) && has(gb)) {  // stream-K: whole row blocks added directly, split ones combined
      Tensor ws = at::empty({(int64_t)c2dsr_ce3_dw_sk_workspace((int)d)}, f32.dtype(at::kByte));
      if (lg_on)
        c2t::launch("c2dsr_ce3_fused_dw_lg_sk", &c2dsr_ce3_fused_dw_lg_sk, (const void*)Hb.data_ptr(),
                    (const float*)F(lg), (int)Mv, (int)n, (int)d, (const float*)F(crow), F(*gW), F(*gb), ws.data_ptr(),
                    (size_t)ws.nbytes(), S());
      else if (mode == 0)
        c2t::launch("c2dsr_ce3_fused_dw_sk", &c2dsr_ce3_fused_dw_sk, (const void*)Hb.data_ptr(),
                    (const void*)Wb.data_ptr(), (const float*)F(bias2), (int)Mv, (int)n, (int)d, (const float*)F(crow),
                    F(*gW), F(*gb), ws.data_ptr(), (size_t)ws.nbytes(), S());
      else
        c2t::launch("c2dsr_ce3b_fused_dw_sk", &c2dsr_ce3b_fused_dw_sk, (const void*)Hb.data_ptr(),
                    (const void*)Wb.data_ptr(), (const float*)F(bias2), (int)Mv, (int)n, (int)d, (const float*)F(crow),
                    F(*gW), F(*gb), ws.data_ptr(), (size_t)ws.nbytes(), S());
    } else if (n_rsplit < 0 && has(gW) && has(gb)) {
      // whole rounds of unsplit row blocks onto the gradients, then the last partial round's row blocks −n_rsplit ways
      const int64_t full = dw_full, rem = n - full, k = -n_rsplit;
      TORCH_CHECK(full > 0 && full % 128 == 0 && rem > 0, "c2dsr::ce_head_backward: a remainder split needs dw_full = "
                  "the whole rounds' rows (a positive multiple of 128 below n = ", n, "), got ", dw_full);
      dw_rows(0, F(*gW), F(*gb), 0, full);
      Tensor dWp = at::empty({k, rem, d}, f32), dbp = at::empty({k, rem}, f32);
      dw_rows((int)k, F(dWp), F(dbp), full, rem);
      c2t::launch("c2dsr_sum_parts", &c2dsr_sum_parts, (const float*)F(dWp), (int)k, (long)(rem * d), 1.f,
                  F(*gW) + full * d, S());
      c2t::launch("c2dsr_sum_parts", &c2dsr_sum_parts, (const float*)F(dbp), (int)k, (long)rem, 1.f, F(*gb) + full,
                  S());
    } else if (n_rsplit <= 1 && has(gW) && has(gb)) {
      dw(0, F(*gW), F(*gb));  // one split: the sweep adds onto the gradients itself (no partials / sum)
    } else {
      n_rsplit = std::max<int64_t>(n_rsplit, 1);
      Tensor dWp = at::empty({n_rsplit, n, d}, f32), dbp = at::empty({n_rsplit, n}, f32);
      dw((int)n_rsplit, F(dWp), F(dbp));
      if (has(gW))
        c2t::launch("c2dsr_sum_parts", &c2dsr_sum_parts, (const float*)F(dWp), (int)n_rsplit, (long)(n * d), 1.f,
                    F(*gW), S());
      if (has(gb))
        c2t::launch("c2dsr_sum_parts", &c2dsr_sum_parts, (const float*)F(dbp), (int)n_rsplit, (long)n, 1.f, F(*gb),
                    S());
    }
    if (has(gW) || has(gb)) {  // the one-hot part: −rw·H[r] into the target's row, deterministic segment sums
      if (has(tplan)) {
        Tensor ws = at::empty({(int64_t)c2dsr_ce_onehot_planned_workspace((int)Mv, (int)n, (int)d)}, f32.dtype(at::kByte));
        c2t::launch("c2dsr_ce_onehot_dw_planned", &c2dsr_ce_onehot_dw_planned, (const void*)tplan->data_ptr(), (int)Mv,
                    (int)n, (const float*)F(Hc), (int)d, (const float*)F(rw), FO(gW), FO(gb), ws.data_ptr(),
                    (size_t)ws.nbytes(), S());
      } else {
        Tensor ws = at::empty({(int64_t)c2dsr_ce_onehot_workspace((int)Mv, (int)n, (int)d)}, f32.dtype(at::kByte));
        c2t::launch("c2dsr_ce_onehot_dw", &c2dsr_ce_onehot_dw, tc.data_ptr<int64_t>(), (int)Mv, (int)n,
                    (const float*)F(Hc), (int)d, (const float*)F(rw), FO(gW), FO(gb), ws.data_ptr(),
                    (size_t)ws.nbytes(), S());
      }
    }
  }
  Tensor dHcat = at::empty({M2, d}, f32), dpad = at::empty({M2}, f32);
  c2t::launch("c2dsr_expand_rows", &c2dsr_expand_rows, (const float*)F(dHc), inv.data_ptr<int>(), (int)M2, (int)d,
              F(dHcat), S());  // 0 on ignored rows
  c2t::launch("c2dsr_expand_rows", &c2dsr_expand_rows, (const float*)F(dpad_c), inv.data_ptr<int>(), (int)M2, 1,
              F(dpad), S());
  if (has(gwpad)) {  // gwpad[0, :] += Σ_r dpad[r]·Hpad[r, :]
    Tensor ws = at::empty({(int64_t)c2dsr_colsum_workspace((int)M2, (int)d)}, f32.dtype(at::kByte));
    c2t::launch("c2dsr_wcolsum", &c2dsr_wcolsum, (const float*)F(Hpad), (int)M2, (int)d, (int)d, (const float*)F(dpad),
                (long)1, 1.f, 1.f, F(*gwpad), ws.data_ptr(), S());
  }
  if (has(gbpad)) colsum(F(dpad), M2, 1, 1, F(*gbpad), f32);
  return {dHcat, dpad};
}

// ---------------------------------------------------------------- discriminators + poolings backward
// fwd: loss_disc_forward's outputs; D / imgT (the transposed images of Da_w, Db_w) / gD (gradients of Da_w, Da_b,
// Db_w, Db_b, each may be absent); heads: [dHcat_a, dpad_a, dHcat_b, dpad_b]; sub: the row subsets of the five
// outputs ([n] idx, or absent for the full layout); maps as in the forward; hshape: the outputs' row counts
// (n, or B·L).  Returns the five encoder outputs' gradients (shaped like the outputs: [n, d] or [B, L, d]).
std::vector<Tensor> loss_disc_backward(const std::vector<Tensor>& fwd, const Tensor& gscale, double lam,
                                       const std::vector<OptT>& D, const std::vector<Tensor>& imgT,
                                       const std::vector<OptT>& gD, const std::vector<Tensor>& heads,
                                       const Tensor& wpad, const std::vector<OptT>& sub, const std::vector<OptT>& maps,
                                       int64_t L, int64_t R, int64_t mode) {
  const char* op = "loss_disc_backward";
  TORCH_CHECK(fwd.size() == 9 && D.size() == 4 && imgT.size() == 2 && gD.size() == 4 && heads.size() == 4 &&
                  sub.size() == 5 && maps.size() == 5,
              "c2dsr::loss_disc_backward: argument lists");
  const Tensor &wa = fwd[0], &wb = fwd[1], &Phx = fwd[2], &Phy = fwd[3], &X2a = fwd[4], &X2b = fwd[5];
  const Tensor &Ua = fwd[6], &Ub = fwd[7], &dS = fwd[8];
  TORCH_CHECK(Phx.dim() == 2, "c2dsr::loss_disc_backward: Phx [B, d]");
  const int64_t B = Phx.size(0), d = Phx.size(1), M2 = 2 * B * R;
  want(wa, op, "wa", at::kFloat, {B, L});
  want(wb, op, "wb", at::kFloat, {B, L});
  for (const Tensor* t : {&Phx, &Phy}) want(*t, op, "pooled", at::kFloat, {B, d});
  for (const Tensor* t : {&X2a, &X2b, &Ua, &Ub}) want(*t, op, "discriminator operand", at::kFloat, {2 * B, d});
  want(dS, op, "dS", at::kFloat, {4, B});
  want(gscale, op, "gscale", at::kFloat, {1});
  for (const Tensor& t : imgT) check_img(t, op, mode, d, d);
  if (has(gD[0])) want(*gD[0], op, "gDa_w", at::kFloat, {1, d, d});
  if (has(gD[2])) want(*gD[2], op, "gDb_w", at::kFloat, {1, d, d});
  if (has(gD[1])) want(*gD[1], op, "gDa_b", at::kFloat, {1});
  if (has(gD[3])) want(*gD[3], op, "gDb_b", at::kFloat, {1});
  want(heads[0], op, "dHcat_a", at::kFloat, {M2, d});
  want(heads[2], op, "dHcat_b", at::kFloat, {M2, d});
  want(heads[1], op, "dpad_a", at::kFloat, {M2});
  want(heads[3], op, "dpad_b", at::kFloat, {M2});
  want(wpad, op, "classifier_pad.weight", at::kFloat, {1, d});
  std::vector<int64_t> nrow(5);
  for (int i = 0; i < 5; ++i) {
    TORCH_CHECK(has(sub[i]) == has(maps[i]), "c2dsr::loss_disc_backward: a row subset comes with its map");
    if (has(sub[i])) {
      TORCH_CHECK(sub[i]->dim() == 1 && sub[i]->scalar_type() == at::kInt, "c2dsr::loss_disc_backward: idx [n] int32");
      nrow[i] = sub[i]->size(0);
      want(*maps[i], op, "row map", at::kInt, {B * L});
    } else {
      nrow[i] = B * L;
    }
  }
  on_device(op, {&wa, &wb, &Phx, &Phy, &X2a, &X2b, &Ua, &Ub, &dS, &gscale, &imgT[0], &imgT[1], &heads[0], &heads[1],
                 &heads[2], &heads[3], &wpad});
  on_device(op, gD);
  on_device(op, sub);
  on_device(op, maps);
  const auto f32 = Phx.options();
  c2t::launch("c2dsr_scale_ds", &c2dsr_scale_ds, F(dS), (int)(4 * B), (const float*)F(gscale), (float)(1.0 - lam), S());
  const Tensor* x1s[2] = {&Phx, &Phy};
  const Tensor* X2s[2] = {&X2a, &X2b};
  const Tensor* Us[2] = {&Ua, &Ub};
  Tensor dx1[2], dX2[2], dUs[2];
  for (int j = 0; j < 2; ++j) {
    dx1[j] = at::empty({B, d}, f32);
    dUs[j] = at::empty({2 * B, d}, f32);
  }
  // both discriminators' row-scale products in one launch
  c2t::launch("c2dsr_bilinear_ds", &c2dsr_bilinear_ds, (const float*)F(*Us[0]), (const float*)F(*Us[1]),
              (const float*)F(*x1s[0]), (const float*)F(*x1s[1]), (const float*)F(dS), (int)B, (int)d, F(dx1[0]),
              F(dx1[1]), F(dUs[0]), F(dUs[1]), S());
  for (int j = 0; j < 2; ++j) {
    const int k = 2 * j;
    const Tensor& dU = dUs[j];
    dX2[j] = at::empty({2 * B, d}, f32);
    proj(mode, 2 * B, d, d, dU, imgT[j], dX2[j]);
    const OptT& gWd = gD[k];
    if (has(gWd) && 2 * B > 0) {  // not deferred: the head range is reduced as this backward returns
      Tensor ws = at::empty({(int64_t)c2dsr_wgemm_workspace((int)d)}, f32.dtype(at::kByte));
      if (mode == 0)
        c2t::launch("c2dsr_wgemm_x3", &c2dsr_wgemm_x3, (int)(2 * B), (int)d, (int)d, (const float*)F(dU), (int)d,
                    (const float*)F(*X2s[j]), (int)d, 1.f, F(*gWd), (float*)nullptr, ws.data_ptr(), S());
      else
        c2t::launch("c2dsr_wgemm", &c2dsr_wgemm, (int)(2 * B), (int)d, (int)d, (const float*)F(dU), (int)d,
                    (const float*)F(*X2s[j]), (int)d, 1.f, F(*gWd), (float*)nullptr, ws.data_ptr(), S());
    }
    if (has(gD[k + 1])) colsum(F(dS) + k * B, 2 * B, 1, 1, F(*gD[k + 1]), f32);
  }
  // the pooling backward WRITES the five encoder-output gradients (no zero fill); the heads then add their
  // last-R-position parts (row-subset outputs get row-subset gradients: pooling writes their rows, heads add
  // through the maps)
  std::vector<Tensor> dh(5);
  for (int i = 0; i < 5; ++i)
    dh[i] = has(sub[i]) ? at::empty({nrow[i], d}, f32) : at::empty({B, L, d}, f32);
  auto pb = [&](const float* d1, const Tensor& w1, const float* d2, const Tensor* w2, int i) {
    c2t::launch("c2dsr_pool2_bwd", &c2dsr_pool2_bwd, d1, (const float*)F(w1), d2,
                w2 ? (const float*)F(*w2) : (const float*)nullptr, (int)B, (int)L, (int)d, IO(sub[i]),
                has(sub[i]) ? (int)nrow[i] : 0, 0, F(dh[i]), S());
  };
  pb(F(dx1[0]), wa, nullptr, nullptr, 1);
  pb(F(dx1[1]), wb, nullptr, nullptr, 2);
  pb(F(dX2[0]), wb, F(dX2[1]), &wa, 0);
  pb(F(dX2[0]) + B * d, wa, nullptr, nullptr, 3);
  pb(F(dX2[1]) + B * d, wb, nullptr, nullptr, 4);
  for (int k = 0; k < 2; ++k)  // classifier_pad's input gradient (pad column ⊗ wpad) folded into the scatter
    c2t::launch("c2dsr_rec_scatter", &c2dsr_rec_scatter, (const float*)F(heads[2 * k]),
                (const float*)F(heads[2 * k + 1]), (long)1, (const float*)F(wpad), (int)B, (int)L, (int)d, (int)R,
                F(dh[0]), IO(maps[0]), F(dh[1 + k]), IO(maps[1 + k]), S());
  return dh;
}

}  // namespace

void register_losshead_ops(torch::Library& m) {
  m.def("loss_disc_forward(Tensor[] h, Tensor?[] maps, Tensor gm_a, Tensor gm_b, Tensor?[] D, Tensor[] img, int mode, "
        "int B_global, Tensor(a!) vec) -> Tensor[]");
  m.def("ce_head_forward(Tensor hs, Tensor? hs_map, Tensor hd, Tensor? hd_map, int B, int L, int R, Tensor W, "
        "Tensor bias, Tensor wpad, Tensor bpad, Tensor idx, Tensor inv, Tensor tc, int Mv0, int Mv1, int n_split, "
        "int mode, int keep_logits=0) -> Tensor[]");
  m.def("loss_partials(Tensor rowsA, Tensor tA, int n_a, Tensor rowsB, Tensor tB, int n_b, int BR, Tensor(a!) vec) -> ()");
  m.def("loss_finalize(Tensor vec, Tensor? cnt, int BR_global, float lam) -> Tensor[]");
  m.def("ce_head_backward(Tensor[] saved, Tensor W, Tensor inv, Tensor tc, int Mv0, int Mv1, Tensor coef, "
        "Tensor gscale, float lam, Tensor(a!)? gW, Tensor(b!)? gb, Tensor(c!)? gwpad, Tensor(d!)? gbpad, "
        "Tensor? tplan, int n_rsplit, int mode, int dw_full=0) -> Tensor[]");
  m.def("loss_disc_backward(Tensor[] fwd, Tensor gscale, float lam, Tensor?[] D, Tensor[] imgT, Tensor(a!)?[] gD, "
        "Tensor[] heads, Tensor wpad, Tensor?[] sub, Tensor?[] maps, int L, int R, int mode) -> Tensor[]");
  m.impl("loss_disc_forward", c10::DispatchKey::CompositeExplicitAutograd, TORCH_FN(loss_disc_forward));
  m.impl("ce_head_forward", c10::DispatchKey::CompositeExplicitAutograd, TORCH_FN(ce_head_forward));
  m.impl("loss_partials", c10::DispatchKey::CompositeExplicitAutograd, TORCH_FN(loss_partials));
  m.impl("loss_finalize", c10::DispatchKey::CompositeExplicitAutograd, TORCH_FN(loss_finalize));
  m.impl("ce_head_backward", c10::DispatchKey::CompositeExplicitAutograd, TORCH_FN(ce_head_backward));
  m.impl("loss_disc_backward", c10::DispatchKey::CompositeExplicitAutograd, TORCH_FN(loss_disc_backward));
}
