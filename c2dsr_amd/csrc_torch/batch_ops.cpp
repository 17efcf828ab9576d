// Stage operators for the training step's bookkeeping launches, each replacing a run of small
// per-kernel calls with one checked operator:
//   step_prepare    the index work a step sizes its launches by (trainer.py:101-154): the five encoder passes' row
//                   sets (c2dsr_need_rows), their padding rows (c2dsr_pad_rows, the attention's keys, Q1) and per
//                   classifier head the stacked last-R targets and their valid-row compaction
//   wgrad_groups    the projections' deferred weight-gradient products, grouped per weight (ops.WGradBatch)
//   weight_images   the projection weights' bf16 / split-bf16 images after an optimizer step (ops._WeightImages),
//                   and the guarded linear1's row norms ‖W1[r]‖² (layout 4)
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
void dev(const Tensor& t, const char* op) {
  TORCH_CHECK(!t.defined() || t.is_cuda(), "c2dsr::", op, ": every tensor must be on the HIP device (no CPU fallback)");
}
void* S() { return c2t::stream(); }
const auto kI32 = at::kInt;

// gm_a / gm_b [B, L] int64 (the pooling masks); seqs: the passes' sequences [B, L] (empty: no padding-row sets);
// code: 3 bits per pass (c2dsr_need_rows); pad: the padding item; heads: per head (t_share, t_spec, n_items), the
// stacked targets [2BR] and their compaction (ignore = n_items).  Returns [need idx [n, M], inv [n, M], cnt [n],
// off [n, B+1], (pad idx, inv, cnt, off if seqs), then per head tcat [2BR] int64, idx [2BR], inv [2BR], tc [2BR] int64,
// cnt [2]].
std::vector<Tensor> step_prepare(const Tensor& gm_a, const Tensor& gm_b, int64_t R, int64_t n_sets, int64_t code,
                                 const std::vector<Tensor>& seqs, int64_t pad, const std::vector<Tensor>& targets,
                                 std::vector<int64_t> n_items, bool need) {
  const char* op = "step_prepare";
  TORCH_CHECK(gm_a.dim() == 2, "c2dsr::step_prepare: gm_a must be [B, L]");
  const int64_t B = gm_a.size(0), L = gm_a.size(1), M = B * L, M2 = 2 * B * R;
  want(gm_a, op, "gm_a", at::kLong, {B, L});
  want(gm_b, op, "gm_b", at::kLong, {B, L});
  TORCH_CHECK(n_sets >= 1 && n_sets <= 8 && R <= L, "c2dsr::step_prepare: 1..8 row sets, R <= L");
  TORCH_CHECK(seqs.empty() || (int64_t)seqs.size() == n_sets, "c2dsr::step_prepare: one sequence tensor per set");
  for (const Tensor& s : seqs) want(s, op, "seq", at::kLong, {B, L});
  TORCH_CHECK(targets.size() == 2 * n_items.size(), "c2dsr::step_prepare: (t_share, t_spec) per head");
  for (const Tensor& t : targets) want(t, op, "targets", at::kLong, {B, L});
  dev(gm_a, op);
  dev(gm_b, op);
  for (const Tensor& s : seqs) dev(s, op);
  for (const Tensor& t : targets) dev(t, op);
  const auto i32 = gm_a.options().dtype(kI32);
  std::vector<Tensor> out;
  if (need) {
    Tensor idx = at::empty({n_sets, M}, i32), inv = at::empty({n_sets, M}, i32), cnt = at::empty({n_sets}, i32);
    Tensor off = at::empty({n_sets, B + 1}, i32);
    Tensor ws = at::empty({(int64_t)(c2dsr_compact_workspace((int)M, (int)n_sets) / 4 + 1)}, i32);
    c2t::launch("c2dsr_need_rows", &c2dsr_need_rows, gm_a.data_ptr<int64_t>(), gm_b.data_ptr<int64_t>(), (int)B,
                (int)L, (int)R, (int)n_sets, (int)code, idx.data_ptr<int>(), inv.data_ptr<int>(), cnt.data_ptr<int>(),
                off.data_ptr<int>(), ws.data_ptr<int>(), S());
    out.insert(out.end(), {idx, inv, cnt, off});
    if (!seqs.empty()) {
      Tensor sq = at::stack(seqs).reshape({n_sets, M});
      Tensor pidx = at::empty({n_sets, M}, i32), pinv = at::empty({n_sets, M}, i32), pcnt = at::empty({n_sets}, i32);
      Tensor poff = at::empty({n_sets, B + 1}, i32);
      Tensor pws = at::empty({(int64_t)(c2dsr_compact_workspace((int)M, (int)n_sets) / 4 + 1)}, i32);
      c2t::launch("c2dsr_pad_rows", &c2dsr_pad_rows, sq.data_ptr<int64_t>(), (int64_t)pad, (int)B, (int)L, (int)n_sets,
                  pidx.data_ptr<int>(), pinv.data_ptr<int>(), pcnt.data_ptr<int>(), poff.data_ptr<int>(),
                  pws.data_ptr<int>(), S());
      out.insert(out.end(), {pidx, pinv, pcnt, poff});
    }
  }
  for (size_t k = 0; k < n_items.size(); ++k) {
    Tensor tcat = at::empty({M2}, gm_a.options());
    c2t::launch("c2dsr_rec_targets", &c2dsr_rec_targets, targets[2 * k].data_ptr<int64_t>(),
                targets[2 * k + 1].data_ptr<int64_t>(), (int)B, (int)L, (int)R, tcat.data_ptr<int64_t>(), S());
    Tensor idx = at::empty({M2}, i32), inv = at::empty({M2}, i32), tc = at::empty({M2}, gm_a.options());
    Tensor cnt = at::empty({2}, i32);
    Tensor ws = at::empty({(int64_t)(c2dsr_compact_workspace((int)M2, 1) / 4 + 1)}, i32);
    c2t::launch("c2dsr_compact_valid", &c2dsr_compact_valid, (const int64_t*)tcat.data_ptr<int64_t>(), (int)M2,
                (int)(B * R), (int)n_items[k], idx.data_ptr<int>(), inv.data_ptr<int>(), tc.data_ptr<int64_t>(),
                cnt.data_ptr<int>(), ws.data_ptr<int>(), c2t::errp(), S());
    out.insert(out.end(), {tcat, idx, inv, tc, cnt});
  }
  return out;
}

// dW[g] (+)= Σ over group g's segments of dY[s]ᵀ·X[s] (and db[g] += Σ dY[s]), segments in order, four per product
// (c2dsr_wgemm_multi / _x3_multi: one set of split partials and one fixed-order sum per product).  seg_group[s]: the
// group of segment s; x3[g]: split-bf16 products (fp32 dY); otherwise bf16 MFMA (dY fp32 or bf16).
void wgrad_groups(const std::vector<Tensor>& dY, const std::vector<Tensor>& X, std::vector<int64_t> seg_group,
                  const std::vector<Tensor>& dW, const std::vector<OptT>& db, std::vector<int64_t> x3) {
  const char* op = "wgrad_groups";
  TORCH_CHECK(dY.size() == X.size() && dY.size() == seg_group.size(), "c2dsr::wgrad_groups: one group per segment");
  TORCH_CHECK(dW.size() == db.size() && dW.size() == x3.size(), "c2dsr::wgrad_groups: dW / db / x3 per group");
  const int64_t G = (int64_t)dW.size();
  for (int64_t g = 0; g < G; ++g) {
    TORCH_CHECK(dW[g].dim() == 2, "c2dsr::wgrad_groups: dW must be [N, D]");
    want(dW[g], op, "dW", at::kFloat, {dW[g].size(0), dW[g].size(1)});
    if (db[g].has_value() && db[g]->defined()) want(*db[g], op, "db", at::kFloat, {dW[g].size(0)});
    TORCH_CHECK(c2dsr_wgemm_supported(1, (int)dW[g].size(0), (int)dW[g].size(1)),
                "c2dsr::wgrad_groups: unsupported weight shape");
  }
  for (size_t s = 0; s < dY.size(); ++s) {
    const int64_t g = seg_group[s];
    TORCH_CHECK(g >= 0 && g < G, "c2dsr::wgrad_groups: segment group out of range");
    const int64_t N = dW[g].size(0), D = dW[g].size(1);
    TORCH_CHECK(dY[s].dim() == 2 && dY[s].size(1) == N && dY[s].is_contiguous() &&
                    (dY[s].scalar_type() == at::kFloat || (!x3[g] && dY[s].scalar_type() == at::kBFloat16)),
                "c2dsr::wgrad_groups: dY must be contiguous [T, N] (fp32; bf16 allowed without x3)");
    want(X[s], op, "X", at::kFloat, {dY[s].size(0), D});
    dev(dY[s], op);
    dev(X[s], op);
  }
  for (int64_t g = 0; g < G; ++g) {
    dev(dW[g], op);
    if (db[g].has_value()) dev(*db[g], op);
  }
  for (int64_t g = 0; g < G; ++g) {
    const int64_t N = dW[g].size(0), D = dW[g].size(1);
    std::vector<size_t> segs;
    for (size_t s = 0; s < dY.size(); ++s)
      if (seg_group[s] == g && dY[s].size(0) > 0) segs.push_back(s);
    if (segs.empty()) continue;
    const bool yb16 = dY[segs[0]].scalar_type() == at::kBFloat16;
    for (size_t s : segs)
      TORCH_CHECK((dY[s].scalar_type() == at::kBFloat16) == yb16, "c2dsr::wgrad_groups: one dY dtype per group");
    Tensor ws = at::empty({(int64_t)c2dsr_wgemm_workspace((int)N)}, dW[g].options().dtype(at::kByte));
    float* dbp = db[g].has_value() && db[g]->defined() ? db[g]->data_ptr<float>() : nullptr;
    for (size_t i = 0; i < segs.size(); i += 4) {
      const size_t nseg = std::min<size_t>(4, segs.size() - i);
      int64_t desc[20];
      for (size_t j = 0; j < nseg; ++j) {
        const size_t s = segs[i + j];
        desc[5 * j + 0] = (int64_t)(uintptr_t)dY[s].data_ptr();
        desc[5 * j + 1] = N;
        desc[5 * j + 2] = (int64_t)(uintptr_t)X[s].data_ptr();
        desc[5 * j + 3] = D;
        desc[5 * j + 4] = dY[s].size(0);
      }
      if (x3[g])
        c2t::launch("c2dsr_wgemm_x3_multi", &c2dsr_wgemm_x3_multi, (const int64_t*)desc, (int)nseg, (int)N, (int)D,
                    1.f, dW[g].data_ptr<float>(), dbp, ws.data_ptr(), S());
      else
        c2t::launch("c2dsr_wgemm_multi", &c2dsr_wgemm_multi, (const int64_t*)desc, (int)nseg, (int)N, (int)D,
                    (int)yb16, 1.f, dW[g].data_ptr<float>(), dbp, ws.data_ptr(), S());
    }
  }
}

// images Y[i] of the fp32 matrices W[i] (trans[i]: of Wᵀ) in layout[i]: 0 bf16 rows, 1 split rows (hi ‖ lo), 2 split
// fragment order (c2dsr_rgemm_x3f), 3 bf16 fragment order (c2dsr_rgemm*, ldb = 0) — up to 64 per launch per layout
void weight_images(const std::vector<Tensor>& W, const std::vector<Tensor>& Y, std::vector<int64_t> trans,
                   std::vector<int64_t> layout) {
  const char* op = "weight_images";
  TORCH_CHECK(W.size() == Y.size() && W.size() == trans.size() && W.size() == layout.size(),
              "c2dsr::weight_images: one image, transpose flag and layout per matrix");
  for (size_t i = 0; i < W.size(); ++i) {
    TORCH_CHECK(W[i].dim() == 2 && W[i].scalar_type() == at::kFloat && W[i].stride(1) == 1,
                "c2dsr::weight_images: W must be fp32 [R, C] with unit column stride");
    if (layout[i] == 4) {  // ‖W[r]‖² (fp32 [R])
      TORCH_CHECK(!trans[i] && Y[i].scalar_type() == at::kFloat && Y[i].is_contiguous() && Y[i].numel() >= W[i].size(0),
                  "c2dsr::weight_images: a row-norm image is fp32 [R] of an untransposed W");
      dev(W[i], op);
      dev(Y[i], op);
      continue;
    }
    TORCH_CHECK(Y[i].scalar_type() == at::kBFloat16 && Y[i].is_contiguous(), "c2dsr::weight_images: bf16 images");
    const int64_t rows = trans[i] ? W[i].size(1) : W[i].size(0), cols = trans[i] ? W[i].size(0) : W[i].size(1);
    const int64_t pad = layout[i] == 2 ? 16 : layout[i] == 3 ? 32 : 1;
    const int64_t need = (rows + pad - 1) / pad * pad * cols * (layout[i] == 1 || layout[i] == 2 ? 2 : 1);
    TORCH_CHECK(layout[i] >= 0 && layout[i] <= 3 && Y[i].numel() >= need, "c2dsr::weight_images: image ", i,
                " too small for its layout (", Y[i].numel(), " < ", need, ")");
    dev(W[i], op);
    dev(Y[i], op);
  }
  using Fn = int (*)(const int64_t*, int, void*);
  const Fn fns[5] = {&c2dsr_to_bf16_multi, &c2dsr_to_split_bf16_multi, &c2dsr_to_split_bf16_frag_multi,
                     &c2dsr_to_bf16_frag_multi, &c2dsr_row_sqnorm_multi};
  const char* names[5] = {"c2dsr_to_bf16_multi", "c2dsr_to_split_bf16_multi", "c2dsr_to_split_bf16_frag_multi",
                          "c2dsr_to_bf16_frag_multi", "c2dsr_row_sqnorm_multi"};
  for (int lay = 0; lay < 5; ++lay) {
    std::vector<int64_t> recs;
    int cnt = 0;
    auto flush = [&] {
      if (cnt) c2t::launch(names[lay], fns[lay], (const int64_t*)recs.data(), cnt, S());
      recs.clear();
      cnt = 0;
    };
    for (size_t i = 0; i < W.size(); ++i) {
      if (layout[i] != lay) continue;
      recs.insert(recs.end(), {(int64_t)(uintptr_t)W[i].data_ptr(), (int64_t)(uintptr_t)Y[i].data_ptr(), W[i].size(0),
                               W[i].size(1), W[i].stride(0), trans[i]});
      if (++cnt == 64) flush();
    }
    flush();
  }
}

}  // namespace

// The range checks of a batch's index tensors (a step whose batch has no host copy: Trainer.prepare), each [B, L]
// int64: tensor i must hold values in [0, hi[i]) in its last cols[i] columns, else bits[i] is ORed into the device's
// index error word.  Returns word 0 copied after the checks (int32 [1]), which the step's deferred count read
// carries to the host (ops.HostCounts raises IndexError on it) — F.embedding / F.cross_entropy raise
// (models/C2DSR.py:65-67,81, encoders.py:30, trainer.py:143-152).
Tensor index_check(const std::vector<Tensor>& idx, std::vector<int64_t> hi, std::vector<int64_t> cols,
                   std::vector<int64_t> bits) {
  const char* op = "index_check";
  TORCH_CHECK(idx.size() == hi.size() && idx.size() == cols.size() && idx.size() == bits.size(),
              "c2dsr::index_check: hi / cols / bits per index tensor");
  for (size_t i = 0; i < idx.size(); ++i) {
    want(idx[i], op, "idx", at::kLong, {-1, -1});
    dev(idx[i], op);
    TORCH_CHECK(cols[i] >= 0 && cols[i] <= idx[i].size(1), "c2dsr::index_check: cols outside [0, L]");
  }
  Tensor w = c2t::err_word();
  for (size_t i = 0; i < idx.size(); ++i)
    c2t::launch("c2dsr_index_check", &c2dsr_index_check, (const int64_t*)idx[i].data_ptr<int64_t>(),
                (long)idx[i].size(0), (int)idx[i].size(1), (int)cols[i], (int64_t)hi[i], (int)bits[i], w.data_ptr<int>(),
                S());
  return w.narrow(0, 0, 1).clone();
}

void register_batch_ops(torch::Library& m) {
  m.def("step_prepare(Tensor gm_a, Tensor gm_b, int R, int n_sets, int code, Tensor[] seqs, int pad, Tensor[] targets, "
        "int[] n_items, bool need) -> Tensor[]");
  m.def("wgrad_groups(Tensor[] dY, Tensor[] X, int[] seg_group, Tensor(a!)[] dW, Tensor(b!)?[] db, int[] x3) -> ()");
  m.def("weight_images(Tensor[] W, Tensor(a!)[] Y, int[] trans, int[] layout) -> ()");
  m.def("index_check(Tensor[] idx, int[] hi, int[] cols, int[] bits) -> Tensor");
  m.impl("step_prepare", c10::DispatchKey::CompositeExplicitAutograd, TORCH_FN(step_prepare));
  m.impl("index_check", c10::DispatchKey::CompositeExplicitAutograd, TORCH_FN(index_check));
  m.impl("wgrad_groups", c10::DispatchKey::CompositeExplicitAutograd, TORCH_FN(wgrad_groups));
  m.impl("weight_images", c10::DispatchKey::CompositeExplicitAutograd, TORCH_FN(weight_images));
}
