// Stage operators of the training step ("TORCH_LIBRARY(c2dsr, m) … one schema per K1–K6 stage").
// Tensor in / Tensor out: every size is derived from the tensors and every extent is checked (TORCH_CHECK →
// RuntimeError) before a kernel of include/c2dsr.h is launched on the current HIP stream.  The host side's
// autograd nodes (c2dsr_amd/ops.py, losshead.py) call one operator per forward / backward:
//   gcn_propagate / gcn_backward_rounds / gcn_backward_final   K1, models/encoders.py:42-48 (C2DSR.py:59-62)
//   embed_fuse / embed_fuse_backward                           K2, models/C2DSR.py:65-71, encoders.py:30-31
//   index_plans                                                 the sort plans of K2's deterministic backward
//   encoder_pass / encoder_pass_backward                        K2 + K3 of one training pass (C2DSR.py:64-85 →
//                                                               encoders.py:29-33 → TransformerEncoderLayer)
//   adamw_step                                                  K6, trainer.py:21-22,158
#include <torch/library.h>

#include <tuple>

#include "c2t.h"

namespace {

using at::Tensor;
using OptT = std::optional<Tensor>;

// ---- checks
void dev(const Tensor& t, const char* op, const char* name) {
  TORCH_CHECK(t.defined(), "c2dsr::", op, ": ", name, " is undefined");
  TORCH_CHECK(t.is_cuda(), "c2dsr::", op, ": ", name, " must be on the HIP device (no CPU fallback)");
}
void want(const Tensor& t, const char* op, const char* name, at::ScalarType dt, std::initializer_list<int64_t> shape) {
  TORCH_CHECK(t.defined(), "c2dsr::", op, ": ", name, " is undefined");
  TORCH_CHECK(t.scalar_type() == dt, "c2dsr::", op, ": ", name, " has dtype ", t.scalar_type(), ", expected ", dt);
  TORCH_CHECK(t.is_contiguous(), "c2dsr::", op, ": ", name, " must be contiguous");
  const std::vector<int64_t> s(shape);
  TORCH_CHECK(t.dim() == (int64_t)s.size(), "c2dsr::", op, ": ", name, " has ", t.dim(), " dims, expected ",
              s.size());
  for (size_t i = 0; i < s.size(); ++i)
    TORCH_CHECK(s[i] < 0 || t.size((int64_t)i) == s[i], "c2dsr::", op, ": ", name, " has shape ", t.sizes(),
                ", expected dim ", i, " = ", s[i]);
}
// at least `bytes` bytes of storage behind a contiguous tensor (workspaces, plans)
void bytes_at_least(const Tensor& t, const char* op, const char* name, size_t bytes) {
  TORCH_CHECK(t.defined() && t.is_contiguous(), "c2dsr::", op, ": ", name, " must be a contiguous tensor");
  TORCH_CHECK((size_t)t.nbytes() >= bytes, "c2dsr::", op, ": ", name, " holds ", t.nbytes(), " bytes, needs ", bytes);
}
// after every shape check of an op: all its tensors on the HIP device
void on_device(const char* op, std::initializer_list<const OptT*> ts) {
  for (const OptT* t : ts)
    if (t->has_value() && (*t)->defined()) dev(**t, op, "every tensor");
}
void on_device(const char* op, std::initializer_list<const Tensor*> ts) {
  for (const Tensor* t : ts)
    if (t->defined()) dev(*t, op, "every tensor");
}
const float* fp(const OptT& t) { return t.has_value() && t->defined() ? t->data_ptr<float>() : nullptr; }
float* fpm(const OptT& t) { return t.has_value() && t->defined() ? t->data_ptr<float>() : nullptr; }
bool has(const OptT& t) { return t.has_value() && t->defined(); }
at::TensorOptions f32(const Tensor& like) { return like.options().dtype(at::kFloat); }
void* S() { return c2t::stream(); }

// ============================================================== K1: GCN propagation
// graph = the SpMM work plan of A (or Aᵀ): work int32 [n_work, 4], split int32 [n_split, 4], col int32 [E],
// val fp32 [E]; part: the split rows' partial slab (n_slots rows)
struct Graph {
  Tensor work, split, col, val;
  int64_t n_slots;
};
// n_rows: the row count the plan was built for (DeviceGraph.n) — it must equal the table's, or the SpMM's rows and
// column indices would walk past (or stop short of) the table
Graph graph(const Tensor& work, const Tensor& split, const Tensor& col, const Tensor& val, int64_t n_rows,
            int64_t n_slots, const Tensor& table, const char* op) {
  TORCH_CHECK(table.dim() == 2 && n_rows == table.size(0), "c2dsr::", op, ": the graph has ", n_rows,
              " rows but the table has ", table.dim() == 2 ? table.size(0) : -1);
  want(work, op, "work", at::kInt, {-1, 4});
  TORCH_CHECK(split.numel() == 0 || (split.dim() == 2 && split.size(1) == 4), "c2dsr::", op, ": split must be [n, 4]");
  if (split.numel()) want(split, op, "split", at::kInt, {-1, 4});
  want(col, op, "col", at::kInt, {-1});
  want(val, op, "val", at::kFloat, {col.size(0)});
  TORCH_CHECK(n_slots >= 0, "c2dsr::", op, ": n_slots < 0");
  return Graph{work, split, col, val, n_slots};
}

void spmm(const Graph& g, const Tensor& part, const Tensor& X, uint32_t k0, uint32_t k1, float p, int mask_out,
          float alpha, const float* Z, float beta, float delta, int pad_row, float gamma, float* Y, float* Y2) {
  const int d = (int)X.size(1);
  if (X.scalar_type() == at::kBFloat16)
    c2t::launch("c2dsr_gcn_spmm_b16", &c2dsr_gcn_spmm_b16, (const int*)g.work.data_ptr(), (int)g.work.size(0),
                g.split.numel() ? (const int*)g.split.data_ptr() : nullptr, (int)g.split.size(0),
                part.data_ptr<float>(), (const int*)g.col.data_ptr(), g.val.data_ptr<float>(), d,
                (const void*)X.data_ptr(), k0, k1, p, mask_out, alpha, (const void*)Z, beta, delta, pad_row, gamma,
                (void*)Y, (void*)Y2, S());
  else
    c2t::launch("c2dsr_gcn_spmm", &c2dsr_gcn_spmm, (const int*)g.work.data_ptr(), (int)g.work.size(0),
                g.split.numel() ? (const int*)g.split.data_ptr() : nullptr, (int)g.split.size(0),
                part.data_ptr<float>(), (const int*)g.col.data_ptr(), g.val.data_ptr<float>(), d, X.data_ptr<float>(),
                k0, k1, p, mask_out, alpha, Z, beta, delta, pad_row, gamma, Y, Y2, S());
}

Tensor part_slab(const Graph& g, const Tensor& X) {
  return at::empty({std::max<int64_t>(g.n_slots, 1), X.size(1)}, f32(X));
}

void check_table(const Tensor& E, const char* op, const char* name) {
  TORCH_CHECK(E.dim() == 2 && E.size(1) % 4 == 0, "c2dsr::", op, ": ", name, " must be [N, d] with d % 4 == 0");
  TORCH_CHECK(E.scalar_type() == at::kFloat || E.scalar_type() == at::kBFloat16, "c2dsr::", op, ": ", name,
              " must be fp32 or bf16");
  TORCH_CHECK(E.is_contiguous(), "c2dsr::", op, ": ", name, " must be contiguous");
}

// H = mean(E, A·drop(E), A·drop(A·drop(E)), …) over n_gnn rounds (models/encoders.py:42-48); keys [2·n_gnn].
// out (optional) receives H (e.g. the first N rows of a larger buffer); returned.
Tensor gcn_propagate(const Tensor& E, const Tensor& work, const Tensor& split, const Tensor& col, const Tensor& val,
                     int64_t n_rows, int64_t n_slots, int64_t n_gnn, double p, std::vector<int64_t> keys,
                     const OptT& out) {
  const char* op = "gcn_propagate";
  check_table(E, op, "E");
  const Graph g = graph(work, split, col, val, n_rows, n_slots, E, op);
  TORCH_CHECK(n_gnn >= 0 && (int64_t)keys.size() == 2 * n_gnn, "c2dsr::gcn_propagate: keys must hold 2·n_gnn values");
  Tensor H = has(out) ? *out : at::empty_like(E);
  TORCH_CHECK(H.sizes() == E.sizes() && H.scalar_type() == E.scalar_type() && H.is_contiguous(),
              "c2dsr::gcn_propagate: out must be a contiguous tensor like E");
  on_device(op, {&E, &H, &work, &split, &col, &val});
  Tensor part = part_slab(g, E);
  const float inv = 1.f / (float)(n_gnn + 1);
  const float* Ep = (const float*)E.data_ptr();
  if (n_gnn == 0) {  // H = E
    spmm(g, part, E, 0, 0, 0.f, 0, 0.f, Ep, 1.f, 0.f, -1, 0.f, (float*)H.data_ptr(), nullptr);
    return H;
  }
  Tensor prev = E;
  for (int64_t k = 0; k < n_gnn; ++k) {
    const bool last = k == n_gnn - 1;
    Tensor hk = last ? Tensor() : at::empty_like(E);
    spmm(g, part, prev, (uint32_t)keys[2 * k], (uint32_t)keys[2 * k + 1], (float)p, 0, inv, k == 0 ? Ep : nullptr,
         inv, 0.f, -1, k == 0 ? 0.f : 1.f, (float*)H.data_ptr(), last ? nullptr : (float*)hk.data_ptr());
    prev = hk;
  }
  return H;
}

// the rounds of the backward before the last: X = T_1 (n_gnn ≥ 2; T_{k-1} = G/(n+1) + M_k ⊙ Aᵀ T_k), G itself for
// n_gnn = 1 (no launch); graph = the plan of Aᵀ
Tensor gcn_backward_rounds(const Tensor& G, const Tensor& work, const Tensor& split, const Tensor& col,
                           const Tensor& val, int64_t n_rows, int64_t n_slots, int64_t n_gnn, double p,
                           std::vector<int64_t> keys) {
  const char* op = "gcn_backward_rounds";
  want(G, op, "G", at::kFloat, {-1, -1});
  const Graph g = graph(work, split, col, val, n_rows, n_slots, G, op);
  TORCH_CHECK(n_gnn >= 1 && (int64_t)keys.size() == 2 * n_gnn, "c2dsr::gcn_backward_rounds: keys must hold 2·n_gnn");
  on_device(op, {&G, &work, &split, &col, &val});
  const float inv = 1.f / (float)(n_gnn + 1);
  Tensor X = G;
  float alpha = inv;
  Tensor part;
  for (int64_t k = n_gnn; k > 1; --k) {
    if (!part.defined()) part = part_slab(g, G);
    Tensor T = at::empty_like(G);
    spmm(g, part, X, (uint32_t)keys[2 * (k - 1)], (uint32_t)keys[2 * (k - 1) + 1], (float)p, 1, alpha,
         G.data_ptr<float>(), inv, 0.f, -1, 0.f, T.data_ptr<float>(), nullptr);
    X = T;
    alpha = 1.f;
  }
  return X;
}

// the last round, into gE (rows of the given work / split slices; the whole plan for a whole-table launch):
//   gE[i] = alpha·drop(Aᵀ X)[i] + (1/(n+1) + [i != pad]·delta)·G[i] + gamma·gE[i]   (alpha = 1/(n+1) for n = 1, else 1)
//   n_gnn = 0: gE[i] = (1 + [i != pad]·delta)·G[i] + gamma·gE[i]
// the training step's form (the table's own lookups and the accumulating .grad): delta = gamma = 1; the module API's
// GCN.forward backward (ops.GCNPropFn): delta = gamma = 0, pad_row = -1
void gcn_backward_final(const Tensor& X, const Tensor& G, const Tensor& gE, const Tensor& work, const Tensor& split,
                        const Tensor& col, const Tensor& val, int64_t n_rows, int64_t n_slots, int64_t n_gnn, double p,
                        int64_t k0,
                        int64_t k1, int64_t pad_row, double delta, double gamma, const OptT& part) {
  const char* op = "gcn_backward_final";
  want(G, op, "G", at::kFloat, {-1, -1});
  want(X, op, "X", at::kFloat, {G.size(0), G.size(1)});
  want(gE, op, "gE", at::kFloat, {G.size(0), G.size(1)});
  const Graph g = graph(work, split, col, val, n_rows, n_slots, G, op);
  TORCH_CHECK(pad_row >= -1 && pad_row < G.size(0), "c2dsr::gcn_backward_final: pad_row out of range");
  Tensor pt = has(part) ? *part : part_slab(g, G);
  TORCH_CHECK(pt.scalar_type() == at::kFloat && pt.is_contiguous() &&
                  pt.numel() >= std::max<int64_t>(g.n_slots, 1) * G.size(1),
              "c2dsr::gcn_backward_final: part slab too small");
  on_device(op, {&X, &G, &gE, &work, &split, &col, &val, &pt});
  if (n_gnn == 0) {
    spmm(g, pt, G, 0, 0, 0.f, 1, 0.f, G.data_ptr<float>(), 1.f, (float)delta, (int)pad_row, (float)gamma,
         gE.data_ptr<float>(), nullptr);
    return;
  }
  const float inv = 1.f / (float)(n_gnn + 1);
  const float alpha = n_gnn == 1 ? inv : 1.f;
  spmm(g, pt, X, (uint32_t)k0, (uint32_t)k1, (float)p, 1, alpha, G.data_ptr<float>(), inv, (float)delta, (int)pad_row,
       (float)gamma, gE.data_ptr<float>(), nullptr);
}

// ============================================================== K2: embedding fuse
void check_idx(const Tensor& t, const char* op, const char* name, int64_t B, int64_t L) {
  want(t, op, name, at::kLong, {B, L});
}

// X = drop((H[seq] + E[seq])·scale + P[pos]) [B, L, d]   (Xin given: X = drop(Xin + P[pos]), H / E unused)
Tensor embed_fuse(const Tensor& seq, const Tensor& pos, const OptT& H, const OptT& E, const OptT& Xin,
                  const Tensor& P, double scale, double p, int64_t k0, int64_t k1, int64_t row_base, const OptT& out) {
  const char* op = "embed_fuse";
  TORCH_CHECK(seq.dim() == 2, "c2dsr::embed_fuse: seq must be [B, L]");
  const int64_t B = seq.size(0), L = seq.size(1);
  check_idx(seq, op, "seq", B, L);
  check_idx(pos, op, "pos", B, L);
  want(P, op, "P", at::kFloat, {-1, -1});
  const int64_t d = P.size(1);
  TORCH_CHECK(d % 4 == 0, "c2dsr::embed_fuse: d % 4 != 0");
  if (has(Xin)) {
    want(*Xin, op, "Xin", at::kFloat, {B, L, d});
  } else {
    TORCH_CHECK(has(H) && has(E), "c2dsr::embed_fuse: H and E (or Xin) required");
    want(*H, op, "H", at::kFloat, {-1, d});
    want(*E, op, "E", at::kFloat, {H->size(0), d});
  }
  if (has(out)) want(*out, op, "out", at::kFloat, {B, L, d});
  on_device(op, {&H, &E, &Xin, &out});
  on_device(op, {&seq, &pos, &P});
  Tensor X = has(out) ? *out : at::empty({B, L, d}, f32(P));
  if (B * L == 0) return X;
  c2t::launch("c2dsr_embed_fwd", &c2dsr_embed_fwd, seq.data_ptr<int64_t>(), pos.data_ptr<int64_t>(), (int)(B * L),
              (int)d, fp(H), fp(E), fp(Xin), P.data_ptr<float>(), (float)scale, (uint32_t)k0, (uint32_t)k1, (float)p,
              (int64_t)(row_base * L), X.data_ptr<float>(), has(H) ? (int)H->size(0) : 0, (int)P.size(0), c2t::errp(),
              S());
  return X;
}

// the sort plans of index tensors (c2dsr_index_plan) packed into `buf` (c2dsr_index_plan_bytes each, in order), on
// the current stream (the caller runs this on its side stream, under the forward)
void index_plans(const std::vector<Tensor>& idx, std::vector<int64_t> n_keys, const Tensor& buf) {
  const char* op = "index_plans";
  TORCH_CHECK(idx.size() == n_keys.size() && !idx.empty(), "c2dsr::index_plans: one n_keys per index tensor");
  TORCH_CHECK(buf.scalar_type() == at::kByte && buf.dim() == 1, "c2dsr::index_plans: buf must be a 1-D uint8 buffer");
  std::vector<size_t> sizes;
  size_t tot = 0;
  for (size_t i = 0; i < idx.size(); ++i) {
    TORCH_CHECK(idx[i].scalar_type() == at::kLong && idx[i].is_contiguous(), "c2dsr::index_plans: int64 indices");
    TORCH_CHECK(n_keys[i] > 0, "c2dsr::index_plans: n_keys must be positive");
    sizes.push_back(c2dsr_index_plan_bytes((int)idx[i].numel()));  // 256-aligned
    tot += sizes.back();
  }
  bytes_at_least(buf, op, "buf", tot);
  for (const Tensor& t : idx) dev(t, op, "idx");
  dev(buf, op, "buf");
  std::vector<int64_t> desc;  // one launch per radix pass for all the plans (c2dsr_index_plans)
  size_t o = 0;
  for (size_t i = 0; i < idx.size(); ++i) {
    desc.insert(desc.end(), {(int64_t)(uintptr_t)idx[i].data_ptr<int64_t>(), (int64_t)idx[i].numel(), n_keys[i],
                             (int64_t)(uintptr_t)((char*)buf.data_ptr() + o), (int64_t)sizes[i]});
    o += sizes[i];
  }
  c2t::launch("c2dsr_index_plans", &c2dsr_index_plans, (const int64_t*)desc.data(), (int)idx.size(), c2t::errp(), S());
}

void check_plan(const OptT& plan, int64_t n, const char* op, const char* name) {
  if (!has(plan)) return;
  TORCH_CHECK(plan->scalar_type() == at::kByte, "c2dsr::", op, ": ", name, " must be a uint8 plan buffer");
  bytes_at_least(*plan, op, name, c2dsr_index_plan_bytes((int)n));
}

// G[seq[r]] += scale·drop(gX[r]), gP[pos[r]] += drop(gX[r]) over prebuilt plans (deterministic segment sums);
// gX as one [B·L, d] tensor, or as two compact row sources (gXa, inv_a, gXb, inv_b: row r = gXa[inv_a[r]] +
// gXb[inv_b[r]], entries < 0 absent).  extra_meta: appended to the launch's timing record (bench accounting).
void embed_fuse_backward(const OptT& seq_plan, const OptT& pos_plan, int64_t n_rows, int64_t d, const OptT& gX,
                         const OptT& gXa, const OptT& inv_a, const OptT& gXb, const OptT& inv_b, double p, int64_t k0,
                         int64_t k1, int64_t idx_base, double scale, const OptT& G, const OptT& gP,
                         std::vector<double> extra_meta) {
  const char* op = "embed_fuse_backward";
  TORCH_CHECK(n_rows >= 0 && d % 4 == 0 && d > 0, "c2dsr::embed_fuse_backward: bad n_rows / d");
  TORCH_CHECK(has(G) == has(seq_plan) && has(gP) == has(pos_plan), "c2dsr::embed_fuse_backward: a plan per output");
  check_plan(seq_plan, n_rows, op, "seq_plan");
  check_plan(pos_plan, n_rows, op, "pos_plan");
  if (has(G)) want(*G, op, "G", at::kFloat, {-1, d});
  if (has(gP)) want(*gP, op, "gP", at::kFloat, {-1, d});
  if (has(gX)) {
    TORCH_CHECK(!has(gXa), "c2dsr::embed_fuse_backward: gX or the two row sources, not both");
    TORCH_CHECK(gX->numel() == n_rows * d && gX->is_contiguous() && gX->scalar_type() == at::kFloat,
                "c2dsr::embed_fuse_backward: gX must hold n_rows × d fp32");
  } else {
    TORCH_CHECK(has(gXa) && has(inv_a) && has(gXb) && has(inv_b), "c2dsr::embed_fuse_backward: gX or two row sources");
    want(*gXa, op, "gXa", at::kFloat, {-1, d});
    want(*gXb, op, "gXb", at::kFloat, {-1, d});
    want(*inv_a, op, "inv_a", at::kInt, {n_rows});
    want(*inv_b, op, "inv_b", at::kInt, {n_rows});
    TORCH_CHECK(d >= 64, "c2dsr::embed_fuse_backward: two row sources need d >= 64");
  }
  on_device(op, {&seq_plan, &pos_plan, &gX, &gXa, &inv_a, &gXb, &inv_b, &G, &gP});
  if (n_rows == 0 || (!has(G) && !has(gP))) return;
  Tensor ws = at::empty({(int64_t)c2dsr_embed_bwd_planned_workspace((int)n_rows, (int)d)},
                        (has(G) ? *G : *gP).options().dtype(at::kByte));
  const void* sp = has(seq_plan) ? seq_plan->data_ptr() : nullptr;
  const void* pp = has(pos_plan) ? pos_plan->data_ptr() : nullptr;
  const int n_items = has(G) ? (int)G->size(0) : 0, n_pos = has(gP) ? (int)gP->size(0) : 0;
  if (has(gX)) {
    c2t::launch_x("c2dsr_embed_bwd_planned", extra_meta, &c2dsr_embed_bwd_planned, sp, pp,
                  (int)n_rows, (int)d, gX->data_ptr<float>(), (uint32_t)k0, (uint32_t)k1, (float)p, (int64_t)idx_base,
                  (float)scale, fpm(G), n_items, fpm(gP), n_pos, (float*)nullptr, ws.data_ptr(), (size_t)ws.nbytes(),
                  S());
    return;
  }
  c2t::launch_x("c2dsr_embed_bwd_planned_rows", extra_meta,
                &c2dsr_embed_bwd_planned_rows, sp, pp, (int)n_rows, (int)d, gXa->data_ptr<float>(),
                inv_a->data_ptr<int>(), gXb->data_ptr<float>(), inv_b->data_ptr<int>(), (uint32_t)k0, (uint32_t)k1,
                (float)p, (int64_t)idx_base, (float)scale, fpm(G), n_items, fpm(gP), n_pos, ws.data_ptr(),
                (size_t)ws.nbytes(), S());
}

// ============================================================== K6: AdamW (amsgrad)
void adamw_step(const Tensor& param, const Tensor& fresh, const OptT& accum, const Tensor& m, const Tensor& v,
                const Tensor& vmax, double lr, double wd, double b1, double b2, double eps, int64_t step) {
  const char* op = "adamw_step";
  const int64_t n = param.numel();
  for (auto* t : {&param, &fresh, &m, &v, &vmax}) want(*t, op, "state", at::kFloat, {n});
  if (has(accum)) want(*accum, op, "accum", at::kFloat, {n});
  on_device(op, {&param, &fresh, &m, &v, &vmax});
  on_device(op, {&accum});
  c2t::launch("c2dsr_adamw", &c2dsr_adamw, param.data_ptr<float>(), fresh.data_ptr<float>(), fpm(accum),
              m.data_ptr<float>(), v.data_ptr<float>(), vmax.data_ptr<float>(), (long)n, (float)lr, (float)wd,
              (float)b1, (float)b2, (float)eps, (int)step, (const int*)c2t::errp(), S());
}

}  // namespace

void register_encoder_ops(torch::Library& m);   // encoder_ops.cpp
void register_losshead_ops(torch::Library& m);  // losshead_ops.cpp
void register_batch_ops(torch::Library& m);     // batch_ops.cpp

TORCH_LIBRARY_FRAGMENT(c2dsr, m) {
  m.def("gcn_propagate(Tensor E, Tensor work, Tensor split, Tensor col, Tensor val, int n_rows, int n_slots, int n_gnn, "
        "float p, int[] keys, Tensor(a!)? out=None) -> Tensor");
  m.def("gcn_backward_rounds(Tensor G, Tensor work, Tensor split, Tensor col, Tensor val, int n_rows, int n_slots, "
        "int n_gnn, float p, int[] keys) -> Tensor");
  m.def("gcn_backward_final(Tensor X, Tensor G, Tensor(a!) gE, Tensor work, Tensor split, Tensor col, Tensor val, "
        "int n_rows, int n_slots, int n_gnn, float p, int k0, int k1, int pad_row, float delta, float gamma, "
        "Tensor(b!)? part=None) -> ()");
  m.def("embed_fuse(Tensor seq, Tensor pos, Tensor? H, Tensor? E, Tensor? Xin, Tensor P, float scale, float p, int k0, "
        "int k1, int row_base, Tensor(a!)? out=None) -> Tensor");
  m.def("index_plans(Tensor[] idx, int[] n_keys, Tensor(a!) buf) -> ()");
  m.def("embed_fuse_backward(Tensor? seq_plan, Tensor? pos_plan, int n_rows, int d, Tensor? gX, Tensor? gXa, "
        "Tensor? inv_a, Tensor? gXb, Tensor? inv_b, float p, int k0, int k1, int idx_base, float scale, "
        "Tensor(a!)? G, Tensor(b!)? gP, float[] extra_meta=[]) -> ()");
  m.def("adamw_step(Tensor(a!) param, Tensor(b!) fresh, Tensor(c!)? accum, Tensor(d!) m, Tensor(e!) v, "
        "Tensor(f!) vmax, float lr, float wd, float b1, float b2, float eps, int step) -> ()");
  register_encoder_ops(m);
  register_losshead_ops(m);
  register_batch_ops(m);
}

TORCH_LIBRARY_IMPL(c2dsr, CompositeExplicitAutograd, m) {
  m.impl("gcn_propagate", &gcn_propagate);
  m.impl("gcn_backward_rounds", &gcn_backward_rounds);
  m.impl("gcn_backward_final", &gcn_backward_final);
  m.impl("embed_fuse", &embed_fuse);
  m.impl("index_plans", &index_plans);
  m.impl("embed_fuse_backward", &embed_fuse_backward);
  m.impl("adamw_step", &adamw_step);
}
