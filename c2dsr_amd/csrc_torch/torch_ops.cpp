// PyTorch-ROCm extension of the gfx950 kernel library (north_star: "exposed through a PyTorch-ROCm C++/HIP
// extension").  Two operator namespaces:
//   * c2dsr_raw:: — every C-ABI entry point of include/c2dsr.h as a schema op (generated from the header:
//     torch_ops_gen.inc): pointers as tensors (written ones annotated Tensor(a!)), checked for device and dtype,
//     sizes as the ABI's ints.  The host side's remaining per-kernel calls (c2dsr_amd/_lib.py `lib`) go here.
//   * c2dsr:: — the stage operators the training step runs on (stage_ops.cpp: Tensor in / Tensor out, every size
//     derived from the tensors and every extent checked), plus the timing hooks below.
// Every op enqueues on the current HIP stream and raises RuntimeError on a bad argument or a hipError.
#include <torch/library.h>

#include <cstdlib>
#include <mutex>
#include <set>
#include <tuple>

#include "c2t.h"

namespace c2t {

// ---- event timing of chosen entry points (bench.py: the K5 / K1 / K2 launches inside the timed region)
static std::atomic<bool> g_any{false};
static std::mutex g_mu;
static std::set<std::string> g_names;
static std::vector<Rec> g_recs;

bool timed(const char* name) {
  if (!g_any.load(std::memory_order_relaxed)) return false;
  std::lock_guard<std::mutex> lk(g_mu);
  return g_names.count(name) != 0;
}

void record(const char* name, hipEvent_t e0, hipEvent_t e1, std::vector<double>&& meta) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_recs.push_back(Rec{name, e0, e1, std::move(meta)});
}

bool debug_sync() {
  static const bool on = [] {
    const char* v = std::getenv("C2DSR_DEBUG_SYNC");
    return v && v[0] == '1';
  }();
  return on;
}

void sync_check(const char* name, const char* where) {
  const hipError_t e = hipStreamSynchronize((hipStream_t)stream());
  TORCH_CHECK(e == hipSuccess, "device fault ", where, " ", name, " (hipError ", (int)e, ")");
}

static std::mutex g_err_mu;
static std::vector<at::Tensor> g_err;  // per device index

at::Tensor err_word() {
  const int dev = (int)c10::hip::current_device();
  std::lock_guard<std::mutex> lk(g_err_mu);
  if ((int)g_err.size() <= dev) g_err.resize(dev + 1);
  if (!g_err[dev].defined())
    g_err[dev] = at::zeros({4}, at::TensorOptions().dtype(at::kInt).device(at::Device(at::kCUDA, (int8_t)dev)));
  return g_err[dev];
}

}  // namespace c2t

#include "torch_ops_gen.inc"

// names of the entry points to bracket with events (empty: off); earlier records are dropped
static void op_timing_set(const std::vector<std::string>& names) {
  std::lock_guard<std::mutex> lk(c2t::g_mu);
  c2t::g_names = std::set<std::string>(names.begin(), names.end());
  for (auto& r : c2t::g_recs) {
    (void)hipEventDestroy(r.e0);
    (void)hipEventDestroy(r.e1);
  }
  c2t::g_recs.clear();
  c2t::g_any.store(!c2t::g_names.empty());
}

// the records since timing_set, in launch order: (names, ms, meta values, meta lengths); synchronises on the events
static std::tuple<std::vector<std::string>, std::vector<double>, std::vector<double>, std::vector<int64_t>>
op_timing_take() {
  std::lock_guard<std::mutex> lk(c2t::g_mu);
  std::vector<std::string> names;
  std::vector<double> ms, meta;
  std::vector<int64_t> lens;
  for (auto& r : c2t::g_recs) {
    float t = 0.f;
    (void)hipEventSynchronize(r.e1);
    (void)hipEventElapsedTime(&t, r.e0, r.e1);
    (void)hipEventDestroy(r.e0);
    (void)hipEventDestroy(r.e1);
    names.push_back(r.name);
    ms.push_back(t);
    meta.insert(meta.end(), r.meta.begin(), r.meta.end());
    lens.push_back((int64_t)r.meta.size());
  }
  c2t::g_recs.clear();
  return {names, ms, meta, lens};
}

static int64_t op_generated_count() { return C2DSR_GENERATED_COUNT; }

// the current device's index error word itself (aliased, not a copy): the host clones it at a sync point, raises
// IndexError when word 0 is nonzero and clears it (c2dsr_amd/trainer.py Trainer.check_index_errors)
static at::Tensor op_error_word() { return c2t::err_word(); }

TORCH_LIBRARY(c2dsr_raw, m) {
  C2DSR_GENERATED_DEFS(m)
  m.def("generated_count() -> int");
}

TORCH_LIBRARY_IMPL(c2dsr_raw, CompositeExplicitAutograd, m) {
  C2DSR_GENERATED_IMPLS(m)
  m.impl("generated_count", &op_generated_count);
}

TORCH_LIBRARY_FRAGMENT(c2dsr, m) {
  m.def("timing_set(str[] names) -> ()", &op_timing_set);
  m.def("timing_take() -> (str[], float[], float[], int[])", &op_timing_take);
  m.def("error_word() -> Tensor", &op_error_word);
}
