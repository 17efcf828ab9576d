// Host-side helpers shared by the PyTorch operator layer (libc2dsr_torch.so): tensor checks, the current HIP
// stream, and `launch`, through which every call into the kernel library (include/c2dsr.h) goes — it turns a
// nonzero hipError_t into a RuntimeError naming the entry point, and optionally (a) brackets the call with HIP
// events for bench.py's in-process kernel timing (timing_set / timing_take) and (b) synchronises around it to pin
// an asynchronous fault on its entry point (C2DSR_DEBUG_SYNC=1).
#pragma once
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime_api.h>

#include <atomic>
#include <cstdint>
#include <optional>
#include <string>
#include <type_traits>
#include <vector>

#include "c2dsr.h"

namespace c2t {

inline void* stream() { return (void*)c10::hip::getCurrentHIPStream().stream(); }

inline void* ptr(const std::optional<at::Tensor>& t) { return t.has_value() && t->defined() ? t->data_ptr() : nullptr; }
inline void* ptr(const at::Tensor& t) { return t.defined() ? t.data_ptr() : nullptr; }

// device / dtype check of a pointer argument (a host descriptor array must be a CPU tensor)
inline void check(const char* op, const char* arg, const std::optional<at::Tensor>& t, bool host,
                  std::optional<at::ScalarType> dt) {
  if (!t.has_value() || !t->defined()) return;
  if (host) {
    TORCH_CHECK(t->device().is_cpu(), "c2dsr::", op, ": ", arg, " is a host array (CPU tensor expected)");
  } else {
    TORCH_CHECK(t->is_cuda(), "c2dsr::", op, ": ", arg, " must be on the HIP device (no CPU fallback)");
  }
  if (dt.has_value()) {
    const auto s = t->scalar_type();
    const bool ok = s == *dt || (*dt == at::kInt && s == at::kUInt32);
    TORCH_CHECK(ok, "c2dsr::", op, ": ", arg, " has dtype ", s, ", expected ", *dt);
  }
}

// extent check of a buffer a raw op writes (tools/raw_extents.py): the bytes from its data pointer to the end of its
// storage must hold `need` elements of `elem` bytes (views of larger buffers are measured against their storage)
inline void extent(const char* op, const char* arg, const std::optional<at::Tensor>& t, int64_t need, int64_t elem) {
  if (!t.has_value() || !t->defined() || need <= 0) return;
  const int64_t avail = (int64_t)t->storage().nbytes() - t->storage_offset() * (int64_t)t->element_size();
  TORCH_CHECK(avail >= need * elem, "c2dsr_raw::", op, ": ", arg, " holds ", avail, " bytes, the call writes up to ",
              need * elem, " (undersized output)");
}
inline int64_t span(int64_t rows, int64_t ld, int64_t cols) { return rows > 0 ? (rows - 1) * ld + cols : 0; }
#define HAS(p) (c2t::ptr(p) != nullptr)
#define SPAN(r, ld, c) c2t::span((int64_t)(r), (int64_t)(ld), (int64_t)(c))

// ---- timing / debug registry (defined in torch_ops.cpp)
struct Rec {
  std::string name;
  hipEvent_t e0, e1;
  std::vector<double> meta;
};
bool timed(const char* name);  // cheap when no name is registered
void record(const char* name, hipEvent_t e0, hipEvent_t e1, std::vector<double>&& meta);
bool debug_sync();
void sync_check(const char* name, const char* where);

// The index error word of the current HIP device (int32 [4], word 0 = the C2DSR_IDX_ERR_* bits; defined in
// torch_ops.cpp): the stage operators pass it to every kernel that range-checks indices, and to AdamW, which
// changes nothing while it is nonzero.  The host reads it through c2dsr::error_word at its sync points.
at::Tensor err_word();
inline int* errp() { return err_word().data_ptr<int>(); }

template <class T>
inline double as_meta(T v) {
  if constexpr (std::is_pointer_v<T>)
    return (double)(uintptr_t)v;
  else
    return (double)v;
}

// one call into the kernel library: F returns 0 or a hipError_t; `extra` values are appended to the timing record
// (bench.py's accounting: e.g. the compact row counts of a fused stage)
template <class F, class... A>
inline int64_t launch_x(const char* name, const std::vector<double>& extra, F fn, A... a) {
  const bool dbg = debug_sync();
  if (dbg) sync_check(name, "before");
  hipEvent_t e0 = nullptr, e1 = nullptr;
  const bool tm = timed(name);
  if (tm) {
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, (hipStream_t)stream());
  }
  const int rc = fn(a...);
  if (tm) {
    (void)hipEventRecord(e1, (hipStream_t)stream());
    std::vector<double> meta{as_meta(a)...};
    meta.insert(meta.end(), extra.begin(), extra.end());
    record(name, e0, e1, std::move(meta));
  }
  if (dbg) sync_check(name, "in");
  TORCH_CHECK(rc == 0, name, " failed with hipError ", rc);
  return rc;
}
template <class F, class... A>
inline int64_t launch(const char* name, F fn, A... a) {
  return launch_x(name, std::vector<double>{}, fn, a...);
}

}  // namespace c2t
