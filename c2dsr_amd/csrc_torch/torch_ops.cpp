// PyTorch-ROCm extension of the gfx950 kernel library (north_star: "exposed through a PyTorch-ROCm C++/HIP
// extension"): TORCH_LIBRARY(c2dsr, m) registers every C-ABI entry point of include/c2dsr.h as a
// schema op (torch.ops.c2dsr.<name without the c2dsr_ prefix>, generated from the header: torch_ops_gen.inc), with
// tensor arguments checked for device and dtype.  The training step's Python host side (c2dsr_amd/ops.py,
// losshead.py) binds the same library through ctypes (c2dsr_amd/_lib.py); these ops are the interface for
// TorchScript / C++ callers, and tests/test_gpu_torch_ops.py holds them bit-equal to the ctypes path.
// Every op enqueues on the current HIP stream and raises (RuntimeError) on a bad argument or a hipError.
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <optional>

#include "c2dsr.h"

namespace c2dsr_torch {

inline void* stream() { return (void*)c10::hip::getCurrentHIPStream().stream(); }

inline void* ptr(const std::optional<at::Tensor>& t) { return t.has_value() && t->defined() ? t->data_ptr() : nullptr; }

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

}  // namespace c2dsr_torch

#include "torch_ops_gen.inc"

TORCH_LIBRARY(c2dsr, m) {
  C2DSR_GENERATED_DEFS(m)
  m.def("generated_count() -> int");
}

static int64_t op_generated_count() { return C2DSR_GENERATED_COUNT; }

TORCH_LIBRARY_IMPL(c2dsr, CompositeExplicitAutograd, m) {
  C2DSR_GENERATED_IMPLS(m)
  m.impl("generated_count", &op_generated_count);
}
