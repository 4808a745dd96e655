// Bindings of the generic HIP ops (csrc/kernels/ops.hip).
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include "kernels/ops.h"

namespace {
hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

at::Tensor gather_rows(at::Tensor src, at::Tensor idx, double scale) {
  TORCH_CHECK(src.is_cuda() && idx.is_cuda(), "gather_rows: GPU tensors expected");
  TORCH_CHECK(src.is_contiguous() && idx.is_contiguous(), "gather_rows: contiguous tensors expected");
  TORCH_CHECK(idx.scalar_type() == at::kInt && idx.dim() == 1, "gather_rows: idx must be int32 [n]");
  const int64_t rows = idx.numel();
  const int64_t row_elems = src.numel() / std::max<int64_t>(src.size(0), 1);
  std::vector<int64_t> shape(src.sizes().begin(), src.sizes().end());
  shape[0] = rows;
  auto out = at::empty(shape, src.options().dtype(at::kFloat));
  if (src.scalar_type() == at::kFloat) {
    tdl::gather_rows_f32(src.data_ptr<float>(), idx.data_ptr<int>(), out.data_ptr<float>(), rows, row_elems,
                         (float)scale, cur_stream());
  } else if (src.scalar_type() == at::kByte) {
    tdl::gather_rows_u8(src.data_ptr<uint8_t>(), idx.data_ptr<int>(), out.data_ptr<float>(), rows, row_elems,
                        (float)scale, cur_stream());
  } else {
    TORCH_CHECK(false, "gather_rows: float32 or uint8 source expected");
  }
  return out;
}

at::Tensor gather_labels(at::Tensor src, at::Tensor idx) {
  TORCH_CHECK(src.is_cuda() && idx.is_cuda() && src.scalar_type() == at::kInt && idx.scalar_type() == at::kInt,
              "gather_labels: int32 GPU tensors expected");
  auto out = at::empty({idx.numel()}, src.options());
  tdl::gather_i32(src.data_ptr<int>(), idx.data_ptr<int>(), out.data_ptr<int>(), idx.numel(), cur_stream());
  return out;
}
}  // namespace

void register_ops(pybind11::module& m) {
  m.def("gather_rows", &gather_rows, "row gather (+u8->f32 scale) of a device-resident dataset");
  m.def("gather_labels", &gather_labels);
}
