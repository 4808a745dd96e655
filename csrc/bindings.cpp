// Python bindings of the HIP kernel library (module `tensorflow_distributed_learning_amd._C`).
//
// Kernels launch on the caller's current HIP stream, so every entry point here is capturable
// into a hipGraph by torch.cuda.graph (the engine captures whole train steps).
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPStream.h>

#include <vector>

#include "kernels/mnist_cnn.h"
#include "kernels/ops.h"
#include "kernels/optim.h"
#include "xgmi_channel.h"

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check_cuda_f32(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
  TORCH_CHECK(t.scalar_type() == at::kFloat, name, " must be float32");
}

// Owns the scratch buffers and the argument block of one replica's fused MNIST step.
class MnistStep {
 public:
  MnistStep(at::Tensor X, at::Tensor Y, at::Tensor idx_buf, at::Tensor W, at::Tensor G,
            std::vector<int64_t> offsets, int64_t b, double scale, at::Tensor lr, at::Tensor metrics)
      : X_(X), Y_(Y), idx_(idx_buf), W_(W), G_(G), lr_(lr), metrics_(metrics) {
    check_cuda_f32(X, "X");
    check_cuda_f32(W, "W");
    check_cuda_f32(G, "G");
    check_cuda_f32(lr, "lr");
    check_cuda_f32(metrics, "metrics");
    TORCH_CHECK(Y.is_cuda() && Y.scalar_type() == at::kInt, "Y must be int32 on GPU");
    TORCH_CHECK(idx_buf.is_cuda() && idx_buf.scalar_type() == at::kInt, "idx must be int32 on GPU");
    TORCH_CHECK(X.numel() % 784 == 0, "X must be [N,28,28,1]");
    TORCH_CHECK(offsets.size() == 8, "8 variable offsets expected");
    TORCH_CHECK(b >= 1 && b <= 256, "fused MNIST step supports 1 <= per-replica batch <= 256");
    TORCH_CHECK(W.numel() == G.numel(), "slab size mismatch");
    for (auto o : offsets) TORCH_CHECK(o % 4 == 0 && o >= 0 && o < W.numel(), "offsets must be 16B aligned");
    auto f = W.options();
    auto u8 = f.dtype(at::kByte);
    P1_ = at::empty({b * 169 * 32}, f);
    A1_ = at::empty({b * 169 * 32}, u8);
    P2_ = at::empty({b * 1600}, f);
    A2_ = at::empty({b * 1600}, u8);
    H_ = at::empty({b * 128}, f);
    dH_ = at::empty({b * 128}, f);
    dL_ = at::zeros({b * tdl::kDLStride}, f);
    cnt_ = at::zeros({b}, f.dtype(at::kInt));
    dHt_ = at::zeros({b * 128}, f.dtype(at::kLong));  // tag 0 never matches (tags start at 1)
    ep_ = at::zeros({1}, f.dtype(at::kInt));
    part3t_ = at::zeros({(int64_t)tdl::kDense1Chunks * b * 128}, f.dtype(at::kLong));
    dP2_ = at::empty({b * 1600}, f);
    part2_ = at::zeros({b * std::max(tdl::kMnistPart2Rows * 64, tdl::kP2QuadFloats)}, f);
    part1_ = at::zeros({(int64_t)tdl::mnist_part1_rows((int)b, true) * tdl::kMnistPart1Cols}, f);
    err_ = at::zeros({1}, f.dtype(at::kInt));
    part3_ = at::zeros({(int64_t)tdl::kDense1Chunks * b * 128}, f);
    a_ = tdl::MnistArgs{};
    a_.X = X_.data_ptr<float>();
    a_.Y = Y_.data_ptr<int>();
    a_.idx = idx_.data_ptr<int>();
    a_.W = W_.data_ptr<float>();
    a_.G = G_.data_ptr<float>();
    a_.ow1 = (int)offsets[0]; a_.ob1 = (int)offsets[1]; a_.ow2 = (int)offsets[2]; a_.ob2 = (int)offsets[3];
    a_.ow3 = (int)offsets[4]; a_.ob3 = (int)offsets[5]; a_.ow4 = (int)offsets[6]; a_.ob4 = (int)offsets[7];
    a_.P1 = P1_.data_ptr<float>();
    a_.A1 = A1_.data_ptr<uint8_t>();
    a_.P2 = P2_.data_ptr<float>();
    a_.A2 = A2_.data_ptr<uint8_t>();
    a_.H = H_.data_ptr<float>();
    a_.dH = dH_.data_ptr<float>();
    a_.dL = dL_.data_ptr<float>();
    a_.cnt = reinterpret_cast<unsigned*>(cnt_.data_ptr<int>());
    a_.dHt = reinterpret_cast<unsigned long long*>(dHt_.data_ptr<int64_t>());
    a_.ep = reinterpret_cast<unsigned*>(ep_.data_ptr<int>());
    a_.part3t = reinterpret_cast<unsigned long long*>(part3t_.data_ptr<int64_t>());
    a_.head = 1;
    {  // A/B switches of the fused kernel (diagnostics; see mnist_cnn.hip)
      const char* v = std::getenv("TDL_MNIST_VARIANT");
      a_.variant = v != nullptr ? std::atoi(v) : tdl::kDefaultMnistVariant;
      const char* g = std::getenv("TDL_FX_GRID");
      a_.fx_grid = g != nullptr ? std::max(0, std::atoi(g)) : 0;
    }
    a_.dp2_fwd = 0;
    a_.fused_bwd = 0;
    a_.err = reinterpret_cast<unsigned*>(err_.data_ptr<int>());
    a_.xchg = 0;
    a_.xtwo = 0;
    a_.dP2 = dP2_.data_ptr<float>();
    a_.part2 = part2_.data_ptr<float>();
    a_.part1 = part1_.data_ptr<float>();
    a_.part3 = part3_.data_ptr<float>();
    a_.metrics = metrics_.data_ptr<float>();
    a_.lr = lr_.data_ptr<float>();
    a_.b = (int)b;
    a_.scale = (float)scale;
    a_.nslab = (int)W.numel();
  }

  // accumulate metrics into another [>= 3] f32 tensor from now on (evaluation reuses step objects)
  void set_metrics(at::Tensor m) {
    check_cuda_f32(m, "metrics");
    TORCH_CHECK(m.numel() >= 3, "metrics needs >= 3 elements");
    metrics_ = m;
    a_.metrics = metrics_.data_ptr<float>();
  }

  void set_idx_offset(int64_t off) {
    TORCH_CHECK(off >= 0 && off + a_.b <= idx_.numel(), "idx offset out of range");
    a_.idx = idx_.data_ptr<int>() + off;
  }

  // Individual stages (tests / profiling): 5 dense weight grads, 6 conv bwd,
  // 8 fwd conv (+dense1, +head), 9 finalize.
  void stage(int64_t k, bool apply_sgd) {
    hipStream_t s = cur_stream();
    switch (k) {
      case 5: tdl::mnist_dense1_bwd(a_, !a_.dp2_fwd, false, s); break;
      case 6: tdl::mnist_conv_bwd(a_, s); break;
      case 8:
        a_.fused_bwd = (fused_bwd_ && a_.dp2_fwd) ? 1 : 0;
        tdl::mnist_fwd_conv(a_, s);
        break;
      case 9: finalize(apply_sgd, false); break;
      default: TORCH_CHECK(false, "unknown stage");
    }
  }

  // forward + loss + backward: leaves the complete gradient in G after finalize(), which also
  // computes the dense weight gradients.
  void forward_backward(int64_t idx_off) {
    set_idx_offset(idx_off);
    hipStream_t s = cur_stream();
    if (fused_bwd_ && a_.dp2_fwd) {  // ONE launch: forward, loss head, dP2 and the conv backward
      a_.fused_bwd = 1;
      tdl::mnist_fwd_conv(a_, s);
    } else {
      a_.fused_bwd = 0;
      tdl::mnist_fwd_conv(a_, s);
      if (!a_.dp2_fwd) tdl::mnist_dense1_bwd(a_, true, false, s);
      tdl::mnist_conv_bwd(a_, s);
    }
    dense_pending_ = true;
  }

  // dP2 inside k_fwd_conv (its workgroups wait for their image's head) or in a K5 launch; the
  // caller enables it only when the step's launches have the GPU to themselves and all 4b
  // workgroups of k_fwd_conv fit on the device at once
  void set_dp2_in_forward(bool on) { a_.dp2_fwd = on ? 1 : 0; }
  bool dp2_in_forward() const { return a_.dp2_fwd != 0; }
  // with dP2 in the forward kernel, also run the conv backward there (forward_backward only)
  void set_fused_bwd(bool on) { fused_bwd_ = on; }
  // keep_grad = false: a single replica's finalize with fused SGD does not write the gradient slab
  // G (nothing reads it on that path; fewer dirty lines for the kernel-end write-back)
  void set_keep_grad(bool on) {
    a_.variant = on ? (a_.variant & ~tdl::kMnistVariantNoG) : (a_.variant | tdl::kMnistVariantNoG);
  }
  bool keep_grad() const { return (a_.variant & tdl::kMnistVariantNoG) == 0; }
  bool fused_bwd() const { return fused_bwd_ && a_.dp2_fwd; }
  // k_finalize_x grid cap (0: one workgroup per range; see MnistArgs::fx_grid)
  void set_fx_grid(int64_t n) { a_.fx_grid = (int)std::max<int64_t>(0, n); }
  int64_t fx_grid() const { return a_.fx_grid; }

  // error word of the in-kernel hand-offs (bit 1: a wait timed out; host sync); reset=true clears it
  int64_t error(bool reset) {
    int64_t v = err_.item<int>();
    if (reset) err_.zero_();
    return v;
  }

  // the same step split at the point where the dense-layer gradients are final in G (after K5):
  // the engine all-reduces that bucket while backward_conv() runs
  void forward_dense(int64_t idx_off) {
    set_idx_offset(idx_off);
    hipStream_t s = cur_stream();
    a_.fused_bwd = 0;
    tdl::mnist_fwd_conv(a_, s);
    tdl::mnist_dense1_bwd(a_, !a_.dp2_fwd, true, s);
    dense_pending_ = false;
  }
  void backward_conv() { tdl::mnist_conv_bwd(a_, cur_stream()); }

  // partial reductions + dense weight gradients (+ SGD).  After a fused forward_backward the
  // fused finalize runs; with `exchange` (fused, apply_sgd, a channel set) it also all-reduces the
  // gradient across the replicas over xGMI before the update (one launch, see k_finalize_x)
  void finalize(bool apply_sgd, bool exchange) {
    if (a_.fused_bwd) {
      TORCH_CHECK(!exchange || (apply_sgd && xchg_ready_), "finalize: the exchange needs apply_sgd and set_exchange()");
      tdl::MnistArgs f = a_;
      f.xchg = exchange ? 1 : 0;
      tdl::mnist_finalize_x(f, apply_sgd, cur_stream());
      return;
    }
    TORCH_CHECK(!exchange, "finalize: the exchange needs the fused backward (forward_backward with fused_bwd)");
    tdl::mnist_finalize(a_, apply_sgd, dense_pending_, cur_stream());
  }

  // the xGMI channel finalize(exchange=true) all-reduces through: exchange slots at slab offsets
  // (capacity >= slab), one signal / epoch slot per finalize workgroup
  void set_exchange(const tdl_host::XgmiChannel& ch) {
    TORCH_CHECK(ch.device() == W_.get_device(), "set_exchange: channel on another device");
    TORCH_CHECK(ch.cap() >= W_.numel(), "set_exchange: channel smaller than the slab");
    TORCH_CHECK(ch.sig_blocks() >= tdl::kFxBlocks, "set_exchange: channel needs >= ", tdl::kFxBlocks, " signal slots");
    TORCH_CHECK(a_.ow4 == a_.ob3 + 128 && a_.ob4 == a_.ow4 + 1280, "set_exchange: dense bias/kernel ranges not contiguous");
    ch.fill_args(a_.xa);
    xchg_ready_ = true;
  }
  bool has_exchange() const { return xchg_ready_; }
  // 0: one-shot exchange in finalize (every rank sums every range); 1: two-shot (reduce-scatter of
  // 1/R of every range + copy of the owners' updated weights: 2 (R-1)/R of the slab over the fabric)
  void set_exchange_algo(int algo) { a_.xtwo = algo != 0; }
  int exchange_algo() const { return a_.xtwo; }

  // forward-only evaluation / inference of the b rows at idx_off: loss, correct count and sample
  // count accumulate into the metrics tensor; logits ([>= b*10] f32, optional) receive the logits
  void forward_eval(int64_t idx_off, c10::optional<at::Tensor> logits) {
    set_idx_offset(idx_off);
    tdl::MnistArgs f = a_;
    f.head = 2;
    f.fused_bwd = 0;
    f.logits = nullptr;
    if (logits.has_value()) {
      check_cuda_f32(*logits, "logits");
      TORCH_CHECK(logits->numel() >= (int64_t)a_.b * 10, "logits buffer too small");
      f.logits = logits->data_ptr<float>();
    }
    tdl::mnist_fwd_conv(f, cur_stream());
  }

  // forward features only (dense1 partials, no loss head / metrics)
  void forward_features(int64_t idx_off) {
    set_idx_offset(idx_off);
    tdl::MnistArgs f = a_;
    f.head = 0;
    f.fused_bwd = 0;
    tdl::mnist_fwd_conv(f, cur_stream());
  }

  // diagnostics: per-workgroup phase timestamps of the next launches (None to disable)
  void set_stamps(c10::optional<at::Tensor> t) {
    if (t.has_value()) {
      TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kLong, "stamps must be int64 on GPU");
      stamps_ = *t;
      a_.stamps = reinterpret_cast<unsigned long long*>(stamps_.data_ptr<int64_t>());
    } else {
      a_.stamps = nullptr;
    }
  }

  std::vector<at::Tensor> buffers() { return {P1_, A1_, P2_, A2_, H_, dH_, dP2_, part2_, part1_, part3_, dL_}; }

 private:
  at::Tensor X_, Y_, idx_, W_, G_, lr_, metrics_;
  at::Tensor P1_, A1_, P2_, A2_, H_, dH_, dP2_, part2_, part1_, part3_, dL_, cnt_, dHt_, ep_, part3t_, err_;
  bool fused_bwd_ = false;
  bool xchg_ready_ = false;
  bool dense_pending_ = true;  // finalize computes the dense weight gradients (forward_backward)
  at::Tensor stamps_;
  tdl::MnistArgs a_;
};

void sgd(at::Tensor w, at::Tensor g, at::Tensor lr, bool zero_grad) {
  check_cuda_f32(w, "w");
  check_cuda_f32(g, "g");
  check_cuda_f32(lr, "lr");
  TORCH_CHECK(w.numel() == g.numel());
  tdl::sgd_apply(w.data_ptr<float>(), g.data_ptr<float>(), lr.data_ptr<float>(), w.numel(), cur_stream(), zero_grad);
}

void sgd_momentum(at::Tensor w, at::Tensor g, at::Tensor v, at::Tensor lr, double m, bool nesterov, bool zero_grad) {
  check_cuda_f32(w, "w");
  check_cuda_f32(g, "g");
  check_cuda_f32(v, "v");
  check_cuda_f32(lr, "lr");
  TORCH_CHECK(w.numel() == g.numel() && v.numel() == w.numel());
  tdl::sgd_momentum_apply(w.data_ptr<float>(), g.data_ptr<float>(), v.data_ptr<float>(), lr.data_ptr<float>(),
                          (float)m, nesterov, w.numel(), cur_stream(), zero_grad);
}

// Flat-slab Adam / AdamW (+AMSGrad): state m, v (vhat), device lr and execution-start step t0
void adam(at::Tensor w, at::Tensor g, at::Tensor m, at::Tensor v, c10::optional<at::Tensor> vhat, at::Tensor lr,
          at::Tensor t0, int64_t t_add, double b1, double b2, double eps, double wd) {
  for (auto* t : {&w, &g, &m, &v, &lr, &t0}) check_cuda_f32(*t, "adam operand");
  TORCH_CHECK(g.numel() == w.numel() && m.numel() == w.numel() && v.numel() == w.numel());
  tdl::OptimArgs a{};
  a.w = w.data_ptr<float>(); a.g = g.data_ptr<float>(); a.s0 = m.data_ptr<float>(); a.s1 = v.data_ptr<float>();
  if (vhat.has_value()) {
    check_cuda_f32(*vhat, "vhat");
    TORCH_CHECK(vhat->numel() == w.numel());
    a.s2 = vhat->data_ptr<float>();
    a.flags = 1;
  }
  a.lr = lr.data_ptr<float>(); a.t0 = t0.data_ptr<float>(); a.t_add = (int)t_add; a.n = w.numel();
  a.b1 = (float)b1; a.b2 = (float)b2; a.eps = (float)eps; a.wd = (float)wd;
  tdl::adam_apply(a, cur_stream());
}

// Flat-slab RMSprop (+momentum, centered)
void rmsprop(at::Tensor w, at::Tensor g, at::Tensor rms, c10::optional<at::Tensor> mom, c10::optional<at::Tensor> mg,
             at::Tensor lr, double rho, double momentum, double eps) {
  for (auto* t : {&w, &g, &rms, &lr}) check_cuda_f32(*t, "rmsprop operand");
  TORCH_CHECK(g.numel() == w.numel() && rms.numel() == w.numel());
  tdl::OptimArgs a{};
  a.w = w.data_ptr<float>(); a.g = g.data_ptr<float>(); a.s0 = rms.data_ptr<float>();
  if (mom.has_value()) { check_cuda_f32(*mom, "mom"); TORCH_CHECK(mom->numel() == w.numel()); a.s1 = mom->data_ptr<float>(); a.flags |= 1; }
  if (mg.has_value()) { check_cuda_f32(*mg, "mg"); TORCH_CHECK(mg->numel() == w.numel()); a.s2 = mg->data_ptr<float>(); a.flags |= 2; }
  a.lr = lr.data_ptr<float>(); a.n = w.numel(); a.b1 = (float)rho; a.b2 = (float)momentum; a.eps = (float)eps;
  tdl::rmsprop_apply(a, cur_stream());
}

// Flat-slab Adagrad
void adagrad(at::Tensor w, at::Tensor g, at::Tensor acc, at::Tensor lr, double eps) {
  for (auto* t : {&w, &g, &acc, &lr}) check_cuda_f32(*t, "adagrad operand");
  TORCH_CHECK(g.numel() == w.numel() && acc.numel() == w.numel());
  tdl::OptimArgs a{};
  a.w = w.data_ptr<float>(); a.g = g.data_ptr<float>(); a.s0 = acc.data_ptr<float>();
  a.lr = lr.data_ptr<float>(); a.n = w.numel(); a.eps = (float)eps;
  tdl::adagrad_apply(a, cur_stream());
}

}  // namespace

void register_ops(pybind11::module& m);
void register_comm(pybind11::module& m);
void register_rccl(pybind11::module& m);

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "gfx950 HIP kernels of tensorflow_distributed_learning_amd";
  pybind11::class_<MnistStep>(m, "MnistStep")
      .def(pybind11::init<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, std::vector<int64_t>, int64_t,
                          double, at::Tensor, at::Tensor>())
      .def("set_idx_offset", &MnistStep::set_idx_offset)
      .def("set_metrics", &MnistStep::set_metrics)
      .def("stage", &MnistStep::stage, pybind11::arg("k"), pybind11::arg("apply_sgd") = false)
      .def("forward_backward", &MnistStep::forward_backward)
      .def("forward_features", &MnistStep::forward_features)
      .def("forward_eval", &MnistStep::forward_eval, pybind11::arg("idx_off"), pybind11::arg("logits") = pybind11::none())
      .def("forward_dense", &MnistStep::forward_dense)
      .def("backward_conv", &MnistStep::backward_conv)
      .def("set_fx_grid", &MnistStep::set_fx_grid)
      .def("fx_grid", &MnistStep::fx_grid)
      .def("finalize", &MnistStep::finalize, pybind11::arg("apply_sgd"), pybind11::arg("exchange") = false)
      .def("set_exchange", &MnistStep::set_exchange)
      .def("has_exchange", &MnistStep::has_exchange)
      .def("set_exchange_algo", &MnistStep::set_exchange_algo)
      .def("exchange_algo", &MnistStep::exchange_algo)
      .def("set_dp2_in_forward", &MnistStep::set_dp2_in_forward)
      .def("dp2_in_forward", &MnistStep::dp2_in_forward)
      .def("set_fused_bwd", &MnistStep::set_fused_bwd)
      .def("fused_bwd", &MnistStep::fused_bwd)
      .def("set_keep_grad", &MnistStep::set_keep_grad)
      .def("keep_grad", &MnistStep::keep_grad)
      .def("error", &MnistStep::error, pybind11::arg("reset") = false)
      .def("buffers", &MnistStep::buffers)
      .def("set_stamps", &MnistStep::set_stamps);
  m.def("sgd", &sgd, "w -= lr * g over a flat slab (zero_grad: g := 0 afterwards)", pybind11::arg("w"),
        pybind11::arg("g"), pybind11::arg("lr"), pybind11::arg("zero_grad") = false);
  m.def("sgd_momentum", &sgd_momentum, "Keras momentum SGD over a flat slab (zero_grad: g := 0 afterwards)",
        pybind11::arg("w"), pybind11::arg("g"), pybind11::arg("v"), pybind11::arg("lr"), pybind11::arg("m"),
        pybind11::arg("nesterov"), pybind11::arg("zero_grad") = false);
  m.def("adam", &adam, pybind11::arg("w"), pybind11::arg("g"), pybind11::arg("m"), pybind11::arg("v"),
        pybind11::arg("vhat"), pybind11::arg("lr"), pybind11::arg("t0"), pybind11::arg("t_add"), pybind11::arg("b1"),
        pybind11::arg("b2"), pybind11::arg("eps"), pybind11::arg("wd") = 0.0);
  m.def("rmsprop", &rmsprop, pybind11::arg("w"), pybind11::arg("g"), pybind11::arg("rms"), pybind11::arg("mom"),
        pybind11::arg("mg"), pybind11::arg("lr"), pybind11::arg("rho"), pybind11::arg("momentum"), pybind11::arg("eps"));
  m.def("adagrad", &adagrad);
  register_ops(m);
  register_comm(m);
  register_rccl(m);
}
