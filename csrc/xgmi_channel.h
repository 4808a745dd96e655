// Host side of the xGMI one-/two-shot all-reduce (csrc/kernels/xgmi.hip): exchange buffers, IPC
// handles and launches.  One XgmiChannel serves one message size of one communicator; kernels
// that run an exchange in their own workgroups (the fused MNIST finalize) take its device view
// with fill_args().
#pragma once
#include <torch/extension.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>

#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "kernels/xgmi.h"

namespace tdl_host {


inline void hip_ok(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, "xgmi: ", what, " failed: ", hipGetErrorString(e));
}

// ONE error word per device, shared by every channel (and by kernels that run an exchange in
// their own workgroups): after the first timed-out wait every xGMI exchange on the device returns
// at entry, so a dead peer costs one timeout instead of one per launch.  Never freed (process
// lifetime; graphs may still reference it).
inline uint32_t* device_error_word(int device) {
  static std::mutex mu;
  static std::map<int, uint32_t*> words;
  std::lock_guard<std::mutex> g(mu);
  auto it = words.find(device);
  if (it != words.end()) return it->second;
  c10::hip::HIPGuard guard((c10::DeviceIndex)device);
  uint32_t* p = nullptr;
  hip_ok(hipMalloc(&p, sizeof(uint32_t)), "hipMalloc(error)");
  hip_ok(hipMemset(p, 0, sizeof(uint32_t)), "hipMemset(error)");
  hip_ok(hipDeviceSynchronize(), "hipDeviceSynchronize");
  words[device] = p;
  return p;
}

class XgmiChannel {
 public:
  // `numel`: the message size of this channel (one-shot calls may be shorter; two-shot calls must
  // use exactly this size, their shard layout depends on it); `algo`: 0 one-shot, 1 two-shot
  // `min_blocks`: at least this many workgroup slots in the signal / epoch arrays (a kernel that
  // runs its own exchange may use more, smaller workgroups than the message has 1024-element blocks)
  XgmiChannel(int64_t rank, int64_t world, int64_t numel, int64_t device, double timeout_s, int64_t algo,
              int64_t min_blocks = 0)
      : rank_((int)rank), world_((int)world), device_((int)device), algo_((int)algo), n_(numel) {
    TORCH_CHECK(world >= 1 && world <= tdl::kXgmiMaxRanks, "xgmi: 1..8 ranks supported");
    TORCH_CHECK(rank >= 0 && rank < world, "xgmi: bad rank");
    TORCH_CHECK(numel > 0, "xgmi: empty channel");
    TORCH_CHECK(algo == 0 || algo == 1, "xgmi: algo is 0 (one-shot) or 1 (two-shot)");
    c10::hip::HIPGuard guard((c10::DeviceIndex)device_);
    blocks_ = tdl::xgmi_blocks(numel);
    cap_ = (int64_t)blocks_ * tdl::kXgmiBlockElems;
    if (min_blocks > blocks_) blocks_ = (int)min_blocks;  // (signal / epoch slots only)
    shard_ = tdl::xgmi_shard(numel, world_);
    timeout_ = (int64_t)(timeout_s * 1e8);
    // 2 parity halves x [input | result]
    hip_ok(hipMalloc(&buf_, (size_t)(4 * cap_) * sizeof(float)), "hipMalloc(exchange)");
    const size_t sig_bytes = (size_t)2 * blocks_ * tdl::kXgmiMaxRanks * sizeof(uint32_t);
    // signal words are polled across the fabric: uncached device memory where the runtime has it
    if (hipExtMallocWithFlags(reinterpret_cast<void**>(&sig_), sig_bytes, hipDeviceMallocUncached) != hipSuccess) {
      (void)hipGetLastError();
      hip_ok(hipMalloc(&sig_, sig_bytes), "hipMalloc(signals)");
    }
    hip_ok(hipMalloc(&epoch_, (size_t)blocks_ * sizeof(uint32_t)), "hipMalloc(epochs)");
    err_ = device_error_word(device_);
    hip_ok(hipMemset(buf_, 0, (size_t)(4 * cap_) * sizeof(float)), "hipMemset");
    hip_ok(hipMemset(sig_, 0, sig_bytes), "hipMemset");
    hip_ok(hipMemset(epoch_, 0, (size_t)blocks_ * sizeof(uint32_t)), "hipMemset");
    hip_ok(hipDeviceSynchronize(), "hipDeviceSynchronize");
    for (int r = 0; r < tdl::kXgmiMaxRanks; ++r) {
      peers_.buf[r] = nullptr;
      peers_.sig[r] = nullptr;
    }
    peers_.buf[rank_] = buf_;
    peers_.sig[rank_] = sig_;
  }

  ~XgmiChannel() {
    c10::hip::HIPGuard guard((c10::DeviceIndex)device_);
    (void)hipDeviceSynchronize();
    for (void* p : opened_) (void)hipIpcCloseMemHandle(p);
    (void)hipFree(buf_);
    (void)hipFree(sig_);
    (void)hipFree(epoch_);
  }

  int64_t cap() const { return cap_; }
  int64_t algo() const { return algo_; }
  bool connected() const { return connected_; }

  pybind11::bytes handle(bool signals) const {
    hipIpcMemHandle_t h;
    hip_ok(hipIpcGetMemHandle(&h, signals ? (void*)sig_ : (void*)buf_), "hipIpcGetMemHandle");
    return pybind11::bytes(reinterpret_cast<const char*>(&h), sizeof(h));
  }

  // peers in other processes: open their IPC handles (index = rank; own entry ignored)
  void open(const std::vector<std::string>& bufs, const std::vector<std::string>& sigs) {
    TORCH_CHECK((int)bufs.size() == world_ && (int)sigs.size() == world_, "xgmi: one handle per rank expected");
    c10::hip::HIPGuard guard((c10::DeviceIndex)device_);
    for (int r = 0; r < world_; ++r) {
      if (r == rank_) continue;
      peers_.buf[r] = reinterpret_cast<float*>(open_one(bufs[r]));
      peers_.sig[r] = reinterpret_cast<uint32_t*>(open_one(sigs[r]));
    }
    connected_ = true;
  }

  // peers in this process (emulated ranks on one device, tests): share the pointers directly
  void connect_local(const std::vector<XgmiChannel*>& group) {
    TORCH_CHECK((int)group.size() == world_, "xgmi: one channel per rank expected");
    for (int r = 0; r < world_; ++r) {
      TORCH_CHECK(group[r]->cap_ == cap_, "xgmi: channel capacities differ");
      peers_.buf[r] = group[r]->buf_;
      peers_.sig[r] = group[r]->sig_;
    }
    connected_ = true;
  }

  void all_reduce(const at::Tensor& src, const at::Tensor& dst, double scale) {
    check(src, "src");
    check(dst, "dst");
    TORCH_CHECK(dst.numel() == src.numel(), "xgmi: src/dst sizes differ");
    launch(src, dst.data_ptr<float>(), nullptr, nullptr, scale, 0);
  }

  void all_reduce_sgd(const at::Tensor& g, const at::Tensor& w, const at::Tensor& lr, double scale) {
    check(g, "gradient");
    check(w, "weights");
    TORCH_CHECK(w.numel() == g.numel(), "xgmi: weights/gradient sizes differ");
    TORCH_CHECK(lr.is_cuda() && lr.scalar_type() == at::kFloat && lr.numel() >= 1, "xgmi: device f32 lr expected");
    launch(g, nullptr, w.data_ptr<float>(), lr.data_ptr<float>(), scale, 1);
  }

  // device view of this channel for a kernel that runs the exchange in its own workgroups
  // (src / dst / w / lr / n / scale are the kernel's own)
  void fill_args(tdl::XgmiArgs& a) const {
    TORCH_CHECK(connected_, "xgmi: channel is not connected");
    a.p = peers_;
    a.epoch = epoch_;
    a.err = err_;
    a.cap = cap_;
    a.shard = shard_;
    a.sig_blocks = blocks_;
    a.timeout = timeout_;
    a.rank = rank_;
    a.world = world_;
    a.n = n_;
  }
  int64_t sig_blocks() const { return blocks_; }
  int64_t device() const { return device_; }

  int64_t error() const {
    c10::hip::HIPGuard guard((c10::DeviceIndex)device_);
    uint32_t v = 0;
    hip_ok(hipMemcpy(&v, err_, sizeof(v), hipMemcpyDeviceToHost), "hipMemcpy(error)");
    return (int64_t)v;
  }

  void reset_error() {
    c10::hip::HIPGuard guard((c10::DeviceIndex)device_);
    hip_ok(hipMemset(err_, 0, sizeof(uint32_t)), "hipMemset(error)");
  }

 private:
  void* open_one(const std::string& s) {
    TORCH_CHECK(s.size() == sizeof(hipIpcMemHandle_t), "xgmi: bad IPC handle size");
    hipIpcMemHandle_t h;
    std::memcpy(&h, s.data(), sizeof(h));
    void* p = nullptr;
    hip_ok(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
    opened_.push_back(p);
    return p;
  }

  void check(const at::Tensor& t, const char* what) const {
    TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous(), "xgmi: ", what,
                " must be a contiguous f32 GPU tensor");
    TORCH_CHECK(t.get_device() == device_, "xgmi: ", what, " is on another device");
    TORCH_CHECK(t.numel() <= cap_, "xgmi: ", what, " exceeds the channel capacity");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, "xgmi: ", what, " must be 16-byte aligned");
  }

  void launch(const at::Tensor& src, float* dst, float* w, const float* lr, double scale, int mode) {
    TORCH_CHECK(connected_, "xgmi: channel is not connected");
    TORCH_CHECK(algo_ == 0 || src.numel() == n_, "xgmi: a two-shot channel serves exactly ", n_, " elements");
    tdl::XgmiArgs a;
    a.p = peers_;
    a.src = src.data_ptr<float>();
    a.dst = dst;
    a.w = w;
    a.lr = lr;
    a.epoch = epoch_;
    a.err = err_;
    a.n = src.numel();
    a.cap = cap_;
    a.shard = shard_;
    a.sig_blocks = blocks_;
    a.timeout = timeout_;
    a.scale = (float)scale;
    a.rank = rank_;
    a.world = world_;
    c10::hip::HIPGuard guard((c10::DeviceIndex)device_);
    tdl::xgmi_all_reduce(a, mode, algo_, c10::hip::getCurrentHIPStream().stream());
  }

  int rank_, world_, device_, algo_;
  int64_t n_;
  int blocks_ = 0;
  int64_t cap_ = 0, shard_ = 0, timeout_ = 0;
  float* buf_ = nullptr;
  uint32_t* sig_ = nullptr;
  uint32_t* epoch_ = nullptr;
  uint32_t* err_ = nullptr;
  tdl::XgmiPeers peers_;
  std::vector<void*> opened_;
  bool connected_ = false;
};

}  // namespace tdl_host
