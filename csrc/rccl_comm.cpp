// Owned RCCL communicator (see rccl_comm.h) + its Python bindings.
#include "rccl_comm.h"

#include <dlfcn.h>
#include <torch/extension.h>

#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>

#include <atomic>
#include <chrono>
#include <cstring>
#include <mutex>
#include <stdexcept>

namespace tdl_host {

namespace {
constexpr int kIdBytes = 128;  // NCCL_UNIQUE_ID_BYTES
struct UniqueId {
  char internal[kIdBytes];
};
typedef int Result;  // ncclResult_t: 0 success, 7 in progress
typedef void* Comm;  // ncclComm_t

// ncclDataType_t / ncclRedOp_t values of rccl.h (stable across RCCL releases)
int nccl_dtype(int d) {
  switch (d) {
    case 0: return 7;  // ncclFloat32
    case 1: return 9;  // ncclBfloat16
    case 2: return 6;  // ncclFloat16
    case 3: return 8;  // ncclFloat64
    case 4: return 2;  // ncclInt32
    case 5: return 4;  // ncclInt64
    case 6: return 1;  // ncclUint8
  }
  throw std::invalid_argument("rccl: unsupported dtype code " + std::to_string(d));
}
int nccl_op(int o) {
  if (o < 0 || o > 4) throw std::invalid_argument("rccl: unsupported reduction op " + std::to_string(o));
  return o;  // ncclSum 0, ncclProd 1, ncclMax 2, ncclMin 3, ncclAvg 4
}
}  // namespace

struct RcclApi {
  Result (*GetVersion)(int*);
  Result (*GetUniqueId)(UniqueId*);
  Result (*CommInitRank)(Comm*, int, UniqueId, int);
  Result (*CommDestroy)(Comm);
  Result (*CommAbort)(Comm);
  Result (*CommGetAsyncError)(Comm, Result*);
  const char* (*GetErrorString)(Result);
  Result (*AllReduce)(const void*, void*, size_t, int, int, Comm, hipStream_t);
  Result (*Broadcast)(const void*, void*, size_t, int, int, Comm, hipStream_t);
  Result (*AllGather)(const void*, void*, size_t, int, Comm, hipStream_t);
  Result (*ReduceScatter)(const void*, void*, size_t, int, int, Comm, hipStream_t);
  Result (*GroupStart)();
  Result (*GroupEnd)();
  Result (*CommInitAll)(Comm*, int, const int*);

  static const RcclApi& get() {
    static RcclApi api;
    static std::once_flag once;
    std::call_once(once, [] { api.load(); });
    return api;
  }

 private:
  void* sym(void* h, const char* name) {
    void* p = dlsym(h, name);
    if (p == nullptr) throw std::runtime_error(std::string("rccl: symbol ") + name + " not found");
    return p;
  }
  void load() {
    // the RCCL torch already loaded (its ProcessGroupNCCL links it): never a second copy
    void* h = dlopen("librccl.so", RTLD_NOW | RTLD_NOLOAD);
    if (h == nullptr) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (h == nullptr) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (h == nullptr) throw std::runtime_error(std::string("rccl: cannot load librccl.so: ") + dlerror());
    GetVersion = reinterpret_cast<decltype(GetVersion)>(sym(h, "ncclGetVersion"));
    GetUniqueId = reinterpret_cast<decltype(GetUniqueId)>(sym(h, "ncclGetUniqueId"));
    CommInitRank = reinterpret_cast<decltype(CommInitRank)>(sym(h, "ncclCommInitRank"));
    CommDestroy = reinterpret_cast<decltype(CommDestroy)>(sym(h, "ncclCommDestroy"));
    CommAbort = reinterpret_cast<decltype(CommAbort)>(sym(h, "ncclCommAbort"));
    CommGetAsyncError = reinterpret_cast<decltype(CommGetAsyncError)>(sym(h, "ncclCommGetAsyncError"));
    GetErrorString = reinterpret_cast<decltype(GetErrorString)>(sym(h, "ncclGetErrorString"));
    AllReduce = reinterpret_cast<decltype(AllReduce)>(sym(h, "ncclAllReduce"));
    Broadcast = reinterpret_cast<decltype(Broadcast)>(sym(h, "ncclBroadcast"));
    AllGather = reinterpret_cast<decltype(AllGather)>(sym(h, "ncclAllGather"));
    ReduceScatter = reinterpret_cast<decltype(ReduceScatter)>(sym(h, "ncclReduceScatter"));
    GroupStart = reinterpret_cast<decltype(GroupStart)>(sym(h, "ncclGroupStart"));
    GroupEnd = reinterpret_cast<decltype(GroupEnd)>(sym(h, "ncclGroupEnd"));
    CommInitAll = reinterpret_cast<decltype(CommInitAll)>(sym(h, "ncclCommInitAll"));
  }
};

RcclComm::RcclComm(const std::string& uid, int rank, int world, int device)
    : api_(RcclApi::get()), rank_(rank), world_(world), device_(device) {
  if ((int)uid.size() != kIdBytes) throw std::invalid_argument("rccl: unique id must be 128 bytes");
  if (world < 1 || rank < 0 || rank >= world) throw std::invalid_argument("rccl: bad rank / world");
  UniqueId id;
  std::memcpy(id.internal, uid.data(), kIdBytes);
  c10::hip::HIPGuard guard((c10::DeviceIndex)device);
  check(api_.CommInitRank(&comm_, world, id, rank), "ncclCommInitRank");
}

RcclComm::~RcclComm() {
  std::lock_guard<std::timed_mutex> lk(mu_);
  if (comm_ != nullptr && !aborted_.load(std::memory_order_acquire)) (void)api_.CommDestroy(comm_);
  comm_ = nullptr;
}

std::string RcclComm::unique_id() {
  UniqueId id;
  const auto& api = RcclApi::get();
  const Result r = api.GetUniqueId(&id);
  if (r != 0) throw std::runtime_error(std::string("rccl: ncclGetUniqueId failed: ") + api.GetErrorString(r));
  return std::string(id.internal, kIdBytes);
}

int RcclComm::version() {
  int v = 0;
  RcclApi::get().GetVersion(&v);
  return v;
}

void RcclComm::check(int r, const char* what) const {
  if (r != 0 && r != 7) throw std::runtime_error(std::string("rccl: ") + what + " failed: " + api_.GetErrorString(r));
}

void RcclComm::all_reduce(void* sb, void* rb, size_t n, int dt, int op, hipStream_t s) {
  std::lock_guard<std::timed_mutex> lk(mu_);
  if (aborted_.load(std::memory_order_acquire)) throw std::runtime_error("rccl: communicator was aborted");
  check(api_.AllReduce(sb, rb, n, nccl_dtype(dt), nccl_op(op), comm_, s), "ncclAllReduce");
}
void RcclComm::broadcast(void* sb, void* rb, size_t n, int dt, int root, hipStream_t s) {
  std::lock_guard<std::timed_mutex> lk(mu_);
  if (aborted_.load(std::memory_order_acquire)) throw std::runtime_error("rccl: communicator was aborted");
  check(api_.Broadcast(sb, rb, n, nccl_dtype(dt), root, comm_, s), "ncclBroadcast");
}
void RcclComm::all_gather(void* sb, void* rb, size_t n, int dt, hipStream_t s) {
  std::lock_guard<std::timed_mutex> lk(mu_);
  if (aborted_.load(std::memory_order_acquire)) throw std::runtime_error("rccl: communicator was aborted");
  check(api_.AllGather(sb, rb, n, nccl_dtype(dt), comm_, s), "ncclAllGather");
}
void RcclComm::reduce_scatter(void* sb, void* rb, size_t n, int dt, int op, hipStream_t s) {
  std::lock_guard<std::timed_mutex> lk(mu_);
  if (aborted_.load(std::memory_order_acquire)) throw std::runtime_error("rccl: communicator was aborted");
  check(api_.ReduceScatter(sb, rb, n, nccl_dtype(dt), nccl_op(op), comm_, s), "ncclReduceScatter");
}
void RcclComm::group_start() { check(api_.GroupStart(), "ncclGroupStart"); }  // (no comm_ use)
void RcclComm::group_end() { check(api_.GroupEnd(), "ncclGroupEnd"); }

int RcclComm::async_error() {
  std::lock_guard<std::timed_mutex> lk(mu_);
  if (aborted_.load(std::memory_order_acquire)) return -1;
  Result e = 0;
  const Result r = api_.CommGetAsyncError(comm_, &e);
  if (r != 0) return r;
  return (e == 0 || e == 7) ? 0 : e;
}

std::string RcclComm::error_string(int code) const {
  if (code < 0) return "communicator aborted";
  return api_.GetErrorString(code);
}

void RcclComm::abort() {
  const bool locked = mu_.try_lock_for(std::chrono::seconds(5));
  bool expected = false;
  if (comm_ != nullptr && aborted_.compare_exchange_strong(expected, true, std::memory_order_acq_rel))
    (void)api_.CommAbort(comm_);  // comm_ stays non-null: the destructor must not destroy it again
  if (locked) mu_.unlock();
}

// ------------------------------------------------------------------ RcclClique
RcclClique::RcclClique(const std::vector<int>& devices) : api_(RcclApi::get()), devices_(devices) {
  if (devices.empty()) throw std::invalid_argument("rccl: a clique needs at least one device");
  for (size_t i = 0; i < devices.size(); ++i)
    for (size_t j = 0; j < i; ++j)
      if (devices[i] == devices[j])
        throw std::invalid_argument("rccl: a clique needs distinct devices (RCCL refuses two ranks on one GPU)");
  comms_.assign(devices.size(), nullptr);
  check(api_.CommInitAll(comms_.data(), (int)devices.size(), devices.data()), "ncclCommInitAll");
}

RcclClique::~RcclClique() {
  std::lock_guard<std::timed_mutex> lk(mu_);
  if (!aborted_.load(std::memory_order_acquire))
    for (void* c : comms_)
      if (c != nullptr) (void)api_.CommDestroy(c);
  comms_.clear();
}

void RcclClique::check(int r, const char* what) const {
  if (r != 0 && r != 7) throw std::runtime_error(std::string("rccl: ") + what + " failed: " + api_.GetErrorString(r));
}

void RcclClique::all_reduce(const std::vector<void*>& bufs, size_t count, int dtype, int op,
                            const std::vector<hipStream_t>& streams) {
  if (bufs.size() != comms_.size() || streams.size() != comms_.size())
    throw std::invalid_argument("rccl: one buffer and one stream per clique device expected");
  std::lock_guard<std::timed_mutex> lk(mu_);
  if (aborted_.load(std::memory_order_acquire)) throw std::runtime_error("rccl: clique was aborted");
  check(api_.GroupStart(), "ncclGroupStart");
  Result first = 0;
  for (size_t i = 0; i < comms_.size(); ++i) {
    const Result r = api_.AllReduce(bufs[i], bufs[i], count, nccl_dtype(dtype), nccl_op(op), comms_[i], streams[i]);
    if (first == 0 && r != 0 && r != 7) first = r;
  }
  const Result e = api_.GroupEnd();  // always closes the group, also after a failed enqueue
  check(first, "ncclAllReduce (grouped)");
  check(e, "ncclGroupEnd");
}

void RcclClique::broadcast(const std::vector<void*>& bufs, size_t count, int dtype, int root,
                           const std::vector<hipStream_t>& streams) {
  if (bufs.size() != comms_.size() || streams.size() != comms_.size())
    throw std::invalid_argument("rccl: one buffer and one stream per clique device expected");
  std::lock_guard<std::timed_mutex> lk(mu_);
  if (aborted_.load(std::memory_order_acquire)) throw std::runtime_error("rccl: clique was aborted");
  check(api_.GroupStart(), "ncclGroupStart");
  Result first = 0;
  for (size_t i = 0; i < comms_.size(); ++i) {
    const Result r = api_.Broadcast(bufs[i], bufs[i], count, nccl_dtype(dtype), root, comms_[i], streams[i]);
    if (first == 0 && r != 0 && r != 7) first = r;
  }
  const Result e = api_.GroupEnd();
  check(first, "ncclBroadcast (grouped)");
  check(e, "ncclGroupEnd");
}

int RcclClique::async_error() {
  std::lock_guard<std::timed_mutex> lk(mu_);
  if (aborted_.load(std::memory_order_acquire)) return -1;
  for (void* c : comms_) {
    Result e = 0;
    const Result r = api_.CommGetAsyncError(c, &e);
    if (r != 0) return r;
    if (e != 0 && e != 7) return e;
  }
  return 0;
}

std::string RcclClique::error_string(int code) const {
  if (code < 0) return "clique aborted";
  return api_.GetErrorString(code);
}

void RcclClique::abort() {
  const bool locked = mu_.try_lock_for(std::chrono::seconds(5));
  bool expected = false;
  if (aborted_.compare_exchange_strong(expected, true, std::memory_order_acq_rel))
    for (void* c : comms_)
      if (c != nullptr) (void)api_.CommAbort(c);
  if (locked) mu_.unlock();
}

}  // namespace tdl_host

namespace {
using tdl_host::RcclComm;

int dtype_code(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return 0;
    case at::kBFloat16: return 1;
    case at::kHalf: return 2;
    case at::kDouble: return 3;
    case at::kInt: return 4;
    case at::kLong: return 5;
    case at::kByte: return 6;
    default: TORCH_CHECK(false, "rccl: unsupported tensor dtype ", t.scalar_type());
  }
}

void check_t(const at::Tensor& t, const RcclComm& c, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "rccl: ", what, " must be a contiguous GPU tensor");
  (void)c;
}

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }
}  // namespace

void register_rccl(pybind11::module& m) {
  pybind11::class_<RcclComm>(m, "RcclComm")
      // the id arrives as std::string (converted while the GIL is held): the constructor runs with
      // the GIL released, so no Python object may be owned by this lambda
      .def(pybind11::init([](const std::string& uid, int rank, int world, int device) {
             return new RcclComm(uid, rank, world, device);
           }),
           pybind11::arg("unique_id"), pybind11::arg("rank"), pybind11::arg("world"), pybind11::arg("device"),
           pybind11::call_guard<pybind11::gil_scoped_release>())
      .def_static("unique_id", []() { return pybind11::bytes(RcclComm::unique_id()); })
      .def_static("version", &RcclComm::version)
      .def_property_readonly("rank", &RcclComm::rank)
      .def_property_readonly("world", &RcclComm::world)
      .def("all_reduce",
           [](RcclComm& c, at::Tensor t, int op) {
             check_t(t, c, "tensor");
             c.all_reduce(t.data_ptr(), t.data_ptr(), t.numel(), dtype_code(t), op, stream());
           },
           pybind11::arg("tensor"), pybind11::arg("op") = 0)
      .def("broadcast",
           [](RcclComm& c, at::Tensor t, int root) {
             check_t(t, c, "tensor");
             c.broadcast(t.data_ptr(), t.data_ptr(), t.numel(), dtype_code(t), root, stream());
           },
           pybind11::arg("tensor"), pybind11::arg("root") = 0)
      .def("all_gather",
           [](RcclComm& c, at::Tensor out, at::Tensor in) {
             check_t(out, c, "out");
             check_t(in, c, "in");
             TORCH_CHECK(out.numel() == in.numel() * c.world() && out.scalar_type() == in.scalar_type(),
                         "rccl: all_gather out must hold world x in");
             c.all_gather(in.data_ptr(), out.data_ptr(), in.numel(), dtype_code(in), stream());
           })
      .def("reduce_scatter",
           [](RcclComm& c, at::Tensor out, at::Tensor in, int op) {
             check_t(out, c, "out");
             check_t(in, c, "in");
             TORCH_CHECK(in.numel() == out.numel() * c.world() && out.scalar_type() == in.scalar_type(),
                         "rccl: reduce_scatter in must hold world x out");
             c.reduce_scatter(in.data_ptr(), out.data_ptr(), out.numel(), dtype_code(in), op, stream());
           },
           pybind11::arg("out"), pybind11::arg("in"), pybind11::arg("op") = 0)
      .def("group_start", &RcclComm::group_start)
      .def("group_end", &RcclComm::group_end)
      .def("async_error", &RcclComm::async_error)
      .def("error_string", &RcclComm::error_string)
      .def("abort", &RcclComm::abort, pybind11::call_guard<pybind11::gil_scoped_release>())
      .def_property_readonly("aborted", &RcclComm::aborted);

  using tdl_host::RcclClique;
  // per-device buffers + streams of one grouped call: tensor i must live on devices()[i]; its part
  // is enqueued on that device's CURRENT stream (the engine's per-device replica stream)
  auto gather = [](RcclClique& c, const std::vector<at::Tensor>& ts, std::vector<void*>& bufs,
                   std::vector<hipStream_t>& streams) {
    TORCH_CHECK((int)ts.size() == c.size(), "rccl clique: one tensor per device expected");
    for (size_t i = 0; i < ts.size(); ++i) {
      const at::Tensor& t = ts[i];
      TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "rccl clique: tensors must be contiguous GPU tensors");
      TORCH_CHECK(t.get_device() == c.devices()[i], "rccl clique: tensor ", i, " is on device ", t.get_device(),
                  ", expected ", c.devices()[i]);
      TORCH_CHECK(t.numel() == ts[0].numel() && t.scalar_type() == ts[0].scalar_type(),
                  "rccl clique: tensors differ in size or dtype");
      bufs.push_back(t.data_ptr());
      streams.push_back(c10::hip::getCurrentHIPStream((c10::DeviceIndex)c.devices()[i]).stream());
    }
  };
  pybind11::class_<RcclClique>(m, "RcclClique")
      .def(pybind11::init<const std::vector<int>&>(), pybind11::arg("devices"),
           pybind11::call_guard<pybind11::gil_scoped_release>())
      .def_property_readonly("size", &RcclClique::size)
      .def_property_readonly("devices", &RcclClique::devices)
      .def("all_reduce",
           [gather](RcclClique& c, const std::vector<at::Tensor>& ts, int op) {
             std::vector<void*> bufs;
             std::vector<hipStream_t> streams;
             gather(c, ts, bufs, streams);
             c.all_reduce(bufs, ts[0].numel(), dtype_code(ts[0]), op, streams);
           },
           pybind11::arg("tensors"), pybind11::arg("op") = 0)
      .def("broadcast",
           [gather](RcclClique& c, const std::vector<at::Tensor>& ts, int root) {
             std::vector<void*> bufs;
             std::vector<hipStream_t> streams;
             gather(c, ts, bufs, streams);
             c.broadcast(bufs, ts[0].numel(), dtype_code(ts[0]), root, streams);
           },
           pybind11::arg("tensors"), pybind11::arg("root") = 0)
      .def("async_error", &RcclClique::async_error)
      .def("error_string", &RcclClique::error_string)
      .def("abort", &RcclClique::abort, pybind11::call_guard<pybind11::gil_scoped_release>())
      .def_property_readonly("aborted", &RcclClique::aborted);
}
