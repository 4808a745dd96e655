// Python bindings of the C++ runtime (module `tensorflow_distributed_learning_amd._native`).
#include <torch/extension.h>

#include <algorithm>
#include <array>
#include <vector>

#include "ring.h"
#include "store.h"

namespace py = pybind11;

namespace {

tdl::DType to_dtype(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return tdl::DType::kF32;
    case at::kDouble: return tdl::DType::kF64;
    case at::kInt: return tdl::DType::kI32;
    case at::kLong: return tdl::DType::kI64;
    default: TORCH_CHECK(false, "ring collectives support float32/float64/int32/int64 CPU tensors");
  }
  return tdl::DType::kF32;
}

tdl::RedOp to_op(const std::string& op) {
  if (op == "sum") return tdl::RedOp::kSum;
  if (op == "prod" || op == "product") return tdl::RedOp::kProd;
  if (op == "max") return tdl::RedOp::kMax;
  if (op == "min") return tdl::RedOp::kMin;
  TORCH_CHECK(false, "unknown reduce op ", op);
  return tdl::RedOp::kSum;
}

void check_cpu(const at::Tensor& t) {
  TORCH_CHECK(!t.is_cuda(), "ring collectives operate on host tensors (stage GPU tensors through host)");
  TORCH_CHECK(t.is_contiguous(), "ring collectives need contiguous tensors");
}

// CRC-32C (Castagnoli), used by the TFRecord event writer and checkpoint checksums.
const std::array<uint32_t, 256>& crc_table() {
  static std::array<uint32_t, 256> t = [] {
    std::array<uint32_t, 256> tab{};
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? (0x82F63B78u ^ (c >> 1)) : (c >> 1);
      tab[i] = c;
    }
    return tab;
  }();
  return t;
}

uint32_t crc32c(const std::string& data, uint32_t crc) {
  const auto& t = crc_table();
  crc = ~crc;
  for (unsigned char ch : data) crc = t[(crc ^ ch) & 0xff] ^ (crc >> 8);
  return ~crc;
}

// tf.data's buffered shuffle on an index sequence (data/dataset.py _shuffle_indices): keep a
// window of `buffer_size` pending elements, emit slot r[k] mod |window|, refill that slot from the
// source, or once the source is drained move the last pending element into it.  r[k] is the k-th
// output of splitmix64 seeded with `seed` (>> 2, i.e. 62 bits); the whole epoch runs without the
// GIL so an input pipeline's producer thread never stalls the launch loop.
static inline uint64_t splitmix64(uint64_t& state) {
  uint64_t z = (state += 0x9E3779B97F4A7C15ULL);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

at::Tensor buffered_shuffle(const at::Tensor& src, int64_t buffer_size, uint64_t seed) {
  TORCH_CHECK(!src.is_cuda() && src.scalar_type() == at::kLong && src.is_contiguous(), "src: int64 CPU");
  TORCH_CHECK(buffer_size > 0, "buffer_size must be > 0");
  const int64_t n = src.numel();
  const int64_t* s = src.data_ptr<int64_t>();
  at::Tensor out = at::empty({n}, src.options());
  int64_t* o = out.data_ptr<int64_t>();
  const int64_t w0 = std::min(buffer_size, n);
  std::vector<int64_t> buf(s, s + w0);
  int64_t nxt = w0;
  uint64_t state = seed;
  for (int64_t k = 0; k < n; ++k) {
    const int64_t len = (int64_t)buf.size();
    const int64_t j = (int64_t)((splitmix64(state) >> 2) % (uint64_t)len);
    o[k] = buf[j];
    if (nxt < n) {
      buf[j] = s[nxt++];
    } else {
      buf[j] = buf.back();
      buf.pop_back();
    }
  }
  return out;
}

}  // namespace

namespace tdl {
bool install_crash_trace();  // crash_trace.cpp
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "C++ runtime of tensorflow_distributed_learning_amd: TCP KV store / rendezvous, ring collectives";
  m.def("install_crash_trace", &tdl::install_crash_trace,
        "SIGABRT/SIGSEGV/SIGBUS/SIGFPE/SIGILL: print the faulting native thread's id, name and backtrace, then "
        "chain to the previous handler (faulthandler) / the default action");

  py::class_<tdl::KVServer>(m, "KVServer")
      .def(py::init<const std::string&, int>(), py::arg("host"), py::arg("port"))
      .def_property_readonly("port", &tdl::KVServer::port)
      .def("stop", &tdl::KVServer::stop, py::call_guard<py::gil_scoped_release>())
      .def("heartbeat_ages", &tdl::KVServer::heartbeat_ages)
      .def("lost_clients", &tdl::KVServer::lost_clients)
      .def("num_keys", &tdl::KVServer::num_keys);

  py::class_<tdl::KVClient>(m, "KVClient")
      .def(py::init<const std::string&, int, int, const std::string&>(), py::arg("host"), py::arg("port"),
           py::arg("timeout_ms") = 60000, py::arg("name") = "", py::call_guard<py::gil_scoped_release>())
      .def("set", [](tdl::KVClient& c, const std::string& k, py::bytes v) {
        std::string s = v;
        py::gil_scoped_release g;
        c.set(k, s);
      })
      .def("append", [](tdl::KVClient& c, const std::string& k, py::bytes v) {
        std::string s = v;
        py::gil_scoped_release g;
        c.append(k, s);
      })
      .def("get", [](tdl::KVClient& c, const std::string& k, int64_t timeout_ms) -> py::object {
        std::string out;
        bool ok;
        {
          py::gil_scoped_release g;
          ok = c.get(k, timeout_ms, &out);
        }
        if (!ok) return py::none();
        return py::bytes(out);
      }, py::arg("key"), py::arg("timeout_ms") = -1)
      .def("add", &tdl::KVClient::add, py::call_guard<py::gil_scoped_release>())
      .def("compare_set", [](tdl::KVClient& c, const std::string& k, py::bytes e, py::bytes d) {
        std::string es = e, ds = d, out;
        {
          py::gil_scoped_release g;
          out = c.compare_set(k, es, ds);
        }
        return py::bytes(out);
      })
      .def("check", &tdl::KVClient::check, py::call_guard<py::gil_scoped_release>())
      .def("delete", &tdl::KVClient::del, py::call_guard<py::gil_scoped_release>())
      .def("num_keys", &tdl::KVClient::num_keys, py::call_guard<py::gil_scoped_release>())
      .def("wait", &tdl::KVClient::wait, py::arg("keys"), py::arg("timeout_ms") = -1,
           py::call_guard<py::gil_scoped_release>())
      .def("ping", &tdl::KVClient::ping, py::call_guard<py::gil_scoped_release>())
      .def("close", &tdl::KVClient::close, py::call_guard<py::gil_scoped_release>());

  py::class_<tdl::RingComm>(m, "RingComm")
      .def(py::init<int, int, const std::string&, int>(), py::arg("rank"), py::arg("world"),
           py::arg("listen_host") = "0.0.0.0", py::arg("timeout_ms") = 300000)
      .def_property_readonly("port", &tdl::RingComm::port)
      .def_property_readonly("rank", &tdl::RingComm::rank)
      .def_property_readonly("world", &tdl::RingComm::world)
      .def("connect", &tdl::RingComm::connect, py::call_guard<py::gil_scoped_release>())
      .def("all_reduce", [](tdl::RingComm& r, at::Tensor t, const std::string& op) {
        check_cpu(t);
        auto dt = to_dtype(t);
        auto o = to_op(op);
        void* p = t.data_ptr();
        int64_t n = t.numel();
        py::gil_scoped_release g;
        r.all_reduce(p, n, dt, o);
      }, py::arg("tensor"), py::arg("op") = "sum")
      .def("broadcast", [](tdl::RingComm& r, at::Tensor t, int root) {
        check_cpu(t);
        void* p = t.data_ptr();
        int64_t nb = t.numel() * t.element_size();
        py::gil_scoped_release g;
        r.broadcast(p, nb, root);
      })
      .def("all_gather", [](tdl::RingComm& r, at::Tensor in, at::Tensor out) {
        check_cpu(in);
        check_cpu(out);
        TORCH_CHECK(out.numel() * out.element_size() == in.numel() * in.element_size() * r.world(),
                    "all_gather: output must hold world * input bytes");
        const void* ip = in.data_ptr();
        void* op = out.data_ptr();
        int64_t nb = in.numel() * in.element_size();
        py::gil_scoped_release g;
        r.all_gather(ip, op, nb);
      })
      .def("barrier", &tdl::RingComm::barrier, py::call_guard<py::gil_scoped_release>())
      .def("close", &tdl::RingComm::close)
      .def("abort", &tdl::RingComm::abort);

  m.def("buffered_shuffle", &buffered_shuffle, py::arg("src"), py::arg("buffer_size"), py::arg("seed"),
        py::call_guard<py::gil_scoped_release>());
  m.def("crc32c", [](py::bytes data, uint32_t crc) { return crc32c(std::string(data), crc); }, py::arg("data"),
        py::arg("crc") = 0u);
}
