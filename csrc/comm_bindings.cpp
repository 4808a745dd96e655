// Python bindings of the xGMI all-reduce channels (csrc/xgmi_channel.h, csrc/kernels/xgmi.hip).
#include "xgmi_channel.h"

using tdl_host::XgmiChannel;

namespace {
// Direct loads/stores from `device` into `peer`'s memory (the xGMI link between them).  One process
// driving several GPUs (single-process MirroredStrategy) maps its replicas' exchange buffers by
// plain pointers instead of IPC handles, so access must be enabled per ordered pair.  Same device:
// nothing to do.  Returns false when the pair has no peer path.
bool enable_peer_access(int64_t device, int64_t peer) {
  if (device == peer) return true;
  int can = 0;
  tdl_host::hip_ok(hipDeviceCanAccessPeer(&can, (int)device, (int)peer), "hipDeviceCanAccessPeer");
  if (!can) return false;
  c10::hip::HIPGuard guard((c10::DeviceIndex)device);
  const hipError_t e = hipDeviceEnablePeerAccess((int)peer, 0);
  if (e == hipErrorPeerAccessAlreadyEnabled) {
    (void)hipGetLastError();
    return true;
  }
  tdl_host::hip_ok(e, "hipDeviceEnablePeerAccess");
  return true;
}
}  // namespace

void register_comm(pybind11::module& m) {
  m.def("enable_peer_access", &enable_peer_access, pybind11::arg("device"), pybind11::arg("peer"));
  pybind11::class_<XgmiChannel>(m, "XgmiChannel")
      .def(pybind11::init<int64_t, int64_t, int64_t, int64_t, double, int64_t, int64_t>(), pybind11::arg("rank"),
           pybind11::arg("world"), pybind11::arg("numel"), pybind11::arg("device"), pybind11::arg("timeout_s") = 60.0,
           pybind11::arg("algo") = 0, pybind11::arg("min_blocks") = 0)
      .def_property_readonly("sig_blocks", &XgmiChannel::sig_blocks)
      .def_property_readonly("cap", &XgmiChannel::cap)
      .def_property_readonly("algo", &XgmiChannel::algo)
      .def_property_readonly("connected", &XgmiChannel::connected)
      .def("handle", &XgmiChannel::handle, pybind11::arg("signals"))
      .def("open", &XgmiChannel::open)
      .def("connect_local", &XgmiChannel::connect_local)
      .def("all_reduce", &XgmiChannel::all_reduce, pybind11::arg("src"), pybind11::arg("dst"),
           pybind11::arg("scale") = 1.0)
      .def("all_reduce_sgd", &XgmiChannel::all_reduce_sgd, pybind11::arg("g"), pybind11::arg("w"),
           pybind11::arg("lr"), pybind11::arg("scale") = 1.0)
      .def("error", &XgmiChannel::error)
      .def("reset_error", &XgmiChannel::reset_error);
}
