// Host TCP ring collectives (see ring.cpp).
#pragma once
#include <string>
#include <vector>

#include "net.h"

namespace tdl {

enum class DType { kF32, kF64, kI32, kI64 };
enum class RedOp { kSum, kProd, kMax, kMin };
size_t dtype_size(DType dt);

class RingComm {
 public:
  RingComm(int rank, int world, const std::string& listen_host, int timeout_ms);
  ~RingComm();
  int port() const { return port_; }
  int rank() const { return rank_; }
  int world() const { return world_; }
  void connect(const std::string& right_host, int right_port);
  void all_reduce(void* data, int64_t n, DType dt, RedOp op);
  void broadcast(void* data, int64_t nbytes, int root);
  void all_gather(const void* in, void* out, int64_t nbytes_per_rank);
  void barrier();
  void close();
  // Unblock a collective running on another thread (its poll/recv sees the shut-down sockets and
  // throws): the job watchdog's abort.  The descriptors stay open until close().
  void abort();

 private:
  void exchange(const char* sbuf, size_t sn, char* rbuf, size_t rn, char* reduce_dst, DType dt, RedOp op);
  int rank_, world_, timeout_ms_;
  int listen_fd_ = -1, port_ = 0, right_fd_ = -1, left_fd_ = -1;
  std::vector<char> scratch_;
};

}  // namespace tdl
