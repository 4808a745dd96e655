// Host TCP ring collectives: the CollectiveCommunication.RING data plane (README.md:23 — TF's
// ring all-reduce over gRPC) and the CPU-replica fallback of README.md:34.
//
// Each rank keeps two persistent sockets: one it connected to its right neighbour and one it
// accepted from its left neighbour.  All-reduce = ring reduce-scatter + ring all-gather over W
// segments; every step is a full-duplex exchange (send segment to the right while receiving from
// the left) driven by one poll() loop, and received elements are reduced as soon as they land, so
// the reduction is pipelined with the transfer.  Reductions happen in a fixed order, so every rank
// ends with bit-identical results.
#include "ring.h"

#include <sys/socket.h>

#include <algorithm>
#include <cmath>
#include <vector>

namespace tdl {

using namespace net;

namespace {

void set_nonblocking(int fd, bool nb) {
  int fl = ::fcntl(fd, F_GETFL, 0);
  ::fcntl(fd, F_SETFL, nb ? (fl | O_NONBLOCK) : (fl & ~O_NONBLOCK));
}

template <typename T>
void reduce_into(T* dst, const T* src, int64_t n, RedOp op) {
  switch (op) {
    case RedOp::kSum:
      for (int64_t i = 0; i < n; ++i) dst[i] += src[i];
      break;
    case RedOp::kProd:
      for (int64_t i = 0; i < n; ++i) dst[i] *= src[i];
      break;
    case RedOp::kMax:
      for (int64_t i = 0; i < n; ++i) dst[i] = std::max(dst[i], src[i]);
      break;
    case RedOp::kMin:
      for (int64_t i = 0; i < n; ++i) dst[i] = std::min(dst[i], src[i]);
      break;
  }
}

void reduce_bytes(void* dst, const void* src, int64_t n, DType dt, RedOp op) {
  switch (dt) {
    case DType::kF32: reduce_into((float*)dst, (const float*)src, n, op); break;
    case DType::kF64: reduce_into((double*)dst, (const double*)src, n, op); break;
    case DType::kI32: reduce_into((int32_t*)dst, (const int32_t*)src, n, op); break;
    case DType::kI64: reduce_into((int64_t*)dst, (const int64_t*)src, n, op); break;
  }
}

}  // namespace

size_t dtype_size(DType dt) {
  switch (dt) {
    case DType::kF32: return 4;
    case DType::kF64: return 8;
    case DType::kI32: return 4;
    case DType::kI64: return 8;
  }
  return 4;
}

RingComm::RingComm(int rank, int world, const std::string& listen_host, int timeout_ms)
    : rank_(rank), world_(world), timeout_ms_(timeout_ms) {
  if (world_ > 1) listen_fd_ = listen_on(listen_host, 0, &port_);
}

RingComm::~RingComm() { close(); }

void RingComm::close() {
  for (int* fd : {&right_fd_, &left_fd_, &listen_fd_}) {
    if (*fd >= 0) {
      ::close(*fd);
      *fd = -1;
    }
  }
}

void RingComm::abort() {
  for (int fd : {right_fd_, left_fd_}) {
    if (fd >= 0) ::shutdown(fd, SHUT_RDWR);
  }
}

void RingComm::connect(const std::string& right_host, int right_port) {
  if (world_ <= 1) return;
  // connect to the right neighbour (announce our rank), accept the left neighbour
  right_fd_ = connect_to(right_host, right_port, timeout_ms_);
  int32_t me = rank_;
  send_all(right_fd_, &me, 4);
  const int left = (rank_ - 1 + world_) % world_;
  auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms_);
  while (left_fd_ < 0) {
    int remain = (int)std::chrono::duration_cast<std::chrono::milliseconds>(deadline - std::chrono::steady_clock::now()).count();
    if (remain <= 0 || !wait_readable(listen_fd_, remain)) throw NetError("ring: timed out waiting for left neighbour");
    int fd = ::accept(listen_fd_, nullptr, nullptr);
    if (fd < 0) continue;
    set_nodelay(fd);
    int32_t who = -1;
    recv_all(fd, &who, 4, timeout_ms_);
    if (who != left) {
      ::close(fd);
      throw NetError("ring: unexpected peer rank " + std::to_string(who) + " (expected " + std::to_string(left) + ")");
    }
    left_fd_ = fd;
  }
  set_bufsizes(right_fd_, 4 << 20);
  set_bufsizes(left_fd_, 4 << 20);
  ::close(listen_fd_);
  listen_fd_ = -1;
}

// Full-duplex exchange: send `sn` bytes to the right while receiving `rn` bytes from the left.
// If reduce_dst is non-null, received elements are reduced into it as they complete.
void RingComm::exchange(const char* sbuf, size_t sn, char* rbuf, size_t rn, char* reduce_dst, DType dt, RedOp op) {
  set_nonblocking(right_fd_, true);
  set_nonblocking(left_fd_, true);
  size_t sent = 0, recvd = 0, reduced = 0;
  const size_t es = dtype_size(dt);
  auto last = std::chrono::steady_clock::now();
  try {
    while (sent < sn || recvd < rn) {
      pollfd p[2];
      int np = 0;
      int is = -1, ir = -1;
      if (sent < sn) { p[np] = {right_fd_, POLLOUT, 0}; is = np++; }
      if (recvd < rn) { p[np] = {left_fd_, POLLIN, 0}; ir = np++; }
      int r = ::poll(p, np, 1000);
      if (r < 0) {
        if (errno == EINTR) continue;
        throw NetError(errstr("poll"));
      }
      bool progress = false;
      if (is >= 0 && (p[is].revents & (POLLOUT | POLLERR | POLLHUP))) {
        if (p[is].revents & (POLLERR | POLLHUP)) throw NetError("ring: right neighbour connection lost");
        ssize_t k = ::send(right_fd_, sbuf + sent, std::min<size_t>(sn - sent, 1 << 20), MSG_NOSIGNAL);
        if (k > 0) { sent += (size_t)k; progress = true; }
        else if (k < 0 && errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR) throw NetError(errstr("ring send"));
      }
      if (ir >= 0 && (p[ir].revents & (POLLIN | POLLERR | POLLHUP))) {
        ssize_t k = ::recv(left_fd_, rbuf + recvd, rn - recvd, 0);
        if (k > 0) {
          recvd += (size_t)k;
          progress = true;
          if (reduce_dst) {
            size_t done = (recvd / es) * es;
            if (done > reduced) {
              reduce_bytes(reduce_dst + reduced, rbuf + reduced, (int64_t)((done - reduced) / es), dt, op);
              reduced = done;
            }
          }
        } else if (k == 0) {
          throw NetError("ring: left neighbour closed the connection");
        } else if (errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR) {
          throw NetError(errstr("ring recv"));
        }
      }
      auto now = std::chrono::steady_clock::now();
      if (progress) {
        last = now;
      } else if (timeout_ms_ >= 0 &&
                 std::chrono::duration_cast<std::chrono::milliseconds>(now - last).count() > timeout_ms_) {
        throw NetError("ring collective timed out: a peer stopped responding");
      }
    }
  } catch (...) {
    set_nonblocking(right_fd_, false);
    set_nonblocking(left_fd_, false);
    throw;
  }
  set_nonblocking(right_fd_, false);
  set_nonblocking(left_fd_, false);
}

void RingComm::all_reduce(void* data, int64_t n, DType dt, RedOp op) {
  if (world_ <= 1 || n == 0) return;
  const size_t es = dtype_size(dt);
  const int W = world_;
  auto seg_lo = [&](int c) { return (int64_t)((__int128)n * c / W); };
  char* base = static_cast<char*>(data);
  int64_t maxseg = 0;
  for (int c = 0; c < W; ++c) maxseg = std::max(maxseg, seg_lo(c + 1) - seg_lo(c));
  scratch_.resize((size_t)maxseg * es);
  // reduce-scatter: after W-1 steps rank r owns the full sum of segment (r+1) % W
  for (int s = 0; s < W - 1; ++s) {
    const int sc = ((rank_ - s) % W + W) % W;
    const int rc = ((rank_ - s - 1) % W + W) % W;
    exchange(base + seg_lo(sc) * es, (size_t)(seg_lo(sc + 1) - seg_lo(sc)) * es, scratch_.data(),
             (size_t)(seg_lo(rc + 1) - seg_lo(rc)) * es, base + seg_lo(rc) * es, dt, op);
  }
  // all-gather of the reduced segments
  for (int s = 0; s < W - 1; ++s) {
    const int sc = ((rank_ + 1 - s) % W + W) % W;
    const int rc = ((rank_ - s) % W + W) % W;
    exchange(base + seg_lo(sc) * es, (size_t)(seg_lo(sc + 1) - seg_lo(sc)) * es, base + seg_lo(rc) * es,
             (size_t)(seg_lo(rc + 1) - seg_lo(rc)) * es, nullptr, dt, op);
  }
}

void RingComm::broadcast(void* data, int64_t nbytes, int root) {
  if (world_ <= 1 || nbytes == 0) return;
  char* p = static_cast<char*>(data);
  const int right = (rank_ + 1) % world_;
  const int64_t piece = 1 << 20;
  for (int64_t off = 0; off < nbytes; off += piece) {
    const size_t len = (size_t)std::min(piece, nbytes - off);
    if (rank_ != root) recv_all(left_fd_, p + off, len, timeout_ms_);
    if (right != root) send_all(right_fd_, p + off, len);
  }
}

void RingComm::all_gather(const void* in, void* out, int64_t nbytes_per_rank) {
  char* o = static_cast<char*>(out);
  std::memcpy(o + (int64_t)rank_ * nbytes_per_rank, in, (size_t)nbytes_per_rank);
  if (world_ <= 1) return;
  const int W = world_;
  for (int s = 0; s < W - 1; ++s) {
    const int sc = ((rank_ - s) % W + W) % W;
    const int rc = ((rank_ - s - 1) % W + W) % W;
    exchange(o + (int64_t)sc * nbytes_per_rank, (size_t)nbytes_per_rank, o + (int64_t)rc * nbytes_per_rank,
             (size_t)nbytes_per_rank, nullptr, DType::kF32, RedOp::kSum);
  }
}

void RingComm::barrier() {
  int64_t one = 1;
  all_reduce(&one, 1, DType::kI64, RedOp::kSum);
  if (one != world_) throw NetError("ring barrier: inconsistent participant count");
}

}  // namespace tdl
