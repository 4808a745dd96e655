// Small POSIX TCP helpers shared by the rendezvous store and the ring communicator.
#pragma once
#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/types.h>
#include <unistd.h>

#include <chrono>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>

namespace tdl {
namespace net {

struct NetError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

inline std::string errstr(const std::string& what) { return what + ": " + std::strerror(errno); }

inline void set_nodelay(int fd) {
  int one = 1;
  ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}

inline void set_bufsizes(int fd, int bytes) {
  ::setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &bytes, sizeof(bytes));
  ::setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &bytes, sizeof(bytes));
}

// Listen on host:port (port 0 = ephemeral).  Returns fd; *bound_port receives the actual port.
inline int listen_on(const std::string& host, int port, int* bound_port, int backlog = 256) {
  int fd = ::socket(AF_INET, SOCK_STREAM, 0);
  if (fd < 0) throw NetError(errstr("socket"));
  int one = 1;
  ::setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_port = htons((uint16_t)port);
  if (host.empty() || host == "0.0.0.0" || host == "*") {
    addr.sin_addr.s_addr = htonl(INADDR_ANY);
  } else {
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    if (::getaddrinfo(host.c_str(), nullptr, &hints, &res) != 0 || !res) {
      ::close(fd);
      throw NetError("cannot resolve listen host '" + host + "'");
    }
    addr.sin_addr = reinterpret_cast<sockaddr_in*>(res->ai_addr)->sin_addr;
    ::freeaddrinfo(res);
  }
  if (::bind(fd, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) < 0) {
    std::string e = errstr("bind " + host + ":" + std::to_string(port));
    ::close(fd);
    throw NetError(e);
  }
  if (::listen(fd, backlog) < 0) {
    ::close(fd);
    throw NetError(errstr("listen"));
  }
  socklen_t len = sizeof(addr);
  ::getsockname(fd, reinterpret_cast<sockaddr*>(&addr), &len);
  if (bound_port) *bound_port = ntohs(addr.sin_port);
  return fd;
}

// Connect with retries until timeout_ms elapses (peers may not be listening yet).
inline int connect_to(const std::string& host, int port, int timeout_ms) {
  auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  std::string last = "timeout";
  while (true) {
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    int rc = ::getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res);
    if (rc == 0 && res) {
      int fd = ::socket(AF_INET, SOCK_STREAM, 0);
      if (fd >= 0) {
        if (::connect(fd, res->ai_addr, res->ai_addrlen) == 0) {
          ::freeaddrinfo(res);
          set_nodelay(fd);
          return fd;
        }
        last = errstr("connect " + host + ":" + std::to_string(port));
        ::close(fd);
      }
      ::freeaddrinfo(res);
    } else {
      last = "cannot resolve '" + host + "'";
    }
    if (std::chrono::steady_clock::now() >= deadline) throw NetError(last);
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
}

// Wait until fd is readable; returns false on timeout (timeout_ms < 0 = forever).
inline bool wait_readable(int fd, int timeout_ms) {
  pollfd p{fd, POLLIN, 0};
  while (true) {
    int r = ::poll(&p, 1, timeout_ms);
    if (r > 0) return true;
    if (r == 0) return false;
    if (errno != EINTR) throw NetError(errstr("poll"));
  }
}

inline void send_all(int fd, const void* buf, size_t n) {
  const char* p = static_cast<const char*>(buf);
  while (n > 0) {
    ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL);
    if (k < 0) {
      if (errno == EINTR) continue;
      throw NetError(errstr("send"));
    }
    p += k;
    n -= (size_t)k;
  }
}

inline void recv_all(int fd, void* buf, size_t n, int timeout_ms = -1) {
  char* p = static_cast<char*>(buf);
  while (n > 0) {
    if (timeout_ms >= 0 && !wait_readable(fd, timeout_ms)) throw NetError("recv timed out (peer unresponsive)");
    ssize_t k = ::recv(fd, p, n, 0);
    if (k < 0) {
      if (errno == EINTR) continue;
      throw NetError(errstr("recv"));
    }
    if (k == 0) throw NetError("connection closed by peer");
    p += k;
    n -= (size_t)k;
  }
}

inline void send_u64(int fd, uint64_t v) { send_all(fd, &v, 8); }
inline uint64_t recv_u64(int fd, int timeout_ms = -1) {
  uint64_t v;
  recv_all(fd, &v, 8, timeout_ms);
  return v;
}
inline void send_str(int fd, const std::string& s) {
  send_u64(fd, s.size());
  if (!s.empty()) send_all(fd, s.data(), s.size());
}
inline std::string recv_str(int fd, int timeout_ms = -1) {
  uint64_t n = recv_u64(fd, timeout_ms);
  if (n > (1ull << 34)) throw NetError("oversized message");
  std::string s(n, '\0');
  if (n) recv_all(fd, &s[0], n, timeout_ms);
  return s;
}

}  // namespace net
}  // namespace tdl
