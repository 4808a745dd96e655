// TCP key-value store: the control plane of cluster bring-up.
//
// Replaces TF's per-task gRPC server + CollectiveParamResolverDistributed for this framework:
// the chief task (TF_CONFIG chief/0, else worker/0 — README.md:51) runs a KVServer on its own
// host:port; every task connects a KVClient, registers itself, learns its global rank layout and
// exchanges the ring / RCCL bootstrap addresses.  Blocking GET / WAIT give the "wait until all
// gRPC services are ready" semantics of README.md:65-66; per-client last-seen times give the
// heartbeat used for failure detection.
#include "store.h"

#include <algorithm>
#include <condition_variable>
#include <map>
#include <mutex>
#include <set>

namespace tdl {

using namespace net;

enum Op : uint8_t {
  OP_SET = 1, OP_GET = 2, OP_ADD = 3, OP_CAS = 4, OP_CHECK = 5, OP_DEL = 6, OP_NUMKEYS = 7,
  OP_WAIT = 8, OP_PING = 9, OP_APPEND = 10, OP_HELLO = 11, OP_BYE = 12
};

struct KVServer::Impl {
  std::mutex mu;
  std::condition_variable cv;
  std::map<std::string, std::string> kv;
  std::map<std::string, double> last_seen;  // client name -> monotonic seconds
  std::set<std::string> departed;
  std::set<std::string> lost;  // clients whose connection dropped without BYE (crashed peers)
  int listen_fd = -1;
  int port = 0;
  bool stopping = false;
  std::thread acceptor;
  std::vector<std::thread> workers;
  std::vector<int> client_fds;

  static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
  }

  void touch(const std::string& who) {
    if (!who.empty()) last_seen[who] = now();
  }

  bool wait_keys(std::unique_lock<std::mutex>& lk, const std::vector<std::string>& keys, int64_t timeout_ms) {
    auto ready = [&] {
      if (stopping) return true;
      for (auto& k : keys)
        if (!kv.count(k)) return false;
      return true;
    };
    if (timeout_ms < 0) {
      cv.wait(lk, ready);
    } else if (!cv.wait_for(lk, std::chrono::milliseconds(timeout_ms), ready)) {
      return false;
    }
    return !stopping;
  }

  void serve(int fd) {
    std::string who;
    try {
      while (true) {
        uint8_t op;
        recv_all(fd, &op, 1);
        switch (op) {
          case OP_HELLO: {
            who = recv_str(fd);
            std::lock_guard<std::mutex> g(mu);
            touch(who);
            departed.erase(who);
            lost.erase(who);
            send_u64(fd, 1);
            break;
          }
          case OP_BYE: {
            std::lock_guard<std::mutex> g(mu);
            if (!who.empty()) departed.insert(who);
            send_u64(fd, 1);
            break;
          }
          case OP_SET: {
            std::string k = recv_str(fd), v = recv_str(fd);
            {
              std::lock_guard<std::mutex> g(mu);
              kv[k] = v;
              touch(who);
            }
            cv.notify_all();
            send_u64(fd, 1);
            break;
          }
          case OP_APPEND: {
            std::string k = recv_str(fd), v = recv_str(fd);
            {
              std::lock_guard<std::mutex> g(mu);
              kv[k] += v;
              touch(who);
            }
            cv.notify_all();
            send_u64(fd, 1);
            break;
          }
          case OP_GET: {
            std::string k = recv_str(fd);
            int64_t tmo = (int64_t)recv_u64(fd);
            std::unique_lock<std::mutex> lk(mu);
            touch(who);
            bool ok = wait_keys(lk, {k}, tmo);
            std::string v = ok ? kv[k] : std::string();
            lk.unlock();
            send_u64(fd, ok ? 1 : 0);
            send_str(fd, v);
            break;
          }
          case OP_ADD: {
            std::string k = recv_str(fd);
            int64_t d = (int64_t)recv_u64(fd);
            int64_t nv;
            {
              std::lock_guard<std::mutex> g(mu);
              auto it = kv.find(k);
              int64_t cur = (it == kv.end() || it->second.empty()) ? 0 : std::stoll(it->second);
              nv = cur + d;
              kv[k] = std::to_string(nv);
              touch(who);
            }
            cv.notify_all();
            send_u64(fd, (uint64_t)nv);
            break;
          }
          case OP_CAS: {
            std::string k = recv_str(fd), expected = recv_str(fd), desired = recv_str(fd);
            std::string out;
            {
              std::lock_guard<std::mutex> g(mu);
              auto it = kv.find(k);
              if (it == kv.end()) {
                if (expected.empty()) kv[k] = desired;
                out = kv.count(k) ? kv[k] : expected;
              } else {
                if (it->second == expected) it->second = desired;
                out = it->second;
              }
              touch(who);
            }
            cv.notify_all();
            send_str(fd, out);
            break;
          }
          case OP_CHECK: {
            uint64_t n = recv_u64(fd);
            std::vector<std::string> keys(n);
            for (auto& k : keys) k = recv_str(fd);
            bool all = true;
            {
              std::lock_guard<std::mutex> g(mu);
              for (auto& k : keys) all = all && kv.count(k);
              touch(who);
            }
            send_u64(fd, all ? 1 : 0);
            break;
          }
          case OP_DEL: {
            std::string k = recv_str(fd);
            size_t n;
            {
              std::lock_guard<std::mutex> g(mu);
              n = kv.erase(k);
              touch(who);
            }
            send_u64(fd, n);
            break;
          }
          case OP_NUMKEYS: {
            size_t n;
            {
              std::lock_guard<std::mutex> g(mu);
              n = kv.size();
            }
            send_u64(fd, n);
            break;
          }
          case OP_WAIT: {
            uint64_t n = recv_u64(fd);
            std::vector<std::string> keys(n);
            for (auto& k : keys) k = recv_str(fd);
            int64_t tmo = (int64_t)recv_u64(fd);
            std::unique_lock<std::mutex> lk(mu);
            touch(who);
            bool ok = wait_keys(lk, keys, tmo);
            lk.unlock();
            send_u64(fd, ok ? 1 : 0);
            break;
          }
          case OP_PING: {
            {
              std::lock_guard<std::mutex> g(mu);
              touch(who);
            }
            send_u64(fd, 1);
            break;
          }
          default:
            throw NetError("bad opcode");
        }
      }
    } catch (const std::exception&) {
      // connection ended: a client that never said BYE died (or lost the network)
      std::lock_guard<std::mutex> g(mu);
      if (!who.empty() && !departed.count(who) && !stopping) lost.insert(who);
    }
    ::close(fd);
  }

  void accept_loop() {
    while (true) {
      {
        std::lock_guard<std::mutex> g(mu);
        if (stopping) break;
      }
      bool r;
      try {
        r = wait_readable(listen_fd, 100);
      } catch (...) {
        break;
      }
      if (!r) continue;
      int fd = ::accept(listen_fd, nullptr, nullptr);
      if (fd < 0) continue;
      set_nodelay(fd);
      std::lock_guard<std::mutex> g(mu);
      if (stopping) {
        ::close(fd);
        break;
      }
      client_fds.push_back(fd);
      workers.emplace_back([this, fd] { serve(fd); });
    }
  }
};

KVServer::KVServer(const std::string& host, int port) : impl_(new Impl) {
  impl_->listen_fd = listen_on(host, port, &impl_->port);
  impl_->acceptor = std::thread([this] { impl_->accept_loop(); });
}

KVServer::~KVServer() { stop(); }

int KVServer::port() const { return impl_->port; }

void KVServer::stop() {
  if (!impl_) return;
  {
    std::lock_guard<std::mutex> g(impl_->mu);
    if (impl_->stopping) return;
    impl_->stopping = true;
    for (int fd : impl_->client_fds) ::shutdown(fd, SHUT_RDWR);
  }
  impl_->cv.notify_all();
  if (impl_->acceptor.joinable()) impl_->acceptor.join();
  for (auto& t : impl_->workers)
    if (t.joinable()) t.join();
  if (impl_->listen_fd >= 0) ::close(impl_->listen_fd);
  impl_->listen_fd = -1;
}

std::map<std::string, double> KVServer::heartbeat_ages() const {
  std::lock_guard<std::mutex> g(impl_->mu);
  std::map<std::string, double> out;
  double t = Impl::now();
  for (auto& kv : impl_->last_seen)
    if (!impl_->departed.count(kv.first)) out[kv.first] = t - kv.second;
  return out;
}

std::vector<std::string> KVServer::lost_clients() const {
  std::lock_guard<std::mutex> g(impl_->mu);
  return std::vector<std::string>(impl_->lost.begin(), impl_->lost.end());
}

size_t KVServer::num_keys() const {
  std::lock_guard<std::mutex> g(impl_->mu);
  return impl_->kv.size();
}

// ------------------------------------------------------------------------------------------------
KVClient::KVClient(const std::string& host, int port, int timeout_ms, const std::string& name)
    : timeout_ms_(timeout_ms) {
  fd_ = connect_to(host, port, timeout_ms);
  if (!name.empty()) {
    std::lock_guard<std::mutex> g(mu_);
    uint8_t op = OP_HELLO;
    send_all(fd_, &op, 1);
    send_str(fd_, name);
    recv_u64(fd_);
  }
}

KVClient::~KVClient() { close(); }

void KVClient::close() {
  std::lock_guard<std::mutex> g(mu_);
  if (fd_ >= 0) {
    try {
      uint8_t op = OP_BYE;
      send_all(fd_, &op, 1);
      recv_u64(fd_, 1000);
    } catch (...) {
    }
    ::close(fd_);
    fd_ = -1;
  }
}

void KVClient::check_open() const {
  if (fd_ < 0) throw NetError("KVClient is closed");
}

void KVClient::set(const std::string& k, const std::string& v) {
  std::lock_guard<std::mutex> g(mu_);
  check_open();
  uint8_t op = OP_SET;
  send_all(fd_, &op, 1);
  send_str(fd_, k);
  send_str(fd_, v);
  recv_u64(fd_, timeout_ms_);
}

void KVClient::append(const std::string& k, const std::string& v) {
  std::lock_guard<std::mutex> g(mu_);
  check_open();
  uint8_t op = OP_APPEND;
  send_all(fd_, &op, 1);
  send_str(fd_, k);
  send_str(fd_, v);
  recv_u64(fd_, timeout_ms_);
}

bool KVClient::get(const std::string& k, int64_t timeout_ms, std::string* out) {
  std::lock_guard<std::mutex> g(mu_);
  check_open();
  uint8_t op = OP_GET;
  send_all(fd_, &op, 1);
  send_str(fd_, k);
  send_u64(fd_, (uint64_t)timeout_ms);
  int rt = timeout_ms < 0 ? -1 : (int)std::min<int64_t>(timeout_ms + 30000, INT32_MAX);
  bool ok = recv_u64(fd_, rt) != 0;
  *out = recv_str(fd_, rt);
  return ok;
}

int64_t KVClient::add(const std::string& k, int64_t d) {
  std::lock_guard<std::mutex> g(mu_);
  check_open();
  uint8_t op = OP_ADD;
  send_all(fd_, &op, 1);
  send_str(fd_, k);
  send_u64(fd_, (uint64_t)d);
  return (int64_t)recv_u64(fd_, timeout_ms_);
}

std::string KVClient::compare_set(const std::string& k, const std::string& expected, const std::string& desired) {
  std::lock_guard<std::mutex> g(mu_);
  check_open();
  uint8_t op = OP_CAS;
  send_all(fd_, &op, 1);
  send_str(fd_, k);
  send_str(fd_, expected);
  send_str(fd_, desired);
  return recv_str(fd_, timeout_ms_);
}

bool KVClient::check(const std::vector<std::string>& keys) {
  std::lock_guard<std::mutex> g(mu_);
  check_open();
  uint8_t op = OP_CHECK;
  send_all(fd_, &op, 1);
  send_u64(fd_, keys.size());
  for (auto& k : keys) send_str(fd_, k);
  return recv_u64(fd_, timeout_ms_) != 0;
}

bool KVClient::del(const std::string& k) {
  std::lock_guard<std::mutex> g(mu_);
  check_open();
  uint8_t op = OP_DEL;
  send_all(fd_, &op, 1);
  send_str(fd_, k);
  return recv_u64(fd_, timeout_ms_) != 0;
}

int64_t KVClient::num_keys() {
  std::lock_guard<std::mutex> g(mu_);
  check_open();
  uint8_t op = OP_NUMKEYS;
  send_all(fd_, &op, 1);
  return (int64_t)recv_u64(fd_, timeout_ms_);
}

bool KVClient::wait(const std::vector<std::string>& keys, int64_t timeout_ms) {
  std::lock_guard<std::mutex> g(mu_);
  check_open();
  uint8_t op = OP_WAIT;
  send_all(fd_, &op, 1);
  send_u64(fd_, keys.size());
  for (auto& k : keys) send_str(fd_, k);
  send_u64(fd_, (uint64_t)timeout_ms);
  int rt = timeout_ms < 0 ? -1 : (int)std::min<int64_t>(timeout_ms + 30000, INT32_MAX);
  return recv_u64(fd_, rt) != 0;
}

bool KVClient::ping() {
  std::lock_guard<std::mutex> g(mu_);
  check_open();
  uint8_t op = OP_PING;
  send_all(fd_, &op, 1);
  return recv_u64(fd_, timeout_ms_) != 0;
}

}  // namespace tdl
