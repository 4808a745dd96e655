// Standalone self-test of the C++ runtime (KV store + TCP ring collectives) for sanitizer builds.
//
// The Python extension cannot run under ASan/TSan without preloading the sanitizer runtime into
// the interpreter, so the same sources (store.cpp, ring.cpp, net.h) are linked into this
// driver instead (build_native.py --sanitize address|thread; tests/test_native_sanitizers.py).
// Ranks are threads over localhost TCP, exactly the protocols the framework runs between
// processes: contended KV traffic (CAS slot claims, counters, blocking waits, heartbeats, a
// crashed client) and ring all-reduce / broadcast / all-gather / barrier for world 1..5 on
// integer-valued data, checked exactly (every rank must hold bit-identical results).
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <thread>
#include <vector>

#include "native/ring.h"
#include "native/store.h"

namespace {

int g_fail = 0;

#define CHECK(cond)                                                          \
  do {                                                                       \
    if (!(cond)) {                                                           \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++g_fail;                                                              \
    }                                                                        \
  } while (0)

void test_kv() {
  tdl::KVServer srv("127.0.0.1", 0);
  const int port = srv.port();
  {
    tdl::KVClient c("127.0.0.1", port, 5000, "main");
    c.set("a", "1");
    std::string v;
    CHECK(c.get("a", 1000, &v) && v == "1");
    CHECK(!c.get("missing", 20, &v));
    CHECK(c.add("n", 5) == 5 && c.add("n", -2) == 3);
    c.append("log", "ab");
    c.append("log", "cd");
    CHECK(c.get("log", 100, &v) && v == "abcd");
    CHECK(c.check({"a", "n"}) && !c.check({"a", "zz"}));
    CHECK(c.del("a") && !c.check({"a"}));
    CHECK(c.ping());
  }
  // contention: 8 clients race for 4 slots (CAS), bump a shared counter, and rendezvous on keys
  constexpr int kClients = 8, kIters = 200;
  std::atomic<int> claimed{0};
  std::vector<std::thread> th;
  for (int t = 0; t < kClients; ++t) {
    th.emplace_back([&, t] {
      tdl::KVClient c("127.0.0.1", port, 10000, "w" + std::to_string(t));
      for (int s = 0; s < 4; ++s) {
        const std::string me = std::to_string(t);
        if (c.compare_set("slot" + std::to_string(s), "", me) == me) claimed.fetch_add(1);
      }
      for (int i = 0; i < kIters; ++i) c.add("ctr", 1);
      c.set("ready" + std::to_string(t), "1");
      std::vector<std::string> keys;
      for (int k = 0; k < kClients; ++k) keys.push_back("ready" + std::to_string(k));
      CHECK(c.wait(keys, 10000));
      c.close();
    });
  }
  for (auto& x : th) x.join();
  CHECK(claimed.load() == 4);
  tdl::KVClient c("127.0.0.1", port, 5000, "checker");
  CHECK(c.add("ctr", 0) == kClients * kIters);
  // a blocking get released by another client's set
  std::string got;
  std::thread waiter([&] {
    tdl::KVClient c2("127.0.0.1", port, 5000, "waiter");
    c2.get("later", 5000, &got);
  });
  std::this_thread::sleep_for(std::chrono::milliseconds(20));
  c.set("later", "x");
  waiter.join();
  CHECK(got == "x");
  CHECK(srv.heartbeat_ages().count("checker") == 1);
  // a client that says HELLO and then drops its connection without BYE is reported as lost
  {
    int fd = tdl::net::connect_to("127.0.0.1", port, 5000);
    uint8_t op = 11;  // OP_HELLO
    tdl::net::send_all(fd, &op, 1);
    tdl::net::send_str(fd, "crasher");
    tdl::net::recv_u64(fd, 5000);
    ::close(fd);
  }
  bool lost = false;
  for (int i = 0; i < 200 && !lost; ++i) {
    for (auto& n : srv.lost_clients()) lost = lost || n == "crasher";
    if (!lost) std::this_thread::sleep_for(std::chrono::milliseconds(5));
  }
  CHECK(lost);
  c.close();
  srv.stop();
}

template <typename T>
void ring_case(int world, int64_t n, tdl::DType dt, tdl::RedOp op) {
  std::vector<std::unique_ptr<tdl::RingComm>> comms;
  for (int r = 0; r < world; ++r) comms.emplace_back(new tdl::RingComm(r, world, "127.0.0.1", 10000));
  std::vector<std::vector<T>> data(world, std::vector<T>(n));
  for (int r = 0; r < world; ++r)
    for (int64_t i = 0; i < n; ++i) data[r][i] = (T)(((i * 7 + r * 13) % 11) - 5 + (op == tdl::RedOp::kProd ? 7 : 0));
  std::vector<T> expect(n);
  for (int64_t i = 0; i < n; ++i) {
    T acc = data[0][i];
    for (int r = 1; r < world; ++r) {
      const T x = data[r][i];
      switch (op) {
        case tdl::RedOp::kSum: acc += x; break;
        case tdl::RedOp::kProd: acc *= x; break;
        case tdl::RedOp::kMax: acc = std::max(acc, x); break;
        case tdl::RedOp::kMin: acc = std::min(acc, x); break;
      }
    }
    expect[i] = acc;
  }
  std::vector<std::thread> th;
  std::vector<std::vector<char>> gathered(world);
  std::vector<int64_t> bc(world);
  for (int r = 0; r < world; ++r) {
    th.emplace_back([&, r] {
      auto& c = *comms[r];
      c.connect("127.0.0.1", comms[(r + 1) % world]->port());
      c.all_reduce(data[r].data(), n, dt, op);
      int64_t token = r == 2 % world ? 4242 : -1;
      c.broadcast(&token, sizeof(token), 2 % world);
      bc[r] = token;
      gathered[r].resize(sizeof(int32_t) * world);
      const int32_t mine = 100 + r;
      c.all_gather(&mine, gathered[r].data(), sizeof(int32_t));
      c.barrier();
      c.close();
    });
  }
  for (auto& x : th) x.join();
  for (int r = 0; r < world; ++r) {
    for (int64_t i = 0; i < n; ++i) CHECK(data[r][i] == expect[i]);
    CHECK(bc[r] == 4242);
    for (int q = 0; q < world; ++q) CHECK(reinterpret_cast<const int32_t*>(gathered[r].data())[q] == 100 + q);
  }
}

void test_ring() {
  for (int world : {1, 2, 3, 4, 5}) {
    for (int64_t n : {1, 3, 17, 1000, 225034}) {  // 225,034 = the reference CNN's gradient
      ring_case<float>(world, n, tdl::DType::kF32, tdl::RedOp::kSum);
      ring_case<int64_t>(world, n, tdl::DType::kI64, tdl::RedOp::kMax);
    }
    ring_case<double>(world, 4099, tdl::DType::kF64, tdl::RedOp::kMin);
    ring_case<int32_t>(world, 513, tdl::DType::kI32, tdl::RedOp::kProd);
  }
}

void test_ring_peer_loss() {
  // rank 1 dies before the collective: rank 0 must fail with an error, not hang
  tdl::RingComm a(0, 2, "127.0.0.1", 2000), b(1, 2, "127.0.0.1", 2000);
  std::thread tb([&] {
    b.connect("127.0.0.1", a.port());
    b.close();
  });
  a.connect("127.0.0.1", b.port());
  tb.join();
  std::vector<float> x(1 << 16, 1.f);
  bool threw = false;
  try {
    a.all_reduce(x.data(), (int64_t)x.size(), tdl::DType::kF32, tdl::RedOp::kSum);
  } catch (const std::exception&) {
    threw = true;
  }
  CHECK(threw);
}

}  // namespace

// Deliberate defects, to prove the sanitizer build is live (tests expect a report + failure).
int inject(const std::string& what) {
  if (what == "race") {
    int counter = 0;
    std::thread a([&] { for (int i = 0; i < 100000; ++i) ++counter; });
    std::thread b([&] { for (int i = 0; i < 100000; ++i) ++counter; });
    a.join();
    b.join();
    return counter == -1;
  }
  if (what == "oob") {
    std::vector<int> v(8, 1);
    volatile int* p = v.data();
    return p[8 + (int)v.size() % 2];
  }
  return 2;
}

int main(int argc, char** argv) {
  if (argc > 1) return inject(argv[1]);
  test_kv();
  test_ring();
  test_ring_peer_loss();
  if (g_fail) {
    std::fprintf(stderr, "native selftest: %d check(s) failed\n", g_fail);
    return 1;
  }
  std::printf("native selftest ok\n");
  return 0;
}
