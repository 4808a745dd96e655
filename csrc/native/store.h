// TCP key-value store (server + client).  See store.cpp.
#pragma once
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "net.h"

namespace tdl {

class KVServer {
 public:
  KVServer(const std::string& host, int port);
  ~KVServer();
  int port() const;
  void stop();
  // client name -> seconds since that client was last heard from (departed clients excluded)
  std::map<std::string, double> heartbeat_ages() const;
  // names of clients whose connection dropped without an orderly BYE (crashed peers)
  std::vector<std::string> lost_clients() const;
  size_t num_keys() const;

 private:
  struct Impl;
  std::unique_ptr<Impl> impl_;
};

class KVClient {
 public:
  KVClient(const std::string& host, int port, int timeout_ms, const std::string& name);
  ~KVClient();
  void set(const std::string& k, const std::string& v);
  void append(const std::string& k, const std::string& v);
  bool get(const std::string& k, int64_t timeout_ms, std::string* out);
  int64_t add(const std::string& k, int64_t d);
  std::string compare_set(const std::string& k, const std::string& expected, const std::string& desired);
  bool check(const std::vector<std::string>& keys);
  bool del(const std::string& k);
  int64_t num_keys();
  bool wait(const std::vector<std::string>& keys, int64_t timeout_ms);
  bool ping();
  void close();

 private:
  void check_open() const;
  int fd_ = -1;
  int timeout_ms_;
  std::mutex mu_;
};

}  // namespace tdl
