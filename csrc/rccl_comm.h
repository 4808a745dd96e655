// Owned RCCL communicator (Communicator over ncclCommInitRank / ncclAllReduce /
// ncclBroadcast / ncclGroupStart+End / ncclCommGetAsyncError / ncclCommAbort), one rank per GPU.
//
// torch.distributed's "nccl" process group is RCCL too, but it owns the communicator: its error
// handling is a watchdog thread with a 10-minute default and a process teardown.  This class gives
// the framework the communicator itself: collectives enqueued on the caller's HIP stream (so they
// record into hipGraphs like any kernel), a non-blocking async-error query for the job watchdog,
// and ncclCommAbort from any thread, which makes a collective that waits for a dead or out-of-step
// peer return instead of hanging the GPU queue.
//
// The RCCL entry points are resolved at run time from the librccl the process already has loaded
// (torch's own copy, RCCL 2.26 at the time of writing -- SURVEY.md §7.4 risk 3: two RCCL builds in
// one process must not be mixed), so only ABI-stable API of RCCL >= 2.18 is used: no config structs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <mutex>
#include <string>
#include <vector>

namespace tdl_host {

struct RcclApi;

class RcclComm {
 public:
  // unique_id: the 128 bytes rank 0 got from unique_id() and shared with every rank
  RcclComm(const std::string& unique_id, int rank, int world, int device);
  ~RcclComm();

  static std::string unique_id();  // ncclGetUniqueId (rank 0)
  static int version();            // ncclGetVersion of the resolved library

  int rank() const { return rank_; }
  int world() const { return world_; }

  // dtype: 0 f32, 1 bf16, 2 f16, 3 f64, 4 i32, 5 i64, 6 u8; op: 0 sum, 1 prod, 2 max, 3 min, 4 avg
  void all_reduce(void* sendbuf, void* recvbuf, size_t count, int dtype, int op, hipStream_t s);
  void broadcast(void* sendbuf, void* recvbuf, size_t count, int dtype, int root, hipStream_t s);
  void all_gather(void* sendbuf, void* recvbuf, size_t sendcount, int dtype, hipStream_t s);
  void reduce_scatter(void* sendbuf, void* recvbuf, size_t recvcount, int dtype, int op, hipStream_t s);
  void group_start();
  void group_end();

  // ncclCommGetAsyncError: 0 = fine (ncclSuccess / ncclInProgress), otherwise the RCCL error code
  int async_error();
  std::string error_string(int code) const;
  // ncclCommAbort: unblocks every pending collective of this communicator; safe from another
  // thread; the communicator is unusable afterwards
  void abort();
  bool aborted() const { return aborted_.load(std::memory_order_acquire); }

 private:
  void check(int r, const char* what) const;
  const RcclApi& api_;
  void* comm_ = nullptr;
  int rank_, world_, device_;
  // abort() may run on the job watchdog's thread while the main thread enqueues: every use of comm_
  // holds mu_ and re-checks aborted_ under it, so no enqueue starts on a communicator that abort()
  // has freed.  abort() waits for the lock only a bounded time: an enqueue that is itself stuck
  // inside RCCL (e.g. connection setup towards a dead peer) is exactly what ncclCommAbort exists to
  // unblock, so after the wait it aborts regardless.
  std::timed_mutex mu_;
  std::atomic<bool> aborted_{false};
};

// One process, G devices (single-process MirroredStrategy, README.md:15-17 "NcclAllReduce" between
// the GPUs of one machine): ncclCommInitAll creates one communicator per device in one call, and
// every collective is issued for all G devices at once inside ncclGroupStart/End (RCCL requires
// the G per-device calls of one process to be grouped, or the first blocks waiting for the others).
// Each device's part is enqueued on the stream passed for that device.
class RcclClique {
 public:
  explicit RcclClique(const std::vector<int>& devices);
  ~RcclClique();

  int size() const { return (int)comms_.size(); }
  const std::vector<int>& devices() const { return devices_; }

  // bufs[i] lives on devices()[i]; in place; every buffer has `count` elements
  void all_reduce(const std::vector<void*>& bufs, size_t count, int dtype, int op,
                  const std::vector<hipStream_t>& streams);
  void broadcast(const std::vector<void*>& bufs, size_t count, int dtype, int root,
                 const std::vector<hipStream_t>& streams);
  // first failing communicator's RCCL error code, 0 if every one is fine
  int async_error();
  std::string error_string(int code) const;
  void abort();
  bool aborted() const { return aborted_.load(std::memory_order_acquire); }

 private:
  void check(int r, const char* what) const;
  const RcclApi& api_;
  std::vector<void*> comms_;
  std::vector<int> devices_;
  std::timed_mutex mu_;
  std::atomic<bool> aborted_{false};
};

}  // namespace tdl_host
