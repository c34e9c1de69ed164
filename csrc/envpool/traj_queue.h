// Time-major trajectory batch queue: the host side of SURVEY.md §2.4 C1-C3
// (the reference's capacity-1 FIFOQueue of unrolls + dequeue_many + the
// time-major transposes + the StagingArea put, experiment.py:530-531,
// 576-597), redesigned so that no host copy or transpose remains:
//
//   * the queue owns K "slabs" in one POSIX shared-memory object; a slab is
//     exactly ONE learner batch in the learner's flat staging layout
//     (every field time-major [T+1, B, ...], 256-B aligned segments);
//   * a producer (actor thread or actor process) Claim()s a column b of the
//     slab currently being filled, writes its unroll straight into
//     [t, b, ...] step by step, and Commit()s; the B-th commit publishes the
//     slab (READY, FIFO by fill order);
//   * the consumer (learner) Acquire()s a READY slab, moves it to HBM with
//     ONE hipMemcpyAsync (the shm is hipHostRegister'ed, so the copy is a DMA
//     from the producers' pages), and Release()s it once that copy is done.
//
// States: FREE -> FILLING (columns being claimed/written) -> READY (all B
// committed) -> READING (consumer) -> FREE.  Column hand-out and slab
// selection run under a tiny process-shared spinlock; blocking waits use a
// process-shared futex on a header word that every transition bumps.
//
// Failure model (fail-stop, by design): a producer that dies between
// ClaimN() and Commit() keeps its columns, so that slab never becomes READY.
// Nothing reclaims them - a half-written unroll must never reach the
// learner.  The learner side detects it instead: actor-group processes are
// supervised (ActorGroups.check() raises as soon as a group exits), and for
// actor threads the learner's Acquire() loop raises 'learner starved' after
// --queue_timeout_secs; either way train() stops and the last checkpoint is
// the restart point (tests/test_traj_queue.py covers a producer that claims
// and never commits).
#pragma once

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <string>
#include <utility>
#include <vector>

namespace sa {

class TrajQueue {
 public:
  enum State : uint32_t { kFree = 0, kFilling = 1, kReady = 2, kReading = 3 };

  // create=true: creates the shm object (K slabs of slab_bytes, batch columns
  // each); false: attaches to an existing one (geometry read from it).
  TrajQueue(const std::string& name, int64_t num_slabs, int64_t slab_bytes,
            int64_t batch, bool create);
  ~TrajQueue();
  TrajQueue(const TrajQueue&) = delete;
  TrajQueue& operator=(const TrajQueue&) = delete;

  // -> (slab, column); (-1, -1) on timeout, (-2, -2) when closed.
  // timeout_ms < 0 waits forever.
  std::pair<int64_t, int64_t> Claim(int64_t timeout_ms);
  // All-or-nothing claim of n columns (a producer that steps several envs in
  // lockstep must never hold some columns while it waits for the rest: the
  // slabs those sit in could then never fill).  -> status 0 and the n
  // (slab, column) pairs, or status -1 timeout / -2 closed and no columns.
  std::pair<int64_t, std::vector<std::pair<int64_t, int64_t>>> ClaimN(int64_t n,
                                                                      int64_t timeout_ms);
  // Marks one claimed column of `slab` written; the last one publishes it.
  void Commit(int64_t slab);
  // Oldest READY slab (by fill order); -1 timeout, -2 closed.
  int64_t Acquire(int64_t timeout_ms);
  void Release(int64_t slab);
  void Close();
  bool closed() const;

  uint8_t* slab_data(int64_t slab) const;
  uint8_t* payload_base() const { return payload_; }
  int64_t payload_bytes() const { return num_slabs_ * slab_bytes_; }
  int64_t num_slabs() const { return num_slabs_; }
  int64_t slab_bytes() const { return slab_bytes_; }
  int64_t batch() const { return batch_; }
  int64_t num_ready() const;
  const std::string& name() const { return name_; }
  static void Unlink(const std::string& name);

 private:
  struct alignas(64) Header {
    uint64_t magic;
    int64_t num_slabs;
    int64_t slab_bytes;
    int64_t batch;
    std::atomic<uint64_t> fill_seq;
    std::atomic<int64_t> filling;      // slab handing out columns, -1 none
    std::atomic<uint32_t> lock;        // spinlock for Claim
    std::atomic<uint32_t> futex_word;  // bumped on every transition
    std::atomic<uint32_t> closed;
  };
  struct alignas(64) SlabHdr {
    std::atomic<uint32_t> state;
    std::atomic<uint32_t> claimed;     // columns handed out
    std::atomic<uint32_t> done;        // columns committed
    std::atomic<uint64_t> seq;         // fill order
  };

  std::pair<int64_t, int64_t> ClaimLocked();  // lock held, capacity checked
  int64_t CapacityLocked() const;
  void Lock();
  void Unlock();
  void Bump();
  bool WaitChange(uint32_t seen, int64_t timeout_ms);

  std::string name_;
  int64_t num_slabs_ = 0;
  int64_t slab_bytes_ = 0;
  int64_t batch_ = 0;
  size_t map_bytes_ = 0;
  void* base_ = nullptr;
  Header* hdr_ = nullptr;
  SlabHdr* slabs_ = nullptr;
  uint8_t* payload_ = nullptr;
  bool owner_ = false;
};

}  // namespace sa
