// Shared-memory slot ring for actor -> learner trajectories and env-worker
// observations (replaces the reference's capacity-1
// tf.FIFOQueue + py_func pipes).
//
// Layout (one POSIX shm object, page aligned):
//   Header { magic, num_slots, slot_bytes, commit_seq, futex word, closed }
//   SlotHdr[num_slots] { state, seq }          (64-B aligned each)
//   payload[num_slots][slot_bytes]             (4 KiB aligned)
//
// Slot states: FREE -> WRITING (producer claimed) -> READY (committed, carries
// a global commit sequence number) -> READING (consumer claimed) -> FREE.
// Transitions are lock-free CAS on the slot state; blocking waits use a
// process-shared futex on the header word (any state change bumps it), so
// producers (actor processes) and the consumer (learner) can live in
// different processes.  Consumers receive slots in commit order (FIFO).
#pragma once

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <string>

namespace sa {

class ShmRing {
 public:
  enum State : uint32_t { kFree = 0, kWriting = 1, kReady = 2, kReading = 3 };

  // create=true: creates (and truncates) the shm object; false: attaches.
  ShmRing(const std::string& name, int64_t num_slots, int64_t slot_bytes,
          bool create);
  ~ShmRing();
  ShmRing(const ShmRing&) = delete;
  ShmRing& operator=(const ShmRing&) = delete;

  // Returns a slot index, or -1 on timeout / -2 if closed. timeout_ms<0: wait forever.
  int64_t AcquireWrite(int64_t timeout_ms);
  void Commit(int64_t slot);
  // Claims the oldest READY slot (FIFO by commit order).
  int64_t AcquireRead(int64_t timeout_ms);
  // Claims up to n READY slots at once (oldest first); returns count.
  int64_t AcquireReadMany(int64_t n, int64_t* out, int64_t timeout_ms);
  void Release(int64_t slot);
  void Close();
  bool closed() const;

  uint8_t* slot_data(int64_t slot) const;
  int64_t num_slots() const { return num_slots_; }
  int64_t slot_bytes() const { return slot_bytes_; }
  int64_t num_ready() const;
  const std::string& name() const { return name_; }
  static void Unlink(const std::string& name);

 private:
  struct alignas(64) Header {
    uint64_t magic;
    int64_t num_slots;
    int64_t slot_bytes;
    std::atomic<uint64_t> commit_seq;
    std::atomic<uint32_t> futex_word;
    std::atomic<uint32_t> closed;
  };
  struct alignas(64) SlotHdr {
    std::atomic<uint32_t> state;
    std::atomic<uint64_t> seq;
  };

  void Bump();
  // Waits until the futex word differs from `seen` or timeout; returns false on timeout.
  bool WaitChange(uint32_t seen, int64_t timeout_ms);
  int64_t ClaimOldestReady();

  std::string name_;
  int64_t num_slots_ = 0;
  int64_t slot_bytes_ = 0;
  size_t map_bytes_ = 0;
  void* base_ = nullptr;
  Header* hdr_ = nullptr;
  SlotHdr* slots_ = nullptr;
  uint8_t* payload_ = nullptr;
  bool owner_ = false;
};

}  // namespace sa
