// Shared-memory slot ring implementation (see shm_ring.h).
#include "envpool/shm_ring.h"

#include <fcntl.h>
#include <linux/futex.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstring>
#include <stdexcept>

namespace sa {
namespace {

constexpr uint64_t kMagic = 0x53414d4952494e47ull;  // "SAMIRING"

size_t AlignUp(size_t x, size_t a) { return (x + a - 1) / a * a; }

long Futex(std::atomic<uint32_t>* addr, int op, uint32_t val,
           const struct timespec* ts) {
  return syscall(SYS_futex, reinterpret_cast<uint32_t*>(addr), op, val, ts,
                 nullptr, 0);
}

}  // namespace

ShmRing::ShmRing(const std::string& name, int64_t num_slots, int64_t slot_bytes,
                 bool create)
    : name_(name), owner_(create) {
  if (name.empty() || name[0] != '/') throw std::invalid_argument("shm name must start with '/'");
  int fd = -1;
  if (create) {
    if (num_slots <= 0 || slot_bytes <= 0) throw std::invalid_argument("bad ring geometry");
    shm_unlink(name.c_str());
    fd = shm_open(name.c_str(), O_CREAT | O_RDWR | O_EXCL, 0600);
    if (fd < 0) throw std::runtime_error("shm_open(create) failed for " + name);
    num_slots_ = num_slots;
    slot_bytes_ = static_cast<int64_t>(AlignUp(slot_bytes, 4096));
    const size_t hdr = AlignUp(sizeof(Header) + sizeof(SlotHdr) * num_slots_, 4096);
    map_bytes_ = hdr + static_cast<size_t>(slot_bytes_) * num_slots_;
    if (ftruncate(fd, static_cast<off_t>(map_bytes_)) != 0) {
      close(fd);
      throw std::runtime_error("ftruncate failed");
    }
  } else {
    fd = shm_open(name.c_str(), O_RDWR, 0600);
    if (fd < 0) throw std::runtime_error("shm_open(attach) failed for " + name);
    struct stat st;
    fstat(fd, &st);
    map_bytes_ = static_cast<size_t>(st.st_size);
  }
  base_ = mmap(nullptr, map_bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (base_ == MAP_FAILED) throw std::runtime_error("mmap failed");
  hdr_ = reinterpret_cast<Header*>(base_);
  if (create) {
    std::memset(base_, 0, AlignUp(sizeof(Header) + sizeof(SlotHdr) * num_slots_, 4096));
    hdr_->num_slots = num_slots_;
    hdr_->slot_bytes = slot_bytes_;
    hdr_->commit_seq.store(0);
    hdr_->futex_word.store(0);
    hdr_->closed.store(0);
    std::atomic_thread_fence(std::memory_order_release);
    hdr_->magic = kMagic;
  } else {
    if (hdr_->magic != kMagic) throw std::runtime_error("not a ShmRing: " + name);
    num_slots_ = hdr_->num_slots;
    slot_bytes_ = hdr_->slot_bytes;
  }
  slots_ = reinterpret_cast<SlotHdr*>(reinterpret_cast<uint8_t*>(base_) + sizeof(Header));
  payload_ = reinterpret_cast<uint8_t*>(base_) +
             AlignUp(sizeof(Header) + sizeof(SlotHdr) * num_slots_, 4096);
}

ShmRing::~ShmRing() {
  if (base_ && base_ != MAP_FAILED) munmap(base_, map_bytes_);
  if (owner_) shm_unlink(name_.c_str());
}

void ShmRing::Unlink(const std::string& name) { shm_unlink(name.c_str()); }

void ShmRing::Bump() {
  hdr_->futex_word.fetch_add(1, std::memory_order_acq_rel);
  Futex(&hdr_->futex_word, FUTEX_WAKE, INT32_MAX, nullptr);
}

bool ShmRing::WaitChange(uint32_t seen, int64_t timeout_ms) {
  if (timeout_ms < 0) {
    Futex(&hdr_->futex_word, FUTEX_WAIT, seen, nullptr);
    return true;
  }
  struct timespec ts;
  ts.tv_sec = timeout_ms / 1000;
  ts.tv_nsec = (timeout_ms % 1000) * 1000000L;
  long r = Futex(&hdr_->futex_word, FUTEX_WAIT, seen, &ts);
  return !(r == -1 && errno == ETIMEDOUT);
}

int64_t ShmRing::AcquireWrite(int64_t timeout_ms) {
  using clock = std::chrono::steady_clock;
  const auto deadline = clock::now() + std::chrono::milliseconds(timeout_ms < 0 ? 0 : timeout_ms);
  while (true) {
    if (hdr_->closed.load()) return -2;
    const uint32_t seen = hdr_->futex_word.load(std::memory_order_acquire);
    for (int64_t i = 0; i < num_slots_; ++i) {
      uint32_t exp = kFree;
      if (slots_[i].state.compare_exchange_strong(exp, kWriting)) return i;
    }
    int64_t left = -1;
    if (timeout_ms >= 0) {
      left = std::chrono::duration_cast<std::chrono::milliseconds>(deadline - clock::now()).count();
      if (left <= 0) return -1;
    }
    WaitChange(seen, left < 0 ? -1 : std::min<int64_t>(left, 100));
  }
}

void ShmRing::Commit(int64_t slot) {
  const uint64_t seq = hdr_->commit_seq.fetch_add(1, std::memory_order_acq_rel);
  slots_[slot].seq.store(seq, std::memory_order_relaxed);
  slots_[slot].state.store(kReady, std::memory_order_release);
  Bump();
}

int64_t ShmRing::ClaimOldestReady() {
  while (true) {
    int64_t best = -1;
    uint64_t best_seq = UINT64_MAX;
    for (int64_t i = 0; i < num_slots_; ++i) {
      if (slots_[i].state.load(std::memory_order_acquire) == kReady) {
        const uint64_t s = slots_[i].seq.load(std::memory_order_relaxed);
        if (s < best_seq) {
          best_seq = s;
          best = i;
        }
      }
    }
    if (best < 0) return -1;
    uint32_t exp = kReady;
    if (slots_[best].state.compare_exchange_strong(exp, kReading)) return best;
  }
}

int64_t ShmRing::AcquireRead(int64_t timeout_ms) {
  int64_t out = -1;
  int64_t n = AcquireReadMany(1, &out, timeout_ms);
  if (n == 1) return out;
  return n;  // -1 timeout, -2 closed
}

int64_t ShmRing::AcquireReadMany(int64_t n, int64_t* out, int64_t timeout_ms) {
  using clock = std::chrono::steady_clock;
  const auto deadline = clock::now() + std::chrono::milliseconds(timeout_ms < 0 ? 0 : timeout_ms);
  int64_t got = 0;
  while (got < n) {
    const uint32_t seen = hdr_->futex_word.load(std::memory_order_acquire);
    int64_t s;
    while (got < n && (s = ClaimOldestReady()) >= 0) out[got++] = s;
    if (got == n) break;
    if (hdr_->closed.load()) {
      for (int64_t i = 0; i < got; ++i) Release(out[i]);
      return -2;
    }
    int64_t left = -1;
    if (timeout_ms >= 0) {
      left = std::chrono::duration_cast<std::chrono::milliseconds>(deadline - clock::now()).count();
      if (left <= 0) {
        // give back partial claims in commit order is not needed: re-mark READY
        for (int64_t i = 0; i < got; ++i) {
          slots_[out[i]].state.store(kReady, std::memory_order_release);
        }
        Bump();
        return -1;
      }
    }
    WaitChange(seen, left < 0 ? 100 : std::min<int64_t>(left, 100));
  }
  return got;
}

void ShmRing::Release(int64_t slot) {
  slots_[slot].state.store(kFree, std::memory_order_release);
  Bump();
}

void ShmRing::Close() {
  hdr_->closed.store(1);
  Bump();
}

bool ShmRing::closed() const { return hdr_->closed.load() != 0; }

uint8_t* ShmRing::slot_data(int64_t slot) const {
  return payload_ + static_cast<size_t>(slot) * static_cast<size_t>(slot_bytes_);
}

int64_t ShmRing::num_ready() const {
  int64_t n = 0;
  for (int64_t i = 0; i < num_slots_; ++i)
    if (slots_[i].state.load() == kReady) ++n;
  return n;
}

}  // namespace sa
