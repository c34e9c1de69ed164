// Time-major trajectory batch queue (see traj_queue.h).
#include "envpool/traj_queue.h"

#include <fcntl.h>
#include <linux/futex.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstring>
#include <stdexcept>

namespace sa {
namespace {

constexpr uint64_t kMagic = 0x5341545241514a31ull;  // "SATRAQJ1"

size_t AlignUp(size_t x, size_t a) { return (x + a - 1) / a * a; }

long Futex(std::atomic<uint32_t>* addr, int op, uint32_t val, const struct timespec* ts) {
  return syscall(SYS_futex, reinterpret_cast<uint32_t*>(addr), op, val, ts, nullptr, 0);
}

}  // namespace

TrajQueue::TrajQueue(const std::string& name, int64_t num_slabs, int64_t slab_bytes,
                     int64_t batch, bool create)
    : name_(name), owner_(create) {
  // an empty name: an anonymous shared mapping (threads, or processes forked
  // after creation) - not bounded by the /dev/shm mount size
  const bool anon = name.empty();
  if (!anon && name[0] != '/') throw std::invalid_argument("shm name must start with '/'");
  if (anon && !create) throw std::invalid_argument("an anonymous queue cannot be attached");
  int fd = -1;
  size_t hdr_bytes = 0;
  if (create) {
    if (num_slabs <= 0 || slab_bytes <= 0 || batch <= 0)
      throw std::invalid_argument("bad trajectory queue geometry");
    if (!anon) {
      shm_unlink(name.c_str());
      fd = shm_open(name.c_str(), O_CREAT | O_RDWR | O_EXCL, 0600);
      if (fd < 0) throw std::runtime_error("shm_open(create) failed for " + name);
    }
    num_slabs_ = num_slabs;
    slab_bytes_ = static_cast<int64_t>(AlignUp(static_cast<size_t>(slab_bytes), 4096));
    batch_ = batch;
    hdr_bytes = AlignUp(sizeof(Header) + sizeof(SlabHdr) * num_slabs_, 4096);
    map_bytes_ = hdr_bytes + static_cast<size_t>(slab_bytes_) * num_slabs_;
    if (!anon && ftruncate(fd, static_cast<off_t>(map_bytes_)) != 0) {
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
  base_ = anon ? mmap(nullptr, map_bytes_, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS,
                      -1, 0)
              : mmap(nullptr, map_bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  if (fd >= 0) close(fd);
  if (base_ == MAP_FAILED) throw std::runtime_error("mmap failed");
  hdr_ = reinterpret_cast<Header*>(base_);
  if (create) {
    std::memset(base_, 0, hdr_bytes);
    hdr_->num_slabs = num_slabs_;
    hdr_->slab_bytes = slab_bytes_;
    hdr_->batch = batch_;
    hdr_->fill_seq.store(0);
    hdr_->filling.store(-1);
    hdr_->lock.store(0);
    hdr_->futex_word.store(0);
    hdr_->closed.store(0);
    std::atomic_thread_fence(std::memory_order_release);
    hdr_->magic = kMagic;
  } else {
    if (hdr_->magic != kMagic) throw std::runtime_error("not a TrajQueue: " + name);
    num_slabs_ = hdr_->num_slabs;
    slab_bytes_ = hdr_->slab_bytes;
    batch_ = hdr_->batch;
    hdr_bytes = AlignUp(sizeof(Header) + sizeof(SlabHdr) * num_slabs_, 4096);
  }
  slabs_ = reinterpret_cast<SlabHdr*>(reinterpret_cast<uint8_t*>(base_) + sizeof(Header));
  payload_ = reinterpret_cast<uint8_t*>(base_) + hdr_bytes;
}

TrajQueue::~TrajQueue() {
  if (base_ && base_ != MAP_FAILED) munmap(base_, map_bytes_);
  if (owner_ && !name_.empty()) shm_unlink(name_.c_str());
}

void TrajQueue::Unlink(const std::string& name) { shm_unlink(name.c_str()); }

void TrajQueue::Lock() {
  for (int spins = 0;; ++spins) {
    uint32_t exp = 0;
    if (hdr_->lock.compare_exchange_weak(exp, 1, std::memory_order_acquire)) return;
    if (spins > 64) sched_yield();
  }
}

void TrajQueue::Unlock() { hdr_->lock.store(0, std::memory_order_release); }

void TrajQueue::Bump() {
  hdr_->futex_word.fetch_add(1, std::memory_order_acq_rel);
  Futex(&hdr_->futex_word, FUTEX_WAKE, INT32_MAX, nullptr);
}

bool TrajQueue::WaitChange(uint32_t seen, int64_t timeout_ms) {
  if (timeout_ms < 0) {
    Futex(&hdr_->futex_word, FUTEX_WAIT, seen, nullptr);
    return true;
  }
  struct timespec ts;
  ts.tv_sec = timeout_ms / 1000;
  ts.tv_nsec = (timeout_ms % 1000) * 1000000L;
  const long r = Futex(&hdr_->futex_word, FUTEX_WAIT, seen, &ts);
  return !(r == -1 && errno == ETIMEDOUT);
}

std::pair<int64_t, int64_t> TrajQueue::Claim(int64_t timeout_ms) {
  auto r = ClaimN(1, timeout_ms);
  if (r.first < 0) return {r.first, r.first};
  return r.second[0];
}

int64_t TrajQueue::CapacityLocked() const {
  int64_t cap = 0;
  const int64_t f = hdr_->filling.load(std::memory_order_relaxed);
  if (f >= 0) cap += batch_ - static_cast<int64_t>(slabs_[f].claimed.load(std::memory_order_relaxed));
  for (int64_t i = 0; i < num_slabs_; ++i)
    if (slabs_[i].state.load(std::memory_order_acquire) == kFree) cap += batch_;
  return cap;
}

std::pair<int64_t, int64_t> TrajQueue::ClaimLocked() {
  const uint32_t B = static_cast<uint32_t>(batch_);
  const int64_t s = hdr_->filling.load(std::memory_order_relaxed);
  if (s >= 0) {
    const uint32_t col = slabs_[s].claimed.fetch_add(1, std::memory_order_relaxed);
    if (col + 1 >= B) hdr_->filling.store(-1, std::memory_order_relaxed);
    return {s, static_cast<int64_t>(col)};
  }
  for (int64_t i = 0; i < num_slabs_; ++i) {
    if (slabs_[i].state.load(std::memory_order_acquire) == kFree) {
      slabs_[i].claimed.store(1, std::memory_order_relaxed);
      slabs_[i].done.store(0, std::memory_order_relaxed);
      slabs_[i].seq.store(hdr_->fill_seq.fetch_add(1), std::memory_order_relaxed);
      slabs_[i].state.store(kFilling, std::memory_order_release);
      hdr_->filling.store(B > 1 ? i : -1, std::memory_order_relaxed);
      return {i, 0};
    }
  }
  return {-1, -1};  // unreachable when the capacity was checked
}

std::pair<int64_t, std::vector<std::pair<int64_t, int64_t>>> TrajQueue::ClaimN(
    int64_t n, int64_t timeout_ms) {
  using clock = std::chrono::steady_clock;
  if (n <= 0 || n > batch_ * num_slabs_) throw std::invalid_argument("ClaimN: bad column count");
  const auto deadline = clock::now() + std::chrono::milliseconds(timeout_ms < 0 ? 0 : timeout_ms);
  std::vector<std::pair<int64_t, int64_t>> out;
  while (true) {
    if (hdr_->closed.load()) return {-2, {}};
    const uint32_t seen = hdr_->futex_word.load(std::memory_order_acquire);
    Lock();
    if (CapacityLocked() >= n) {
      out.reserve(static_cast<size_t>(n));
      for (int64_t k = 0; k < n; ++k) out.push_back(ClaimLocked());
      Unlock();
      return {0, std::move(out)};
    }
    Unlock();
    int64_t left = -1;
    if (timeout_ms >= 0) {
      left = std::chrono::duration_cast<std::chrono::milliseconds>(deadline - clock::now()).count();
      if (left <= 0) return {-1, {}};
    }
    WaitChange(seen, left < 0 ? 100 : std::min<int64_t>(left, 100));
  }
}

void TrajQueue::Commit(int64_t slab) {
  if (slab < 0 || slab >= num_slabs_) throw std::out_of_range("slab index");
  // release: the producer's payload writes happen-before the consumer's
  // acquire of the READY state
  const uint32_t done = slabs_[slab].done.fetch_add(1, std::memory_order_acq_rel) + 1;
  if (done >= static_cast<uint32_t>(batch_)) {
    slabs_[slab].state.store(kReady, std::memory_order_release);
    Bump();
  }
}

int64_t TrajQueue::Acquire(int64_t timeout_ms) {
  using clock = std::chrono::steady_clock;
  const auto deadline = clock::now() + std::chrono::milliseconds(timeout_ms < 0 ? 0 : timeout_ms);
  while (true) {
    if (hdr_->closed.load()) return -2;
    const uint32_t seen = hdr_->futex_word.load(std::memory_order_acquire);
    int64_t best = -1;
    uint64_t best_seq = UINT64_MAX;
    for (int64_t i = 0; i < num_slabs_; ++i) {
      if (slabs_[i].state.load(std::memory_order_acquire) == kReady) {
        const uint64_t q = slabs_[i].seq.load(std::memory_order_relaxed);
        if (q < best_seq) {
          best_seq = q;
          best = i;
        }
      }
    }
    if (best >= 0) {
      uint32_t exp = kReady;
      if (slabs_[best].state.compare_exchange_strong(exp, kReading)) return best;
      continue;
    }
    int64_t left = -1;
    if (timeout_ms >= 0) {
      left = std::chrono::duration_cast<std::chrono::milliseconds>(deadline - clock::now()).count();
      if (left <= 0) return -1;
    }
    WaitChange(seen, left < 0 ? 100 : std::min<int64_t>(left, 100));
  }
}

void TrajQueue::Release(int64_t slab) {
  if (slab < 0 || slab >= num_slabs_) throw std::out_of_range("slab index");
  slabs_[slab].state.store(kFree, std::memory_order_release);
  Bump();
}

void TrajQueue::Close() {
  hdr_->closed.store(1);
  Bump();
}

bool TrajQueue::closed() const { return hdr_->closed.load() != 0; }

uint8_t* TrajQueue::slab_data(int64_t slab) const {
  if (slab < 0 || slab >= num_slabs_) throw std::out_of_range("slab index");
  return payload_ + static_cast<size_t>(slab) * slab_bytes_;
}

int64_t TrajQueue::num_ready() const {
  int64_t n = 0;
  for (int64_t i = 0; i < num_slabs_; ++i)
    n += slabs_[i].state.load(std::memory_order_relaxed) == kReady;
  return n;
}

}  // namespace sa
