// Shared-memory env request/response channel (see env_channel.h).
#include "envpool/env_channel.h"

#include <linux/futex.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <climits>
#include <cstring>
#include <stdexcept>

namespace sa {
namespace {

void FutexWait(std::atomic<uint32_t>* w, uint32_t seen, int64_t timeout_ms) {
  struct timespec ts;
  ts.tv_sec = timeout_ms / 1000;
  ts.tv_nsec = (timeout_ms % 1000) * 1000000L;
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), FUTEX_WAIT, seen, &ts, nullptr, 0);
}

void FutexWake(std::atomic<uint32_t>* w) {
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), FUTEX_WAKE, INT_MAX, nullptr, nullptr, 0);
}

int64_t NowMs() {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return static_cast<int64_t>(ts.tv_sec) * 1000 + ts.tv_nsec / 1000000;
}

}  // namespace

EnvDoorbell::EnvDoorbell() {
  bytes_ = 4096;
  void* p = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
  if (p == MAP_FAILED) throw std::runtime_error("EnvDoorbell: mmap failed");
  std::memset(p, 0, bytes_);
  word_ = reinterpret_cast<std::atomic<uint32_t>*>(p);
}

EnvDoorbell::~EnvDoorbell() {
  if (word_) munmap(word_, bytes_);
}

uint32_t EnvDoorbell::value() const { return word_->load(std::memory_order_acquire); }

uint32_t EnvDoorbell::Wait(uint32_t seen, int64_t timeout_ms) {
  const int64_t deadline = NowMs() + std::max<int64_t>(0, timeout_ms);
  while (true) {
    const uint32_t v = word_->load(std::memory_order_acquire);
    if (v != seen) return v;
    const int64_t left = deadline - NowMs();
    if (left <= 0) return v;
    FutexWait(word_, seen, std::min<int64_t>(left, 50));
  }
}

EnvChannel::EnvChannel() {
  bytes_ = (sizeof(Slot) + 4095) / 4096 * 4096;
  void* p = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
  if (p == MAP_FAILED) throw std::runtime_error("EnvChannel: mmap failed");
  std::memset(p, 0, bytes_);
  slot_ = reinterpret_cast<Slot*>(p);
  slot_->instr_len = -1;
}

EnvChannel::~EnvChannel() {
  if (slot_) munmap(slot_, bytes_);
}

uint32_t EnvChannel::Request(int32_t method, int32_t kind, const std::vector<double>& action) {
  if (action.size() > static_cast<size_t>(kMaxAction))
    throw std::invalid_argument("EnvChannel: action has more than 16 values");
  slot_->method = method;
  slot_->kind = kind;
  slot_->naction = static_cast<int32_t>(action.size());
  std::copy(action.begin(), action.end(), slot_->action);
  // release: the request body happens-before the worker's acquire of req_seq
  const uint32_t seq = slot_->req_seq.load(std::memory_order_relaxed) + 1;
  slot_->req_seq.store(seq, std::memory_order_release);
  FutexWake(&slot_->req_seq);
  if (bell_) {
    // after req_seq: a worker woken by the bell finds the request posted
    bell_->fetch_add(1, std::memory_order_acq_rel);
    FutexWake(bell_);
  }
  return seq;
}

int EnvChannel::WaitResponse(uint32_t seq, int64_t timeout_ms) {
  const int64_t deadline = NowMs() + std::max<int64_t>(0, timeout_ms);
  int spins = 0;
  while (true) {
    const uint32_t r = slot_->resp_seq.load(std::memory_order_acquire);
    if (r == seq) return 1;
    if (++spins < 64) continue;  // env steps are often tens of microseconds
    const int64_t left = deadline - NowMs();
    if (left <= 0) return 0;
    FutexWait(&slot_->resp_seq, r, std::min<int64_t>(left, 50));
  }
}

int32_t EnvChannel::status() const { return slot_->status; }
float EnvChannel::reward() const { return slot_->reward; }
bool EnvChannel::done() const { return slot_->done != 0; }
bool EnvChannel::has_instr() const { return slot_->instr_len >= 0; }
std::string EnvChannel::instr() const {
  return slot_->instr_len > 0 ? std::string(slot_->instr, slot_->instr_len) : std::string();
}

std::tuple<int64_t, int32_t, int32_t, std::vector<double>> EnvChannel::WaitRequest(
    int64_t timeout_ms) {
  const int64_t deadline = NowMs() + std::max<int64_t>(0, timeout_ms);
  while (true) {
    const uint32_t q = slot_->req_seq.load(std::memory_order_acquire);
    if (q != slot_->resp_seq.load(std::memory_order_relaxed) &&
        q != slot_->skip_seq.load(std::memory_order_relaxed)) {
      std::vector<double> a(slot_->action, slot_->action + slot_->naction);
      return std::make_tuple(static_cast<int64_t>(q), slot_->method, slot_->kind, std::move(a));
    }
    const int64_t left = deadline - NowMs();
    if (left <= 0) return std::make_tuple(int64_t{-1}, 0, 0, std::vector<double>());
    FutexWait(&slot_->req_seq, q, std::min<int64_t>(left, 50));
  }
}

void EnvChannel::DiscardPending() {
  slot_->skip_seq.store(slot_->req_seq.load(std::memory_order_acquire),
                        std::memory_order_release);
}

void EnvChannel::Respond(uint32_t seq, int32_t status, float reward, bool done, bool has_instr,
                         const std::string& instr) {
  slot_->status = status;
  slot_->reward = reward;
  slot_->done = done ? 1 : 0;
  if (!has_instr) {
    slot_->instr_len = -1;
  } else {
    const size_t n = std::min(instr.size(), static_cast<size_t>(kMaxInstr));
    std::memcpy(slot_->instr, instr.data(), n);
    slot_->instr_len = static_cast<int32_t>(n);
  }
  slot_->resp_seq.store(seq, std::memory_order_release);
  FutexWake(&slot_->resp_seq);
}

}  // namespace sa
