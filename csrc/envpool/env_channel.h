// Shared-memory request/response channel between an actor and its env worker
// process.  The reference moves every env call through a
// pickled multiprocessing.Pipe (py_process.py:97-113, worker :151-170); here
// the hot calls (initial / step) are a fixed-layout slot in an anonymous
// MAP_SHARED page inherited by the forked worker:
//
//   caller:  write method + action, bump req_seq, FUTEX_WAKE  -> wait resp_seq
//   worker:  FUTEX_WAIT on req_seq, run the env, write reward / done /
//            instruction bytes, set resp_seq = req_seq, FUTEX_WAKE
//
// The observation frame itself never crosses the channel: the worker writes
// it into a shared frame buffer (py_process.EnvProcess).  Waits release the
// GIL and take a timeout, so the caller can watch for a dead or hung worker
// (supervisor restarts, the env watchdog) between slices.
#pragma once

#include <atomic>
#include <cstdint>
#include <string>
#include <tuple>
#include <vector>

namespace sa {

// One wake-up word shared by the channels of the envs ONE worker process
// hosts (py_process.start_group: k envs per worker).  Every request on an
// attached channel also bumps the word and wakes it, so the worker sleeps
// on one futex for all its envs and serves every pending request per wake
// (one wake per batch of steps instead of one per env).
class EnvDoorbell {
 public:
  EnvDoorbell();  // anonymous shared mapping: create BEFORE forking the worker
  ~EnvDoorbell();
  EnvDoorbell(const EnvDoorbell&) = delete;
  EnvDoorbell& operator=(const EnvDoorbell&) = delete;

  uint32_t value() const;
  // worker side: sleeps until the word differs from `seen` or timeout_ms
  // passes; returns the current value
  uint32_t Wait(uint32_t seen, int64_t timeout_ms);
  std::atomic<uint32_t>* word() { return word_; }

 private:
  std::atomic<uint32_t>* word_ = nullptr;
  size_t bytes_ = 0;
};

class EnvChannel {
 public:
  static constexpr int kMaxAction = 16;
  static constexpr int kMaxInstr = 1024;
  enum Kind : int32_t { kScalarInt = 0, kIntVector = 1, kFloatVector = 2 };

  EnvChannel();  // anonymous shared mapping: create BEFORE forking the worker
  ~EnvChannel();
  EnvChannel(const EnvChannel&) = delete;
  EnvChannel& operator=(const EnvChannel&) = delete;

  // ---- caller side
  // Posts a request (and rings the attached doorbell); returns its sequence
  // number.
  uint32_t Request(int32_t method, int32_t kind, const std::vector<double>& action);
  // Rings `bell` after every request from now on (the bell must outlive the
  // channel; attach before forking the worker).
  void AttachDoorbell(EnvDoorbell* bell) { bell_ = bell ? bell->word() : nullptr; }
  // Waits up to timeout_ms for the response to `seq`: 1 = answered, 0 = not
  // yet (call again; lets the caller check the worker's health in between).
  int WaitResponse(uint32_t seq, int64_t timeout_ms);
  // The response of the last answered request.
  int32_t status() const;
  float reward() const;
  bool done() const;
  // instruction bytes, or has_instr() == false for None
  bool has_instr() const;
  std::string instr() const;

  // ---- worker side
  // Waits up to timeout_ms for a request newer than the last response:
  // -> (seq, method, kind, action values); seq < 0 on timeout.
  std::tuple<int64_t, int32_t, int32_t, std::vector<double>> WaitRequest(int64_t timeout_ms);
  // A replacement worker ignores the request its dead predecessor never
  // answered - without answering it: the caller learns of the restart on the
  // pipe and re-issues.
  void DiscardPending();
  // status 0 = ok, 1 = error (the exception itself travels on the pipe).
  void Respond(uint32_t seq, int32_t status, float reward, bool done, bool has_instr,
               const std::string& instr);

 private:
  struct alignas(64) Slot {
    std::atomic<uint32_t> req_seq;
    std::atomic<uint32_t> resp_seq;
    std::atomic<uint32_t> skip_seq;  // a request no worker will answer
    int32_t method;
    int32_t kind;
    int32_t naction;
    int32_t status;
    double action[kMaxAction];
    float reward;
    int32_t done;
    int32_t instr_len;  // -1: None
    char instr[kMaxInstr];
  };
  Slot* slot_ = nullptr;
  size_t bytes_ = 0;
  std::atomic<uint32_t>* bell_ = nullptr;
};

}  // namespace sa
