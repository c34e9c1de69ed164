// Clang thread-safety annotations + an annotated mutex (static lock checking
// under -Wthread-safety).  Expands to nothing on other
// compilers.
#pragma once

#include <condition_variable>
#include <mutex>

#if defined(__clang__)
#define SA_TSA(x) __attribute__((x))
#else
#define SA_TSA(x)
#endif

#define SA_CAPABILITY(x) SA_TSA(capability(x))
#define SA_SCOPED_CAPABILITY SA_TSA(scoped_lockable)
#define SA_GUARDED_BY(x) SA_TSA(guarded_by(x))
#define SA_PT_GUARDED_BY(x) SA_TSA(pt_guarded_by(x))
#define SA_REQUIRES(...) SA_TSA(requires_capability(__VA_ARGS__))
#define SA_EXCLUDES(...) SA_TSA(locks_excluded(__VA_ARGS__))
#define SA_ACQUIRE(...) SA_TSA(acquire_capability(__VA_ARGS__))
#define SA_RELEASE(...) SA_TSA(release_capability(__VA_ARGS__))
#define SA_NO_TSA SA_TSA(no_thread_safety_analysis)

namespace sa {

class SA_CAPABILITY("mutex") Mutex {
 public:
  void lock() SA_ACQUIRE() { mu_.lock(); }
  void unlock() SA_RELEASE() { mu_.unlock(); }
  std::mutex& native() { return mu_; }

 private:
  std::mutex mu_;
};

class SA_SCOPED_CAPABILITY MutexLock {
 public:
  explicit MutexLock(Mutex* mu) SA_ACQUIRE(mu) : mu_(mu) { mu_->lock(); }
  ~MutexLock() SA_RELEASE() { mu_->unlock(); }
  MutexLock(const MutexLock&) = delete;
  MutexLock& operator=(const MutexLock&) = delete;

 private:
  Mutex* mu_;
};

// Condition variable working on sa::Mutex (caller must hold the mutex).
class CondVar {
 public:
  void Wait(Mutex* mu) SA_REQUIRES(mu) SA_NO_TSA {
    std::unique_lock<std::mutex> l(mu->native(), std::adopt_lock);
    cv_.wait(l);
    l.release();
  }
  // Returns false on timeout.
  template <class Duration>
  bool WaitFor(Mutex* mu, Duration d) SA_REQUIRES(mu) SA_NO_TSA {
    std::unique_lock<std::mutex> l(mu->native(), std::adopt_lock);
    auto st = cv_.wait_for(l, d);
    l.release();
    return st == std::cv_status::no_timeout;
  }
  void NotifyOne() { cv_.notify_one(); }
  void NotifyAll() { cv_.notify_all(); }

 private:
  std::condition_variable cv_;
};

}  // namespace sa
