// Native serving thread of the inference board (runtime/inference_board.py).
//
// The board is the shared-memory request/response table that CPU-only
// actor-group processes post their rows to; the learner process serves it
// with ONE captured inference graph over every row.  The Python server loop
// shared the learner's interpreter (GIL) with the training loop, so each
// batch waited behind learner-side Python work.  This
// thread runs the same loop with no Python in it:
//
//   futex-wait on the board's sequence word -> collect REQUEST slots (for
//   up to a short batching window while fewer than min_ready are ready) ->
//   row mask into pinned memory -> H2D of the whole input region + mask ->
//   hipGraphLaunch of the captured graph (plain or with-instruction variant,
//   picked from the instruction lengths) -> D2H of each ready slot's output
//   block -> wait on this batch's event -> RESPONSE + futex wake per slot.
//
// Everything is enqueued on the inference model's own stream, the stream the
// learner's weight publish (inference.py InferenceModel.publish) also copies
// on, so stream order keeps a replay from reading a half-copied snapshot.
// The graphs are captured by Python before start() (no capture may run on
// that stream while the thread serves).  Reference counterpart: the
// dynamic-batching inference of experiment.py:534-546 + batcher.cc.
#include <torch/extension.h>
#include <hip/hip_runtime.h>

#include <linux/futex.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <atomic>
#include <climits>
#include <cstring>
#include <ctime>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace {

constexpr uint32_t kRequest = 1, kResponse = 2;

long futex(uint32_t* addr, int op, uint32_t val, const timespec* ts) {
  return syscall(SYS_futex, addr, op, val, ts, nullptr, 0);
}

class NativeBoardServer {
 public:
  // Board layout (inference_board.py InferenceBoard): header words
  // [0] seq, [1] closed, [16 + s] slot state, [16 + S + s] rows of slot s;
  // inputs at base + hdr (in_bytes, field-major over all S * M rows);
  // outputs at base + hdr + in_bytes (slot-major, slot_out_bytes each).
  NativeBoardServer(uintptr_t base, int64_t hdr, int64_t in_bytes, int64_t slot_out_bytes,
                    int64_t num_slots, int64_t rows_per_slot, int64_t instr_len_off,
                    uintptr_t in_dev, uintptr_t out_dev, uintptr_t mask_dev, uintptr_t mask_host,
                    uintptr_t stream, uintptr_t exec_plain, uintptr_t exec_instr, int64_t device)
      : base_(reinterpret_cast<uint8_t*>(base)), hdr_(hdr), in_bytes_(in_bytes),
        so_(slot_out_bytes), S_(num_slots), M_(rows_per_slot), instr_off_(instr_len_off),
        in_dev_(reinterpret_cast<void*>(in_dev)), out_dev_(reinterpret_cast<uint8_t*>(out_dev)),
        mask_dev_(reinterpret_cast<void*>(mask_dev)),
        mask_host_(reinterpret_cast<float*>(mask_host)),
        stream_(reinterpret_cast<hipStream_t>(stream)),
        exec_plain_(reinterpret_cast<hipGraphExec_t>(exec_plain)),
        exec_instr_(reinterpret_cast<hipGraphExec_t>(exec_instr)), device_(static_cast<int>(device)) {
    TORCH_CHECK(base_ && in_dev_ && out_dev_ && mask_dev_ && mask_host_, "null board pointer");
    TORCH_CHECK(S_ > 0 && S_ <= 250 && M_ > 0, "board geometry");
    TORCH_CHECK(exec_plain_ || exec_instr_, "no captured inference graph");
    words_ = reinterpret_cast<uint32_t*>(base_);
    ready_.reserve(S_);
  }

  ~NativeBoardServer() {
    stop();
    if (done_ev_) (void)hipEventDestroy(done_ev_);
  }

  void start() {
    TORCH_CHECK(!thread_.joinable(), "server already started");
    stop_.store(false);
    thread_ = std::thread([this] { run(); });
  }

  void stop() {
    stop_.store(true);
    futex(&words_[0], FUTEX_WAKE, INT_MAX, nullptr);
    if (thread_.joinable()) thread_.join();
  }

  // batching window (see serve): launch once >= min_ready slots are ready
  // or gather_us microseconds after the first one; gather_us 0 = off
  void set_batching(int64_t min_ready, int64_t gather_us) {
    min_ready_ = min_ready < 1 ? 1 : (min_ready > S_ ? S_ : min_ready);
    gather_us_ = gather_us < 0 ? 0 : (gather_us > 100000 ? 100000 : gather_us);
  }
  int64_t gathered() const { return gathered_.load(); }
  int64_t batches() const { return batches_.load(); }
  int64_t rows_served() const { return rows_.load(); }
  bool running() const { return thread_.joinable() && !done_.load(); }

  std::string error() const {
    std::lock_guard<std::mutex> g(err_mu_);
    return error_;
  }

  // one pass of the loop on the caller's thread (tests); false = no request
  bool serve_once(int64_t timeout_ms) {
    if (hipSetDevice(device_) != hipSuccess) fail("hipSetDevice failed");
    return serve(static_cast<int>(timeout_ms));
  }

 private:
  void fail(const std::string& what) {
    {
      std::lock_guard<std::mutex> g(err_mu_);
      if (error_.empty()) error_ = what;
    }
    // close the board: every waiting worker sees it and raises EOFError
    __atomic_store_n(&words_[1], 1u, __ATOMIC_RELEASE);
    futex(&words_[0], FUTEX_WAKE, INT_MAX, nullptr);
    for (int64_t s = 0; s < S_; ++s) futex(&words_[16 + s], FUTEX_WAKE, INT_MAX, nullptr);
    throw std::runtime_error(what);
  }

  void check(hipError_t e, const char* what) {
    if (e != hipSuccess) fail(std::string(what) + ": " + hipGetErrorString(e));
  }

  bool closed() const { return __atomic_load_n(&words_[1], __ATOMIC_ACQUIRE) != 0; }

  void scan() {
    ready_.clear();
    for (int64_t s = 0; s < S_; ++s)
      if (__atomic_load_n(&words_[16 + s], __ATOMIC_ACQUIRE) == kRequest) ready_.push_back(s);
  }

  static int64_t now_us() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return static_cast<int64_t>(t.tv_sec) * 1000000 + t.tv_nsec / 1000;
  }

  bool serve(int timeout_ms) {
    uint32_t seq = __atomic_load_n(&words_[0], __ATOMIC_ACQUIRE);
    scan();
    if (ready_.empty()) {
      timespec ts{timeout_ms / 1000, (timeout_ms % 1000) * 1000000L};
      futex(&words_[0], FUTEX_WAIT, seq, &ts);
      return false;
    }
    // Batching window: every launch runs the graph over the WHOLE board and
    // copies its whole input region, so a launch that serves few slots
    // wastes most of that.  With fewer than min_ready_ slots ready, wait up
    // to gather_us_ for more posts (the board's sequence word) first.
    if (gather_us_ > 0 && static_cast<int64_t>(ready_.size()) < min_ready_) {
      const int64_t deadline = now_us() + gather_us_;
      while (static_cast<int64_t>(ready_.size()) < min_ready_ && !closed()) {
        const int64_t left = deadline - now_us();
        if (left <= 0) break;
        timespec ts{0, left * 1000L};
        futex(&words_[0], FUTEX_WAIT, seq, &ts);
        seq = __atomic_load_n(&words_[0], __ATOMIC_ACQUIRE);
        scan();
      }
      gathered_.fetch_add(1);
    }
    const int64_t R = S_ * M_;
    std::memset(mask_host_, 0, sizeof(float) * R);
    int64_t rows = 0;
    for (int64_t s : ready_) {
      int64_t n = __atomic_load_n(&words_[16 + S_ + s], __ATOMIC_ACQUIRE);
      n = n < 0 ? 0 : (n > M_ ? M_ : n);
      for (int64_t r = 0; r < n; ++r) mask_host_[s * M_ + r] = 1.f;
      rows += n;
    }
    // the with-instruction graph when any row carries an instruction (the
    // Python server's rule: over the whole board)
    bool instr = false;
    if (exec_instr_) {
      const int64_t* len = reinterpret_cast<const int64_t*>(base_ + hdr_ + instr_off_);
      for (int64_t r = 0; r < R && !instr; ++r) instr = len[r] > 0;
    }
    hipGraphExec_t g = instr ? exec_instr_ : exec_plain_;
    if (!g) fail(instr ? "no with-instruction graph captured" : "no plain graph captured");
    check(hipMemcpyAsync(in_dev_, base_ + hdr_, in_bytes_, hipMemcpyHostToDevice, stream_),
          "board H2D");
    check(hipMemcpyAsync(mask_dev_, mask_host_, sizeof(float) * R, hipMemcpyHostToDevice, stream_),
          "mask H2D");
    check(hipGraphLaunch(g, stream_), "hipGraphLaunch");
    uint8_t* host_out = base_ + hdr_ + in_bytes_;
    for (int64_t s : ready_)
      check(hipMemcpyAsync(host_out + s * so_, out_dev_ + s * so_, so_, hipMemcpyDeviceToHost,
                           stream_),
            "slot D2H");
    // wait on an event of this batch, not on the stream: the learner thread
    // keeps enqueueing weight publishes onto the same stream meanwhile
    // (a stream-wide synchronise held it off: 15.6 ms of learner-loop host
    // time per step at 96 actors)
    if (!done_ev_) check(hipEventCreateWithFlags(&done_ev_, hipEventDisableTiming), "hipEventCreate");
    check(hipEventRecord(done_ev_, stream_), "hipEventRecord");
    check(hipEventSynchronize(done_ev_), "hipEventSynchronize");
    for (int64_t s : ready_) {
      __atomic_store_n(&words_[16 + s], kResponse, __ATOMIC_RELEASE);
      futex(&words_[16 + s], FUTEX_WAKE, INT_MAX, nullptr);
    }
    batches_.fetch_add(1);
    rows_.fetch_add(rows);
    return true;
  }

  void run() {
    try {
      if (hipSetDevice(device_) != hipSuccess) fail("hipSetDevice failed");
      while (!stop_.load() && !closed()) serve(50);
    } catch (const std::exception&) {
      // error_ is set and the board closed by fail()
    }
    done_.store(true);
  }

  uint8_t* base_;
  uint32_t* words_ = nullptr;
  int64_t hdr_, in_bytes_, so_, S_, M_, instr_off_;
  void* in_dev_;
  uint8_t* out_dev_;
  void* mask_dev_;
  float* mask_host_;
  hipStream_t stream_;
  hipGraphExec_t exec_plain_, exec_instr_;
  hipEvent_t done_ev_ = nullptr;
  int device_;
  std::vector<int64_t> ready_;
  std::thread thread_;
  std::atomic<bool> stop_{false}, done_{false};
  std::atomic<int64_t> batches_{0}, rows_{0}, gathered_{0};
  int64_t min_ready_ = 1, gather_us_ = 0;  // set_batching (before start)
  mutable std::mutex err_mu_;
  std::string error_;
};

}  // namespace

void register_board_server(pybind11::module& m) {
  namespace py = pybind11;
  py::class_<NativeBoardServer>(m, "NativeBoardServer")
      .def(py::init<uintptr_t, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, uintptr_t,
                    uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t, int64_t>(),
           py::arg("base"), py::arg("hdr"), py::arg("in_bytes"), py::arg("slot_out_bytes"),
           py::arg("num_slots"), py::arg("rows_per_slot"), py::arg("instr_len_off"),
           py::arg("in_dev"), py::arg("out_dev"), py::arg("mask_dev"), py::arg("mask_host"),
           py::arg("stream"), py::arg("exec_plain"), py::arg("exec_instr"), py::arg("device"))
      .def("start", &NativeBoardServer::start)
      .def("stop", &NativeBoardServer::stop, py::call_guard<py::gil_scoped_release>())
      .def("serve_once", &NativeBoardServer::serve_once, py::arg("timeout_ms") = 50,
           py::call_guard<py::gil_scoped_release>())
      .def("set_batching", &NativeBoardServer::set_batching, py::arg("min_ready"),
           py::arg("gather_us"))
      .def("gathered", &NativeBoardServer::gathered)
      .def("batches", &NativeBoardServer::batches)
      .def("rows_served", &NativeBoardServer::rows_served)
      .def("running", &NativeBoardServer::running)
      .def("error", &NativeBoardServer::error);
}
