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
// The row mask normally lives in the board's input region (one H2D carries
// it), and with set_direct_output the graph's epilogue writes the ready rows
// straight into the registered host board, so a launch is ONE copy and one
// graph: the per-slot D2H copies cost ~40-150 us each on the queue
// (profiles/r6_e2e.md).
//
// Depth 2 (add_buffer, a second set of device buffers and graphs): batch k+1
// is enqueued before batch k is answered.  Its input H2D runs on a copy
// stream of its own while batch k's graph runs (the compute stream waits on
// the copy's event), and the host half of the loop (event wait, responses,
// scan, mask) overlaps the GPU instead of sitting between two launches.  A
// slot is in at most one batch at a time: it stays REQUEST until answered,
// so the scan skips the in-flight ones.  The LSTM state is one device array
// updated under the row mask in stream order, so batch k+1 sees batch k's
// update for every row batch k served.
//
// Everything else is enqueued on the inference model's own stream, the stream the
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
        stream_(reinterpret_cast<hipStream_t>(stream)), device_(static_cast<int>(device)) {
    TORCH_CHECK(base_, "null board pointer");
    TORCH_CHECK(S_ > 0 && S_ <= 250 && M_ > 0, "board geometry");
    words_ = reinterpret_cast<uint32_t*>(base_);
    ready_.reserve(S_);
    pend_slots_.reserve(S_);
    inflight_.assign(S_, 0);
    add_buffer(in_dev, out_dev, mask_dev, mask_host, exec_plain, exec_instr);
  }

  // a second buffer set (inputs, outputs, mask, graphs captured over them)
  // turns on depth-2 serving; before start()
  void add_buffer(uintptr_t in_dev, uintptr_t out_dev, uintptr_t mask_dev, uintptr_t mask_host,
                  uintptr_t exec_plain, uintptr_t exec_instr) {
    TORCH_CHECK(!thread_.joinable(), "add_buffer after start");
    TORCH_CHECK(bufs_.size() < 2, "at most two buffer sets");
    Buf b;
    b.in_dev = reinterpret_cast<void*>(in_dev);
    b.out_dev = reinterpret_cast<uint8_t*>(out_dev);
    b.mask_dev = reinterpret_cast<void*>(mask_dev);
    b.mask_host = reinterpret_cast<float*>(mask_host);
    b.plain = reinterpret_cast<hipGraphExec_t>(exec_plain);
    b.instr = reinterpret_cast<hipGraphExec_t>(exec_instr);
    TORCH_CHECK(b.in_dev && b.out_dev && b.mask_dev && b.mask_host, "null board pointer");
    TORCH_CHECK(b.plain || b.instr, "no captured inference graph");
    // a host mask inside the board's input region (its row_mask field)
    // travels with the input H2D; its device copy must then be the same
    // offset of in_dev
    const uint8_t* mh = reinterpret_cast<const uint8_t*>(b.mask_host);
    const uint8_t* in0 = base_ + hdr_;
    if (mh >= in0 && mh < in0 + in_bytes_) {
      TORCH_CHECK(mh + sizeof(float) * S_ * M_ <= in0 + in_bytes_ &&
                      static_cast<uint8_t*>(b.mask_dev) ==
                          static_cast<uint8_t*>(b.in_dev) + (mh - in0),
                  "a mask inside the board's inputs must be the same field of in_dev");
      b.mask_in_board = true;
    }
    bufs_.push_back(b);
  }

  ~NativeBoardServer() {
    stop();
    for (Buf& b : bufs_) {
      if (b.done_ev) (void)hipEventDestroy(b.done_ev);
      if (b.in_ev) (void)hipEventDestroy(b.in_ev);
    }
    if (copy_) (void)hipStreamDestroy(copy_);
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
  // direct output: the graph's epilogue writes the ready rows into the
  // host board itself, so no D2H copy per slot (before start)
  void set_direct_output(bool on) { direct_out_ = on; }
  int64_t gathered() const { return gathered_.load(); }
  int64_t depth() const { return static_cast<int64_t>(bufs_.size()); }
  int64_t batches() const { return batches_.load(); }
  int64_t rows_served() const { return rows_.load(); }
  bool running() const { return thread_.joinable() && !done_.load(); }

  std::string error() const {
    std::lock_guard<std::mutex> g(err_mu_);
    return error_;
  }

  // one pass of the loop on the caller's thread (tests); false = no request
  // (drain: a depth-2 batch is answered before it returns; drain=false
  // leaves it in flight, as the serving thread does)
  bool serve_once(int64_t timeout_ms, bool drain) {
    if (hipSetDevice(device_) != hipSuccess) fail("hipSetDevice failed");
    const bool r = serve(static_cast<int>(timeout_ms));
    if (drain && pending_) finish();
    return r;
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

  // REQUEST slots not already in the batch in flight
  void scan() {
    ready_.clear();
    for (int64_t s = 0; s < S_; ++s)
      if (!inflight_[s] && __atomic_load_n(&words_[16 + s], __ATOMIC_ACQUIRE) == kRequest)
        ready_.push_back(s);
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
      if (pending_) {  // nothing new: answer the batch in flight
        finish();
        return true;
      }
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
    const int k = bufs_.size() > 1 && pending_ ? 1 - pend_buf_ : 0;
    const int64_t rows = launch(k);
    if (pending_) finish();  // batch k-1 finishes while batch k runs
    pending_ = true;
    pend_buf_ = k;
    pend_rows_ = rows;
    pend_slots_.assign(ready_.begin(), ready_.end());
    for (int64_t s : pend_slots_) inflight_[s] = 1;
    if (bufs_.size() == 1) finish();
    return true;
  }

  // enqueue one batch over the ready_ slots into buffer set k; returns rows
  int64_t launch(int k) {
    Buf& b = bufs_[k];
    const int64_t R = S_ * M_;
    std::memset(b.mask_host, 0, sizeof(float) * R);
    int64_t rows = 0;
    for (int64_t s : ready_) {
      int64_t n = __atomic_load_n(&words_[16 + S_ + s], __ATOMIC_ACQUIRE);
      n = n < 0 ? 0 : (n > M_ ? M_ : n);
      for (int64_t r = 0; r < n; ++r) b.mask_host[s * M_ + r] = 1.f;
      rows += n;
    }
    // the with-instruction graph when any row carries an instruction (the
    // Python server's rule: over the whole board)
    bool instr = false;
    if (b.instr) {
      const int64_t* len = reinterpret_cast<const int64_t*>(base_ + hdr_ + instr_off_);
      for (int64_t r = 0; r < R && !instr; ++r) instr = len[r] > 0;
    }
    hipGraphExec_t g = instr ? b.instr : b.plain;
    if (!g) fail(instr ? "no with-instruction graph captured" : "no plain graph captured");
    if (!b.done_ev) check(hipEventCreateWithFlags(&b.done_ev, hipEventDisableTiming), "hipEventCreate");
    if (bufs_.size() > 1) {
      // set k's previous batch is answered (its event waited), so its
      // input buffers are free: copy on the copy stream, under the graph
      // of the batch in flight
      if (!copy_) check(hipStreamCreateWithFlags(&copy_, hipStreamNonBlocking), "hipStreamCreate");
      if (!b.in_ev) check(hipEventCreateWithFlags(&b.in_ev, hipEventDisableTiming), "hipEventCreate");
      check(hipMemcpyAsync(b.in_dev, base_ + hdr_, in_bytes_, hipMemcpyHostToDevice, copy_),
            "board H2D");
      if (!b.mask_in_board)
        check(hipMemcpyAsync(b.mask_dev, b.mask_host, sizeof(float) * R, hipMemcpyHostToDevice,
                             copy_),
              "mask H2D");
      check(hipEventRecord(b.in_ev, copy_), "hipEventRecord");
      check(hipStreamWaitEvent(stream_, b.in_ev, 0), "hipStreamWaitEvent");
    } else {
      check(hipMemcpyAsync(b.in_dev, base_ + hdr_, in_bytes_, hipMemcpyHostToDevice, stream_),
            "board H2D");
      if (!b.mask_in_board)
        check(hipMemcpyAsync(b.mask_dev, b.mask_host, sizeof(float) * R, hipMemcpyHostToDevice,
                             stream_),
              "mask H2D");
    }
    check(hipGraphLaunch(g, stream_), "hipGraphLaunch");
    uint8_t* host_out = base_ + hdr_ + in_bytes_;
    if (!direct_out_)
      for (int64_t s : ready_)
        check(hipMemcpyAsync(host_out + s * so_, b.out_dev + s * so_, so_, hipMemcpyDeviceToHost,
                             stream_),
              "slot D2H");
    // an event of this batch, not a stream synchronise: the learner thread
    // keeps enqueueing weight publishes onto the same stream meanwhile
    // (a stream-wide synchronise held it off: 15.6 ms of learner-loop host
    // time per step at 96 actors)
    check(hipEventRecord(b.done_ev, stream_), "hipEventRecord");
    return rows;
  }

  // wait for the batch in flight and answer its slots
  void finish() {
    check(hipEventSynchronize(bufs_[pend_buf_].done_ev), "hipEventSynchronize");
    for (int64_t s : pend_slots_) {
      inflight_[s] = 0;
      __atomic_store_n(&words_[16 + s], kResponse, __ATOMIC_RELEASE);
      futex(&words_[16 + s], FUTEX_WAKE, INT_MAX, nullptr);
    }
    pending_ = false;
    batches_.fetch_add(1);
    rows_.fetch_add(pend_rows_);
  }

  void run() {
    try {
      if (hipSetDevice(device_) != hipSuccess) fail("hipSetDevice failed");
      while (!stop_.load() && !closed()) serve(50);
      if (pending_) finish();
    } catch (const std::exception&) {
      // error_ is set and the board closed by fail()
    }
    done_.store(true);
  }

  struct Buf {
    void* in_dev = nullptr;
    uint8_t* out_dev = nullptr;
    void* mask_dev = nullptr;
    float* mask_host = nullptr;
    hipGraphExec_t plain = nullptr, instr = nullptr;
    hipEvent_t done_ev = nullptr, in_ev = nullptr;
    bool mask_in_board = false;
  };

  uint8_t* base_;
  uint32_t* words_ = nullptr;
  int64_t hdr_, in_bytes_, so_, S_, M_, instr_off_;
  hipStream_t stream_;
  hipStream_t copy_ = nullptr;  // depth 2: the input H2D
  int device_;
  std::vector<Buf> bufs_;
  std::vector<int64_t> ready_, pend_slots_;
  std::vector<char> inflight_;
  bool pending_ = false;
  bool direct_out_ = false;
  int pend_buf_ = 0;
  int64_t pend_rows_ = 0;
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
           py::arg("drain") = true,
           py::call_guard<py::gil_scoped_release>())
      .def("add_buffer", &NativeBoardServer::add_buffer, py::arg("in_dev"), py::arg("out_dev"),
           py::arg("mask_dev"), py::arg("mask_host"), py::arg("exec_plain"),
           py::arg("exec_instr"))
      .def("depth", &NativeBoardServer::depth)
      .def("set_direct_output", &NativeBoardServer::set_direct_output, py::arg("on"))
      .def("set_batching", &NativeBoardServer::set_batching, py::arg("min_ready"),
           py::arg("gather_us"))
      .def("gathered", &NativeBoardServer::gathered)
      .def("batches", &NativeBoardServer::batches)
      .def("rows_served", &NativeBoardServer::rows_served)
      .def("running", &NativeBoardServer::running)
      .def("error", &NativeBoardServer::error);
}
