// Dynamic request batcher (MI355X-native equivalent of the reference's TF
// custom op, batcher.cc:35-547).  Standalone C++17, no TF/torch dependency.
//
// Contract kept from the reference (so the ported tests can assert on it):
//   * Compute(inputs) blocks the caller until its slice of a batched result
//     arrives; every input must have dim0 == 1.
//   * GetInputs() returns min(queued, max) requests once >= min are queued,
//     or once `timeout_ms` elapsed with >= 1 queued (-1 = no timeout; the
//     wait then polls every 100 ms to notice cancellation).
//   * Every batch gets a fresh computation id; SetOutputs(outputs, id) may be
//     called in any order across ids (out-of-order completion).
//   * Errors: "Batcher requires batch size 1 but was N", "Shapes of inputs
//     much be equal...", "Output shape must have a batch dimension", "Output
//     shape must have the same batch dimension as the input batch size.
//     Expected: X Observed: Y", "Invalid computation id. Id: N" (all
//     InvalidArgument, each cancels and closes the batcher); "Batcher is
//     closed", "GetInputs operation was cancelled", "Compute was cancelled"
//     (Cancelled).
//
// Beyond the reference: GetInputsInto() gathers the request rows straight into
// caller-provided buffers (a pinned-host staging slab), so the batched
// inference input reaches the GPU with ONE hipMemcpyAsync.
#pragma once

#include <chrono>
#include <cstdint>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <vector>

#include "batcher/thread_annotations.h"

namespace sa {

enum class Code { kOk = 0, kCancelled = 1, kInvalidArgument = 2 };

struct Status {
  Code code = Code::kOk;
  std::string msg;
  bool ok() const { return code == Code::kOk; }
  static Status OK() { return Status(); }
  static Status Cancelled(std::string m) { return {Code::kCancelled, std::move(m)}; }
  static Status Invalid(std::string m) { return {Code::kInvalidArgument, std::move(m)}; }
};

struct TensorMeta {
  std::string dtype;      // numpy dtype string, e.g. "<f4"
  size_t itemsize = 1;
  std::vector<int64_t> shape;
  size_t nbytes() const {
    size_t n = itemsize;
    for (auto d : shape) n *= static_cast<size_t>(d);
    return n;
  }
  size_t row_bytes() const {  // bytes of one dim0 slice
    size_t n = itemsize;
    for (size_t i = 1; i < shape.size(); ++i) n *= static_cast<size_t>(shape[i]);
    return n;
  }
};

// Caller-owned memory, valid until the call that received it returns.
struct TensorView {
  TensorMeta meta;
  const void* data = nullptr;
};

struct OwnedTensor {
  TensorMeta meta;
  std::shared_ptr<uint8_t> data;
  static OwnedTensor Alloc(const TensorMeta& m);
};

std::string ShapeString(const std::vector<int64_t>& s);

class Batcher {
 public:
  Batcher(int64_t minimum_batch_size, int64_t maximum_batch_size,
          int64_t timeout_ms);
  ~Batcher();

  Status Compute(const std::vector<TensorView>& inputs,
                 std::vector<OwnedTensor>* outputs) SA_EXCLUDES(mu_);

  Status GetInputs(std::vector<OwnedTensor>* batched, int64_t* computation_id)
      SA_EXCLUDES(mu_);

  // Gathers rows into dst[i] (capacity cap[i] bytes each).  On success fills
  // metas (batched shapes) and the batch size.
  Status GetInputsInto(const std::vector<void*>& dst,
                       const std::vector<size_t>& cap,
                       std::vector<TensorMeta>* metas, int64_t* batch_size,
                       int64_t* computation_id) SA_EXCLUDES(mu_);

  // Packed staging: the n rows of input k land at dst + offsets[k], the
  // segments back to back (each start aligned to `align` bytes), so the
  // whole batched input is ONE contiguous range [0, *used) of the slab and
  // reaches the GPU with a single host->device copy.
  // layout_pow2: segments are laid out for `*layout_rows` = the batch size
  // rounded up to a power of two (capped at the maximum batch size), so a
  // consumer can keep one fixed layout (and one captured graph) per bucket.
  Status GetInputsPacked(void* dst, size_t cap, size_t align, bool layout_pow2,
                         std::vector<TensorMeta>* metas,
                         std::vector<size_t>* offsets, size_t* used,
                         int64_t* layout_rows, int64_t* batch_size,
                         int64_t* computation_id) SA_EXCLUDES(mu_);

  Status SetOutputs(const std::vector<TensorView>& outputs,
                    int64_t computation_id) SA_EXCLUDES(mu_);

  // Graceful close (QueueRunner stop): pending Computes fail with
  // "Compute was cancelled", waiting GetInputs with "Batcher is closed".
  void Close() SA_EXCLUDES(mu_);
  // Session-close semantics: a waiting GetInputs fails with "GetInputs
  // operation was cancelled" and the batcher is cancelled+closed.
  void Cancel() SA_EXCLUDES(mu_);
  bool closed() SA_EXCLUDES(mu_);

  int64_t minimum_batch_size() const { return min_; }
  int64_t maximum_batch_size() const { return max_; }
  int64_t timeout_ms() const { return timeout_ms_; }

  // Stats (for observability): total batches, total requests.
  int64_t num_batches() SA_EXCLUDES(mu_);
  int64_t num_requests() SA_EXCLUDES(mu_);

 private:
  struct Request {
    const std::vector<TensorView>* inputs = nullptr;
    std::vector<OwnedTensor>* outputs = nullptr;
    Status status;
    bool done = false;
    CondVar cv;
  };

  // Waits for a batch and moves it to being_computed_. Returns the requests.
  Status TakeBatch(std::vector<Request*>* reqs, int64_t* id) SA_EXCLUDES(mu_);
  Status ValidateBatch(const std::vector<Request*>& reqs) SA_REQUIRES(mu_);
  void FinishRequest(Request* r, Status s) SA_REQUIRES(mu_);
  void CancelAndCloseLocked() SA_REQUIRES(mu_);
  void EndCopy(int64_t id, Status* st) SA_EXCLUDES(mu_);

  const int64_t min_;
  const int64_t max_;
  const int64_t timeout_ms_;

  Mutex mu_;
  CondVar batch_cv_;  // full batch or cancelled
  std::deque<Request*> inputs_ SA_GUARDED_BY(mu_);
  std::map<int64_t, std::vector<Request*>> being_computed_ SA_GUARDED_BY(mu_);
  std::set<int64_t> copying_ SA_GUARDED_BY(mu_);
  int64_t next_id_ SA_GUARDED_BY(mu_) = 0;
  bool closed_ SA_GUARDED_BY(mu_) = false;
  bool cancelled_ SA_GUARDED_BY(mu_) = false;
  int waiting_get_inputs_ SA_GUARDED_BY(mu_) = 0;
  int64_t n_batches_ SA_GUARDED_BY(mu_) = 0;
  int64_t n_requests_ SA_GUARDED_BY(mu_) = 0;
};

}  // namespace sa
