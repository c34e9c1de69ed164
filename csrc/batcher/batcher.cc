// Dynamic request batcher implementation (see batcher.h for the contract).
#include "batcher/batcher.h"

#include <algorithm>
#include <cstring>
#include <sstream>

namespace sa {

OwnedTensor OwnedTensor::Alloc(const TensorMeta& m) {
  OwnedTensor t;
  t.meta = m;
  const size_t n = std::max<size_t>(m.nbytes(), 1);
  t.data = std::shared_ptr<uint8_t>(new uint8_t[n],
                                    std::default_delete<uint8_t[]>());
  return t;
}

std::string ShapeString(const std::vector<int64_t>& s) {
  std::ostringstream o;
  o << "[";
  for (size_t i = 0; i < s.size(); ++i) o << (i ? "," : "") << s[i];
  o << "]";
  return o.str();
}

Batcher::Batcher(int64_t minimum_batch_size, int64_t maximum_batch_size,
                 int64_t timeout_ms)
    : min_(std::max<int64_t>(1, minimum_batch_size)),
      max_(std::max<int64_t>(1, maximum_batch_size)),
      timeout_ms_(timeout_ms) {}

Batcher::~Batcher() { Close(); }

void Batcher::FinishRequest(Request* r, Status s) {
  r->status = std::move(s);
  r->done = true;
  // Notify while holding mu_: the waiter cannot destroy `r` before we unlock.
  r->cv.NotifyOne();
}

void Batcher::CancelAndCloseLocked() {
  closed_ = true;
  for (Request* r : inputs_) FinishRequest(r, Status::Cancelled("Compute was cancelled"));
  inputs_.clear();
  for (auto it = being_computed_.begin(); it != being_computed_.end();) {
    if (copying_.count(it->first)) {  // finished by EndCopy()
      ++it;
      continue;
    }
    for (Request* r : it->second)
      FinishRequest(r, Status::Cancelled("Compute was cancelled"));
    it = being_computed_.erase(it);
  }
  batch_cv_.NotifyAll();
}

void Batcher::Close() {
  MutexLock l(&mu_);
  CancelAndCloseLocked();
}

void Batcher::Cancel() {
  MutexLock l(&mu_);
  cancelled_ = true;
  CancelAndCloseLocked();
}

bool Batcher::closed() {
  MutexLock l(&mu_);
  return closed_;
}

int64_t Batcher::num_batches() {
  MutexLock l(&mu_);
  return n_batches_;
}

int64_t Batcher::num_requests() {
  MutexLock l(&mu_);
  return n_requests_;
}

Status Batcher::Compute(const std::vector<TensorView>& inputs,
                        std::vector<OwnedTensor>* outputs) {
  Request req;
  req.inputs = &inputs;
  req.outputs = outputs;
  MutexLock l(&mu_);
  if (closed_) return Status::Cancelled("Batcher is closed");
  inputs_.push_back(&req);
  if (static_cast<int64_t>(inputs_.size()) >= min_) batch_cv_.NotifyOne();
  while (!req.done) req.cv.Wait(&mu_);
  return req.status;
}

Status Batcher::ValidateBatch(const std::vector<Request*>& reqs) {
  const auto& first = *reqs[0]->inputs;
  for (Request* r : reqs) {
    const auto& in = *r->inputs;
    if (in.size() != first.size())
      return Status::Invalid("Number of inputs must be equal. Observed: " +
                             std::to_string(first.size()) + ", " +
                             std::to_string(in.size()));
    for (size_t k = 0; k < in.size(); ++k) {
      const auto& m = in[k].meta;
      if (m.shape.empty() || m.shape[0] != 1) {
        return Status::Invalid(
            "Batcher requires batch size 1 but was " +
            (m.shape.empty() ? std::string("a scalar")
                             : std::to_string(m.shape[0])));
      }
      const auto& m0 = first[k].meta;
      if (m.shape != m0.shape)
        return Status::Invalid("Shapes of inputs much be equal. Shapes observed: " +
                               ShapeString(m0.shape) + ", " + ShapeString(m.shape));
      if (m.dtype != m0.dtype)
        return Status::Invalid("Dtypes of inputs must be equal. Observed: " +
                               m0.dtype + ", " + m.dtype);
    }
  }
  return Status::OK();
}

Status Batcher::TakeBatch(std::vector<Request*>* reqs, int64_t* id) {
  using clock = std::chrono::steady_clock;
  const auto poll = std::chrono::milliseconds(100);
  MutexLock l(&mu_);
  const auto start = clock::now();
  Status st;
  ++waiting_get_inputs_;
  while (true) {
    if (cancelled_) {
      st = Status::Cancelled("GetInputs operation was cancelled");
      break;
    }
    if (closed_) {
      st = Status::Cancelled("Batcher is closed");
      break;
    }
    const int64_t n = static_cast<int64_t>(inputs_.size());
    const bool has_timeout = timeout_ms_ >= 0;
    const auto elapsed = clock::now() - start;
    const auto timeout = std::chrono::milliseconds(has_timeout ? timeout_ms_ : 0);
    const bool timed_out = has_timeout && elapsed >= timeout;
    if (n >= min_ || (timed_out && n > 0)) break;
    if (has_timeout && !timed_out) {
      auto remaining = std::chrono::duration_cast<std::chrono::milliseconds>(
          timeout - elapsed) + std::chrono::milliseconds(1);
      batch_cv_.WaitFor(&mu_, std::min<std::chrono::milliseconds>(remaining, poll));
    } else {
      batch_cv_.WaitFor(&mu_, poll);
    }
  }
  --waiting_get_inputs_;
  if (!st.ok()) {
    CancelAndCloseLocked();
    return st;
  }
  const int64_t batch = std::min<int64_t>(static_cast<int64_t>(inputs_.size()), max_);
  reqs->assign(inputs_.begin(), inputs_.begin() + batch);
  inputs_.erase(inputs_.begin(), inputs_.begin() + batch);
  st = ValidateBatch(*reqs);
  if (!st.ok()) {
    for (Request* r : *reqs) FinishRequest(r, Status::Cancelled("Compute was cancelled"));
    reqs->clear();
    CancelAndCloseLocked();
    return st;
  }
  *id = next_id_++;
  being_computed_[*id] = *reqs;
  copying_.insert(*id);
  ++n_batches_;
  n_requests_ += batch;
  return Status::OK();
}

void Batcher::EndCopy(int64_t id, Status* st) {
  MutexLock l(&mu_);
  copying_.erase(id);
  if (closed_) {  // closed while rows were being gathered
    auto it = being_computed_.find(id);
    if (it != being_computed_.end()) {
      for (Request* r : it->second)
        FinishRequest(r, Status::Cancelled("Compute was cancelled"));
      being_computed_.erase(it);
    }
    *st = Status::Cancelled(cancelled_ ? "GetInputs operation was cancelled"
                                       : "Batcher is closed");
  }
}

Status Batcher::GetInputs(std::vector<OwnedTensor>* batched,
                          int64_t* computation_id) {
  std::vector<Request*> reqs;
  int64_t id = -1;
  Status st = TakeBatch(&reqs, &id);
  if (!st.ok()) return st;
  // Rows are copied outside the lock: the requests sit in being_computed_
  // under `copying_`, so neither Close() nor SetOutputs() can complete them.
  const auto& first = *reqs[0]->inputs;
  batched->clear();
  batched->reserve(first.size());
  const int64_t n = static_cast<int64_t>(reqs.size());
  for (size_t k = 0; k < first.size(); ++k) {
    TensorMeta m = first[k].meta;
    m.shape[0] = n;
    OwnedTensor t = OwnedTensor::Alloc(m);
    const size_t row = m.row_bytes();
    for (int64_t i = 0; i < n; ++i)
      std::memcpy(t.data.get() + i * row, (*reqs[i]->inputs)[k].data, row);
    batched->push_back(std::move(t));
  }
  EndCopy(id, &st);
  if (!st.ok()) {
    batched->clear();
    return st;
  }
  *computation_id = id;
  return Status::OK();
}

Status Batcher::GetInputsInto(const std::vector<void*>& dst,
                              const std::vector<size_t>& cap,
                              std::vector<TensorMeta>* metas,
                              int64_t* batch_size, int64_t* computation_id) {
  std::vector<Request*> reqs;
  int64_t id = -1;
  Status st = TakeBatch(&reqs, &id);
  if (!st.ok()) return st;
  const auto& first = *reqs[0]->inputs;
  const int64_t n = static_cast<int64_t>(reqs.size());
  metas->clear();
  if (dst.size() != first.size() || cap.size() != first.size()) {
    st = Status::Invalid("GetInputsInto: expected " + std::to_string(first.size()) +
                         " destination buffers");
  } else {
    for (size_t k = 0; k < first.size() && st.ok(); ++k) {
      TensorMeta m = first[k].meta;
      m.shape[0] = n;
      if (m.nbytes() > cap[k]) {
        st = Status::Invalid("GetInputsInto: destination buffer " + std::to_string(k) +
                             " too small");
        break;
      }
      const size_t row = m.row_bytes();
      uint8_t* base = static_cast<uint8_t*>(dst[k]);
      for (int64_t i = 0; i < n; ++i)
        std::memcpy(base + i * row, (*reqs[i]->inputs)[k].data, row);
      metas->push_back(m);
    }
  }
  if (!st.ok()) {
    MutexLock l(&mu_);
    copying_.erase(id);
    CancelAndCloseLocked();
    return st;
  }
  EndCopy(id, &st);
  if (!st.ok()) return st;
  *batch_size = n;
  *computation_id = id;
  return Status::OK();
}

Status Batcher::GetInputsPacked(void* dst, size_t cap, size_t align,
                                bool layout_pow2, std::vector<TensorMeta>* metas,
                                std::vector<size_t>* offsets, size_t* used,
                                int64_t* layout_rows, int64_t* batch_size,
                                int64_t* computation_id) {
  std::vector<Request*> reqs;
  int64_t id = -1;
  Status st = TakeBatch(&reqs, &id);
  if (!st.ok()) return st;
  const auto& first = *reqs[0]->inputs;
  const int64_t n = static_cast<int64_t>(reqs.size());
  int64_t rows = n;
  if (layout_pow2) {
    rows = 1;
    while (rows < n) rows <<= 1;
    if (rows > max_) rows = max_;
  }
  if (align == 0) align = 1;
  metas->clear();
  offsets->clear();
  size_t off = 0;
  for (size_t k = 0; k < first.size(); ++k) {
    TensorMeta m = first[k].meta;
    m.shape[0] = n;
    off = (off + align - 1) / align * align;
    offsets->push_back(off);
    off += m.row_bytes() * static_cast<size_t>(rows);
    metas->push_back(m);
  }
  if (off > cap) {
    st = Status::Invalid("GetInputsPacked: staging slab too small (" +
                         std::to_string(off) + " > " + std::to_string(cap) + " bytes)");
    MutexLock l(&mu_);
    copying_.erase(id);
    CancelAndCloseLocked();
    return st;
  }
  uint8_t* base = static_cast<uint8_t*>(dst);
  for (size_t k = 0; k < first.size(); ++k) {
    const size_t row = (*metas)[k].row_bytes();
    uint8_t* seg = base + (*offsets)[k];
    for (int64_t i = 0; i < n; ++i)
      std::memcpy(seg + i * row, (*reqs[i]->inputs)[k].data, row);
  }
  EndCopy(id, &st);
  if (!st.ok()) return st;
  *used = off;
  *layout_rows = rows;
  *batch_size = n;
  *computation_id = id;
  return Status::OK();
}

Status Batcher::SetOutputs(const std::vector<TensorView>& outputs,
                           int64_t computation_id) {
  std::vector<Request*> reqs;
  {
    MutexLock l(&mu_);
    if (closed_) return Status::Cancelled("Batcher is closed");
    auto it = being_computed_.find(computation_id);
    if (it == being_computed_.end() || copying_.count(computation_id)) {
      CancelAndCloseLocked();
      return Status::Invalid("Invalid computation id. Id: " +
                             std::to_string(computation_id));
    }
    const int64_t n = static_cast<int64_t>(it->second.size());
    for (const auto& o : outputs) {
      if (o.meta.shape.empty()) {
        CancelAndCloseLocked();
        return Status::Invalid("Output shape must have a batch dimension");
      }
      if (o.meta.shape[0] != n) {
        CancelAndCloseLocked();
        return Status::Invalid(
            "Output shape must have the same batch dimension as the input batch "
            "size. Expected: " + std::to_string(n) +
            " Observed: " + std::to_string(o.meta.shape[0]));
      }
    }
    reqs = std::move(it->second);
    being_computed_.erase(it);
  }
  // Scatter rows to the waiters outside the lock (unreachable from Close()).
  for (size_t i = 0; i < reqs.size(); ++i) {
    auto* outs = reqs[i]->outputs;
    outs->clear();
    outs->reserve(outputs.size());
    for (const auto& o : outputs) {
      TensorMeta m = o.meta;
      m.shape[0] = 1;
      OwnedTensor t = OwnedTensor::Alloc(m);
      const size_t row = m.row_bytes();
      std::memcpy(t.data.get(), static_cast<const uint8_t*>(o.data) + i * row, row);
      outs->push_back(std::move(t));
    }
  }
  MutexLock l(&mu_);
  for (Request* r : reqs) FinishRequest(r, Status::OK());
  return Status::OK();
}

}  // namespace sa
