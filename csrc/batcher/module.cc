// pybind11 module `scalable_agent_amd.runtime._native`: host runtime pieces
// (dynamic batcher; trajectory ring and env-pool primitives register
// themselves from csrc/envpool/).  Numpy arrays cross the boundary; every
// blocking call releases the GIL.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "batcher/batcher.h"

namespace py = pybind11;

namespace sa {

void register_envpool(py::module& m);  // csrc/envpool/module_part.cc
void register_image_ops(py::module& m);  // csrc/envpool/image_ops.cc
void register_crc(py::module& m);        // csrc/envpool/crc32c.cc

namespace {

// Raw pointers (intentionally never released): py::object globals would be
// destroyed after interpreter finalisation.
PyObject* g_cancelled = nullptr;
PyObject* g_invalid = nullptr;

}  // namespace

[[noreturn]] void RaiseStatus(const Status& s) {
  PyObject* exc = s.code == Code::kCancelled ? g_cancelled : g_invalid;
  PyErr_SetString(exc, s.msg.c_str());
  throw py::error_already_set();
}

void SetExceptionTypes(PyObject* cancelled, PyObject* invalid) {
  g_cancelled = cancelled;
  g_invalid = invalid;
}

namespace {

[[noreturn]] void Raise(const Status& s) { RaiseStatus(s); }

TensorMeta MetaOf(const py::array& a) {
  TensorMeta m;
  m.dtype = py::str(a.dtype().attr("str"));
  m.itemsize = static_cast<size_t>(a.itemsize());
  for (py::ssize_t i = 0; i < a.ndim(); ++i) m.shape.push_back(a.shape(i));
  return m;
}

// Converts a Python list of arrays to views; keeps contiguous copies alive.
std::vector<TensorView> Views(const py::list& arrays,
                              std::vector<py::array>* keep) {
  std::vector<TensorView> v;
  for (auto h : arrays) {
    py::array a = py::array::ensure(h, py::array::c_style);
    if (!a) throw py::value_error("batcher inputs must be array-like");
    if (a.dtype().kind() == 'O')
      throw py::type_error("object arrays are not supported by the batcher");
    keep->push_back(a);
    TensorView tv;
    tv.meta = MetaOf(a);
    tv.data = a.data();
    v.push_back(tv);
  }
  return v;
}

py::array ToArray(const OwnedTensor& t) {
  auto holder = new std::shared_ptr<uint8_t>(t.data);
  py::capsule cap(holder, [](void* p) {
    delete reinterpret_cast<std::shared_ptr<uint8_t>*>(p);
  });
  std::vector<py::ssize_t> shape(t.meta.shape.begin(), t.meta.shape.end());
  return py::array(py::dtype(t.meta.dtype), shape, t.data.get(), cap);
}

class PyBatcher {
 public:
  PyBatcher(int64_t min_b, int64_t max_b, int64_t timeout_ms)
      : b_(min_b, max_b, timeout_ms) {}

  py::list Compute(const py::list& inputs) {
    std::vector<py::array> keep;
    auto views = Views(inputs, &keep);
    std::vector<OwnedTensor> outs;
    Status s;
    {
      py::gil_scoped_release nogil;
      s = b_.Compute(views, &outs);
    }
    if (!s.ok()) Raise(s);
    py::list r;
    for (auto& o : outs) r.append(ToArray(o));
    return r;
  }

  py::tuple GetInputs() {
    std::vector<OwnedTensor> batched;
    int64_t id = -1;
    Status s;
    {
      py::gil_scoped_release nogil;
      s = b_.GetInputs(&batched, &id);
    }
    if (!s.ok()) Raise(s);
    py::list r;
    for (auto& o : batched) r.append(ToArray(o));
    return py::make_tuple(r, id);
  }

  // dst: list of (address:int, capacity_bytes:int) pairs (e.g. pinned torch
  // tensors' data_ptr/nbytes).  Returns (batch_size, id, [(dtype, shape)]).
  py::tuple GetInputsInto(const py::list& dst) {
    std::vector<void*> ptrs;
    std::vector<size_t> caps;
    for (auto h : dst) {
      auto t = h.cast<py::tuple>();
      ptrs.push_back(reinterpret_cast<void*>(t[0].cast<uintptr_t>()));
      caps.push_back(t[1].cast<size_t>());
    }
    std::vector<TensorMeta> metas;
    int64_t n = 0, id = -1;
    Status s;
    {
      py::gil_scoped_release nogil;
      s = b_.GetInputsInto(ptrs, caps, &metas, &n, &id);
    }
    if (!s.ok()) Raise(s);
    py::list m;
    for (auto& x : metas) m.append(py::make_tuple(x.dtype, py::cast(x.shape)));
    return py::make_tuple(n, id, m);
  }

  // Packed variant: one slab (address, capacity); returns (batch_size, id,
  // used_bytes, layout_rows, [(dtype, shape, offset)]).
  py::tuple GetInputsPacked(uintptr_t addr, size_t cap, size_t align,
                            bool layout_pow2) {
    std::vector<TensorMeta> metas;
    std::vector<size_t> offs;
    size_t used = 0;
    int64_t n = 0, id = -1, rows = 0;
    Status s;
    {
      py::gil_scoped_release nogil;
      s = b_.GetInputsPacked(reinterpret_cast<void*>(addr), cap, align, layout_pow2,
                             &metas, &offs, &used, &rows, &n, &id);
    }
    if (!s.ok()) Raise(s);
    py::list m;
    for (size_t k = 0; k < metas.size(); ++k)
      m.append(py::make_tuple(metas[k].dtype, py::cast(metas[k].shape), offs[k]));
    return py::make_tuple(n, id, used, rows, m);
  }

  void SetOutputs(const py::list& outputs, int64_t id) {
    std::vector<py::array> keep;
    std::vector<TensorView> views;
    for (auto h : outputs) {
      py::array a = py::array::ensure(h, py::array::c_style);
      if (!a) throw py::value_error("outputs must be array-like");
      keep.push_back(a);
      TensorView tv;
      tv.meta = MetaOf(a);
      tv.data = a.data();
      views.push_back(tv);
    }
    Status s;
    {
      py::gil_scoped_release nogil;
      s = b_.SetOutputs(views, id);
    }
    if (!s.ok()) Raise(s);
  }

  void Close() {
    py::gil_scoped_release nogil;
    b_.Close();
  }
  void Cancel() {
    py::gil_scoped_release nogil;
    b_.Cancel();
  }
  bool closed() { return b_.closed(); }
  int64_t num_batches() { return b_.num_batches(); }
  int64_t num_requests() { return b_.num_requests(); }
  int64_t min_b() const { return b_.minimum_batch_size(); }
  int64_t max_b() const { return b_.maximum_batch_size(); }
  int64_t timeout() const { return b_.timeout_ms(); }

 private:
  Batcher b_;
};

}  // namespace
}  // namespace sa

PYBIND11_MODULE(_native, m) {
  using sa::PyBatcher;
  m.doc() = "scalable_agent_amd host runtime (C++17)";
  static py::exception<std::runtime_error> cancelled(m, "CancelledError");
  static py::exception<std::runtime_error> invalid(m, "InvalidArgumentError");
  sa::SetExceptionTypes(cancelled.ptr(), invalid.ptr());
  py::class_<PyBatcher>(m, "Batcher")
      .def(py::init<int64_t, int64_t, int64_t>(), py::arg("minimum_batch_size"),
           py::arg("maximum_batch_size"), py::arg("timeout_ms"))
      .def("compute", &PyBatcher::Compute)
      .def("get_inputs", &PyBatcher::GetInputs)
      .def("get_inputs_into", &PyBatcher::GetInputsInto)
      .def("get_inputs_packed", &PyBatcher::GetInputsPacked, py::arg("address"),
           py::arg("capacity"), py::arg("align") = 256,
           py::arg("layout_pow2") = false)
      .def("set_outputs", &PyBatcher::SetOutputs)
      .def("close", &PyBatcher::Close)
      .def("cancel", &PyBatcher::Cancel)
      .def_property_readonly("closed", &PyBatcher::closed)
      .def_property_readonly("num_batches", &PyBatcher::num_batches)
      .def_property_readonly("num_requests", &PyBatcher::num_requests)
      .def_property_readonly("minimum_batch_size", &PyBatcher::min_b)
      .def_property_readonly("maximum_batch_size", &PyBatcher::max_b)
      .def_property_readonly("timeout_ms", &PyBatcher::timeout);
  sa::register_envpool(m);
  sa::register_image_ops(m);
  sa::register_crc(m);
}
