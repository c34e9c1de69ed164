// pybind11 registration of the shared-memory ring (part of module _native).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <vector>

#include <linux/futex.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>
#include <atomic>
#include <climits>

#include "envpool/env_channel.h"
#include "envpool/shm_ring.h"
#include "envpool/traj_queue.h"

namespace py = pybind11;

namespace sa {

namespace {
// Futex wait/wake on a 32-bit word of a process-shared mapping (inference
// board slots): wait returns when *addr != expected or after timeout_ms.
int FutexWaitAddr(uintptr_t addr, uint32_t expected, int64_t timeout_ms) {
  auto* w = reinterpret_cast<std::atomic<uint32_t>*>(addr);
  if (w->load(std::memory_order_acquire) != expected) return 1;
  struct timespec ts;
  ts.tv_sec = timeout_ms / 1000;
  ts.tv_nsec = (timeout_ms % 1000) * 1000000L;
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(addr), FUTEX_WAIT, expected,
          timeout_ms < 0 ? nullptr : &ts, nullptr, 0);
  return w->load(std::memory_order_acquire) != expected ? 1 : 0;
}
}  // namespace

void register_envpool(py::module& m) {
  m.def("futex_wait", [](uintptr_t addr, uint32_t expected, int64_t timeout_ms) {
          py::gil_scoped_release nogil;
          return FutexWaitAddr(addr, expected, timeout_ms);
        }, py::arg("addr"), py::arg("expected"), py::arg("timeout_ms"));
  m.def("futex_wake", [](uintptr_t addr) {
          return static_cast<int>(syscall(SYS_futex, reinterpret_cast<uint32_t*>(addr),
                                          FUTEX_WAKE, INT_MAX, nullptr, nullptr, 0));
        }, py::arg("addr"));
  m.def("atomic_store_u32", [](uintptr_t addr, uint32_t v) {
          reinterpret_cast<std::atomic<uint32_t>*>(addr)->store(v, std::memory_order_release);
        });
  m.def("atomic_load_u32", [](uintptr_t addr) {
          return reinterpret_cast<std::atomic<uint32_t>*>(addr)->load(std::memory_order_acquire);
        });
  m.def("atomic_add_u32", [](uintptr_t addr, uint32_t v) {
          return reinterpret_cast<std::atomic<uint32_t>*>(addr)->fetch_add(
              v, std::memory_order_acq_rel);
        });

  py::class_<EnvDoorbell>(m, "EnvDoorbell")
      .def(py::init<>())
      .def_property_readonly("value", &EnvDoorbell::value)
      .def("wait", [](EnvDoorbell& b, uint32_t seen, int64_t t) {
             py::gil_scoped_release nogil;
             return b.Wait(seen, t);
           }, py::arg("seen"), py::arg("timeout_ms"));

  py::class_<EnvChannel>(m, "EnvChannel")
      .def(py::init<>())
      // keep_alive: the channel holds a raw pointer into the bell's page
      .def("attach_doorbell", &EnvChannel::AttachDoorbell, py::keep_alive<1, 2>())
      .def("request", &EnvChannel::Request, py::arg("method"), py::arg("kind"),
           py::arg("action"))
      .def("wait_response", [](EnvChannel& c, uint32_t seq, int64_t t) {
             py::gil_scoped_release nogil;
             return c.WaitResponse(seq, t);
           }, py::arg("seq"), py::arg("timeout_ms"))
      .def_property_readonly("status", &EnvChannel::status)
      .def_property_readonly("reward", &EnvChannel::reward)
      .def_property_readonly("done", &EnvChannel::done)
      .def_property_readonly("instr", [](EnvChannel& c) -> py::object {
             if (!c.has_instr()) return py::none();
             return py::bytes(c.instr());
           })
      .def("wait_request", [](EnvChannel& c, int64_t t) {
             std::tuple<int64_t, int32_t, int32_t, std::vector<double>> r;
             {
               py::gil_scoped_release nogil;
               r = c.WaitRequest(t);
             }
             return r;
           }, py::arg("timeout_ms"))
      .def("discard_pending", &EnvChannel::DiscardPending)
      .def("respond", [](EnvChannel& c, uint32_t seq, int32_t status, float reward,
                         bool done, py::object instr) {
             const bool has = !instr.is_none();
             std::string s = has ? instr.cast<std::string>() : std::string();
             c.Respond(seq, status, reward, done, has, s);
           }, py::arg("seq"), py::arg("status"), py::arg("reward"), py::arg("done"),
           py::arg("instr"));

  py::class_<ShmRing>(m, "ShmRing", py::buffer_protocol())
      .def(py::init<const std::string&, int64_t, int64_t, bool>(),
           py::arg("name"), py::arg("num_slots") = 0, py::arg("slot_bytes") = 0,
           py::arg("create") = false)
      .def("acquire_write", [](ShmRing& r, int64_t t) {
             py::gil_scoped_release nogil;
             return r.AcquireWrite(t);
           }, py::arg("timeout_ms") = -1)
      .def("commit", &ShmRing::Commit)
      .def("acquire_read", [](ShmRing& r, int64_t t) {
             py::gil_scoped_release nogil;
             return r.AcquireRead(t);
           }, py::arg("timeout_ms") = -1)
      .def("acquire_read_many", [](ShmRing& r, int64_t n, int64_t t) {
             std::vector<int64_t> out(static_cast<size_t>(n));
             int64_t got;
             {
               py::gil_scoped_release nogil;
               got = r.AcquireReadMany(n, out.data(), t);
             }
             if (got < 0) return py::object(py::int_(got));
             out.resize(static_cast<size_t>(got));
             return py::object(py::cast(out));
           }, py::arg("n"), py::arg("timeout_ms") = -1)
      .def("release", &ShmRing::Release)
      .def("close", &ShmRing::Close)
      .def_property_readonly("closed", &ShmRing::closed)
      .def_property_readonly("num_slots", &ShmRing::num_slots)
      .def_property_readonly("slot_bytes", &ShmRing::slot_bytes)
      .def_property_readonly("num_ready", &ShmRing::num_ready)
      .def_property_readonly("name", &ShmRing::name)
      .def("slot_address", [](ShmRing& r, int64_t s) {
             return reinterpret_cast<uintptr_t>(r.slot_data(s));
           })
      .def("slot_view", [](ShmRing& r, int64_t s) {
             return py::memoryview::from_memory(r.slot_data(s), r.slot_bytes(), false);
           }, py::keep_alive<0, 1>())
      .def_static("unlink", &ShmRing::Unlink);

  py::class_<TrajQueue>(m, "TrajQueue")
      .def(py::init<const std::string&, int64_t, int64_t, int64_t, bool>(),
           py::arg("name"), py::arg("num_slabs") = 0, py::arg("slab_bytes") = 0,
           py::arg("batch") = 0, py::arg("create") = false)
      .def("claim", [](TrajQueue& q, int64_t t) {
             py::gil_scoped_release nogil;
             return q.Claim(t);
           }, py::arg("timeout_ms") = -1)
      .def("claim_n", [](TrajQueue& q, int64_t n, int64_t t) {
             py::gil_scoped_release nogil;
             return q.ClaimN(n, t);
           }, py::arg("n"), py::arg("timeout_ms") = -1)
      .def("commit", &TrajQueue::Commit)
      .def("acquire", [](TrajQueue& q, int64_t t) {
             py::gil_scoped_release nogil;
             return q.Acquire(t);
           }, py::arg("timeout_ms") = -1)
      .def("release", &TrajQueue::Release)
      .def("close", &TrajQueue::Close)
      .def_property_readonly("closed", &TrajQueue::closed)
      .def_property_readonly("num_slabs", &TrajQueue::num_slabs)
      .def_property_readonly("slab_bytes", &TrajQueue::slab_bytes)
      .def_property_readonly("batch", &TrajQueue::batch)
      .def_property_readonly("num_ready", &TrajQueue::num_ready)
      .def_property_readonly("name", &TrajQueue::name)
      .def_property_readonly("payload_address", [](TrajQueue& q) {
             return reinterpret_cast<uintptr_t>(q.payload_base());
           })
      .def_property_readonly("payload_bytes", &TrajQueue::payload_bytes)
      .def("slab_view", [](TrajQueue& q, int64_t s) {
             return py::memoryview::from_memory(q.slab_data(s), q.slab_bytes(), false);
           }, py::keep_alive<0, 1>())
      .def_static("unlink", &TrajQueue::Unlink);
}

}  // namespace sa
