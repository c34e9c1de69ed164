// CRC-32C (Castagnoli), slicing-by-8, for the TF event-file writer
// (scalable_agent_amd/summary.py) and the TF checkpoint reader/writer
// (scalable_agent_amd/tf_checkpoint.py): multi-MB tensors would take seconds
// through the byte-at-a-time Python table loop.
#include <pybind11/pybind11.h>

#include <cstdint>
#include <cstring>

namespace py = pybind11;

namespace sa {
namespace {

struct Tables {
  uint32_t t[8][256];
  Tables() {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
      t[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; ++i)
      for (int s = 1; s < 8; ++s) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xFF];
  }
};

const Tables& tables() {
  static const Tables tb;
  return tb;
}

}  // namespace

uint32_t Crc32c(const uint8_t* p, size_t n, uint32_t crc) {
  const auto& T = tables().t;
  crc = ~crc;
  while (n >= 8) {
    uint32_t lo, hi;
    std::memcpy(&lo, p, 4);
    std::memcpy(&hi, p + 4, 4);
    lo ^= crc;
    crc = T[7][lo & 0xFF] ^ T[6][(lo >> 8) & 0xFF] ^ T[5][(lo >> 16) & 0xFF] ^
          T[4][lo >> 24] ^ T[3][hi & 0xFF] ^ T[2][(hi >> 8) & 0xFF] ^
          T[1][(hi >> 16) & 0xFF] ^ T[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) crc = T[0][(crc ^ *p++) & 0xFF] ^ (crc >> 8);
  return ~crc;
}

void register_crc(py::module& m) {
  m.def("crc32c", [](py::buffer b, uint32_t init) {
        py::buffer_info info = b.request();
        const size_t n = static_cast<size_t>(info.size) * static_cast<size_t>(info.itemsize);
        const auto* p = static_cast<const uint8_t*>(info.ptr);
        py::gil_scoped_release nogil;
        return Crc32c(p, n, init);
      }, py::arg("data"), py::arg("init") = 0u,
      "CRC-32C of a contiguous buffer (continues from `init`).");
}

}  // namespace sa
