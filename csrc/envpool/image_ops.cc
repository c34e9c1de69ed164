// Host-side image ops used by the env wrappers (the reference calls OpenCV:
// envs/env_wrappers.py:196-260 cv2.resize / cv2.cvtColor).  These run inside
// env worker processes on every frame, so they are native, GIL-free and
// allocation-light:
//   resize_u8(src[H,W,C] or [H,W], out_h, out_w, mode)  mode: 0 nearest
//       (cv2.INTER_NEAREST index rule), 1 area (exact fractional box filter,
//       cv2.INTER_AREA for downscaling), 2 bilinear (half-pixel centres,
//       cv2.INTER_LINEAR convention)
//   rgb_to_gray(src[H,W,3]) -> [H,W]   (BT.601 0.299/0.587/0.114, rounded)
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <stdexcept>
#include <vector>

namespace py = pybind11;

namespace sa {
namespace {

using U8Array = py::array_t<uint8_t, py::array::c_style | py::array::forcecast>;

void ResizeNearest(const uint8_t* src, int sh, int sw, int c, uint8_t* dst,
                   int dh, int dw) {
  const double fy = static_cast<double>(sh) / dh;
  const double fx = static_cast<double>(sw) / dw;
  std::vector<int> xs(dw);
  for (int x = 0; x < dw; ++x)
    xs[x] = std::min(static_cast<int>(std::floor(x * fx)), sw - 1);
  for (int y = 0; y < dh; ++y) {
    const int sy = std::min(static_cast<int>(std::floor(y * fy)), sh - 1);
    const uint8_t* row = src + static_cast<size_t>(sy) * sw * c;
    uint8_t* out = dst + static_cast<size_t>(y) * dw * c;
    for (int x = 0; x < dw; ++x)
      for (int k = 0; k < c; ++k) out[x * c + k] = row[xs[x] * c + k];
  }
}

// Per-axis box-filter taps: destination cell i covers source interval
// [i*s, (i+1)*s) with s = src/dst; each source pixel contributes its overlap.
struct Tap {
  int src;
  float w;
};

std::vector<std::vector<Tap>> AreaTaps(int src_n, int dst_n) {
  std::vector<std::vector<Tap>> taps(dst_n);
  const double s = static_cast<double>(src_n) / dst_n;
  for (int i = 0; i < dst_n; ++i) {
    const double a = i * s, b = std::min((i + 1) * s, double(src_n));
    for (int j = static_cast<int>(std::floor(a)); j < b && j < src_n; ++j) {
      const double lo = std::max(a, double(j)), hi = std::min(b, j + 1.0);
      if (hi > lo) taps[i].push_back({j, static_cast<float>((hi - lo) / s)});
    }
  }
  return taps;
}

std::vector<std::vector<Tap>> LinearTaps(int src_n, int dst_n) {
  std::vector<std::vector<Tap>> taps(dst_n);
  const double s = static_cast<double>(src_n) / dst_n;
  for (int i = 0; i < dst_n; ++i) {
    double f = (i + 0.5) * s - 0.5;
    f = std::max(0.0, std::min(f, double(src_n - 1)));
    const int j0 = static_cast<int>(std::floor(f));
    const int j1 = std::min(j0 + 1, src_n - 1);
    const float w1 = static_cast<float>(f - j0);
    taps[i].push_back({j0, 1.f - w1});
    if (j1 != j0 && w1 > 0.f) taps[i].push_back({j1, w1});
  }
  return taps;
}

void ResizeSeparable(const uint8_t* src, int sh, int sw, int c, uint8_t* dst,
                     int dh, int dw, bool area) {
  const auto ty = area ? AreaTaps(sh, dh) : LinearTaps(sh, dh);
  const auto tx = area ? AreaTaps(sw, dw) : LinearTaps(sw, dw);
  std::vector<float> rowbuf(static_cast<size_t>(sw) * c);
  for (int y = 0; y < dh; ++y) {
    std::fill(rowbuf.begin(), rowbuf.end(), 0.f);
    for (const Tap& t : ty[y]) {
      const uint8_t* row = src + static_cast<size_t>(t.src) * sw * c;
      for (int i = 0; i < sw * c; ++i) rowbuf[i] += t.w * row[i];
    }
    uint8_t* out = dst + static_cast<size_t>(y) * dw * c;
    for (int x = 0; x < dw; ++x) {
      for (int k = 0; k < c; ++k) {
        float acc = 0.f;
        for (const Tap& t : tx[x]) acc += t.w * rowbuf[t.src * c + k];
        out[x * c + k] = static_cast<uint8_t>(
            std::min(255.f, std::max(0.f, std::nearbyint(acc))));
      }
    }
  }
}

py::array ResizeU8(U8Array src, int out_h, int out_w, int mode) {
  if (src.ndim() != 2 && src.ndim() != 3)
    throw std::invalid_argument("resize_u8 expects [H,W] or [H,W,C] uint8");
  if (out_h <= 0 || out_w <= 0)
    throw std::invalid_argument("resize_u8: output size must be positive");
  const int sh = static_cast<int>(src.shape(0));
  const int sw = static_cast<int>(src.shape(1));
  const int c = src.ndim() == 3 ? static_cast<int>(src.shape(2)) : 1;
  std::vector<py::ssize_t> shape = {out_h, out_w};
  if (src.ndim() == 3) shape.push_back(c);
  U8Array out(shape);
  const uint8_t* s = src.data();
  uint8_t* d = out.mutable_data();
  {
    py::gil_scoped_release nogil;
    if (sh == out_h && sw == out_w) {
      std::copy(s, s + static_cast<size_t>(sh) * sw * c, d);
    } else if (mode == 0) {
      ResizeNearest(s, sh, sw, c, d, out_h, out_w);
    } else if (mode == 1 || mode == 2) {
      // INTER_AREA only differs from bilinear when shrinking (OpenCV falls
      // back to bilinear for enlargement); mirror that.
      const bool area = mode == 1 && out_h <= sh && out_w <= sw;
      ResizeSeparable(s, sh, sw, c, d, out_h, out_w, area);
    } else {
      throw std::invalid_argument("resize_u8: mode must be 0, 1 or 2");
    }
  }
  return std::move(out);
}

py::array RgbToGray(U8Array src) {
  if (src.ndim() != 3 || src.shape(2) != 3)
    throw std::invalid_argument("rgb_to_gray expects [H,W,3] uint8");
  const py::ssize_t h = src.shape(0), w = src.shape(1);
  U8Array out({h, w});
  const uint8_t* s = src.data();
  uint8_t* d = out.mutable_data();
  {
    py::gil_scoped_release nogil;
    // Fixed-point BT.601 weights (x2^14) with round-to-nearest.
    constexpr int kR = 4899, kG = 9617, kB = 1868;
    for (py::ssize_t i = 0; i < h * w; ++i) {
      const int v = kR * s[3 * i] + kG * s[3 * i + 1] + kB * s[3 * i + 2];
      d[i] = static_cast<uint8_t>((v + (1 << 13)) >> 14);
    }
  }
  return std::move(out);
}

}  // namespace

void register_image_ops(py::module& m) {
  m.def("resize_u8", &ResizeU8, py::arg("src"), py::arg("out_h"),
        py::arg("out_w"), py::arg("mode") = 0);
  m.def("rgb_to_gray", &RgbToGray, py::arg("src"));
}

}  // namespace sa
