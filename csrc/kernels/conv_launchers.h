// Launchers for the NHWC implicit-GEMM conv / pool kernels (conv*.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace sa {}  // namespace sa
