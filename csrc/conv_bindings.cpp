// Torch bindings for the conv torso kernels.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <c10/core/DeviceGuard.h>

#include "kernels/conv_launchers.h"

void register_conv_ops(pybind11::module& m) {}
