"""Hand-written CDNA4 (gfx950) HIP kernels for the learner/actor hot path.

Every op here is backed by the in-tree extension `scalable_agent_amd/_C*.so`
built from `csrc/kernels/*.hip` by `csrc/build.py` (hipcc --offload-arch=gfx950,
no hipify, no CUDA shims).  On a GPU the ops FAIL LOUDLY if the extension is
missing; the pure-PyTorch oracles they are tested against live next to the
callers (models/layers.py, vtrace.py, losses.py, optim.py).
"""

from ._ext import available, load, ext  # noqa: F401
from .rmsprop import poison_on_error, rmsprop_step  # noqa: F401
from .vtrace_loss import vtrace_loss, vtrace_fused_forward  # noqa: F401
from .lstm import lstm_unroll  # noqa: F401
from .conv import torso_forward, linear_relu  # noqa: F401
from .conv_f32 import torso_forward_f32, linear_relu_f32  # noqa: F401
from .core import core_lstm  # noqa: F401
from .lang import language_lstm  # noqa: F401
from .heads import heads_vtrace_loss, actor_heads_sample, PhiloxStream  # noqa: F401
from .grad_sink import direct_grads  # noqa: F401
