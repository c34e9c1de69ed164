"""Data-parallel learners over RCCL (xGMI) — new capability.

The reference has exactly one learner (experiment.py:508).  Here N learners,
one process per GPU, each consume their own B-sized batches; after backward the
flat gradient buffer (see optim.FlatParams) is summed (or averaged) with one
`torch.distributed.all_reduce` — backend "nccl" is RCCL on ROCm.  With
`--grad_reduce=sum`, N learners x batch B is exactly one learner with batch N*B
under the reference's sum losses.
"""

from .dist import (init_distributed, GradientSynchronizer, broadcast_params,
                   param_checksum_consistent, world_info, cleanup,
                   backend_info)
from .affinity import auto_pin_wanted, gpu_numa_node, pin_to_gpu_numa
