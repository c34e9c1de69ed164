"""Data-parallel learners over RCCL (xGMI) — new capability.

The reference has exactly one learner (experiment.py:508).  Here N learners,
one process per GPU, each consume their own B-sized batches; after backward the
flat gradient buffer (see optim.FlatParams) is summed (or averaged) with one
`torch.distributed.all_reduce` — backend "nccl" is RCCL on ROCm.  The default
`--grad_reduce=mean` scales the summed gradient by 1/N inside the RMSProp
update (N learners x B == one learner with batch N*B and --grad_scale 1/N);
`--grad_reduce=sum` is exactly one learner with batch N*B under the
reference's sum losses, which at N*B = 256 does not learn at the reference
learning rate (profiles/r4_learning_dp_equiv.md).
"""

from .dist import (init_distributed, GradientSynchronizer, broadcast_params,
                   param_checksum_consistent, world_info, cleanup,
                   backend_info)
from .streams import (stream_plan, warmup_collective, reset_stream_plans,
                      reserve_hw_queues, StreamPlan)
from .affinity import (auto_pin_wanted, gpu_numa_node, pin_to_gpu_numa,
                       visible_gpu_count)
