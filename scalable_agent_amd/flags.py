"""Command-line flags of the IMPALA engine.

Reproduces the flag surface of the reference `experiment.py:46-95` (same names,
same defaults, `--flag=value` syntax) and adds the MI355X-native knobs listed in
SURVEY.md §5.6 (torso choice, synthetic env, data-parallel learners, dtype,
inference batching, PopArt, fault injection).

absl is not installed in this image, so the parser is argparse; argparse accepts
both `--flag=value` and `--flag value`.
"""

import argparse
import dataclasses
from typing import List, Optional


def _str2bool(v):
  if isinstance(v, bool):
    return v
  v = str(v).lower()
  if v in ('1', 'true', 't', 'yes', 'y'):
    return True
  if v in ('0', 'false', 'f', 'no', 'n'):
    return False
  raise argparse.ArgumentTypeError('boolean expected, got %r' % v)


def build_parser() -> argparse.ArgumentParser:
  p = argparse.ArgumentParser(
      description='MI355X-native IMPALA (scalable_agent capabilities).')
  # --- reference flags (experiment.py:49-95) ---
  p.add_argument('--logdir', default='/tmp/agent', help='Log/checkpoint dir.')
  p.add_argument('--mode', default='train', choices=['train', 'test'])
  p.add_argument('--test_num_episodes', type=int, default=10,
                 help='Number of episodes per level.')
  p.add_argument('--task', type=int, default=-1,
                 help='Task id. Use -1 for local training.')
  p.add_argument('--job_name', default='learner', choices=['learner', 'actor'],
                 help='Job name. Ignored when task is set to -1.')
  p.add_argument('--total_environment_frames', type=int, default=int(1e9))
  p.add_argument('--num_actors', type=int, default=4)
  p.add_argument('--batch_size', type=int, default=2)
  p.add_argument('--unroll_length', type=int, default=100)
  p.add_argument('--num_action_repeats', type=int, default=4)
  p.add_argument('--seed', type=int, default=1)
  p.add_argument('--entropy_cost', type=float, default=0.00025)
  p.add_argument('--baseline_cost', type=float, default=.5)
  p.add_argument('--discounting', type=float, default=.99)
  p.add_argument('--reward_clipping', default='abs_one',
                 choices=['abs_one', 'soft_asymmetric'])
  p.add_argument('--dataset_path', default='')
  p.add_argument('--level_name', default='explore_goal_locations_small')
  p.add_argument('--width', type=int, default=96)
  p.add_argument('--height', type=int, default=72)
  p.add_argument('--renderer', default='software')
  p.add_argument('--benchmark_mode', type=int, default=0)
  p.add_argument('--learning_rate', type=float, default=0.00048)
  p.add_argument('--decay', type=float, default=.99)
  p.add_argument('--momentum', type=float, default=0.)
  p.add_argument('--epsilon', type=float, default=.1)
  # --- MI355X-native additions ---
  p.add_argument('--torso', default='shallow', choices=['shallow', 'deep'],
                 help='shallow = experiment.py:178-183 (active in reference); '
                      'deep = IMPALA ResNet experiment.py:156-176.')
  p.add_argument('--env', default='auto',
                 choices=['auto', 'synthetic', 'dmlab', 'doom'],
                 help='auto: doom_* -> doom, synthetic* -> synthetic, else dmlab.')
  p.add_argument('--obs_shape', default='',
                 help='Synthetic env frame shape HxWxC (default height x width x 3).')
  p.add_argument('--synthetic_episode_length', type=int, default=200,
                 help='Mean (geometric) episode length of the synthetic env.')
  p.add_argument('--num_learners', type=int, default=0,
                 help='Data-parallel learners (one process per GPU, RCCL '
                      'all-reduce), launched with torch.distributed.run; '
                      '0 = WORLD_SIZE decides, else it must equal WORLD_SIZE.')
  p.add_argument('--grad_reduce', default='mean', choices=['sum', 'mean'],
                 help='Data-parallel gradient reduction.  mean (default): '
                      'the all-reduced sum times 1/N, folded into the RMSProp '
                      'update - each update has the size of one B-column '
                      'learner\'s.  sum: N learners x B == one learner with '
                      'N*B under the reference sum losses, which at N=8 does '
                      'not learn at the reference learning rate '
                      '(profiles/r4_learning_dp_equiv.md).')
  p.add_argument('--grad_scale', type=float, default=1.0,
                 help='Multiplies the (all-reduced) gradient inside the '
                      'RMSProp update; a single learner with batch N*B and '
                      'grad_scale 1/N reproduces N learners with '
                      '--grad_reduce=mean (DP-semantics experiments).')
  p.add_argument('--grad_overlap', type=_str2bool, default=True,
                 help='Data-parallel: all-reduce the heads/core/FC gradients '
                      'while the conv-torso backward runs (two-phase '
                      'backward), then the torso gradients.')
  p.add_argument('--dtype', default='fp32', choices=['fp32', 'bf16'],
                 help='Compute dtype of convs/GEMMs: fp32 = the reference\'s '
                      'precision (exact-fp32 MFMA kernels on HIP); bf16 = '
                      'bf16 operands, fp32 accumulation (V-trace/loss/'
                      'optimizer state always fp32).')
  p.add_argument('--device', default='auto',
                 help='auto | cpu | cuda | cuda:N')
  p.add_argument('--backend', default='auto', choices=['auto', 'hip', 'torch'],
                 help='Model backend: hip = the hand-written gfx950 kernels '
                      '(default on a GPU), torch = the pure-PyTorch oracle.')
  p.add_argument('--inference_min_batch', type=int, default=1)
  p.add_argument('--inference_max_batch', type=int, default=1024)
  p.add_argument('--inference_timeout_ms', type=int, default=100)
  p.add_argument('--inference_dtype', default='auto',
                 choices=['auto', 'fp32', 'bf16'],
                 help='Actor-inference compute dtype (auto = --dtype); bf16 '
                      'trades behaviour-policy precision (V-trace corrects '
                      'for the policy lag either way) for actor throughput.')
  p.add_argument('--inference_device', default='auto',
                 help='Device of the actor-inference model: auto = the '
                      'learner device; e.g. cuda:1 or cpu.')
  p.add_argument('--trajectory_queue', type=_str2bool, default=True,
                 help='Local actors write time-major batches in place into '
                      'a pinned shared-memory slab queue (one H2D copy per '
                      'learner step); false: per-unroll queue + stacking.')
  p.add_argument('--actor_groups', type=int, default=-1,
                 help='Run the num_actors envs as G vectorised actor-group '
                      'processes (each: its envs stepped in parallel, one '
                      'captured inference graph per step, writes into the '
                      'trajectory queue); 0 = actor threads in the learner '
                      'process; -1 = auto: on a GPU from 32 actors on CPU '
                      'groups of ~40 envs (at least 2) with '
                      '--inference_server (profiles/r6_e2e.md), below that '
                      '1 GPU group (more GPU processes share the card badly: '
                      'profiles/r2_e2e_actors.md); threads on CPU.')
  p.add_argument('--inference_server', type=_str2bool, default=False,
                 help='Actor groups stay CPU-only and post their rows to a '
                      'shared-memory inference board served by a thread of '
                      'the learner process (one GPU context in total).')
  p.add_argument('--inference_gather_us', type=int, default=0,
                 help='Inference board: with fewer than half of the board\'s '
                      'slots requesting, the server waits up to this many '
                      'microseconds for more before launching (every launch '
                      'runs the whole board).  0 = launch at once.')
  p.add_argument('--inference_lanes', type=int, default=2,
                 help='Inference board: boards served side by side, each by '
                      'its own thread, model snapshot and stream (actor '
                      'group g posts to lane g %% lanes; at most one lane per '
                      'group).  2 measured 1-3 %% above 1 at configs #2 and #4 '
                      '(profiles/r6_e2e.md).')
  p.add_argument('--inference_board_depth', type=int, default=1,
                 choices=(1, 2),
                 help='Inference board: batches in flight in the native '
                      'serving loop (2 = the next batch\'s input copy and '
                      'host work overlap the current batch\'s graph; '
                      'measured slower at config #4, profiles/r6_e2e.md).')
  p.add_argument('--actor_group_splits', type=int, default=2,
                 help='Pipeline stages per actor group: split k\'s inference '
                      'runs on the GPU while the envs of another split step.')
  p.add_argument('--envs_per_worker', type=int, default=1,
                 help='Envs hosted by one supervised env worker process '
                      '(py_process.start_group: the envs share one doorbell '
                      'futex, so a step of all of them costs one wake-up). '
                      '1 = one process per env, as the reference.')
  p.add_argument('--popart', type=_str2bool, default=False,
                 help='PopArt value normalisation (north-star config #4).')
  p.add_argument('--popart_beta', type=float, default=3e-4)
  p.add_argument('--save_checkpoint_secs', type=float, default=600)
  p.add_argument('--import_tf_checkpoint', type=str, default='',
                 help='TF V2 checkpoint prefix (or a logdir with a '
                      '`checkpoint` file) of a reference run to start from '
                      'when --logdir has no checkpoint of its own.')
  p.add_argument('--checkpoint_format', default='pt', choices=['pt', 'tf'],
                 help='pt: checkpoint_<frames>.pt (torch, weights_only); tf: '
                      'the reference\'s model.ckpt-<frames>.{index,data} + '
                      '`checkpoint` (TF V2 bundle, no TensorFlow needed).  '
                      'Restore and --mode=test read either.')
  p.add_argument('--save_summaries_secs', type=float, default=30)
  p.add_argument('--keep_checkpoints', type=int, default=5)
  p.add_argument('--log_every_frames', type=int, default=50000,
                 help='Throughput log period (reference log_step_count_steps).')
  p.add_argument('--use_hip_graph', type=_str2bool, default=True)
  p.add_argument('--pipeline_chunks', type=int, default=1,
                 help='HIP learner: split the unroll into N time chunks and '
                      'overlap chunk k\'s LSTM recurrence (side stream) with '
                      'the conv torso of chunk k+1 (1 = off).')
  p.add_argument('--fault_inject', default='',
                 help='e.g. env_crash:0.01,actor_stall:50 (tests only).')
  p.add_argument('--deterministic', type=_str2bool, default=False)
  p.add_argument('--max_learner_steps', type=int, default=0,
                 help='Stop after N learner steps (0 = frames limit only).')
  p.add_argument('--queue_timeout_secs', type=float, default=600.,
                 help='Learner starvation timeout (diagnostic failure).')
  p.add_argument('--env_timeout_secs', type=float, default=0.,
                 help='Env-call watchdog: a worker that does not answer in '
                      'time is killed and respawned (0 = off).')
  p.add_argument('--numa_affinity', default='auto', choices=['auto', 'on', 'off'],
                 help='pin each learner rank (and the actor processes it forks) '
                 'to the NUMA node of its GPU before any pinned allocation; '
                 'auto: when the learner runs on a GPU')
  p.add_argument('--consistency_check_steps', type=int, default=1000,
                 help='Data-parallel: every N steps all-reduce a parameter '
                      'checksum and fail on divergence (0 = off).')
  p.add_argument('--collective_timeout_secs', type=float, default=600.,
                 help='RCCL/gloo collective timeout: a hung rank aborts the '
                      'job (restart it to resume from the last checkpoint).')
  p.add_argument('--skip_nonfinite', type=_str2bool, default=True,
                 help='Skip (and count) optimizer steps with NaN/inf grads.')
  return p


def parse_flags(argv: Optional[List[str]] = None):
  """Parses argv (without program name) and returns an argparse Namespace."""
  parser = build_parser()
  flags, unknown = parser.parse_known_args(argv)
  if unknown:
    raise SystemExit('Unknown flags: %s' % ' '.join(unknown))
  check_flags(flags)
  return flags


def check_flags(flags):
  """Rejects combinations the kernels do not implement (instead of quietly
  running something else): the shallow torso has exact-fp32 HIP kernels
  only, so `--dtype bf16 --torso shallow` on the HIP backend is refused."""
  if (getattr(flags, 'dtype', 'fp32') == 'bf16' and
      getattr(flags, 'torso', 'deep') == 'shallow' and
      getattr(flags, 'backend', 'auto') != 'torch'):
    raise SystemExit('--dtype bf16 --torso shallow: the shallow torso has no '
                     'bf16 HIP kernels (its fp32 kernels would run); use '
                     '--dtype fp32, the deep torso, or --backend torch')


def default_flags(**overrides):
  """Default flags with keyword overrides (library/test convenience)."""
  flags = parse_flags([])
  for k, v in overrides.items():
    if not hasattr(flags, k):
      raise AttributeError('unknown flag %s' % k)
    setattr(flags, k, v)
  return flags


def frames_per_step(flags, world_size=1):
  """Env frames consumed per learner step (experiment.py:419-420)."""
  return (flags.batch_size * flags.unroll_length * flags.num_action_repeats *
          world_size)
