"""Base class for gym-style RL agents (reference algorithms/utils/agent.py:
26-238): CLI arguments, seeding, checkpoint rotation (`.pth`, keep N),
cfg.json persistence, summary/save-rate schedules and the
train-step/env-step/time stopping rules.

Checkpoints are plain tensors/scalars and are loaded with
`torch.load(..., weights_only=True)`; summaries go through the framework's
own TF-event writer (`summary.SummaryWriter`, tensorboardX is not needed).
"""

import glob
import json
import math
import os
import time
from os.path import join

import numpy as np
import torch

from ..summary import SummaryWriter
from ..utils.decay import LinearDecay
from ..utils.utils import (cfg_file, ensure_dir_exists, experiment_dir, log,
                           memory_consumption_mb, summaries_dir)


class TrainStatus(object):
  SUCCESS, FAILURE = range(2)


class AgentBase(object):

  @classmethod
  def add_cli_args(cls, parser):
    p = parser
    p.add_argument('--seed', default=42, type=int,
                   help='Set a fixed seed value')
    p.add_argument('--initial_save_rate', default=1000, type=int,
                   help='Save model every N steps in the beginning of training')
    p.add_argument('--keep_checkpoints', default=4, type=int,
                   help='Number of model checkpoints to keep')
    p.add_argument('--stats_episodes', default=100, type=int,
                   help='How many episodes to average to measure performance')
    p.add_argument('--learning_rate', default=1e-4, type=float, help='LR')
    p.add_argument('--train_for_steps', default=int(1e10), type=int,
                   help='Stop training after this many SGD steps')
    p.add_argument('--train_for_env_steps', default=int(1e10), type=int,
                   help='Stop training after this many environment steps')
    p.add_argument('--train_for_seconds', default=int(1e10), type=int,
                   help='Stop training after this many seconds')
    p.add_argument('--obs_subtract_mean', default=0.0, type=float,
                   help='Observation preprocessing: value to subtract')
    p.add_argument('--obs_scale', default=1.0, type=float,
                   help='Observation preprocessing: divide by this scalar')
    p.add_argument('--gamma', default=0.99, type=float, help='Discount factor')
    p.add_argument('--reward_scale', default=1.0, type=float,
                   help='Multiply all rewards by this factor')
    p.add_argument('--reward_clip', default=10.0, type=float,
                   help='Clip rewards to [-c, c]')
    p.add_argument('--encoder', default='convnet_simple', type=str,
                   help='Type of the observation encoder')
    p.add_argument('--hidden_size', default=512, type=int,
                   help='Size of the hidden layer / RNN state')
    p.add_argument('--device', default='auto', type=str,
                   help="'cuda' (HIP), 'cpu' or 'auto'")

  def __init__(self, cfg):
    self.cfg = cfg
    if self._get('seed') is not None:
      log.info('Settings fixed seed %d', cfg.seed)
      torch.manual_seed(cfg.seed)
      np.random.seed(cfg.seed)
    dev = self._get('device', 'auto')
    if dev == 'auto':
      dev = 'cuda' if torch.cuda.is_available() else 'cpu'
    self.device = torch.device(dev)
    self.train_step = self.env_steps = 0
    self.total_train_seconds = 0
    self.last_training_step = time.time()
    self.best_avg_reward = math.nan
    self.summary_rate_decay = LinearDecay([(0, 100), (1000000, 2000),
                                           (10000000, 10000)])
    self.last_summary_written = -1e9
    self.save_rate_decay = LinearDecay(
        [(0, self._get('initial_save_rate', 1000)), (1000000, 5000)],
        staircase=100)
    self.writer = SummaryWriter(summaries_dir(experiment_dir(cfg=cfg)))

  def _get(self, key, default=None):
    if isinstance(self.cfg, dict):
      return self.cfg.get(key, default)
    return getattr(self.cfg, key, default)

  def initialize(self):
    ckpt = self._load_checkpoint(self._checkpoint_dir())
    if ckpt is None:
      log.debug('Did not load from checkpoint, starting from scratch!')
    else:
      log.debug('Loading model from checkpoint')
      self._load_state(ckpt)
    log.debug('Experiment parameters:')
    for k, v in self._cfg_dict().items():
      log.debug('\t %s: %r', k, v)

  def finalize(self):
    self.writer.close()

  def _should_end_training(self):
    return (self.train_step >= self._get('train_for_steps', int(1e10)) or
            self.env_steps > self._get('train_for_env_steps', int(1e10)) or
            self.total_train_seconds > self._get('train_for_seconds',
                                                 int(1e10)))

  def _after_optimizer_step(self):
    self.train_step += 1
    self._maybe_save()
    now = time.time()
    self.total_train_seconds += now - self.last_training_step
    self.last_training_step = now

  def _on_finished_training(self):
    log.info('Finished training at train_steps %d, env_steps %d, seconds %d',
             self.train_step, self.env_steps, self.total_train_seconds)
    self._save()

  def _load_state(self, checkpoint_dict):
    self.train_step = int(checkpoint_dict['train_step'])
    self.env_steps = int(checkpoint_dict['env_steps'])
    self.best_avg_reward = float(checkpoint_dict['best_avg_reward'])
    self.total_train_seconds = float(checkpoint_dict['total_train_seconds'])
    log.info('Loaded experiment state at training iteration %d, env step %d',
             self.train_step, self.env_steps)

  def _maybe_save(self):
    every = self.save_rate_decay.at(self.train_step)
    if (self.train_step + 1) % every == 0 or self.train_step <= 1:
      self._save()

  def _checkpoint_dir(self):
    return ensure_dir_exists(join(experiment_dir(cfg=self.cfg), 'checkpoint'))

  @staticmethod
  def _get_checkpoints(checkpoints_dir):
    return sorted(glob.glob(join(checkpoints_dir, 'checkpoint_*')))

  def _load_checkpoint(self, checkpoints_dir):
    ckpts = self._get_checkpoints(checkpoints_dir)
    if not ckpts:
      log.warning('No checkpoints found in %s', experiment_dir(cfg=self.cfg))
      return None
    log.warning('Loading state from checkpoint %s...', ckpts[-1])
    return torch.load(ckpts[-1], map_location=self.device, weights_only=True)

  def _get_checkpoint_dict(self):
    return {'train_step': self.train_step, 'env_steps': self.env_steps,
            'best_avg_reward': self.best_avg_reward,
            'total_train_seconds': self.total_train_seconds}

  def _save(self):
    checkpoint = self._get_checkpoint_dict()
    assert checkpoint is not None
    path = join(self._checkpoint_dir(), 'checkpoint_%09d_%d.pth' %
                (self.train_step, self.env_steps))
    log.info('Saving %s...', path)
    tmp = path + '.tmp'
    torch.save(checkpoint, tmp)
    os.replace(tmp, path)
    keep = self._get('keep_checkpoints', 4)
    ckpts = self._get_checkpoints(self._checkpoint_dir())
    for old in ckpts[:max(0, len(ckpts) - keep)]:
      log.debug('Removing %s', old)
      os.remove(old)
    self._save_cfg()

  def _cfg_dict(self):
    return self.cfg if isinstance(self.cfg, dict) else vars(self.cfg)

  def _save_cfg(self):
    with open(cfg_file(self.cfg), 'w') as f:
      json.dump(self._cfg_dict(), f, indent=2)

  def _should_write_summaries(self):
    every = self.summary_rate_decay.at(self.train_step)
    return self.train_step - self.last_summary_written > every

  def _maybe_print(self, avg_rewards, avg_length, fps, t):
    log.info('<====== Step %d, env step %.2fM ======>', self.train_step,
             self.env_steps / 1e6)
    log.info('Avg FPS: %.1f', fps)
    log.info('Timing: %s', t)
    if math.isnan(avg_rewards) or math.isnan(avg_length):
      return
    n = self._get('stats_episodes', 100)
    log.info('Avg. %d episode length: %.3f', n, avg_length)
    best = '' if math.isnan(self.best_avg_reward) else \
        '(best: %.3f)' % self.best_avg_reward
    log.info('Avg. %d episode reward: %.3f %s', n, avg_rewards, best)

  def _maybe_update_avg_reward(self, avg_reward, stats_num_episodes):
    if stats_num_episodes > self._get('stats_episodes', 100):
      if math.isnan(avg_reward):
        return
      if math.isnan(self.best_avg_reward) or \
          avg_reward > self.best_avg_reward + 1e-6:
        log.warning('New best reward %.6f (was %.6f)!', avg_reward,
                    self.best_avg_reward)
        self.best_avg_reward = avg_reward

  def _report_train_summaries(self, stats):
    for key, scalar in stats.items():
      self.writer.add_scalar('train/%s' % key, scalar, self.env_steps)
    self.last_summary_written = self.train_step

  def _report_basic_summaries(self, fps, avg_reward, avg_length):
    w, s = self.writer, self.env_steps
    w.add_scalar('0_aux/fps', fps, s)
    w.add_scalar('0_aux/master_process_memory_mb',
                 float(memory_consumption_mb()), s)
    if math.isnan(avg_reward) or math.isnan(avg_length):
      return
    w.add_scalar('0_aux/avg_reward', float(avg_reward), s)
    w.add_scalar('0_aux/avg_length', float(avg_length), s)
    w.add_scalar('0_aux/best_reward_ever', float(self.best_avg_reward), s)


Agent = AgentBase  # reference name
