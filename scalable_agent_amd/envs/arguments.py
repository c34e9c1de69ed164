"""Experiment configuration for the gym-side env stack (reference
algorithms/utils/arguments.py:12-99): `parse_args` (algo + env + optional
evaluation arguments, env-specific defaults), `default_cfg` for tests and
the IMPALA Doom adaptor, and cfg.json restore.

Algorithm classes: only the agent base class exists in the reference
(its PPO/APPO modules were trimmed from the fork), so every algo name
resolves to `AgentBase` with a warning for unknown names.
"""

import argparse
import json
import os
import sys

from ..algo.agent_base import AgentBase
from ..algo.evaluation_config import add_eval_args
from ..utils.utils import AttrDict, cfg_file, log
from .env_config import add_env_args, env_override_defaults

ALGORITHMS = {'IMPALA': AgentBase, 'PPO': AgentBase, 'APPO': AgentBase}


def get_algo_class(algo):
  if algo not in ALGORITHMS:
    log.warning('Algorithm %s is not supported', algo)
  return ALGORITHMS.get(algo, AgentBase)


def parse_args(argv=None, evaluation=False):
  if argv is None:
    argv = sys.argv[1:]
  parser = argparse.ArgumentParser(
      formatter_class=argparse.ArgumentDefaultsHelpFormatter)
  parser.add_argument('--algo', type=str, default=None, required=True)
  parser.add_argument('--env', type=str, default=None, required=True)
  parser.add_argument('--experiment', type=str, default=None, required=True)
  parser.add_argument('--experiments_root', type=str, default=None,
                      help='Sub-folder of train_dir for groups of experiments')
  basic, _ = parser.parse_known_args(argv)
  get_algo_class(basic.algo).add_cli_args(parser)
  add_env_args(basic.env, parser)
  env_override_defaults(basic.env, parser)
  if evaluation:
    add_eval_args(parser)
  args = parser.parse_args(argv)
  args.command_line = ' '.join(argv)
  return args


def default_cfg(algo='IMPALA', env='env', experiment='test'):
  """Defaults for an env (used by tests and the IMPALA Doom adaptor)."""
  return parse_args(argv=['--algo=%s' % algo, '--env=%s' % env,
                          '--experiment=%s' % experiment])


def load_from_checkpoint(cfg):
  filename = cfg_file(cfg)
  if not os.path.isfile(filename):
    raise Exception('Could not load saved parameters for experiment %s' %
                    cfg.experiment)
  with open(filename) as f:
    loaded = AttrDict(json.load(f))
  log.warning('Loading existing experiment configuration from %s', filename)
  log.warning('Command-line parameters will be ignored!\nIf you want to '
              'resume experiment with different parameters, you should edit '
              '%s!', filename)
  for key, value in vars(cfg).items():
    if key not in loaded:
      loaded[key] = value
  return loaded


def maybe_load_from_checkpoint(cfg):
  if not os.path.isfile(cfg_file(cfg)):
    log.warning('Saved parameter configuration for experiment %s not found!',
                cfg.experiment)
    log.warning('Starting experiment from scratch!')
    return AttrDict(vars(cfg))
  return load_from_checkpoint(cfg)
