"""Evaluation-mode CLI arguments (reference
algorithms/utils/evaluation_config.py)."""

from os.path import join

from ..utils.utils import project_root


def add_eval_args(parser):
  parser.add_argument('--fps', default=0, type=int,
                      help='Enable sync mode with adjustable FPS. 0 means the '
                      'env default (e.g. ~35 for Doom) or unlimited')
  parser.add_argument('--render_action_repeat', default=None, type=int,
                      help='Repeat an action that many frames during '
                      'evaluation (default: env frameskip from training)')
  parser.add_argument('--record_to',
                      default=join(project_root(), '..', 'recorded_episodes'),
                      type=str, help='Record episodes to this folder')
  parser.add_argument('--no_render', action='store_true',
                      help='Do not render the environment during evaluation')
  parser.add_argument('--policy_index', default=0, type=int,
                      help='Policy to evaluate in multi-policy training')
