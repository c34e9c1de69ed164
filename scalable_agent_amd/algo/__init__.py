"""Gym-side algorithm utilities (reference algorithms/): agent base class,
action distributions, vectorised envs, numerical helpers, spaces."""

from .algo_utils import (EPS, RunningMeanStd, calculate_discounted_sum,  # noqa
                         calculate_gae, num_env_steps)
from .spaces import Discretized  # noqa
