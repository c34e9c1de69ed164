"""Doom action spaces (reference envs/doom/action_space.py:13-138).

Each space is a Tuple of independent heads whose order matches the
`available_buttons` of the scenario it is used with; index 0 of every
Discrete head is the no-op.  Turning is either 2 buttons (Discrete(3)), a
continuous delta (Box) or a discretized delta (Discretized).
"""

from ..gym_compat import Box, Discrete, Tuple
from ...algo.spaces import Discretized


def key_to_action_basic(key):
  from pynput.keyboard import Key  # pylint: disable=import-outside-toplevel
  return {Key.left: 0, Key.right: 1, Key.up: 2, Key.down: 3}.get(key, None)


def doom_action_space_basic():
  """TURN_LEFT TURN_RIGHT MOVE_FORWARD MOVE_BACKWARD."""
  space = Tuple((Discrete(3),    # noop, turn left, turn right
                 Discrete(3)))   # noop, forward, backward
  space.key_to_action = key_to_action_basic
  return space


def doom_action_space():
  """MOVE_FORWARD MOVE_BACKWARD MOVE_RIGHT MOVE_LEFT SELECT_NEXT_WEAPON
  SELECT_PREV_WEAPON ATTACK SPEED TURN_LEFT_RIGHT_DELTA."""
  return Tuple((Discrete(3),   # noop, forward, backward
                Discrete(3),   # noop, move right, move left
                Discrete(3),   # noop, next weapon, prev weapon
                Discrete(2),   # noop, attack
                Discrete(2),   # noop, sprint
                Box(-1.0, 1.0, (1,))))


def doom_action_space_discretized():
  return Tuple((Discrete(3), Discrete(3), Discrete(3), Discrete(2),
                Discrete(2),
                Discretized(11, min_action=-10.0, max_action=10.0)))


def doom_action_space_discretized_no_weap():
  return Tuple((Discrete(3), Discrete(3), Discrete(2), Discrete(2),
                Discretized(11, min_action=-10.0, max_action=10.0)))


def doom_action_space_continuous_no_weap():
  return Tuple((Discrete(3), Discrete(3), Discrete(2), Discrete(2),
                Box(-1.0, 1.0, (1,))))


def doom_action_space_discrete():
  return Tuple((Discrete(3), Discrete(3), Discrete(3), Discrete(3),
                Discrete(2), Discrete(2)))


def doom_action_space_discrete_no_weap():
  return Tuple((Discrete(3), Discrete(3), Discrete(3), Discrete(2),
                Discrete(2)))


def doom_action_space_full_discretized(with_use=False):
  """MOVE_FORWARD MOVE_BACKWARD MOVE_RIGHT MOVE_LEFT SELECT_WEAPON1..7
  ATTACK SPEED [USE] TURN_LEFT_RIGHT_DELTA."""
  heads = [Discrete(3),   # noop, forward, backward
           Discrete(3),   # noop, move right, move left
           Discrete(8),   # noop, select weapon 1..7
           Discrete(2),   # noop, attack
           Discrete(2)]   # noop, sprint
  if with_use:
    heads.append(Discrete(2))  # noop, use
  heads.append(Discretized(21, min_action=-12.5, max_action=12.5))
  return Tuple(heads)
