"""DMLab defaults: same as Doom (reference envs/dmlab/dmlab_params.py)."""


def dmlab_override_defaults(env, parser):
  from ..doom.doom_params import doom_override_defaults  # pylint: disable=import-outside-toplevel
  doom_override_defaults(env, parser)
