"""VizDoom support (reference environments_doom.py + envs/doom/).

Real ViZDoom is used when importable.  This image does not ship it, so
`SA_DOOM_BACKEND=sim` (or cfg.doom_backend='sim') selects the in-tree
`SimDoomGame` test double; without either, constructing a Doom env raises a
clear ImportError.
"""

from .impala_adapter import DOOM_W, DOOM_H, DOOM_ACTION_SET, PyProcessDoom  # noqa
