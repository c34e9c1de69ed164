"""VizDoom support (reference environments_doom.py + envs/doom/).

ViZDoom is not installed in this image; everything here imports it lazily
and raises a clear ImportError when an env is actually constructed.
"""

from .impala_adapter import DOOM_W, DOOM_H, DOOM_ACTION_SET, PyProcessDoom  # noqa
