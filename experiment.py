#!/usr/bin/env python3
"""CLI entry point with the reference's invocation: `python experiment.py
--level_name=... --num_actors=... --batch_size=...` (see
scalable_agent_amd/experiment.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from scalable_agent_amd.experiment import main  # noqa: E402

if __name__ == '__main__':
  main()
