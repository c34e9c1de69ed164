"""DeepMind Lab gym env (reference envs/dmlab/)."""
