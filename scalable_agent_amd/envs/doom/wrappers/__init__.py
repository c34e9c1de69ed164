"""Doom gym wrappers (reference envs/doom/wrappers/)."""
