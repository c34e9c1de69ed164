"""Atari (ALE via gym) factory (reference envs/atari/)."""
