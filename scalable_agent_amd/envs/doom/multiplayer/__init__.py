"""Doom multiplayer: UDP host/join game instances and the multi-agent
wrappers (reference envs/doom/multiplayer/)."""
