from .agent import Agent, torso_spec, CORE_SIZE
from . import layers
from .instruction import tokenize, hash_bucket
