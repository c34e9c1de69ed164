"""`--fault_inject` parsing (tests and drills only).

Spec: comma-separated `kind:value` items:
  env_crash:P    every env step hard-kills the env worker with probability P
                 (exercises the supervisor respawn + dropped-unroll path)
  env_hang:P     every env step hangs the worker with probability P (needs
                 --env_timeout_secs > 0; exercises the hang watchdog)
  actor_stall:MS every actor unroll starts with an MS-millisecond stall
  learner_nan:K  the learner step K (1-based) poisons one gradient with NaN
                 (exercises the non-finite-update guard)
"""


class FaultSpec(object):

  KINDS = ('env_crash', 'env_hang', 'actor_stall', 'learner_nan')

  def __init__(self, spec=''):
    self.spec = spec or ''
    self.values = {}
    for part in filter(None, self.spec.split(',')):
      kind, sep, value = part.partition(':')
      if kind not in self.KINDS or not sep:
        raise ValueError('bad --fault_inject item %r (kinds: %s)' %
                         (part, ', '.join(self.KINDS)))
      self.values[kind] = float(value)

  def get(self, kind, default=0.0):
    return self.values.get(kind, default)

  def env_spec(self):
    """The part forwarded to env workers."""
    return ','.join('%s:%g' % (k, v) for k, v in self.values.items()
                    if k.startswith('env_'))

  def __bool__(self):
    return bool(self.values)
