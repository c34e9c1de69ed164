"""Minimal nested-structure utilities (the reference uses tf.contrib nest).

Supports tuples, namedtuples, lists and dicts (sorted keys); everything else
is a leaf.  `None` is a leaf too.
"""


def _is_namedtuple(x):
  return isinstance(x, tuple) and hasattr(x, '_fields')


def is_sequence(x):
  return isinstance(x, (tuple, list, dict))


def flatten(structure):
  out = []

  def rec(s):
    if isinstance(s, dict):
      for k in sorted(s):
        rec(s[k])
    elif isinstance(s, (tuple, list)):
      for e in s:
        rec(e)
    else:
      out.append(s)

  rec(structure)
  return out


def pack_sequence_as(structure, flat):
  flat = list(flat)
  it = iter(flat)

  def rec(s):
    if isinstance(s, dict):
      return {k: rec(s[k]) for k in sorted(s)}
    if _is_namedtuple(s):
      return type(s)(*[rec(e) for e in s])
    if isinstance(s, tuple):
      return tuple(rec(e) for e in s)
    if isinstance(s, list):
      return [rec(e) for e in s]
    return next(it)

  out = rec(structure)
  rest = list(it)
  if rest:
    raise ValueError('pack_sequence_as: %d leftover elements' % len(rest))
  return out


def map_structure(fn, *structures):
  flats = [flatten(s) for s in structures]
  n = len(flats[0])
  for f in flats[1:]:
    if len(f) != n:
      raise ValueError('structures have different numbers of leaves')
  return pack_sequence_as(structures[0], [fn(*xs) for xs in zip(*flats)])
