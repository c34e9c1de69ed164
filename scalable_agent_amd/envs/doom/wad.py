"""Doom WAD files: the lump container and UDMF (TEXTMAP) maps.

The scenario maps of the reference (`envs/doom/scenarios/*.wad`, read by
ViZDoom through `doom_scenario_path` / `doom_map` in each .cfg) are game
assets.  This module lets the framework author its own: a PWAD writer /
reader for the lump directory (12-byte header "PWAD", count, directory
offset; 16-byte entries: offset, size, 8-byte name) and a writer / parser
for ZDoom's text map format (UDMF, `namespace = "zdoom";` with `thing`,
`vertex`, `linedef`, `sidedef` and `sector` blocks), the format most of the
reference's scenario WADs use.  A map is stored as the lumps MAPxx (empty
marker), TEXTMAP, SCRIPTS (ACS source; compiled into BEHAVIOR when an ACS
compiler is available, `tools/doom_build_wads.py --acc`) and ENDMAP.  No
node lumps are written: ZDoom builds the BSP of a UDMF map that has none.

`MapBuilder` assembles maps from closed polygons: rooms (one sector each,
one-sided walls) and pillars (holes cut into the surrounding sector).
"""

import re
import struct

HEADER = struct.Struct('<4sii')
ENTRY = struct.Struct('<ii8s')

# Doom editor numbers used by the scenario builders (and read back by the
# simulator backend, sim_game.py)
PLAYER1_START = 1
DEATHMATCH_START = 11
MONSTERS = {3001: 'DoomImp', 3002: 'Demon', 3004: 'ZombieMan', 9: 'ShotgunGuy',
            3005: 'Cacodemon', 65: 'ChaingunGuy'}
HEALTH_ITEMS = {2011: 'Stimpack', 2012: 'Medikit', 2014: 'HealthBonus'}
ARMOR_ITEMS = {2018: 'GreenArmor', 2019: 'BlueArmor'}
AMMO_ITEMS = {2007: 'Clip', 2008: 'Shell', 2048: 'ClipBox', 2049: 'ShellBox',
              2010: 'RocketAmmo', 2047: 'Cell'}
WEAPON_ITEMS = {2001: 'Shotgun', 82: 'SuperShotgun', 2002: 'Chaingun',
                2003: 'RocketLauncher', 2004: 'PlasmaRifle'}


# --------------------------------------------------------------- container
def write_wad(path, lumps):
  """lumps: sequence of (name, bytes).  Writes a PWAD (data, then the
  directory) atomically enough for a cache (tmp file + rename)."""
  import os
  body = bytearray()
  entries = []
  off = HEADER.size
  for name, data in lumps:
    nm = name.upper().encode('ascii')
    if len(nm) > 8 or not nm:
      raise ValueError('bad lump name %r' % name)
    data = bytes(data)
    entries.append((off if data else 0, len(data), nm.ljust(8, b'\0')))
    body += data
    off += len(data)
  out = bytearray(HEADER.pack(b'PWAD', len(entries), off))
  out += body
  for e in entries:
    out += ENTRY.pack(*e)
  tmp = '%s.%d.tmp' % (path, os.getpid())
  with open(tmp, 'wb') as f:
    f.write(out)
  os.replace(tmp, path)


def read_wad(path):
  """-> list of (name, bytes) in directory order.  Validates the header and
  that every lump lies inside the file."""
  with open(path, 'rb') as f:
    data = f.read()
  if len(data) < HEADER.size:
    raise ValueError('%s: too short for a WAD header' % path)
  ident, n, diro = HEADER.unpack_from(data, 0)
  if ident not in (b'PWAD', b'IWAD'):
    raise ValueError('%s: not a WAD (%r)' % (path, ident))
  if n < 0 or diro < HEADER.size or diro + n * ENTRY.size > len(data):
    raise ValueError('%s: directory out of range' % path)
  lumps = []
  for i in range(n):
    off, size, nm = ENTRY.unpack_from(data, diro + i * ENTRY.size)
    if size < 0 or (size and (off < 0 or off + size > len(data))):
      raise ValueError('%s: lump %d out of range' % (path, i))
    lumps.append((nm.rstrip(b'\0').decode('ascii'), data[off:off + size]))
  return lumps


def map_lumps(lumps, map_name):
  """The lumps of map `map_name` (marker .. ENDMAP or the next marker) as a
  dict name -> bytes; KeyError when the WAD has no such map."""
  names = [n for n, _ in lumps]
  want = map_name.upper()
  if want not in names:
    raise KeyError('map %s not in WAD (maps: %s)' %
                   (want, ', '.join(map_names(lumps))))
  i = names.index(want) + 1
  out = {}
  while i < len(lumps) and lumps[i][0] != 'ENDMAP' and not _is_marker(lumps[i][0]):
    out[lumps[i][0]] = lumps[i][1]
    i += 1
  return out


def _is_marker(name):
  return re.match(r'^(MAP\d\d|E\dM\d)$', name) is not None


def map_names(lumps):
  return [n for n, _ in lumps if _is_marker(n)]


# --------------------------------------------------------------------- UDMF
def _fmt(v):
  if isinstance(v, bool):
    return 'true' if v else 'false'
  if isinstance(v, float):
    return '%.3f' % v
  if isinstance(v, int):
    return str(v)
  return '"%s"' % str(v).replace('\\', '\\\\').replace('"', '\\"')


def udmf_text(m):
  """m: dict with lists 'things', 'vertices', 'linedefs', 'sidedefs',
  'sectors' of field dicts -> TEXTMAP text (namespace zdoom)."""
  out = ['namespace = "zdoom";', '']
  for kind, key in (('thing', 'things'), ('vertex', 'vertices'),
                    ('linedef', 'linedefs'), ('sidedef', 'sidedefs'),
                    ('sector', 'sectors')):
    for i, block in enumerate(m[key]):
      out.append('%s // %d' % (kind, i))
      out.append('{')
      for k, v in block.items():
        out.append('%s = %s;' % (k, _fmt(v)))
      out.append('}')
      out.append('')
  return '\n'.join(out)


_TOKEN = re.compile(r'\s*(//[^\n]*|/\*.*?\*/|"(?:[^"\\]|\\.)*"|[{};=]|[^\s{};=/]+)',
                    re.S)


def _value(tok):
  if tok.startswith('"'):
    return tok[1:-1].replace('\\"', '"').replace('\\\\', '\\')
  low = tok.lower()
  if low in ('true', 'false'):
    return low == 'true'
  try:
    return int(tok, 0)
  except ValueError:
    return float(tok)


def parse_udmf(text):
  """TEXTMAP text -> dict like udmf_text's input (plus 'namespace')."""
  toks = [t for t in (m.group(1) for m in _TOKEN.finditer(text))
          if t and not t.startswith('//') and not t.startswith('/*')]
  kinds = {'thing': 'things', 'vertex': 'vertices', 'linedef': 'linedefs',
           'sidedef': 'sidedefs', 'sector': 'sectors'}
  m = {v: [] for v in kinds.values()}
  m['namespace'] = None
  i = 0
  while i < len(toks):
    t = toks[i]
    if i + 1 < len(toks) and toks[i + 1] == '=':
      # top-level assignment: key = value ;
      if t.lower() == 'namespace':
        m['namespace'] = _value(toks[i + 2])
      i += 4
      continue
    if i + 1 < len(toks) and toks[i + 1] == '{':
      block, i = {}, i + 2
      while toks[i] != '}':
        if toks[i + 1] != '=' or toks[i + 3] != ';':
          raise ValueError('UDMF: malformed field near %r' % toks[i])
        block[toks[i].lower()] = _value(toks[i + 2])
        i += 4
      i += 1
      if t.lower() in kinds:
        m[kinds[t.lower()]].append(block)
      continue
    raise ValueError('UDMF: unexpected token %r' % t)
  return m


# ------------------------------------------------------------------ builder
class MapBuilder(object):
  """Closed-polygon map assembly.

  room(poly, ...) adds a sector bounded by one-sided walls (poly in
  counter-clockwise order); pillar(poly, room) cuts a solid hole out of a
  room (its walls face outwards into the room).  Vertices are shared by
  coordinate."""

  def __init__(self):
    self.m = {'things': [], 'vertices': [], 'linedefs': [], 'sidedefs': [],
              'sectors': []}
    self._vid = {}

  def _vertex(self, x, y):
    key = (float(x), float(y))
    if key not in self._vid:
      self._vid[key] = len(self.m['vertices'])
      self.m['vertices'].append({'x': float(x), 'y': float(y)})
    return self._vid[key]

  def _walls(self, poly, sector, texture, reverse):
    pts = list(poly)[::-1] if reverse else list(poly)
    for a, b in zip(pts, pts[1:] + pts[:1]):
      side = len(self.m['sidedefs'])
      self.m['sidedefs'].append({'sector': sector, 'texturemiddle': texture})
      self.m['linedefs'].append({'v1': self._vertex(*a), 'v2': self._vertex(*b),
                                 'sidefront': side, 'blocking': True})

  def room(self, poly, wall='STARTAN2', floor='FLOOR0_1', ceiling='CEIL1_1',
           floor_h=0, ceiling_h=128, light=192, **sector_fields):
    """poly: counter-clockwise [(x, y), ...].  Doom walls face the sector on
    their right, so the boundary is emitted clockwise.  Returns the sector."""
    sec = len(self.m['sectors'])
    fields = {'heightfloor': int(floor_h), 'heightceiling': int(ceiling_h),
              'texturefloor': floor, 'textureceiling': ceiling,
              'lightlevel': int(light)}
    fields.update(sector_fields)
    self.m['sectors'].append(fields)
    self._walls(poly, sec, wall, reverse=True)
    return sec

  def pillar(self, poly, room_sector, wall='STARTAN2'):
    """A solid column inside `room_sector` (poly counter-clockwise): its
    walls are emitted counter-clockwise so they face the room."""
    self._walls(poly, room_sector, wall, reverse=False)

  def thing(self, x, y, type_, angle=0, tid=0, **fields):
    t = {'x': float(x), 'y': float(y), 'type': int(type_), 'angle': int(angle)}
    if tid:
      t['id'] = int(tid)
    for k in ('skill1', 'skill2', 'skill3', 'skill4', 'skill5', 'single',
              'dm', 'coop'):
      t[k] = True
    t.update(fields)
    self.m['things'].append(t)

  def textmap(self):
    return udmf_text(self.m)


def rect(x0, y0, x1, y1):
  """Counter-clockwise rectangle."""
  return [(x0, y0), (x1, y0), (x1, y1), (x0, y1)]


def map_lump_list(name, textmap, scripts=None, behavior=None):
  lumps = [(name.upper(), b''), ('TEXTMAP', textmap.encode('ascii'))]
  if behavior:
    lumps.append(('BEHAVIOR', behavior))
  if scripts:
    lumps.append(('SCRIPTS', scripts.encode('ascii')))
  lumps.append(('ENDMAP', b''))
  return lumps


def check_map(m):
  """Structural checks of a parsed map; returns a list of problems (empty =
  sound): index ranges, zero-length walls, and that every sector is closed -
  its boundary, the front sides of its lines walked v1 -> v2 and the back
  sides v2 -> v1, enters every vertex as often as it leaves it."""
  import collections
  errs = []
  nv, ns, nsec = len(m['vertices']), len(m['sidedefs']), len(m['sectors'])
  deg = collections.defaultdict(int)  # (sector, vertex) -> out - in
  for i, s in enumerate(m['sidedefs']):
    if not 0 <= s.get('sector', -1) < nsec:
      errs.append('sidedef %d: sector out of range' % i)
  for i, l in enumerate(m['linedefs']):
    v1, v2 = l.get('v1', -1), l.get('v2', -1)
    if not (0 <= v1 < nv and 0 <= v2 < nv):
      errs.append('linedef %d: vertex out of range' % i)
      continue
    if v1 == v2:
      errs.append('linedef %d: zero length' % i)
    for key, a, b in (('sidefront', v1, v2), ('sideback', v2, v1)):
      sd = l.get(key, -1)
      if sd == -1 and key == 'sideback':
        continue
      if not 0 <= sd < ns:
        errs.append('linedef %d: %s out of range' % (i, key))
        continue
      sec = m['sidedefs'][sd].get('sector', -1)
      deg[(sec, a)] += 1
      deg[(sec, b)] -= 1
  bad = sorted(k for k, d in deg.items() if d != 0)
  if bad:
    errs.append('open sector boundary at (sector, vertex) %s' % bad[:8])
  if not any(t.get('type') in (PLAYER1_START, DEATHMATCH_START)
             for t in m['things']):
    errs.append('no player start')
  return errs
