"""Self-authored Doom scenario WADs (envs/doom/wad.py, scenario_maps.py):
container round trip, UDMF write/parse, map soundness, one WAD per scenario
the table names, and the simulator backend running on them.

Parity with the reference's own WADs is not the claim (they are binary
assets with compiled ACS); the reference UDMF maps are only used, read-only,
to check that the parser reads real ZDoom TEXTMAPs."""
import glob
import os

import numpy as np
import pytest

from scalable_agent_amd.envs.doom import scenario_maps, scenarios
from scalable_agent_amd.envs.doom import wad as W

REF_SCEN = '/root/reference/envs/doom/scenarios'


def test_wad_container_roundtrip(tmp_path):
  lumps = [('MAP01', b''), ('TEXTMAP', b'namespace = "zdoom";'),
           ('SCRIPTS', b'script 1 OPEN {}'), ('ENDMAP', b'')]
  p = str(tmp_path / 'x.wad')
  W.write_wad(p, lumps)
  assert W.read_wad(p) == lumps
  assert W.map_names(W.read_wad(p)) == ['MAP01']
  with open(p, 'rb') as f:
    assert f.read(4) == b'PWAD'
  with pytest.raises(ValueError):
    W.write_wad(p, [('TOOLONGNAME', b'')])
  bad = tmp_path / 'bad.wad'
  bad.write_bytes(b'XWAD' + b'\0' * 8)
  with pytest.raises(ValueError, match='not a WAD'):
    W.read_wad(str(bad))


def test_udmf_roundtrip_and_checks():
  b = W.MapBuilder()
  sec = b.room(W.rect(0, 0, 512, 256), light=160, damageamount=5)
  b.pillar(W.rect(200, 100, 260, 160), sec)
  b.thing(32, 32, W.PLAYER1_START, angle=90, tid=7)
  m = W.parse_udmf(b.textmap())
  assert m['namespace'] == 'zdoom'
  assert len(m['vertices']) == 8 and len(m['linedefs']) == 8
  assert m['sectors'][0]['damageamount'] == 5
  assert m['things'][0]['type'] == 1 and m['things'][0]['id'] == 7
  assert m['things'][0]['angle'] == 90 and m['things'][0]['single'] is True
  assert W.check_map(m) == []
  # an open boundary and a dangling index are reported
  m['linedefs'].pop()
  assert any('open sector boundary' in e for e in W.check_map(m))
  m['linedefs'].append({'v1': 0, 'v2': 99, 'sidefront': 0})
  assert any('vertex out of range' in e for e in W.check_map(m))


def test_room_walls_face_inwards():
  # Doom's front side is on the right of v1 -> v2: for a room the interior
  # must be on the right of every wall, for a pillar the room must be
  b = W.MapBuilder()
  sec = b.room(W.rect(0, 0, 100, 100))
  b.pillar(W.rect(40, 40, 60, 60), sec)
  m = W.parse_udmf(b.textmap())
  vx = [(v['x'], v['y']) for v in m['vertices']]
  for i, l in enumerate(m['linedefs']):
    (x1, y1), (x2, y2) = vx[l['v1']], vx[l['v2']]
    mx, my = (x1 + x2) / 2, (y1 + y2) / 2
    # a point just to the right of the wall
    rx, ry = mx + (y2 - y1) * 0.01, my - (x2 - x1) * 0.01
    in_room = 0 < rx < 100 and 0 < ry < 100
    in_pillar = 40 < rx < 60 and 40 < ry < 60
    assert in_room and not in_pillar, i


def test_every_scenario_wad_is_built_and_sound(tmp_path):
  needed = {s.wad for s in scenarios.SCENARIOS.values()}
  assert needed <= set(scenario_maps.BUILDERS)
  paths = scenario_maps.build_all(str(tmp_path))
  assert len(paths) == len(scenario_maps.BUILDERS)
  for p in paths:
    lumps = W.read_wad(p)
    maps = W.map_names(lumps)
    assert maps and maps[0] == 'MAP01', p
    for mn in maps:
      ml = W.map_lumps(lumps, mn)
      assert 'TEXTMAP' in ml and 'SCRIPTS' in ml, (p, mn)
      m = W.parse_udmf(ml['TEXTMAP'].decode())
      assert W.check_map(m) == [], (p, mn)
  # deterministic: the same bytes on a second build
  again = scenario_maps.build_all(str(tmp_path / 'b'))
  for a, b in zip(paths, again):
    with open(a, 'rb') as fa, open(b, 'rb') as fb:
      assert fa.read() == fb.read()


@pytest.mark.skipif(not os.path.isdir(REF_SCEN), reason='reference not present')
def test_parser_reads_reference_udmf_maps():
  n = 0
  for p in sorted(glob.glob(os.path.join(REF_SCEN, '*.wad'))):
    lumps = W.read_wad(p)
    for mn in W.map_names(lumps):
      ml = W.map_lumps(lumps, mn)
      if 'TEXTMAP' not in ml:
        continue  # binary (Hexen-format) map
      m = W.parse_udmf(ml['TEXTMAP'].decode('latin1'))
      assert m['namespace'] == 'zdoom' and m['vertices'] and m['things']
      n += 1
  assert n >= 5


def test_wad_path_falls_back_to_generated(monkeypatch, tmp_path):
  monkeypatch.setenv('SA_DOOM_SCENARIOS_DIR', str(tmp_path / 'empty'))
  p = scenarios.wad_path('health_gathering.wad')
  assert os.path.exists(p) and W.map_names(W.read_wad(p)) == ['MAP01']
  # a user directory holding the file wins
  user = tmp_path / 'user'
  user.mkdir()
  (user / 'basic.wad').write_bytes(open(scenarios.wad_path('basic.wad'), 'rb').read())
  monkeypatch.setenv('SA_DOOM_SCENARIOS_DIR', str(user))
  assert scenarios.wad_path('basic.wad') == str(user / 'basic.wad')


def _sim(cfg_name, tmp_path, **args):
  from scalable_agent_amd.envs.doom.sim_game import SimDoomGame
  sc = scenarios.SCENARIOS[cfg_name]
  g = SimDoomGame()
  g.load_config(sc.write_cfg(str(tmp_path)))
  for a in args.get('game_args', ()):
    g.add_game_args(a)
  g.set_seed(3)
  g.init()
  return g


def test_sim_runs_on_the_scenario_maps(monkeypatch, tmp_path):
  monkeypatch.setenv('SA_DOOM_SCENARIOS_DIR', str(tmp_path / 'none'))
  g = _sim('basic.cfg', tmp_path)
  assert g.map_loaded
  # basic: one room 512 x 448, player start at (64, 224) facing east
  np.testing.assert_allclose(g._lo, [0, 0])
  np.testing.assert_allclose(g._hi, [512, 448])
  np.testing.assert_allclose(g._pos, [64, 224])
  assert g._angle == 0
  g = _sim('deadly_corridor.cfg', tmp_path)
  assert len(g._monsters) == 6           # the six alcove gunners
  g = _sim('health_gathering.cfg', tmp_path)
  assert g._floor_damage == 5 and len(g._medkits) == 16
  h0 = g._health
  for _ in range(64):
    g.make_action([0, 0, 0])
  assert g._health < h0                  # the floor hurts
  g = _sim('two_colors_hard.cfg', tmp_path)
  assert len(g._poison_items) == 10 and len(g._medkits) == 10
  g = _sim('dwango5_dm.cfg', tmp_path, game_args=('-host 2',))
  dm = {tuple(map(float, p)) for p, _ in g._starts}
  assert len(dm) == 8                    # deathmatch starts in multiplayer
  assert tuple(map(float, g._pos)) in dm
  for _ in range(20):
    g.make_action([0] * g.get_available_buttons_size())
  st = g.get_state()
  assert st.screen_buffer.shape[0] == 3
