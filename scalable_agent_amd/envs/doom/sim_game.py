"""`SimDoomGame`: a small stand-in for `vizdoom.DoomGame`.

ViZDoom is not installed in this image (and the GPU boxes have no network),
so the Doom stack - action conversion, game-variable parsing, every wrapper,
the multiplayer/bot logic and the IMPALA adaptor - would otherwise be
untestable.  This module implements the subset of the DoomGame API that
`doom_gym.VizdoomEnv` uses, on top of a tiny 2D arena with a column-projected
first-person view:

  * buttons are read from the cfg's `available_buttons` in order and act on
    the player (move/strafe/turn/turn-delta/attack/speed/weapon select/use);
  * `available_game_variables` are produced in cfg order (position, angle,
    health, armor, weapons/ammo, kill/frag/death/hit/damage counters,
    player counts and per-player frags for multiplayer);
  * rewards: living_reward per tic, the scenario's kill reward, death
    penalty; episodes end on death (single player) or `episode_timeout`;
  * `screen_buffer` is [3, H, W] uint8 (CRCGCB) at the set resolution;
  * the map comes from the cfg's `doom_scenario_path` / `doom_map` when that
    WAD holds a UDMF map (the self-authored scenario WADs of
    scenario_maps.py, or any TEXTMAP WAD): the arena is its bounding box, the
    player spawns at its player / deathmatch starts, its monsters and health
    pickups are the ones the episode starts with, and a damaging floor
    (sector `damageamount`) hurts every 32 tics; without a readable map a
    1024 x 1024 arena with random monsters and medikits is used.

It is selected with `SA_DOOM_BACKEND=sim` (or `doom_gym.doom_backend('sim')`);
real ViZDoom is used whenever it is importable and not overridden.  It is a
test double for the framework plumbing, not a Doom reimplementation.
"""

import math
import os
import re

import numpy as np

from . import wad as wadlib
from .scenarios import parse_cfg

RESOLUTIONS = ['160x120', '200x125', '200x150', '256x144', '256x160',
               '256x192', '320x180', '320x200', '320x240', '320x256',
               '400x225', '400x250', '400x300', '512x288', '512x320',
               '512x384', '640x360', '640x400', '640x480', '800x450',
               '800x500', '800x600', '1024x576', '1024x640', '1024x768',
               '1280x720', '1280x800', '1280x960', '1280x1024', '1400x787',
               '1400x875', '1400x1050', '1600x900', '1600x1000', '1600x1200',
               '1920x1080']


class ScreenResolution(object):
  pass


for _r in RESOLUTIONS:
  setattr(ScreenResolution, 'RES_' + _r.upper(), 'RES_' + _r.upper())


class Mode(object):
  PLAYER, SPECTATOR, ASYNC_PLAYER, ASYNC_SPECTATOR = range(4)


class AutomapMode(object):
  NORMAL, WHOLE, OBJECTS, OBJECTS_WITH_SIZE = range(4)


class GameState(object):

  def __init__(self, number, screen_buffer, game_variables):
    self.number = number
    self.screen_buffer = screen_buffer
    self.game_variables = game_variables
    self.automap_buffer = None
    self.depth_buffer = None
    self.labels_buffer = None


def _res_wh(res):
  m = re.match(r'RES_(\d+)X(\d+)', str(res))
  return (int(m.group(1)), int(m.group(2))) if m else (640, 480)


ARENA = 1024.0
FOV = math.radians(90.0)


class SimDoomGame(object):
  """See module docstring."""

  def __init__(self):
    self._cfg = {}
    self._buttons = []
    self._vars = []
    self._res = 'RES_640X480'
    self._seed = 0
    self._args = []
    self._initialized = False
    self._finished = True
    self._last_reward = 0.0
    self._pending_action = None
    self._bots = 0
    self._max_players = 1
    self._player_number = 1

  # -- configuration -------------------------------------------------------
  def load_config(self, path):
    with open(path) as f:
      self._cfg = parse_cfg(f.read())
    self._buttons = list(self._cfg.get('available_buttons', []))
    self._vars = list(self._cfg.get('available_game_variables', []))
    if 'screen_resolution' in self._cfg:
      self._res = self._cfg['screen_resolution']
    return True

  def set_screen_resolution(self, res):
    self._res = res

  def set_seed(self, seed):
    self._seed = int(seed)

  def set_window_visible(self, visible):
    pass

  def set_mode(self, mode):
    pass

  def set_automap_buffer_enabled(self, enabled):
    pass

  def set_automap_mode(self, mode):
    pass

  def set_automap_rotate(self, rotate):
    pass

  def set_automap_render_textures(self, textures):
    pass

  def add_game_args(self, args):
    self._args.append(args)
    m = re.search(r'-host (\d+)', args)
    if m:
      self._max_players = int(m.group(1))
    m = re.search(r'\+name AI(\d+)', args)
    if m:
      self._player_number = int(m.group(1)) + 1
      self._max_players = max(self._max_players, self._player_number)

  def get_available_buttons_size(self):
    return len(self._buttons)

  def get_available_game_variables_size(self):
    return len(self._vars)

  def init(self):
    self._rng = np.random.RandomState(self._seed % (2 ** 32))
    self._timeout = int(self._cfg.get('episode_timeout', 2100))
    self._living = float(self._cfg.get('living_reward', 0))
    self._death_penalty = float(self._cfg.get('death_penalty', 0))
    self._kill_reward = 1.0
    self._load_map()
    self._initialized = True
    self._deaths = 0
    self.new_episode()
    return True

  def close(self):
    self._initialized = False

  def _load_map(self):
    """Arena, starts, monsters, pickups and floor damage of the cfg's map
    (see the module docstring); None fields = the default arena."""
    self._lo = np.zeros(2)
    self._hi = np.full(2, ARENA)
    self._starts = []
    self._map_monsters = None
    self._map_medkits = None
    self._poison = np.zeros((0, 2))
    self._floor_damage = 0.0
    self.map_loaded = False
    path = self._cfg.get('doom_scenario_path')
    if not path:
      return
    try:
      lumps = wadlib.read_wad(path)
      ml = wadlib.map_lumps(lumps, self._cfg.get('doom_map', 'map01'))
      m = wadlib.parse_udmf(ml['TEXTMAP'].decode('latin1'))
    except (OSError, ValueError, KeyError):
      return  # binary-format or missing map: the default arena
    vx = np.array([[v['x'], v['y']] for v in m['vertices']], np.float64)
    if len(vx) < 3:
      return
    self._lo, self._hi = vx.min(0), vx.max(0)
    things = m['things']

    def pos(types):
      return np.array([[t['x'], t['y']] for t in things if t.get('type') in types],
                      np.float64).reshape(-1, 2)
    multi = self._max_players > 1 or self._bots > 0
    starts = pos({wadlib.DEATHMATCH_START} if multi else {wadlib.PLAYER1_START})
    if not len(starts):
      starts = pos({wadlib.PLAYER1_START, wadlib.DEATHMATCH_START})
    self._starts = [(p, next((t.get('angle', 0) for t in things
                              if (t['x'], t['y']) == tuple(p)), 0)) for p in starts]
    mons = pos(set(wadlib.MONSTERS))
    self._map_monsters = mons if len(mons) else None
    # two-colour scenarios: stimpacks are the poison pickups
    poison = 'two_colors' in os.path.basename(path)
    heal = set(wadlib.HEALTH_ITEMS) - ({2011} if poison else set())
    meds = pos(heal)
    self._map_medkits = meds if len(meds) else None
    if poison:
      self._poison = pos({2011})
    self._floor_damage = float(max((sec.get('damageamount', 0)
                                    for sec in m['sectors']), default=0))
    self.map_loaded = True

  def _uniform(self, rng, n, margin=50.0):
    return rng.uniform(self._lo + margin, self._hi - margin, size=(n, 2))

  # -- episode ---------------------------------------------------------------
  def new_episode(self, recording_path=''):
    del recording_path
    rng = self._rng
    self._tic = 0
    self._finished = False
    if self._starts:
      p, a = self._starts[rng.randint(len(self._starts))]
      self._pos = np.array(p, np.float64)
      self._angle = float(a)
    else:
      self._pos = self._uniform(rng, 1, 200.0)[0]
      self._angle = rng.uniform(0, 360)
    self._health = 100.0
    self._armor = 0.0
    self._weapons = np.zeros(10)
    self._weapons[1] = self._weapons[2] = 1
    self._ammo = np.zeros(10)
    self._ammo[2] = 50
    self._selected = 2
    self._kills = 0.0
    self._hits = 0.0
    self._damage = 0.0
    self._cooldown = 0
    self._dead = False
    self._monsters = (self._map_monsters.copy() if self._map_monsters is not None
                      else self._uniform(rng, 8))
    self._medkits = (self._map_medkits.copy() if self._map_medkits is not None
                     else self._uniform(rng, 6))
    self._poison_items = self._poison.copy()
    self._bot_frags = np.zeros(9)

  def is_episode_finished(self):
    return self._finished

  def is_player_dead(self):
    return self._dead

  def get_episode_time(self):
    return self._tic

  def get_last_reward(self):
    return self._last_reward

  def send_game_command(self, cmd):
    if cmd.startswith('removebots'):
      self._bots = 0
    elif cmd.startswith('addbot'):
      self._bots += 1

  def replay_episode(self, path):
    raise NotImplementedError('demo replay needs real ViZDoom')

  # -- actions ---------------------------------------------------------------
  def _apply_buttons(self, action):
    a = list(action) + [0] * (len(self._buttons) - len(action))
    speed = 1.0
    move = np.zeros(2)
    turn = 0.0
    attack = False
    for name, v in zip(self._buttons, a):
      if not v:
        continue
      if name == 'MOVE_FORWARD':
        move[0] += 1
      elif name == 'MOVE_BACKWARD':
        move[0] -= 1
      elif name == 'MOVE_RIGHT':
        move[1] -= 1
      elif name == 'MOVE_LEFT':
        move[1] += 1
      elif name == 'TURN_LEFT':
        turn += 6.0
      elif name == 'TURN_RIGHT':
        turn -= 6.0
      elif name == 'TURN_LEFT_RIGHT_DELTA':
        turn -= float(v)
      elif name == 'SPEED':
        speed = 2.0
      elif name == 'ATTACK':
        attack = True
      elif name.startswith('SELECT_WEAPON'):
        w = int(name[len('SELECT_WEAPON'):])
        if self._weapons[w] > 0:
          self._selected = w
      elif name == 'SELECT_NEXT_WEAPON':
        self._selected = self._selected % 7 + 1
      elif name == 'SELECT_PREV_WEAPON':
        self._selected = (self._selected - 2) % 7 + 1
    return move, turn, speed, attack

  def _tick(self, move, turn, speed, attack):
    rng = self._rng
    self._angle = (self._angle + turn) % 360.0
    th = math.radians(self._angle)
    fwd = np.array([math.cos(th), math.sin(th)])
    left = np.array([-math.sin(th), math.cos(th)])
    self._pos = np.clip(self._pos + 8.0 * speed * (move[0] * fwd +
                                                   move[1] * left),
                        self._lo + 16, self._hi - 16)
    reward = self._living
    # monsters drift towards the player and bite when close
    d = self._pos[None] - self._monsters
    dist = np.linalg.norm(d, axis=1) + 1e-6
    self._monsters += 2.0 * d / dist[:, None]
    close = dist < 64
    if close.any():
      dmg = 1.0 * close.sum()
      self._health -= dmg
    # medkits
    dm = np.linalg.norm(self._medkits - self._pos[None], axis=1)
    for i in np.nonzero(dm < 40)[0]:
      self._health = min(100.0, self._health + 25.0)
      self._medkits[i] = self._uniform(rng, 1)[0]
    if len(self._poison_items):
      dp = np.linalg.norm(self._poison_items - self._pos[None], axis=1)
      for i in np.nonzero(dp < 40)[0]:
        self._health -= 25.0
        self._poison_items[i] = self._uniform(rng, 1)[0]
    if self._floor_damage and self._tic % 32 == 31:
      self._health -= self._floor_damage
    self._cooldown = max(0, self._cooldown - 1)
    if attack and self._cooldown == 0 and self._ammo[self._selected] > 0:
      self._cooldown = 4
      self._ammo[self._selected] -= 1
      rel = self._monsters - self._pos[None]
      ang = np.degrees(np.arctan2(rel[:, 1], rel[:, 0])) - self._angle
      ang = (ang + 180.0) % 360.0 - 180.0
      rd = np.linalg.norm(rel, axis=1)
      hit = np.nonzero((np.abs(ang) < 8.0) & (rd < 600))[0]
      if len(hit):
        j = hit[np.argmin(rd[hit])]
        self._hits += 1
        self._damage += 20
        self._kills += 1
        reward += self._kill_reward
        self._monsters[j] = self._uniform(rng, 1)[0]
        if rng.rand() < 0.5:
          self._ammo[self._selected] += 5
    if self._bots and rng.rand() < 0.002 * self._bots:
      self._bot_frags[rng.randint(1, 1 + min(self._bots, 8))] += 1
    self._tic += 1
    if self._health <= 0:
      self._dead = True
      self._deaths += 1
      reward -= self._death_penalty
      if self._max_players > 1 or self._bots > 0:
        self._health = 100.0   # multiplayer: respawn
        self._dead = False
      else:
        self._finished = True
    if self._tic >= self._timeout:
      self._finished = True
    return reward

  def make_action(self, action, tics=1):
    move, turn, speed, attack = self._apply_buttons(action)
    r = 0.0
    for _ in range(max(1, int(tics))):
      if self._finished:
        break
      r += self._tick(move, turn, speed, attack)
    self._last_reward = r
    return r

  def set_action(self, action):
    self._pending_action = list(action)

  def advance_action(self, tics=1, update_state=True):
    del update_state
    self.make_action(self._pending_action or [0] * len(self._buttons), tics)

  # -- observation -----------------------------------------------------------
  def _variables(self):
    frag = self._kills if (self._max_players > 1 or self._bots) else 0.0
    v = {'POSITION_X': self._pos[0], 'POSITION_Y': self._pos[1],
         'ANGLE': self._angle, 'HEALTH': self._health, 'ARMOR': self._armor,
         'SELECTED_WEAPON': self._selected,
         'SELECTED_WEAPON_AMMO': self._ammo[self._selected],
         'USER2': self._kills, 'FRAGCOUNT': frag,
         'DEATHCOUNT': self._deaths, 'HITCOUNT': self._hits,
         'DAMAGECOUNT': self._damage, 'DEAD': float(self._dead),
         'ATTACK_READY': float(self._cooldown == 0),
         'PLAYER_NUMBER': self._player_number,
         'PLAYER_COUNT': max(self._max_players, 1) + self._bots,
         'KILLCOUNT': self._kills}
    for i in range(10):
      v['WEAPON%d' % i] = self._weapons[i]
      v['AMMO%d' % i] = self._ammo[i]
    for i in range(1, 10):
      v['PLAYER%d_FRAGCOUNT' % i] = (frag if i == self._player_number
                                     else self._bot_frags[i - 1])
    return np.array([v.get(name, 0.0) for name in self._vars], np.float64)

  def _render(self):
    w, h = _res_wh(self._res)
    img = np.empty((3, h, w), np.uint8)
    horizon = h // 2
    sky = np.linspace(40, 110, horizon, dtype=np.float32)
    floor = np.linspace(70, 140, h - horizon, dtype=np.float32)
    img[0, :horizon] = sky[:, None].astype(np.uint8)
    img[1, :horizon] = (sky[:, None] * 0.8).astype(np.uint8)
    img[2, :horizon] = (sky[:, None] * 1.2).clip(0, 255).astype(np.uint8)
    img[:, horizon:] = floor[None, :, None].astype(np.uint8)
    cols = np.arange(w)
    ray = self._angle + np.degrees(FOV) * (0.5 - (cols + 0.5) / w)
    for objs, color in ((self._monsters, (200, 40, 40)),
                        (self._medkits, (40, 200, 60)),
                        (self._poison_items, (200, 60, 200))):
      rel = objs - self._pos[None]
      dist = np.linalg.norm(rel, axis=1) + 1e-3
      ang = np.degrees(np.arctan2(rel[:, 1], rel[:, 0]))
      for a, dd in sorted(zip(ang, dist), key=lambda t: -t[1]):
        off = (ray - a + 180.0) % 360.0 - 180.0
        half_w = np.degrees(math.atan2(24.0, dd))
        mask = np.abs(off) < half_w
        if not mask.any():
          continue
        half_h = int(min(horizon, 32.0 * h / dd))
        for c in range(3):
          img[c, horizon - half_h:horizon + half_h, mask] = int(
              color[c] * min(1.0, 200.0 / dd + 0.3))
    return img

  def get_state(self):
    if self._finished:
      return None
    return GameState(self._tic, self._render(), self._variables())
