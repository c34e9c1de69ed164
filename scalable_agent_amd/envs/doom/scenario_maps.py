"""Self-authored Doom scenario maps for every WAD the scenario table names.

The reference ships its scenario WADs (`envs/doom/scenarios/*.wad`) as
binary game assets; this module builds this framework's own version of each
one from the scenario's description, as UDMF maps (wad.py) plus the ACS
source of the scenario rules:

  basic             one room; a monster appears at a random spot on the far
                    wall; killing it pays, every shot costs
  deadly_corridor   a long corridor with gunners in side alcoves and armor at
                    the far end; reward for progress towards the armor
  health_gathering  a square room with a damaging floor; medikits keep
                    spawning and are the only way to survive
  two_colors_*      a room with good (medikit) and bad (stimpack = poison)
                    pickups; hard = more bad ones and a harsher floor
  battle / D3_battle, battle2 / D4_battle2 / D4_battle
                    arenas with pillars, respawning monsters, ammo and health
                    (D4 / battle2: larger, more pillars and monsters)
  cig, dwango5, ssl2, freedm
                    deathmatch arenas: 8 deathmatch starts, weapons, ammo,
                    armor and health (cig: MAP01-MAP02, dwango5: MAP01-MAP04)

`build_all(directory)` writes every WAD (idempotent; `ensure_wads` caches
them per user).  The simulator backend (sim_game.py) reads the maps - room
bounds, player / deathmatch starts, monsters, pickups and floor damage - so
the Doom stack runs on them without ViZDoom.  For real ViZDoom the SCRIPTS
lumps must be compiled into BEHAVIOR with ZDoom's ACS compiler
(`tools/doom_build_wads.py --acc /path/to/acc`); without BEHAVIOR the maps
load but the scenario scripts (rewards beyond the .cfg's living reward and
death penalty, respawns) do not run.
"""

import os
import subprocess
import tempfile

import numpy as np

from . import wad as W

_ACS_HEAD = '#include "zcommon.acs"\n\nglobal int 0:reward;\nglobal int 1:shaping_reward;\n\n'


# ------------------------------------------------------------------ basic
def _basic():
  b = W.MapBuilder()
  b.room(W.rect(0, 0, 512, 448), wall='BRICK9', floor='FLOOR0_1',
         ceiling='FLAT4', ceiling_h=104, light=210)
  b.thing(64, 224, W.PLAYER1_START, angle=0, tid=100)
  acs = _ACS_HEAD + """// basic: shoot the monster that appears on the far wall.
// Rules (the scenario's published reward): +106 when it dies (the episode
// ends), -5 per shot fired, -1 per tic from the .cfg's living_reward.

#define MONSTER 10

script "basic_setup" OPEN
{
    reward = 0;
    // one motionless, one-hit Cacodemon at a random height on the east wall
    Spawn("Cacodemon", 448.0, Random(32.0, 416.0), 0.0, MONSTER, 128);
    SetActorProperty(MONSTER, APROP_Speed, 0);
    SetActorProperty(MONSTER, APROP_Health, 1);
    SetThingSpecial(MONSTER, ACS_NamedExecuteAlways, "basic_kill");
}

script "basic_player" ENTER
{
    TakeInventory("Fist", 1);
    int clips = CheckInventory("Clip");
    for (;;)
    {
        // every clip spent since the last tic is a shot
        int now = CheckInventory("Clip");
        reward -= 5.0 * (clips - now);
        clips = now;
        Delay(1);
    }
}

script "basic_kill" (void)
{
    reward += 106.0;
    Exit_Normal(0);
}
"""
  return {'MAP01': (b, acs)}


# -------------------------------------------------------- deadly_corridor
def _deadly_corridor():
  b = W.MapBuilder()
  L, Wd = 1536, 128
  # the corridor and, on both sides, alcoves holding the gunners
  poly = [(0, 0)]
  for x0 in (320, 704, 1088):
    poly += [(x0, 0), (x0, -96), (x0 + 128, -96), (x0 + 128, 0)]
  poly += [(L, 0), (L, Wd)]
  for x0 in (1088, 704, 320):
    poly += [(x0 + 128, Wd), (x0 + 128, Wd + 96), (x0, Wd + 96), (x0, Wd)]
  poly += [(0, Wd)]
  b.room(poly, wall='STONE2', floor='FLOOR4_8', ceiling='CEIL3_5',
         ceiling_h=128, light=176)
  b.thing(32, 64, W.PLAYER1_START, angle=0, tid=100)
  for i, x0 in enumerate((320, 704, 1088)):
    b.thing(x0 + 64, -48, 9 if i else 3004, angle=90, tid=20 + 2 * i)
    b.thing(x0 + 64, Wd + 48, 3004 if i else 9, angle=270, tid=21 + 2 * i)
  b.thing(L - 48, 64, 2018, tid=30)
  acs = _ACS_HEAD + """int goal_x = 1488.0;

script "dc_setup" OPEN
{
    reward = 0;
    shaping_reward = 0;
}

// reward = progress towards the armor (x distance travelled this tic)
script "dc_player" ENTER
{
    int last_x = GetActorX(0);
    while (true)
    {
        int x = GetActorX(0);
        reward = reward + (x - last_x);
        last_x = x;
        if (x >= goal_x)
        {
            reward = reward + 100.0;
            Exit_Normal(0);
        }
        delay(1);
    }
}
"""
  return {'MAP01': (b, acs)}


# ------------------------------------------------------- health_gathering
def _pickup_room(size, n_good, n_bad, damage, seed, wall, floor):
  b = W.MapBuilder()
  b.room(W.rect(0, 0, size, size), wall=wall, floor=floor, ceiling='CEIL4_1',
         ceiling_h=104, light=210, damageamount=damage, damageinterval=32)
  b.thing(size / 2, size / 2, W.PLAYER1_START, angle=0, tid=100)
  rng = np.random.RandomState(seed)
  for _ in range(n_good):
    x, y = rng.uniform(32, size - 32, size=2)
    b.thing(round(x), round(y), 2012, tid=111)
  for _ in range(n_bad):
    x, y = rng.uniform(32, size - 32, size=2)
    b.thing(round(x), round(y), 2011, tid=112)
  return b


def _health_gathering():
  size = 1216
  b = _pickup_room(size, 16, 0, 5, 1, 'GSTONE1', 'NUKAGE1')
  acs = _ACS_HEAD + """// health_gathering: the floor hurts; medikits (tid 111) are the only
// healing.  The map starts with 16 of them; one more appears every 30 tics.
// shaping_reward (USER1) counts +100 per medikit picked up.

#define MEDIKIT 111

function void drop_medikit(void)
{
    // retry until the spot is free
    int ok = 0;
    while (!ok)
        ok = Spawn("Medikit", Random(32.0, 1184.0), Random(32.0, 1184.0), 20.0, MEDIKIT);
    SetThingSpecial(MEDIKIT, ACS_NamedExecuteAlways, "hg_pickup");
}

script "hg_setup" OPEN
{
    reward = 0;
    shaping_reward = 0;
    SetThingSpecial(MEDIKIT, ACS_NamedExecuteAlways, "hg_pickup");
    for (;;)
    {
        Delay(30);
        drop_medikit();
    }
}

script "hg_player" ENTER
{
    ClearInventory();
}

script "hg_pickup" (void)
{
    shaping_reward += 100.0;
}
"""
  return {'MAP01': (b, acs)}


def _two_colors(hard):
  size = 1024
  b = _pickup_room(size, 10 if hard else 12, 10 if hard else 4,
                   8 if hard else 4, 2 + hard, 'BROWN1', 'FLOOR7_1')
  acs = _ACS_HEAD + """int good_tid = 111;
int bad_tid = 112;

// medikits heal; stimpacks are poison in this scenario
script "tc_setup" OPEN
{
    reward = 0;
    SetThingSpecial(good_tid, ACS_NamedExecuteAlways, "tc_good");
    SetThingSpecial(bad_tid, ACS_NamedExecuteAlways, "tc_bad");
}

script "tc_player" ENTER
{
    ClearInventory();
}

script "tc_good" (void)
{
    shaping_reward += 100.0;
}

script "tc_bad" (void)
{
    DamageThing(%d);
    shaping_reward -= 100.0;
}
""" % (40 if hard else 25)
  return {'MAP01': (b, acs)}


# ------------------------------------------------------------------ battle
def _arena(size, pillars, monsters, items, seed, wall, floor, dm=False):
  b = W.MapBuilder()
  sec = b.room(W.rect(0, 0, size, size), wall=wall, floor=floor,
               ceiling='CEIL5_1', ceiling_h=160, light=176)
  rng = np.random.RandomState(seed)
  step = size / (pillars + 1)
  for i in range(pillars):
    for j in range(pillars):
      cx, cy = step * (i + 1), step * (j + 1)
      h = 48
      b.pillar(W.rect(cx - h, cy - h, cx + h, cy + h), sec, wall=wall)

  def free_spot():
    while True:
      x, y = rng.uniform(48, size - 48, size=2)
      if all(abs(x - step * (i + 1)) > 80 or abs(y - step * (j + 1)) > 80
             for i in range(pillars) for j in range(pillars)):
        return round(x), round(y)

  if dm:
    for k in range(8):
      x, y = free_spot()
      b.thing(x, y, W.DEATHMATCH_START, angle=45 * k)
    x, y = free_spot()
    b.thing(x, y, W.PLAYER1_START)
  else:
    b.thing(size / 2, 64, W.PLAYER1_START, angle=90, tid=100)
  for t in monsters:
    x, y = free_spot()
    b.thing(x, y, t, angle=int(rng.randint(0, 8)) * 45, tid=50)
  for t in items:
    x, y = free_spot()
    b.thing(x, y, t)
  return b


_BATTLE_ACS = _ACS_HEAD + """global int 2:kills;  // ViZDoom's USER2

int monster_tid = 50;

// kills count into USER2; a dead monster comes back after a while
script "battle_setup" OPEN
{
    reward = 0;
    kills = 0;
    SetThingSpecial(monster_tid, ACS_NamedExecuteAlways, "battle_kill");
}

script "battle_player" ENTER
{
    ClearInventory();
    GiveInventory("Pistol", 1);
    GiveInventory("Clip", 50);
}

script "battle_kill" (void)
{
    reward = reward + 1.0;
    kills = kills + 1;
    delay(105);
    Thing_Spawn(monster_tid, 0, 0, monster_tid);
}
"""


def _battle(large):
  if large:
    b = _arena(2304, 4, [3001] * 6 + [3002] * 4 + [3004] * 4 + [9] * 2,
               [2007] * 8 + [2012] * 6 + [2008] * 4 + [2001], 7, 'STONE3',
               'FLOOR5_1')
  else:
    b = _arena(1536, 2, [3001] * 4 + [3002] * 3 + [3004] * 3,
               [2007] * 6 + [2012] * 4, 5, 'STARTAN2', 'FLOOR0_1')
  return {'MAP01': (b, _BATTLE_ACS)}


# -------------------------------------------------------------- deathmatch
_DM_ITEMS = ([2001, 82, 2002, 2003, 2004] + [2007, 2008, 2048, 2049, 2010, 2047] * 2 +
             [2018, 2019] + [2012] * 4 + [2011] * 4)

_DM_ACS = _ACS_HEAD + """// deathmatch: the frag counters of the engine are the score
script "dm_setup" OPEN
{
    reward = 0;
}
"""


def _deathmatch(nmaps, seed, size=2048):
  out = {}
  for k in range(nmaps):
    b = _arena(size - 256 * (k % 2), 2 + (k % 3), [], _DM_ITEMS, seed + k,
               ('STARTAN2', 'STONE2', 'BROWN1', 'METAL1')[k % 4],
               ('FLOOR0_1', 'FLOOR4_8', 'FLOOR7_1', 'FLAT5_4')[k % 4], dm=True)
    out['MAP%02d' % (k + 1)] = (b, _DM_ACS)
  return out


BUILDERS = {
    'basic.wad': _basic,
    'deadly_corridor.wad': _deadly_corridor,
    'health_gathering.wad': _health_gathering,
    'two_colors_easy.wad': lambda: _two_colors(False),
    'two_colors_hard.wad': lambda: _two_colors(True),
    'battle.wad': lambda: _battle(False),
    'D3_battle.wad': lambda: _battle(False),
    'battle2.wad': lambda: _battle(True),
    'D4_battle2.wad': lambda: _battle(True),
    'D4_battle.wad': lambda: _battle(True),
    'cig.wad': lambda: _deathmatch(2, 11),
    'dwango5.wad': lambda: _deathmatch(4, 21),
    'ssl2.wad': lambda: _deathmatch(1, 31, size=2560),
    'freedm.wad': lambda: _deathmatch(2, 41),
}


def wad_lumps(name, acc=None):
  """The lump list of scenario WAD `name`.  acc: path of an ACS compiler;
  when given, each map's SCRIPTS is compiled into BEHAVIOR."""
  lumps = []
  for map_name, (b, acs) in sorted(BUILDERS[name]().items()):
    behavior = _compile_acs(acs, acc) if acc else None
    lumps += W.map_lump_list(map_name, b.textmap(), acs, behavior)
  return lumps


def _compile_acs(source, acc):
  with tempfile.TemporaryDirectory() as d:
    src, out = os.path.join(d, 'scripts.acs'), os.path.join(d, 'behavior.o')
    with open(src, 'w') as f:
      f.write(source)
    subprocess.run([acc, src, out], check=True, capture_output=True,
                   cwd=os.path.dirname(acc) or None)
    with open(out, 'rb') as f:
      return f.read()


def build_all(directory, acc=None, names=None):
  """Writes every scenario WAD (or `names`) into `directory`; returns the
  paths."""
  os.makedirs(directory, exist_ok=True)
  paths = []
  for name in names or sorted(BUILDERS):
    path = os.path.join(directory, name)
    W.write_wad(path, wad_lumps(name, acc))
    paths.append(path)
  return paths


def default_cache_dir():
  return os.path.join(tempfile.gettempdir(), 'sa_doom_wads_%d' % os.getuid())


def ensure_wads(directory=None):
  """Builds the WADs once into `directory` (default: a per-user cache) and
  returns the directory."""
  directory = directory or default_cache_dir()
  if not all(os.path.exists(os.path.join(directory, n)) for n in BUILDERS):
    build_all(directory)
  return directory
