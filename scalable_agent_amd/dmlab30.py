"""DMLab-30 suite: level mapping, human/random scores, normalised score.

Data and semantics of the reference dmlab30.py:27-218 (the published DMLab-30
human and random reference scores), with the reference's Python-2-only code
paths fixed for Python 3 (`dict.iteritems`, indexing `dict_keys`; SURVEY.md
§2.1 "Dangling or broken references").
"""

import collections
import logging

import numpy as np

_TRAIN_TEST = [
    ('rooms_collect_good_objects_train', 'rooms_collect_good_objects_test'),
    ('rooms_exploit_deferred_effects_train',
     'rooms_exploit_deferred_effects_test'),
    ('rooms_select_nonmatching_object',) * 2,
    ('rooms_watermaze',) * 2,
    ('rooms_keys_doors_puzzle',) * 2,
    ('language_select_described_object',) * 2,
    ('language_select_located_object',) * 2,
    ('language_execute_random_task',) * 2,
    ('language_answer_quantitative_question',) * 2,
    ('lasertag_one_opponent_small',) * 2,
    ('lasertag_three_opponents_small',) * 2,
    ('lasertag_one_opponent_large',) * 2,
    ('lasertag_three_opponents_large',) * 2,
    ('natlab_fixed_large_map',) * 2,
    ('natlab_varying_map_regrowth',) * 2,
    ('natlab_varying_map_randomized',) * 2,
    ('skymaze_irreversible_path_hard',) * 2,
    ('skymaze_irreversible_path_varied',) * 2,
    ('psychlab_arbitrary_visuomotor_mapping',) * 2,
    ('psychlab_continuous_recognition',) * 2,
    ('psychlab_sequential_comparison',) * 2,
    ('psychlab_visual_search',) * 2,
    ('explore_object_locations_small',) * 2,
    ('explore_object_locations_large',) * 2,
    ('explore_obstructed_goals_small',) * 2,
    ('explore_obstructed_goals_large',) * 2,
    ('explore_goal_locations_small',) * 2,
    ('explore_goal_locations_large',) * 2,
    ('explore_object_rewards_few',) * 2,
    ('explore_object_rewards_many',) * 2,
]
LEVEL_MAPPING = collections.OrderedDict(_TRAIN_TEST)

# (human, random) episode-return reference scores per test level.
_SCORES = {
    'rooms_collect_good_objects_test': (10, 0.073),
    'rooms_exploit_deferred_effects_test': (85.65, 8.501),
    'rooms_select_nonmatching_object': (65.9, 0.312),
    'rooms_watermaze': (54, 4.065),
    'rooms_keys_doors_puzzle': (53.8, 4.135),
    'language_select_described_object': (389.5, -0.07),
    'language_select_located_object': (280.7, 1.929),
    'language_execute_random_task': (254.05, -5.913),
    'language_answer_quantitative_question': (184.5, -0.33),
    'lasertag_one_opponent_small': (12.65, -0.224),
    'lasertag_three_opponents_small': (18.55, -0.214),
    'lasertag_one_opponent_large': (18.6, -0.083),
    'lasertag_three_opponents_large': (31.5, -0.102),
    'natlab_fixed_large_map': (36.9, 2.173),
    'natlab_varying_map_regrowth': (24.45, 2.989),
    'natlab_varying_map_randomized': (42.35, 7.346),
    'skymaze_irreversible_path_hard': (100, 0.1),
    'skymaze_irreversible_path_varied': (100, 14.4),
    'psychlab_arbitrary_visuomotor_mapping': (58.75, 0.163),
    'psychlab_continuous_recognition': (58.3, 0.224),
    'psychlab_sequential_comparison': (39.5, 0.129),
    'psychlab_visual_search': (78.5, 0.085),
    'explore_object_locations_small': (74.45, 3.575),
    'explore_object_locations_large': (65.65, 4.673),
    'explore_obstructed_goals_small': (206, 6.76),
    'explore_obstructed_goals_large': (119.5, 2.61),
    'explore_goal_locations_small': (267.5, 7.66),
    'explore_goal_locations_large': (194.5, 3.14),
    'explore_object_rewards_few': (77.7, 2.073),
    'explore_object_rewards_many': (106.7, 2.438),
}
HUMAN_SCORES = {k: v[0] for k, v in _SCORES.items()}
RANDOM_SCORES = {k: v[1] for k, v in _SCORES.items()}

ALL_LEVELS = frozenset(list(LEVEL_MAPPING.keys()) +
                       list(LEVEL_MAPPING.values()))


def _transform_level_returns(level_returns):
  """Converts training level names to test level names (reference :165-183)."""
  new_level_returns = {}
  for level_name, returns in level_returns.items():
    new_level_returns[LEVEL_MAPPING.get(level_name, level_name)] = returns
  test_set = set(LEVEL_MAPPING.values())
  diff = test_set - set(new_level_returns.keys())
  if diff:
    raise ValueError('Missing levels: %s' % sorted(diff))
  for level_name, returns in new_level_returns.items():
    if level_name in test_set:
      if not returns:
        raise ValueError('Missing returns for level: \'%s\': ' % level_name)
    else:
      logging.info('Skipping level %s for calculation.', level_name)
  return new_level_returns


def compute_human_normalized_score(level_returns, per_level_cap):
  """Mean human-normalised score in percent (reference :186-218)."""
  new_level_returns = _transform_level_returns(level_returns)

  def human_normalized_score(level_name, returns):
    score = np.mean(returns)
    human = HUMAN_SCORES[level_name]
    random = RANDOM_SCORES[level_name]
    s = (score - random) / (human - random) * 100
    if per_level_cap is not None:
      s = min(s, per_level_cap)
    return s

  return np.mean([human_normalized_score(k, v)
                  for k, v in new_level_returns.items()
                  if k in HUMAN_SCORES])
