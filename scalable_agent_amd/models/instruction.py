"""Host-side instruction tokenizer (reference experiment.py:123-132).

The reference splits the instruction string on whitespace and maps every word
to one of 1000 buckets with `tf.string_to_hash_bucket_fast` (FarmHash
Fingerprint64).  FarmHash is not available in this image, so words are hashed
with FNV-1a-64 instead: the bucket *ids* differ from TF's (parity unpinned; it
only matters for importing a TF-trained embedding table), the semantics
(split, hash, embed, LSTM over words, take the last valid output) are the same.
Only integer ids travel to the GPU.
"""

import functools

import numpy as np

NUM_HASH_BUCKETS = 1000
_FNV_OFFSET = 0xcbf29ce484222325
_FNV_PRIME = 0x100000001b3
_MASK = (1 << 64) - 1


@functools.lru_cache(maxsize=65536)
def hash_bucket(word: str, num_buckets: int = NUM_HASH_BUCKETS) -> int:
  h = _FNV_OFFSET
  for byte in word.encode('utf-8'):
    h ^= byte
    h = (h * _FNV_PRIME) & _MASK
  return h % num_buckets


def tokenize(instructions, max_len=None, num_buckets=NUM_HASH_BUCKETS):
  """Tokenizes a flat sequence of strings.

  Returns:
    ids: int64 [N, L] (0 where padded), lengths: int64 [N].  L >= 1 (the
    reference pads the embedding to at least one step, experiment.py:138-140).
  """
  words = [(s.decode('utf-8') if isinstance(s, bytes) else str(s)).split()
           for s in instructions]
  lengths = np.array([len(w) for w in words], dtype=np.int64)
  L = max(1, int(lengths.max()) if len(words) else 1)
  if max_len is not None:
    L = max(L, max_len)
  ids = np.zeros((len(words), L), dtype=np.int64)
  for i, ws in enumerate(words):
    for j, w in enumerate(ws):
      ids[i, j] = hash_bucket(w, num_buckets)
  return ids, lengths
