"""The 16-hex cas_id string contract and its consumers (CPU only, no kernel calls).

* cas_id = ``Hash::to_hex()[..16]`` (core/src/object/cas.rs:61): lowercase hex of the
  first 8 digest bytes; the engine carries it as a big-endian u64 key (SURVEY.md §8
  definitions), so ``format(key, '016x') == cas_id`` and numeric key order is the string
  order of cas_ids.
* Thumbnail shard directory = the first three hex chars, 4,096 shards 000..fff
  (core/src/object/media/thumbnail/shard.rs:10-13) — the top 12 bits of the key.
"""
import json
import os
import random

from spacedrive_amd.cas import cas_id_to_key, get_shard_hex, key_to_cas_id

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "golden.json")


def _golden_ids():
    with open(GOLDEN) as f:
        return [e["cas_id"] for e in json.load(f)["cas"]["files"]]


def test_golden_cas_ids_round_trip_through_keys():
    ids = _golden_ids()
    assert ids
    for cid in ids:
        assert len(cid) == 16 and cid == cid.lower() and all(c in "0123456789abcdef" for c in cid)
        k = cas_id_to_key(cid)
        assert 0 <= k < 1 << 64
        assert key_to_cas_id(k) == cid == format(k, "016x")


def test_key_order_is_cas_id_string_order():
    rng = random.Random(0x5DCA5)
    keys = [rng.getrandbits(64) for _ in range(2000)] + [0, 1, (1 << 64) - 1, 1 << 63]
    assert sorted(keys, key=key_to_cas_id) == sorted(keys)


def test_shard_hex_is_top_12_bits():
    rng = random.Random(7)
    seen = set()
    for k in [rng.getrandbits(64) for _ in range(5000)] + [0, (1 << 64) - 1]:
        cid = key_to_cas_id(k)
        s = get_shard_hex(cid)
        assert s == cid[0:3] == format(k >> 52, "03x")
        seen.add(s)
    assert len(seen) > 2500 and all(len(s) == 3 for s in seen)  # 4,096 possible shards
    for cid in _golden_ids():
        assert int(get_shard_hex(cid), 16) == cas_id_to_key(cid) >> 52
