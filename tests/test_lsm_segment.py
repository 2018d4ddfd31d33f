"""LSM on-disk format (flat's vectors bucket): the oracle restatement pinned
to the reference's own segment files, and the C-ABI segment reader checked
against it.  Host-only calls: runs without a GPU.

Fixtures tests/golden/lsm/*.db are data files copied from the reference's
test data (usecases/backup/test_data/node1/*_lsm/...): two replace-strategy
"objects" segments (version 0, one secondary index) and two segments of
other strategies.
"""
import glob
import os
import struct

import numpy as np
import pytest

import lsm  # oracle/lsm.py (test infrastructure)

GOLD = os.path.join(os.path.dirname(__file__), "golden", "lsm")
REPLACE = sorted(glob.glob(os.path.join(GOLD, "objects_*.db")))


def read(p):
    with open(p, "rb") as f:
        return f.read()


@pytest.mark.parametrize("path", REPLACE)
def test_oracle_walk_matches_reference_disk_tree(path):
    b = read(path)
    h = lsm.parse_header(b)
    assert h["strategy"] == lsm.STRATEGY_REPLACE and h["secondary_indices"] == 1
    nodes = lsm.walk_nodes(b)
    tree = lsm.disk_tree_nodes(lsm.primary_index(b))
    assert len(nodes) == len(tree) > 0
    assert sorted(tree) == sorted((n["key"], n["start"], n["end"]) for n in nodes)


@pytest.mark.parametrize("path", REPLACE)
def test_c_scan_matches_oracle_on_reference_segments(wv, path):
    b = read(path)
    nodes = lsm.walk_nodes(b)
    hdr = wv.lsm_segment_header(path)
    assert hdr["index_start"] == lsm.parse_header(b)["index_start"] and hdr["size"] == len(b)
    assert hdr["secondary_indices"] == 1 and hdr["version"] == 0
    r = wv.lsm_segment_scan(path)
    np.testing.assert_array_equal(r["start"], [n["start"] for n in nodes])
    np.testing.assert_array_equal(r["end"], [n["end"] for n in nodes])
    np.testing.assert_array_equal(r["tombstone"], [n["tombstone"] for n in nodes])
    # 16-byte UUID keys are not BE uint64 ids -> UINT64_MAX
    assert all(int(k) == 2**64 - 1 for k in r["key_id"])


@pytest.mark.parametrize("name,strategy", [("property_id_setcollection.db", "setcollection"),
                                           ("property_title_roaringset.db", "roaringset")])
def test_other_strategies_rejected(wv, name, strategy):
    path = os.path.join(GOLD, name)
    assert wv.lsm_segment_header(path)["strategy"] == lsm.parse_header(read(path))["strategy"]
    with pytest.raises(wv.WeaviateError, match=f"unsupported strategy in segment: strategy {strategy}"):
        wv.lsm_segment_scan(path)


def _vector_segment(tmp_path, name, ids, vecs, version=1):
    p = tmp_path / name
    p.write_bytes(lsm.write_segment(lsm.vector_entries(ids, vecs), version=version))
    return str(p)


@pytest.mark.parametrize("version", [0, 1])
def test_c_scan_of_written_vector_segment(wv, tmp_path, version):
    rng = np.random.default_rng(5)
    ids = rng.choice(10**6, 300, replace=False).astype(np.uint64)
    vecs = rng.standard_normal((300, 33)).astype(np.float32)
    p = _vector_segment(tmp_path, "s.db", ids, vecs, version)
    b = read(p)
    if version == 1:
        assert lsm.checksum_ok(b)
    nodes = lsm.walk_nodes(b)
    r = wv.lsm_segment_scan(p, validate_checksum=True)
    np.testing.assert_array_equal(r["key_id"], [struct.unpack(">Q", n["key"])[0] for n in nodes])
    np.testing.assert_array_equal(r["key_id"], np.sort(ids))
    np.testing.assert_array_equal(r["end"], [n["end"] for n in nodes])
    assert not r["tombstone"].any()


def test_checksum_and_format_errors(wv, tmp_path):
    ids = np.arange(20, dtype=np.uint64)
    vecs = np.ones((20, 8), np.float32)
    p = _vector_segment(tmp_path, "v1.db", ids, vecs, 1)
    b = bytearray(read(p))
    b[40] ^= 0xFF  # inside a value
    bad = tmp_path / "bad.db"
    bad.write_bytes(bytes(b))
    with pytest.raises(wv.WeaviateError, match="invalid checksum"):
        wv.lsm_segment_scan(str(bad), validate_checksum=True)
    assert len(wv.lsm_segment_scan(str(bad), validate_checksum=False)["start"]) == 20
    v2 = bytearray(read(p))
    v2[2:4] = struct.pack("<H", 2)
    (tmp_path / "v2.db").write_bytes(bytes(v2))
    with pytest.raises(wv.WeaviateError, match="unsupported version 2"):
        wv.lsm_segment_header(str(tmp_path / "v2.db"))
    # truncated data region: index start beyond what the nodes hold
    tr = bytearray(read(p))
    tr[8:16] = struct.pack("<Q", len(tr) - 4)
    (tmp_path / "tr.db").write_bytes(bytes(tr))
    with pytest.raises(wv.WeaviateError):
        wv.lsm_segment_scan(str(tmp_path / "tr.db"), validate_checksum=False)
    with pytest.raises(wv.WeaviateError, match="open segment"):
        wv.lsm_segment_scan(str(tmp_path / "missing.db"))


def test_oracle_replay_newest_wins(tmp_path):
    a = lsm.write_segment(lsm.vector_entries([1, 2, 3], np.eye(3, dtype=np.float32)))
    b = lsm.write_segment(lsm.vector_entries([2], None) + lsm.vector_entries([3], np.full((1, 3), 7, np.float32)))
    st = lsm.replay_segments([a, b])
    assert st[2] is None and st[3].tolist() == [7, 7, 7] and st[1].tolist() == [1, 0, 0]
