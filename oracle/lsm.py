"""Test infrastructure (oracle) -- NOT product code.

CPU restatement of Weaviate's LSM "replace"-strategy segment format, used by
tests/ only, to check the C-ABI segment reader (weaviate_amd/csrc/lsm_segment.hip)
and to write synthetic vectors-bucket segments the GPU restore path loads.

Pinned by the reference's own segment files (usecases/backup/test_data/
node1/*_lsm/*/segment-*.db, copied as data into tests/golden/lsm/): the
node walk over the data region must reproduce exactly the [start, end)
offsets and keys that the reference's writer recorded in the segment's
primary disk-tree index.

Followed:
  header       lsmkv/segmentindex/header.go:24-42 (WriteTo), :117-134 (ParseHeader)
  node         lsmkv/segment_serialization.go:34-104 (KeyIndexAndWriteTo),
               :106-166 (ParseReplaceNode)
  data region  lsmkv/segment.go:288-289 ([HeaderSize, IndexStart))
  disk tree    lsmkv/segmentindex/disk_tree.go:84-103 (readNode: u32 keylen,
               key, u64 start, u64 end, i64 left, i64 right)
  primary idx  lsmkv/segmentindex/header.go:64-93 (PrimaryIndex), segment.go:282-284
               (v1 without secondaries: drop the 4 checksum bytes)
  checksum     lsmkv/segmentindex/segment_file.go:274-341 (CRC32-IEEE over the
               body, then the header; hash.Sum(nil) = big endian)
  flat values  flat/index.go:204-208 (BE uint64 key), :317-336 (LE float32)
"""
from __future__ import annotations

import struct
import zlib
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

HEADER_SIZE = 16
CHECKSUM_SIZE = 4
STRATEGY_REPLACE = 0


def parse_header(b: bytes) -> dict:
    level, version, sec, strategy, index_start = struct.unpack_from("<HHHHQ", b, 0)
    return {"level": level, "version": version, "secondary_indices": sec, "strategy": strategy,
            "index_start": index_start}


def checksum_ok(b: bytes) -> bool:
    body = b[HEADER_SIZE:len(b) - CHECKSUM_SIZE]
    crc = zlib.crc32(b[:HEADER_SIZE], zlib.crc32(body))
    return crc == struct.unpack(">I", b[-CHECKSUM_SIZE:])[0]


def walk_nodes(b: bytes) -> List[dict]:
    """ParseReplaceNode over [HeaderSize, IndexStart)."""
    h = parse_header(b)
    out = []
    pos = HEADER_SIZE
    while pos < h["index_start"]:
        start = pos
        tomb = b[pos] == 1
        vlen = struct.unpack_from("<Q", b, pos + 1)[0]
        pos += 9
        value = b[pos:pos + vlen]
        pos += vlen
        klen = struct.unpack_from("<I", b, pos)[0]
        pos += 4
        key = b[pos:pos + klen]
        pos += klen
        sec = []
        for _ in range(h["secondary_indices"]):
            sl = struct.unpack_from("<I", b, pos)[0]
            pos += 4
            sec.append(b[pos:pos + sl])
            pos += sl
        out.append({"start": start, "end": pos, "tombstone": tomb, "value": value, "key": key,
                    "secondary": sec})
    if pos != h["index_start"]:
        raise ValueError(f"node walk ended at {pos}, index starts at {h['index_start']}")
    return out


def primary_index(b: bytes) -> bytes:
    h = parse_header(b)
    if h["secondary_indices"] == 0:
        idx = b[h["index_start"]:]
        if h["version"] >= 1:
            idx = idx[:-CHECKSUM_SIZE]
        return idx
    ist = h["index_start"]
    first_sec = struct.unpack_from("<Q", b, ist)[0]
    return b[ist + 8 * h["secondary_indices"]:first_sec]


def disk_tree_nodes(idx: bytes) -> List[Tuple[bytes, int, int]]:
    """All (key, start, end) of a disk tree, read node after node."""
    out = []
    pos = 0
    while pos + 36 <= len(idx):
        klen = struct.unpack_from("<I", idx, pos)[0]
        key = idx[pos + 4:pos + 4 + klen]
        start, end, _l, _r = struct.unpack_from("<QQqq", idx, pos + 4 + klen)
        out.append((key, start, end))
        pos += 4 + klen + 32
    return out


def write_segment(entries: Sequence[Tuple[bytes, Optional[bytes]]], version: int = 1, level: int = 0) -> bytes:
    """A replace segment with no secondary index: entries = (key, value or None
    for a tombstone), written in the given order (callers pass sorted keys, as
    the memtable flush does).  The primary index here is a flat list of
    disk-tree nodes with no children (-1), enough for readers that walk the
    data region; the reference's balanced tree layout is not restated."""
    body = bytearray()
    keys = []
    for key, value in entries:
        start = HEADER_SIZE + len(body)
        tomb = value is None
        v = b"" if tomb else value
        body += struct.pack("<BQ", 1 if tomb else 0, len(v)) + v + struct.pack("<I", len(key)) + key
        keys.append((key, start, HEADER_SIZE + len(body)))
    index_start = HEADER_SIZE + len(body)
    for key, s, e in keys:
        body += struct.pack("<I", len(key)) + key + struct.pack("<QQqq", s, e, -1, -1)
    header = struct.pack("<HHHHQ", level, version, 0, STRATEGY_REPLACE, index_start)
    out = header + bytes(body)
    if version >= 1:
        out += struct.pack(">I", zlib.crc32(header, zlib.crc32(bytes(body))))
    return out


def vector_entries(ids: Iterable[int], vecs: Optional[np.ndarray]) -> List[Tuple[bytes, Optional[bytes]]]:
    """flat's vectors bucket entries: BE uint64 key, LE float32 value (None = tombstone)."""
    ids = list(ids)
    out = []
    for i, id_ in enumerate(ids):
        key = struct.pack(">Q", int(id_))
        out.append((key, None if vecs is None else np.asarray(vecs[i], "<f4").tobytes()))
    return sorted(out, key=lambda kv: kv[0])


def replay_segments(segments: Sequence[bytes]) -> Dict[int, Optional[np.ndarray]]:
    """Final bucket state, newest segment wins (SegmentGroup replace semantics)."""
    state: Dict[int, Optional[np.ndarray]] = {}
    for b in segments:
        for n in walk_nodes(b):
            id_ = struct.unpack(">Q", n["key"])[0]
            state[id_] = None if n["tombstone"] else np.frombuffer(n["value"], "<f4").copy()
    return state
