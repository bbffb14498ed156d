"""CPU restatement of the per-buffer metadata SDFS writes after dedup — TEST INFRASTRUCTURE ONLY.

Only ``tests/`` (and the smoke/bench checkers) may import this module; the product path
(``sdfs_amd``) never does.  It follows, for one flushed write buffer:

* SparseDedupFile.writeCache's HashLocPair per chunk (SparseDedupFile.java:535-556): hash = the
  chunk's digest, hashloc = the fingerprint's position (InsertRecord.getHashLocs =
  Longs.toByteArray(pos), InsertRecord.java:29-33), len = nlen = chunk length, pos = chunk start,
  offset = 0, dup = not the copy that was inserted;
* HashLocPair.asArray (HashLocPair.java:37-59): hash | hashloc[8] | BE32 len, pos, offset, nlen;
* SparseDataChunk.getBytes for map versions >= 2 (SparseDataChunk.java:295-318):
  u8 flags | BE32 capacity | BE32 n | n records (TreeMap order = ascending pos) | BE32 doop;
* the LongByteArrayMap slot length (LongByteArrayMap.java:55-60: 13 + BAL * 2 * max_hash_cluster).
Parity status: pinned by the reference's own serialisation code (no fixtures exist for it).
"""
from __future__ import annotations

import struct


def bal(hash_len: int) -> int:
    """HashLocPair.BAL = hashLength + 8 + 4 + 4 + 4 + 4."""
    return hash_len + 24


def slot_bytes(hash_len: int, chunk_length: int, min_len: int) -> int:
    """LongByteArrayMap._v2arrayLength with max_hash_cluster = CHUNK_LENGTH / minLen."""
    return 13 + bal(hash_len) * 2 * (chunk_length // min_len)


def hashlocpair_as_array(digest: bytes, hashloc_pos: int, ln: int, pos: int, offset: int = 0,
                         nlen: int | None = None) -> bytes:
    nlen = ln if nlen is None else nlen
    if ln < 0 or pos < 0 or offset < 0 or nlen < 0:
        raise IOError("data is corrupt")  # HashLocPair.checkCorrupt
    return bytes(digest) + struct.pack(">qiiii", hashloc_pos, ln, pos, offset, nlen)


def sparse_data_chunk_bytes(pairs) -> bytes:
    """pairs: iterable of (digest, hashloc_pos, len, pos, dup) in ascending pos."""
    pairs = sorted(pairs, key=lambda p: p[3])
    body = b"".join(hashlocpair_as_array(d, hl, ln, pos) for d, hl, ln, pos, _ in pairs)
    doop = sum(ln for _, _, ln, _, dup in pairs if dup)
    return struct.pack(">BII", 0, 13 + len(body), len(pairs)) + body + struct.pack(">I", doop)
