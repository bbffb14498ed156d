"""CPU restatement of SDFS's dedup-hit step (test infrastructure only — never imported by the
product path; tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg are its only users).

Follows, per flushed buffer in order:
  * SparseDedupFile.writeCache groups the buffer's Fingers by hash, the first Finger of a hash
    carrying `claims` = its number of occurrences (SparseDedupFile.java:435-446);
  * every distinct hash goes to the hash store with its claims (Finger.java:50-60 ->
    HashChunkService.writeChunk, HashChunkService.java:98-118 -> RocksDBMap.put,
    RocksDBMap.java:785-870): present -> refcount += claims, InsertRecord(inserted=false, pos);
    absent -> chunk persisted at a new pos, {pos, refcount = claims} inserted,
    InsertRecord(inserted=true, pos);
  * each Finger becomes a HashLocPair with hashloc = its hash's pos, dup = not inserted for the
    Finger that was written and dup = true for the buffer's other copies, whose `hl` stays null
    (SparseDedupFile.java:541-560).
New positions are pos_base + the number of insertions before it, in buffer order (the
reference's archive positions come from HashBlobArchive; here the caller owns them).
Parity status: pinned by the reference's own control flow only (no fixtures exist for it).
"""
from __future__ import annotations

from dataclasses import dataclass, field


@dataclass
class Entry:
    pos: int
    refcount: int


@dataclass
class HashesMap:
    """The hash store's map: fingerprint -> {pos, refcount} (RocksDBMap value = pos | ct)."""

    entries: dict = field(default_factory=dict)

    def put(self, key: bytes, claims: int, new_pos: int):
        """RocksDBMap.put(cm, persist) with cm.references = claims (RocksDBMap.java:785-870)."""
        e = self.entries.get(key)
        if e is not None:
            e.refcount += claims if claims > 0 else 1
            return False, e.pos
        self.entries[key] = Entry(new_pos, claims if claims > 0 else 1)
        return True, new_pos


def write_buffers(m: HashesMap, digests: list, buffer_ids: list, pos_base: int):
    """Apply a batch of fingerprint records (in buffer order) as consecutive writeCache calls.

    Returns (dup[list of 0/1], hashloc[list of int], new_list[list of record indices])."""
    n = len(digests)
    dup = [1] * n
    hashloc = [0] * n
    new_list = []
    r = 0
    while r < n:
        b = buffer_ids[r]
        e = r
        while e < n and buffer_ids[e] == b:
            e += 1
        # mp: hash -> first Finger of the buffer, with claims (SparseDedupFile.java:435-446)
        first = {}
        claims = {}
        for i in range(r, e):
            k = digests[i]
            if k not in first:
                first[k] = i
                claims[k] = 1
            else:
                claims[k] += 1
        # writeChunk per distinct hash (executor order is irrelevant: keys are distinct)
        result = {}
        for k, i in sorted(first.items(), key=lambda kv: kv[1]):
            inserted, pos = m.put(k, claims[k], pos_base + len(new_list))
            if inserted:
                new_list.append(i)
            result[k] = (inserted, pos)
        for i in range(r, e):
            inserted, pos = result[digests[i]]
            hashloc[i] = pos
            dup[i] = 0 if (first[digests[i]] == i and inserted) else 1
        r = e
    return dup, hashloc, new_list
