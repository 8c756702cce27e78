"""Iteration order of ``list(frozenset(range(n)) - frozenset(excluded))`` for small non-negative
ints, simulated from CPython 3.10's set implementation (Objects/setobject.c).

TEST INFRASTRUCTURE (oracle/): the ByteTrack scipy branch of ``linear_assignment``
(ultralytics/trackers/utils/matching.py:52-59) returns its unmatched indices as
``list(frozenset(np.arange(N)) - frozenset(matches[:, k]))``, and BYTETracker.update
(byte_tracker.py:356, 376, 387) iterates them in that order -- which decides, e.g., the order in
which new tracks are activated and so their track ids.  The device tracker reproduces the
order with the same algorithm (csrc/bytetrack.hip, ``pyset_diff``); this restatement is what it
is checked against, and tests/test_bytetrack_cpu.py checks this restatement against the running
interpreter.

The parts of setobject.c used (int keys: hash(i) == i, no dummies while building):
  * set_add_entry: slot i = hash & mask; probe i..i+LINEAR_PROBES (9) when i + 9 <= mask, else
    just i; then perturb >>= 5; i = (i * 5 + 1 + perturb) & mask.  After a new slot is filled,
    resize when fill * 5 >= mask * 3 to the smallest power of two > used * 4 (>= 8).
  * set_table_resize / set_insert_clean: old entries re-inserted in old-table order.
  * set_difference(so, other): if len(so) >> 2 > len(other): copy so (set_merge into an empty
    set pre-sized to 2 * len(so): keys < table size, so ascending) then discard -> the surviving
    keys in ascending order; else a new set built by adding so's keys not in other, in so's
    iteration order (ascending for frozenset(range(n))).
"""
from __future__ import annotations

LINEAR_PROBES = 9
PERTURB_SHIFT = 5
MINSIZE = 8


class _Table:
    def __init__(self):
        self.keys = [None] * MINSIZE
        self.mask = MINSIZE - 1
        self.fill = 0
        self.used = 0

    def _insert_clean(self, keys, mask, key):
        perturb = key
        i = key & mask
        while True:
            if keys[i] is None:
                keys[i] = key
                return
            if i + LINEAR_PROBES <= mask:
                for j in range(1, LINEAR_PROBES + 1):
                    if keys[i + j] is None:
                        keys[i + j] = key
                        return
            perturb >>= PERTURB_SHIFT
            i = (i * 5 + 1 + perturb) & mask

    def _resize(self, minused):
        size = MINSIZE
        while size <= minused:
            size <<= 1
        old = [k for k in self.keys if k is not None]
        self.keys = [None] * size
        self.mask = size - 1
        for k in old:
            self._insert_clean(self.keys, self.mask, k)
        self.fill = self.used = len(old)

    def add(self, key):
        mask = self.mask
        perturb = key
        i = key & mask
        while True:
            probes = LINEAR_PROBES if i + LINEAR_PROBES <= mask else 0
            j = 0
            while True:
                k = self.keys[i + j]
                if k is None:
                    self.keys[i + j] = key
                    self.fill += 1
                    self.used += 1
                    if self.fill * 5 >= mask * 3:
                        self._resize(self.used * 2 if self.used > 50000 else self.used * 4)
                    return
                if k == key:
                    return
                if j == probes:
                    break
                j += 1
            perturb >>= PERTURB_SHIFT
            i = (i * 5 + 1 + perturb) & mask

    def order(self):
        return [k for k in self.keys if k is not None]


def frozenset_diff_order(n: int, excluded) -> list[int]:
    """list(frozenset(range(n)) - frozenset(excluded)) as CPython 3.10 iterates it."""
    ex = list(excluded)
    n_other = len(set(ex))
    if (n >> 2) > n_other:
        s = set(ex)
        return [k for k in range(n) if k not in s]
    s = set(ex)
    t = _Table()
    for k in range(n):
        if k not in s:
            t.add(k)
    return t.order()
