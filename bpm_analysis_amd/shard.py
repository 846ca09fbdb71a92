"""Placement of ragged batches: recordings over ranks, and their
order inside one GPU batch.

Recordings are independent (no exchange), so placement is pure scheduling:

* ``lpt_partition`` — longest-processing-time-first over ranks: recordings in
  descending length, each to the rank with the least total so far (ties to
  the lower rank).  Every rank computes the same partition from the same
  lengths, so no collective is needed to agree on it.  Greedy LPT is within
  4/3 of the optimal makespan.
* ``longest_first`` — the order a rank hands its recordings to one
  ``bpmx_run``: the per-recording kernels give recording f workgroup f and the
  hardware dispatches workgroups in index order, so longest-first is LPT over
  the CUs and a long recording never starts last (the ragged C5 tail).
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np


def longest_first(lengths: Sequence[int]) -> np.ndarray:
    """Permutation putting the longest recordings first (stable for equal lengths)."""
    n = np.asarray(lengths, dtype=np.int64)
    return np.argsort(-n, kind="stable")


def lpt_partition(lengths: Sequence[int], world: int) -> List[List[int]]:
    """Recording indices per rank; each rank's list is longest first."""
    if world < 1:
        raise ValueError("world must be >= 1")
    n = np.asarray(lengths, dtype=np.int64)
    load = np.zeros(world, dtype=np.int64)
    parts: List[List[int]] = [[] for _ in range(world)]
    for i in longest_first(n):
        r = int(np.argmin(load))                    # first minimum: ties go to the lower rank
        parts[r].append(int(i))
        load[r] += n[i]
    return parts


def makespan(lengths: Sequence[int], parts: List[List[int]]) -> int:
    n = np.asarray(lengths, dtype=np.int64)
    return max((int(n[p].sum()) if p else 0) for p in parts)
