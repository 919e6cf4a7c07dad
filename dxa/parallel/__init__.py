"""Multi-GPU execution: one engine process per MI355X, RCCL (``torch.distributed`` "nccl" backend) over xGMI.

The reference scales by data-partition parallelism with Spark hash exchanges under GROUP BY / JOIN / DISTINCT
(SURVEY §2.G X2), broadcasts for small tables (X3) and driver reductions for counts/metrics (X5).  Here:

* every rank owns a disjoint share of the stream (its source partitions) and runs the full per-batch plan;
* tables carry a distribution tag — ``partitioned`` (rank-local share), ``hashed`` (partitioned by a key hash) or
  ``replicated`` (identical on every rank: reference data, constants, global aggregates);
* GROUP BY over partitioned input is two-phase: rank-local partial aggregates → ONE variable-size all-to-all of a
  packed [rows × cols] int64 matrix (+ one for string bytes) routed by ``hash(keys) % world`` → merge on the owner.
  Only partials cross xGMI (kilobytes per batch for the IoT flow), so the exchange is latency-, not link-bound;
* joins of two partitioned inputs shuffle both sides by join-key hash; partitioned ⨝ replicated joins are local;
* batch metrics have a rank-independent key set (checked by digest before any value moves); counts are summed and
  latencies maxed over ranks; rank 0 emits them.

``init`` is a no-op for world size 1, which keeps the single-GPU path free of collectives.  Multi-process CPU
tests run the same code over gloo.
"""
from __future__ import annotations

import threading
from typing import List, Optional, Tuple

import torch

_GROUP = None
_WORLD = 1
_RANK = 0
_DEVICE = None
_TLS = threading.local()          # per-thread communicator override (concurrent views)
_BRANCH_GROUPS: List = []

PARTITIONED = "partitioned"
HASHED = "hashed"
REPLICATED = "replicated"


def init(group=None, device=None):
    global _GROUP, _WORLD, _RANK, _DEVICE
    import torch.distributed as dist
    _GROUP = group or dist.group.WORLD
    _WORLD = dist.get_world_size(_GROUP)
    _RANK = dist.get_rank(_GROUP)
    _DEVICE = torch.device(device) if device is not None else None
    # the host-side (gloo) communicator for small host-byte broadcasts under RCCL: created HERE, on every rank of
    # the job's group at the same point (new_group is itself a collective — created lazily by one rank's reference
    # data refresh it would deadlock the others)
    from . import exchange as X
    X._HOST_GROUP = None
    if _WORLD > 1 and dist.get_backend(_GROUP) != "gloo":
        X._HOST_GROUP = dist.new_group(ranks=_group_ranks(_GROUP), backend="gloo")


def _group_ranks(g):
    import torch.distributed as dist
    try:
        return dist.get_process_group_ranks(g)
    except Exception:                                  # the default group
        return list(range(dist.get_world_size()))


def shutdown():
    global _GROUP, _WORLD, _RANK
    _GROUP, _WORLD, _RANK = None, 1, 0
    _BRANCH_GROUPS.clear()


def group():
    """The communicator of this thread's collectives: the job's group, or the branch group a concurrent view
    runs on (``use_branch``)."""
    g = getattr(_TLS, "group", None)
    return g if g is not None else _GROUP


def branch_groups(n: int) -> List:
    """``n`` extra communicators over the job's ranks, created once, in the same order on every rank (a
    collective).  Concurrent views run branch ``i`` of a level on group ``i``: each group sees its branch's
    collectives in program order on every rank, so branches on different threads cannot interleave one
    communicator's operations differently across ranks.  With RCCL each group is its own communicator (own
    channels over xGMI), so the branches' exchanges also overlap on the links."""
    import torch.distributed as dist
    ranks = list(range(_WORLD))
    while len(_BRANCH_GROUPS) < n:
        _BRANCH_GROUPS.append(dist.new_group(ranks=ranks, backend=dist.get_backend(_GROUP)))
    return _BRANCH_GROUPS[:n]


class use_branch:
    """``with use_branch(g):`` — collectives issued by this thread go to ``g``."""

    def __init__(self, g):
        self.g = g

    def __enter__(self):
        self.prev = getattr(_TLS, "group", None)
        _TLS.group = self.g
        return self.g

    def __exit__(self, *exc):
        _TLS.group = self.prev


def active() -> bool:
    return _WORLD > 1


def world() -> int:
    return _WORLD


def rank() -> int:
    return _RANK


def owner_of(h: torch.Tensor) -> torch.Tensor:
    """Owning rank of each 64-bit key hash."""
    return (h & 0x7FFFFFFFFFFFFFFF) % _WORLD


def dist_of(table) -> str:
    return getattr(table, "dist", REPLICATED)


def set_dist(table, d: str):
    table.dist = d
    return table


from .exchange import (MetricKeysMismatch, all_reduce_sum, allgather_table, broadcast_bytes,  # noqa: E402
                       broadcast_device_bytes,
                       broadcast_table, broadcast_tensor, is_max_metric, order_point, rebalance_table, reduce_metrics,
                       shuffle_table, split_by_destination)
