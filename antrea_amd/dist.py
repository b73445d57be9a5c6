"""Multi-GPU plumbing of the path: one process per GPU, packets sharded, rule
image replicated, and ONE collective -- the sum all-reduce of the per-rule counters that
NetworkPolicyMetrics reports (network_policy.go:2034; collector.go:114 reads it every 60 s).

The counters are the library's device buffer (gpc_counters: n_slots x {packets, bytes, sessions}
uint64), wrapped zero-copy and reduced in place over RCCL ("nccl" backend = RCCL on ROCm); the
same functions run over gloo on CPU tensors in the tests.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np

COUNTER_WORDS = 3  # core.hpp kCounterWords


class _CAI:
    def __init__(self, ptr, n):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "<i8", "data": (ptr, False), "version": 2}


def device_counters(ptr: int, n_slots: int, device):
    """int64 torch view (no copy) of the library's device counter buffer."""
    import torch
    return torch.as_tensor(_CAI(ptr, COUNTER_WORDS * n_slots), device=device)


def allreduce_counters(t, group=None):
    """Sum the per-rule counters of all ranks in place (u64 counters carried as int64: sums of
    packet/byte counts stay far below 2^63)."""
    import torch.distributed as dist
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


def shard_range(n_total: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous packet range of `rank` (strong-scaling split; bench.py uses weak scaling with
    a per-rank seed instead)."""
    per = (n_total + world - 1) // world
    lo = min(n_total, rank * per)
    return lo, min(n_total, lo + per)


def metrics_from_counters(counters: np.ndarray, slot_conj: Sequence[int]) -> Dict[int, Tuple[int, int, int]]:
    """NetworkPolicyMetrics shape: conj id -> (packets, bytes, sessions), skipping released slots
    (the same mapping gpc_metrics applies on one device)."""
    c = np.asarray(counters, dtype=np.uint64).reshape(-1, COUNTER_WORDS)
    out = {}
    for s, conj in enumerate(slot_conj):
        if conj:
            out[int(conj)] = tuple(int(x) for x in c[s])
    return out
