"""Stripe sharding across GPUs / ranks.

Stripes are independent, so the multi-GPU path is pure partitioning: rank r
owns a contiguous stripe range and no collective touches the data path.
torch.distributed (gloo) is used only by the benchmark for the barrier and
the max-over-ranks timing reduction.
"""
from __future__ import annotations

import contextlib
import os
import sys
from typing import Optional, Tuple


def shard_range(nstripes: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous [lo, hi) of `nstripes` for `rank`; sizes differ by at most one."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(nstripes, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


@contextlib.contextmanager
def _stdout_to_stderr():
    """Point fd 1 at stderr for the block: gloo's C++ side prints its
    "[Gloo] Rank r is connected to ..." lines on stdout, where the bench's
    single JSON result line must be the only output."""
    sys.stdout.flush()
    saved = os.dup(1)
    try:
        os.dup2(2, 1)
        yield
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


class RankGroup:
    """Barrier + scalar reductions over ranks (gloo), or no-ops for one rank."""

    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self._dist = None
        if self.world > 1:
            import torch.distributed as dist

            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if not dist.is_initialized():
                with _stdout_to_stderr():
                    dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
                    self._dist = dist
                    self.barrier()  # gloo's mesh is connected (and reported) by now
            self._dist = dist

    def barrier(self) -> None:
        if self._dist is not None:
            self._dist.barrier()

    def _reduce(self, x: float, op: str) -> float:
        if self._dist is None:
            return float(x)
        import torch

        t = torch.tensor([float(x)], dtype=torch.float64)
        self._dist.all_reduce(t, op=getattr(self._dist.ReduceOp, op))
        return float(t.item())

    def max(self, x: float) -> float:
        return self._reduce(x, "MAX")

    def gather(self, x: float) -> list:
        """Every rank's x, in rank order, on every rank."""
        if self._dist is None:
            return [float(x)]
        import torch

        t = torch.zeros(self.world, dtype=torch.float64)
        t[self.rank] = float(x)
        self._dist.all_reduce(t, op=self._dist.ReduceOp.SUM)
        return [float(v) for v in t.tolist()]

    def sum(self, x: float) -> float:
        return self._reduce(x, "SUM")

    def close(self) -> None:
        if self._dist is not None and self._dist.is_initialized():
            self._dist.destroy_process_group()
