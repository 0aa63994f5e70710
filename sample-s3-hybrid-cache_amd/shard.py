"""Multi-GPU sharding of a block batch: blocks are independent, so a batch is
split into contiguous ranges, one per rank, with no data-path collective. torch.distributed
(gloo, CPU) is used only for the barrier and the max/sum of per-rank timings."""
from __future__ import annotations

import os


def shard_range(n_total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous [lo, hi) block range of `rank`: ceil-split, every block exactly once."""
    per = -(-n_total // world) if world else 0
    lo = min(n_total, rank * per)
    return lo, min(n_total, lo + per)


class Group:
    """gloo process group from torchrun's env (RANK/WORLD_SIZE/MASTER_*); no-op when world == 1."""

    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.dist = None
        if self.world > 1:
            import torch.distributed as dist

            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if not dist.is_initialized():
                dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
            self.dist = dist

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def _reduce(self, x: float, op) -> float:
        if self.dist is None:
            return x
        import torch

        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=op)
        return float(t.item())

    def max(self, x: float) -> float:
        return self._reduce(x, self.dist.ReduceOp.MAX) if self.dist else x

    def sum(self, x: float) -> float:
        return self._reduce(x, self.dist.ReduceOp.SUM) if self.dist else x

    def close(self):
        if self.dist is not None:
            self.dist.destroy_process_group()
            self.dist = None
