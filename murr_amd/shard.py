"""Key-range sharding across GPUs: one process per GPU, each
decoding its own contiguous key range; no data-path collective.

torch.distributed (gloo, CPU tensors) carries only the start/stop barriers and
the max-over-ranks time / sum-over-ranks bytes the bench reports, so the data
path never touches RCCL: every output cell depends on exactly one input row
(src/io/row/read.rs:85-91) and the utf8 offset prefix is local to a block.
"""
from __future__ import annotations

import os


def shard_rows(rank: int, world: int, total: int) -> tuple[int, int]:
    """Contiguous key range [start, start + count) of `rank` out of `world`
    over `total` rows (earlier ranks take the remainder, one row each)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} of {world}")
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


class Group:
    """The bench's process group: None-safe wrappers (world size 1 = no group)."""

    def __init__(self, backend: str = "gloo"):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.dist = None
        self.rank, self.local_rank = 0, 0
        if self.world > 1:
            import torch.distributed as dist
            if not dist.is_initialized():
                dist.init_process_group(backend)
            self.dist = dist
            self.rank = dist.get_rank()
            self.local_rank = int(os.environ.get("LOCAL_RANK", str(self.rank)))

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
        return self._reduce(x, self.dist.ReduceOp.MAX if self.dist else None)

    def sum(self, x: float) -> float:
        return self._reduce(x, self.dist.ReduceOp.SUM if self.dist else None)

    def close(self):
        if self.dist is not None:
            self.dist.destroy_process_group()
            self.dist = None
