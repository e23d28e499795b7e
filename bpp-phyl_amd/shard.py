"""Site-pattern sharding across GPUs (one process per GPU, torch.distributed over RCCL).

Patterns are independent, so each rank evaluates a contiguous pattern range with no
data-path communication.  The single exchange of an evaluation is the final
log-likelihood: every rank contributes its fixed-order 4096-pattern block sums
(plk_root_loglik's block_sums), they are all-gathered and summed in global block
order, so the total is bitwise identical for any GPU count as long as shard
boundaries fall on block boundaries.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np

BLOCK = 4096  # plk_block_size()


def shard_range(rank: int, world: int, n_patterns: int, align: int = BLOCK) -> Tuple[int, int]:
    """Strong-scaling split of [0, n_patterns) into `world` contiguous ranges whose
    boundaries are multiples of `align` (the last range takes the remainder)."""
    n_blocks = (n_patterns + align - 1) // align
    per, extra = divmod(n_blocks, world)
    b0 = rank * per + min(rank, extra)
    b1 = b0 + per + (1 if rank < extra else 0)
    return min(b0 * align, n_patterns), min(b1 * align, n_patterns)


def bench_range(scaling: str, rank: int, world: int, patterns: int) -> Tuple[int, int, int]:
    """bench.py's pattern range of a rank and the job's total: weak = `patterns` per rank
    (rank r holds [r * patterns, (r + 1) * patterns) of one global alignment, so per-GPU work
    is fixed as N grows); strong = `patterns` in total, split into contiguous block-aligned
    ranges by shard_range (the lnL is then bitwise the same for every N)."""
    if scaling == "weak":
        return rank * patterns, (rank + 1) * patterns, patterns * world
    if scaling == "strong":
        a, b = shard_range(rank, world, patterns)
        return a, b, patterns
    raise ValueError(scaling)


def fixed_order_sum(blocks: np.ndarray) -> float:
    """Sequential left-to-right sum (np.add.accumulate is strictly sequential, unlike
    np.sum's pairwise summation), i.e. the same order plk_root_loglik uses."""
    b = np.asarray(blocks, dtype=np.float64)
    return float(np.add.accumulate(b)[-1]) if b.size else 0.0


def allgather_lnl(blocks: np.ndarray, dist=None, device=None) -> float:
    """All-gather per-rank block sums (variable counts allowed) and sum in global order."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return fixed_order_sum(blocks)
    import torch

    world = dist.get_world_size()
    n = torch.tensor([len(blocks)], dtype=torch.int64, device=device)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n)
    cmax = int(max(int(c.item()) for c in counts))
    buf = torch.zeros(cmax, dtype=torch.float64, device=device)
    buf[: len(blocks)] = torch.from_numpy(np.asarray(blocks, dtype=np.float64)).to(buf.device)
    out = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(out, buf)
    allb = np.concatenate([o[: int(c.item())].cpu().numpy() for o, c in zip(out, counts)])
    return fixed_order_sum(allb)


class BlockExchange:
    """The one exchange of a sharded evaluation, sized at setup: every rank's block count
    is all-gathered ONCE here, so each evaluation is a single fixed-size all-gather of the
    padded block sums (no count exchange, no per-rank .item() syncs) followed by the
    fixed-order sum on the host -- bitwise identical for any GPU count."""

    def __init__(self, dist, n_blocks: int, device=None):
        import torch

        self.dist = dist
        self.world = dist.get_world_size()
        n = torch.tensor([n_blocks], dtype=torch.int64, device=device)
        counts = [torch.zeros_like(n) for _ in range(self.world)]
        dist.all_gather(counts, n)
        self.counts = [int(c.item()) for c in counts]
        self.cmax = max(self.counts)
        self.n = n_blocks
        self.buf = torch.zeros(self.cmax, dtype=torch.float64, device=device)
        self.out = torch.empty(self.world * self.cmax, dtype=torch.float64, device=device)
        self.host = torch.empty(self.world * self.cmax, dtype=torch.float64,
                                pin_memory=str(device).startswith("cuda"))
        try:
            self._gather = dist.all_gather_into_tensor
            self._gather(self.out, self.buf)   # probe once: gloo may not provide it
        except (RuntimeError, AttributeError, NotImplementedError):
            self._gather = None
        self.views = list(self.out.view(self.world, self.cmax))

    def lnl(self, blocks: np.ndarray) -> float:
        import torch

        self.buf[: self.n].copy_(torch.from_numpy(np.asarray(blocks, dtype=np.float64)))
        if self._gather is not None:
            self._gather(self.out, self.buf)
        else:
            self.dist.all_gather(self.views, self.buf)
        self.host.copy_(self.out)
        allb = self.host.numpy().reshape(self.world, self.cmax)
        return fixed_order_sum(np.concatenate([allb[r, : self.counts[r]] for r in range(self.world)]))
