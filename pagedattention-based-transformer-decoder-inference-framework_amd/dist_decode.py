"""Batch-sharded multi-GPU decode (one process per GPU, torch.distributed).

The reference is single-GPU, batch 1 (decoder/decoder_block.hpp:48); there is
no collective anywhere in it.  Decode rows are independent, so the multi-GPU
design shards SEQUENCES across ranks (each rank owns its rows' KV pages and a
full weight replica) and exchanges nothing inside a step.  The one collective
is the gather of each step's final logits (or of the generated ids) to rank 0
over RCCL (`backend="nccl"` is RCCL on ROCm), which receives from every peer
over its own xGMI link.

Device-agnostic: the same code runs with the gloo backend on CPU tensors,
which is how tests/test_dist_gloo.py exercises it at world_size 2.
"""
from __future__ import annotations

from typing import Callable, Sequence


def shard_range(n: int, world: int, rank: int) -> tuple[int, int]:
    """Rows [lo, hi) of a global batch of n owned by `rank` (contiguous, sizes
    differ by at most one)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    hi = lo + base + (1 if rank < extra else 0)
    return lo, hi


class LogitsGatherer:
    """Double-buffered asynchronous gather of per-step logits to rank 0.

    Per step: t = buffer() (waits for the gather that last used this slot),
    write the step's logits into t, push().  A slot is re-used only after its
    previous gather completed, so step s+1 computes while step s's logits move.
    With keep=True rank 0 accumulates every gathered step (per-rank tensors
    concatenated along rows) in `completed`, in step order."""

    def __init__(self, shape, dtype, device, world: int, rank: int, shard_rows=None,
                 keep: bool = False):
        import torch
        self.world, self.rank, self.keep = world, rank, keep
        rows = shard_rows or [shape[0]] * world
        self.bufs = [torch.empty(shape, dtype=dtype, device=device) for _ in range(2)]
        self.recv = [[torch.empty((rows[r],) + tuple(shape[1:]), dtype=dtype, device=device)
                      for r in range(world)] if rank == 0 else None for _ in range(2)]
        self.works = [None, None]
        self.slot = 0
        self.completed = []

    def _retire(self, s):
        w = self.works[s]
        if w is not None:
            w.wait()
            self.works[s] = None
            if self.keep and self.rank == 0:
                import torch
                self.completed.append(torch.cat(self.recv[s]).clone())

    def buffer(self):
        """The tensor the next step should write its logits into."""
        self._retire(self.slot)
        return self.bufs[self.slot]

    def push(self):
        s = self.slot
        if self.world > 1:
            self.works[s] = _gather(self.bufs[s], self.recv[s], self.rank)
        elif self.keep:
            self.completed.append(self.bufs[s].clone())
        self.slot ^= 1

    def finish(self):
        """Wait for every pending gather (oldest first); returns `completed`."""
        self._retire(self.slot)      # older pending step
        self._retire(self.slot ^ 1)  # newest step
        return self.completed


def _gather(t, recv, rank):
    """gather with unequal shard sizes: point-to-point receives on rank 0 (each
    peer on its own link), a single send elsewhere."""
    import torch.distributed as dist
    world = dist.get_world_size()
    if rank == 0:
        recv[0].copy_(t)
        ops = [dist.P2POp(dist.irecv, recv[r], r) for r in range(1, world)]
    else:
        ops = [dist.P2POp(dist.isend, t, 0)]
    reqs = dist.batch_isend_irecv(ops)
    return _Works(reqs)


class _Works:
    def __init__(self, reqs):
        self.reqs = reqs

    def wait(self):
        for r in self.reqs:
            r.wait()


def distributed_generate(make_decoder: Callable, prompts: Sequence[Sequence[int]],
                         max_gen_len: int, temperature: float = 1.0):
    """Shard `prompts` over the ranks of the default process group, generate on
    each rank with `make_decoder(n_rows)` (an object with generate_batch), and
    gather the results to rank 0 (returned there; None elsewhere)."""
    import torch.distributed as dist
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    lo, hi = shard_range(len(prompts), world, rank)
    mine = [list(p) for p in prompts[lo:hi]]
    out = make_decoder(len(mine)).generate_batch(mine, max_gen_len, temperature) if mine else []
    if world == 1:
        return out
    gathered = [None] * world if rank == 0 else None
    dist.gather_object(out, gathered, dst=0)
    if rank != 0:
        return None
    res = []
    for part in gathered:
        res.extend(part)
    return res
