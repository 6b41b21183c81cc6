"""Batch-sharded multi-GPU decode (one process per GPU, torch.distributed).

The reference is single-GPU, batch 1 (decoder/decoder_block.hpp:48); there is
no collective anywhere in it.  Decode rows are independent, so the multi-GPU
design shards SEQUENCES across ranks (each rank owns its rows' KV pages and a
full weight replica) and exchanges nothing inside a step.  The one collective
is the gather of each step's output to rank 0 over RCCL (`backend="nccl"` is
RCCL on ROCm): either the final logits ([rows][V] fp32, 12.9 MB per 64-row
shard) or, for greedy decoding, only the argmax ids ([rows] int32).
Rank 0 receives from every peer on its own xGMI link.

This module is THE multi-rank decode loop: bench.py times it on the GPU ranks
(HipDecoderStep over the HIP decoder) and tests/test_dist_gloo.py runs the
same code with the gloo backend on CPU tensors (an oracle-backed step) at world
sizes 2, 3 and 4, weak and strong (ragged: padded to the largest shard, one
gather) sharding, bit-exact against one process.
"""
from __future__ import annotations

import time
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


def shard_sizes(n: int, world: int) -> list[int]:
    return [hi - lo for lo, hi in (shard_range(n, world, r) for r in range(world))]


class RowGatherer:
    """Double-buffered asynchronous gather of per-step row outputs (logits
    [rows][V] or ids [rows]) to rank 0.

    Per step: t = buffer() (waits for the gather that last used this slot),
    write the step's rows into t, push().  A slot is re-used only after its
    previous gather completed, so step s+1 computes while step s's rows move.
    With keep=True rank 0 accumulates every gathered step (per-rank rows
    concatenated in rank order) in `completed`, in step order.

    Ragged shards (strong scaling at a world size that does not divide the
    batch) take the SAME collective as equal ones: every rank's buffers hold
    `pad` = max(shard_rows) rows, the step writes its own rows into the first
    ones (buffer() returns that prefix view), one torch.distributed gather
    moves `pad` rows per rank, and rank 0 trims each peer's block to its row
    count.  So every world size runs the one gather path the single-rank RCCL
    test and the gloo tests cover; there is no point-to-point branch."""

    def __init__(self, shape, dtype, device, world: int, rank: int, shard_rows=None,
                 keep: bool = False):
        import torch
        self.world, self.rank, self.keep = world, rank, keep
        self.rows = list(shard_rows) if shard_rows else [shape[0]] * world
        if len(self.rows) != world or self.rows[rank] != shape[0]:
            raise ValueError("shard_rows must give every rank's row count, this rank's = shape[0]")
        self.pad = max(self.rows)
        full = (self.pad,) + tuple(shape[1:])
        self.bufs = [torch.empty(full, dtype=dtype, device=device) for _ in range(2)]
        self.recv = [[torch.empty(full, dtype=dtype, device=device) for _ in range(world)]
                     if rank == 0 else None for _ in range(2)]
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
                self.completed.append(
                    torch.cat([self.recv[s][r][:n] for r, n in enumerate(self.rows)]).clone())

    def buffer(self):
        """The tensor the next step should write its rows into (this rank's
        rows: a prefix of the padded slot)."""
        self._retire(self.slot)
        return self.bufs[self.slot][:self.rows[self.rank]]

    def push(self):
        s = self.slot
        if self.world > 1:
            self.works[s] = _gather(self.bufs[s], self.recv[s], self.rank)
        elif self.keep:
            self.completed.append(self.bufs[s][:self.rows[0]].clone())
        self.slot ^= 1

    def finish(self):
        """Wait for every pending gather (oldest first); returns `completed`."""
        self._retire(self.slot)      # older pending step
        self._retire(self.slot ^ 1)  # newest step
        return self.completed


LogitsGatherer = RowGatherer  # the name of the round-1 API


def _gather(t, recv, rank):
    """One torch.distributed gather of equal-sized (padded) blocks to rank 0."""
    import torch.distributed as dist
    return dist.gather(t, recv if rank == 0 else None, dst=0, async_op=True)


class HipDecoderStep:
    """One decode step of an llm_decoder INT8Decoder / CUDADecoder on a HIP
    stream: logits (if asked) go to a device tensor, greedy ids to an int32
    device tensor, without a host synchronisation.

    The stream must be the one the caller's torch work (staging copies,
    gathers, events) is ordered on, and it cannot be torch's default stream:
    its handle is 0, which the C ABI reads as "the decoder's own stream" (a
    non-blocking stream that does not synchronise with the default one).  Run
    under torch.cuda.stream(torch.cuda.Stream()) or pass such a stream."""

    def __init__(self, dec, stream=None):
        import torch
        self.dec = dec
        self.sp = (stream or torch.cuda.current_stream()).cuda_stream
        if not self.sp:
            raise ValueError("HipDecoderStep needs a non-default torch stream (the C ABI reads "
                             "stream 0 as the decoder's own stream): run it under "
                             "torch.cuda.stream(torch.cuda.Stream())")

    def __call__(self, tokens, logits_out):
        self.dec.step(tokens, logits_ptr=logits_out.data_ptr() if logits_out is not None else 0,
                      stream=self.sp, want_next=False)

    def ids_into(self, out):
        self.dec.copy_next_ids(out.data_ptr(), self.sp)


class ShardedDecode:
    """This rank's part of a batch-sharded decode: `step_fn` decodes the rank's
    `rows` (step_fn(tokens or None, logits_out or None); step_fn.ids_into(t)
    for gather="ids"), and each step's output goes to rank 0.

    gather: "logits" (the step's [rows][V] fp32 logits), "ids" (the greedy
    next ids, int32 [rows]) or "none".  A single rank gathers nothing unless
    keep=True.  staging="host" copies each step's output to host memory
    before the gather (a gloo rehearsal of the GPU path)."""

    def __init__(self, step_fn, rows: int, vocab: int, *, world: int = 1, rank: int = 0,
                 shard_rows: Sequence[int] | None = None, gather: str = "logits",
                 device="cuda", staging: str = "device", keep: bool = False):
        import torch
        if gather not in ("logits", "ids", "none"):
            raise ValueError("gather must be 'logits', 'ids' or 'none'")
        self.step_fn, self.world, self.rank, self.gather = step_fn, world, rank, gather
        self.active = gather != "none" and (world > 1 or keep)
        self.host = staging == "host"
        shape, dtype = ((rows, vocab), torch.float32) if gather == "logits" else ((rows,), torch.int32)
        gdev = "cpu" if self.host else device
        self.dev_buf = torch.empty(shape, dtype=dtype, device=device) if self.host else None
        self.g = RowGatherer(shape, dtype, gdev, world, rank, shard_rows, keep) if self.active else None

    def step(self, tokens=None):
        if not self.active:
            self.step_fn(tokens, None)
            return
        buf = self.g.buffer()
        out = self.dev_buf if self.host else buf
        if self.gather == "logits":
            self.step_fn(tokens, out)
        else:
            self.step_fn(tokens, None)
            self.step_fn.ids_into(out)
        if self.host:
            buf.copy_(out)
        self.g.push()

    def finish(self):
        return self.g.finish() if self.g else []


def timed_run(sd: ShardedDecode, warmup: int, steps: int, first_tokens, *,
              sync: Callable[[], None] | None = None, timer_device="cuda",
              step_times: list | None = None, rank_times: list | None = None) -> float:
    """bench.py's measured loop: `warmup` untimed steps (the first feeds
    first_tokens, later steps feed back the device's ids), then exactly `steps`
    timed ones bracketed by a barrier + device synchronisation on both sides.
    Returns the elapsed seconds, the MAX over ranks.  step_times (a list, GPU
    ranks only): filled with this rank's per-step device times in seconds,
    from HIP events recorded on torch's current stream (the stream the steps
    run on) between consecutive steps.  rank_times (a list): filled with every
    rank's own elapsed seconds, in rank order (one entry in a single process)."""
    import torch
    import torch.distributed as dist
    multi = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
    if sync is None:
        sync = torch.cuda.synchronize
    for i in range(warmup):
        sd.step(first_tokens if i == 0 else None)
    sd.finish()
    sync()
    if multi:
        dist.barrier()
    sync()
    ev = None
    if step_times is not None:
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    t0 = time.perf_counter()
    if ev:
        ev[0].record()
    for i in range(steps):
        sd.step(first_tokens if warmup == 0 and i == 0 else None)
        if ev:
            ev[i + 1].record()
    sd.finish()
    sync()
    if multi:
        dist.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    if ev:
        step_times[:] = [ev[i].elapsed_time(ev[i + 1]) * 1e-3 for i in range(steps)]
    per_rank = [elapsed]
    if multi:
        t = torch.tensor([elapsed], dtype=torch.float64, device=timer_device)
        ts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
        dist.all_gather(ts, t)
        per_rank = [float(x.item()) for x in ts]
    if rank_times is not None:
        rank_times[:] = per_rank
    return max(per_rank)


def time_gather(sd: ShardedDecode, iters: int = 10, *, sync: Callable[[], None] | None = None,
                timer_device="cuda") -> float | None:
    """Seconds one step's gather takes on its own (no decode step beside it):
    `iters` back-to-back gathers of the step buffer, barrier + sync on both
    sides, the MAX over ranks.  None when this loop gathers nothing."""
    import torch
    import torch.distributed as dist
    if sd.g is None or sd.world == 1:
        return None
    if sync is None:
        sync = torch.cuda.synchronize
    g = sd.g
    buf, recv = g.bufs[0], g.recv[0]
    _gather(buf, recv, g.rank).wait()  # warm the communicator's path
    sync()
    dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(iters):
        _gather(buf, recv, g.rank).wait()
    sync()
    dist.barrier()
    sync()
    t = torch.tensor([(time.perf_counter() - t0) / iters], dtype=torch.float64,
                     device=timer_device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


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
