"""The multi-GPU decode loop on the GPU: two gloo ranks, both on cuda:0, each
running bench.py's loop (dist_decode.ShardedDecode + timed_run) over its own
HIP INT8Decoder (HipDecoderStep), staging every step's output through host
memory for the gloo gather.  Weak sharding (3 rows per rank) and ragged
strong sharding (5 rows over 2 ranks), logits and greedy-id gathers.  Rank
0's gathered steps must equal ONE process stepping all rows, bit for bit.

The model's context stays below one attention split (max_seq 48: every launch
is the direct single-split form at any row count) and its LayerNorms run in
the GEMM prologue at every row count, so a row's results do not depend on how
many rows share its decoder; the weight GEMMs' int32 sums are exact in every
tile form.  On the 8-GPU node the same loop runs one rank per GPU over RCCL
(bench.py --gpus N); this test keeps the driver's GPU run exercising it."""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "pagedattention-based-transformer-decoder-inference-framework_amd"
WARMUP, STEPS, ROWS_PER_RANK, V = 2, 4, 3, 300


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


PROMPT = 600  # long-context case: every row prefilled with its own prompt


def _prompt(row):
    return np.random.default_rng(7000 + row).integers(0, V, PROMPT).astype(np.int32).tolist()


def _decoder(rows, row0=None):
    """A fresh INT8 decoder of `rows` rows.  row0 is None: context 0 (every
    launch the single-split form); else rows row0 .. row0 + rows - 1 of the
    global batch are first prefilled with their own PROMPT-token prompts (a
    row's KV depends only on its own tokens, so it is the same whichever
    process holds the row), and every decode step then attends >= PROMPT
    tokens in several splits whose count depends on the rows per process."""
    import llm_decoder
    from oracle.oracle import Oracle, synthetic_int8_model
    max_seq = 48 if row0 is None else PROMPT + 48
    w = synthetic_int8_model(Oracle(), L=2, H=4, D=64, V=V, max_seq=max_seq, seed=23)
    c = w["cfg"]
    dec = llm_decoder.INT8Decoder(c["L"], c["H"], c["D"], c["hid"], c["V"], c["max_seq"],
                                  max_batch=rows)
    d = {k: np.ascontiguousarray(v) for k, v in w.items() if k != "cfg"}
    d["emb"] = w["emb"].view(np.uint16)
    dec.set_weights(d)
    dec.begin_synthetic(rows, 0, 0, False)
    if row0 is not None:
        for r in range(rows):
            dec.prefill(r, _prompt(row0 + r))
    return dec


def _tokens(mode, world, rank, global_rows):
    from dist_decode import shard_range
    if mode == "weak":
        return np.random.default_rng(1234 + rank).integers(0, V, ROWS_PER_RANK).astype(np.int32)
    lo, hi = shard_range(global_rows, world, rank)
    return np.random.default_rng(1234).integers(0, V, global_rows).astype(np.int32)[lo:hi]


def _run(rows, world, rank, shard_rows, gather, first, row0=None, staging="host"):
    import torch
    import dist_decode
    dec = _decoder(rows, row0)
    with torch.cuda.stream(torch.cuda.Stream()):  # bench.py's explicit stream
        sd = dist_decode.ShardedDecode(dist_decode.HipDecoderStep(dec), rows, V, world=world,
                                       rank=rank, shard_rows=shard_rows, gather=gather,
                                       staging=staging, keep=True)
        elapsed = dist_decode.timed_run(sd, WARMUP, STEPS, [int(t) for t in first],
                                        timer_device="cpu")
        return [t.cpu().numpy().copy() for t in sd.finish()], elapsed


def test_hip_step_refuses_the_default_stream(gpu):
    """torch's default stream is handle 0, which the C ABI reads as the
    decoder's own (non-blocking) stream: HipDecoderStep refuses it rather than
    letting staging copies and gathers race the step."""
    import dist_decode
    with pytest.raises(ValueError, match="non-default"):
        dist_decode.HipDecoderStep(_decoder(1))


def _worker(rank, world, port, mode, gather, global_rows, q, long_ctx=False, staging="host"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    for p in (str(ROOT), str(PKG)):
        sys.path.insert(0, p)
    import torch
    import torch.distributed as dist
    import dist_decode
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    shard_rows = None
    if mode == "weak":
        rows = ROWS_PER_RANK
    else:
        shard_rows = dist_decode.shard_sizes(global_rows, world)
        rows = shard_rows[rank]
    row0 = None
    if long_ctx:
        row0 = rank * ROWS_PER_RANK if mode == "weak" else dist_decode.shard_range(global_rows, world, rank)[0]
    collected, elapsed = _run(rows, world, rank, shard_rows, gather,
                              _tokens(mode, world, rank, global_rows), row0, staging)
    if rank == 0:
        q.put((collected, elapsed))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode,gather,global_rows", [
    ("weak", "logits", 0),
    ("weak", "ids", 0),
    ("strong", "logits", 5),  # ragged: 3 + 2, point-to-point receives on rank 0
    ("strong", "ids", 5),
])
def test_sharded_hip_decode_matches_one_process(gpu, mode, gather, global_rows):
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mode, gather, global_rows, q))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        collected, elapsed = q.get(timeout=100)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.exitcode is None:
                p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert elapsed > 0 and len(collected) == WARMUP + STEPS
    first = np.concatenate([_tokens(mode, world, r, global_rows) for r in range(world)])
    ref, _ = _run(len(first), 1, 0, None, gather, first)
    for s in range(WARMUP + STEPS):
        assert collected[s].shape == ref[s].shape, (s, collected[s].shape, ref[s].shape)
        assert np.array_equal(collected[s].view(np.uint32) if gather == "logits" else collected[s],
                              ref[s].view(np.uint32) if gather == "logits" else ref[s]), s


@pytest.mark.timeout(300)
@pytest.mark.parametrize("mode,global_rows", [("weak", 0), ("strong", 5)])
def test_sharded_hip_decode_long_context(gpu, mode, global_rows):
    """The sharded loop at a real context: every row prefilled with its own
    600-token prompt, so each step's attention runs several splits, and the
    split count follows the rows per process (3 or 2 per rank here, 6 or 5 in
    the one-process reference), so the split merge sums in another order.
    The tolerance for that is stated: logits within 1e-3 of the one-process
    run, tensor-normalised, over every gathered step (the free-running decode
    lets an int8 rounding flip propagate; measured far below it), greedy ids
    equal unless the one-process logits tie within 1e-3 of their scale."""
    import torch.multiprocessing as mp
    from _util import rel_err
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mode, "logits", global_rows, q, True))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        collected, _ = q.get(timeout=200)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.exitcode is None:
                p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    first = np.concatenate([_tokens(mode, world, r, global_rows) for r in range(world)])
    ref, _ = _run(len(first), 1, 0, None, "logits", first, row0=0)
    worst = 0.0
    for s_ in range(WARMUP + STEPS):
        a, b = collected[s_], ref[s_]
        assert a.shape == b.shape, (s_, a.shape, b.shape)
        err = rel_err(a, b)
        worst = max(worst, err)
        assert err < 1e-3, (s_, err)
        ga, gb = a.argmax(axis=1), b.argmax(axis=1)
        for r in np.nonzero(ga != gb)[0]:
            assert b[r, gb[r]] - b[r, ga[r]] <= 1e-3 * np.abs(b[r]).max(), (s_, r)
    print(f"sharded vs one process at {PROMPT}+ tokens: worst logits rel err {worst:.2e}")


@pytest.mark.parametrize("gather", ["logits", "ids"])
def test_sharded_hip_decode_device_staging(gpu, gather):
    """The staging="device" branch bench.py runs over RCCL: each step's rows
    are written straight into the RowGatherer's device buffers and the gather
    takes the device tensors (gloo's gather accepts them and moves them
    through host memory itself; on the 8-GPU node the same tensors go to
    RCCL).  Weak sharding: the equal-shard torch.distributed gather.  Rank 0's
    gathered steps must equal one process stepping all rows, bit for bit."""
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, "weak", gather, 0, q, False, "device"))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        collected, _ = q.get(timeout=100)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.exitcode is None:
                p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    first = np.concatenate([_tokens("weak", world, r, 0) for r in range(world)])
    ref, _ = _run(len(first), 1, 0, None, gather, first)
    assert len(collected) == WARMUP + STEPS
    for s in range(WARMUP + STEPS):
        a, b = collected[s], ref[s]
        assert a.shape == b.shape, (s, a.shape, b.shape)
        assert np.array_equal(a.view(np.uint32) if gather == "logits" else a,
                              b.view(np.uint32) if gather == "logits" else b), s


def _rccl_worker(port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    for p in (str(ROOT), str(PKG)):
        sys.path.insert(0, p)
    import torch
    import torch.distributed as dist
    import dist_decode
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    with torch.cuda.stream(torch.cuda.Stream()):
        t = torch.arange(3 * V, dtype=torch.float32, device="cuda").view(3, V)
        recv = [torch.full((3, V), -1.0, device="cuda")]
        dist_decode._gather(t, recv, 0).wait()
        ids = torch.arange(7, dtype=torch.int32, device="cuda")
        rids = [torch.zeros(7, dtype=torch.int32, device="cuda")]
        dist_decode._gather(ids, rids, 0).wait()
        torch.cuda.synchronize()
        q.put((torch.equal(recv[0], t), torch.equal(rids[0], ids), dist.get_backend()))
    dist.destroy_process_group()


def test_rccl_gather_of_device_rows(gpu):
    """The RCCL leg of the device-staged gather on the one-GPU box: a one-rank
    nccl (= RCCL) group gathers device logits and id rows with the same
    dist_decode._gather call the multi-GPU loop makes (RCCL refuses two ranks
    on one device, so this is as far as one GPU takes it)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), q))
    p.start()
    try:
        ok_logits, ok_ids, backend = q.get(timeout=100)
    finally:
        p.join(timeout=30)
        if p.exitcode is None:
            p.kill()
    assert p.exitcode == 0, p.exitcode
    assert backend == "nccl" and ok_logits and ok_ids
