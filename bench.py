#!/usr/bin/env python3
"""Decode throughput of the MI355X paged-attention INT8 decoder (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2|c4|c5|c1]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

Workload (default, BASELINE config C3): INT8Decoder with 24 layers, 16 heads,
head_dim 128 (hidden 2048, inter 8192, vocab 50257), a batch of 64 sequences,
every sequence holding a KV context of 8192 tokens in shuffled 16-token pages
(synthetic random fp16 K/V, random-init int8 weights — no checkpoints exist).
A step = one full decode step of all rows (embed, 24 x {LN, qkv GEMM, KV
append, paged attention, o GEMM, LN, fc1, fc2}, tied LM head, argmax), replayed
as a hipGraph; generation continues from step to step (the context grows).

Multi-GPU: one process per GPU.  `--gpus N` with no WORLD_SIZE in the
environment starts the N ranks itself (before torch or any GPU is touched);
under torch.distributed.run it checks that the launcher started exactly N.
Sequences are sharded by rank, no exchange inside a step; the final logits of
every step are gathered to rank 0 over RCCL (the one collective of the design).
The headline follows the metric's own mode: C3 / C2 scale STRONG,
the config's batch (64 for C3) split over the N ranks; C5 (64 rows per GPU by
definition) and C4 scale weak.  At N > 1 a strong line also carries the weak
figure (the config's batch on EVERY rank) as `weak_scaling`.  value = tokens/s
of the whole job = rows of all ranks / t_step, t_step = max over ranks.

Also reported (one JSON line on rank 0):
  roofline     the paged-attention launch (the dominant kernel), timed live with
               HIP events on the stream it runs on, against 8 TB/s HBM
  cpu_baseline the oracle's restated INT8Decoder step on this host's cores
               (bounded sample, see `sample`)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
PKG = ROOT / "pagedattention-based-transformer-decoder-inference-framework_amd"
sys.path.insert(0, str(PKG))
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

CONFIGS = {
    # BASELINE.json configs[2]: the metric's config
    "c3": dict(cls="INT8Decoder", L=24, H=16, D=128, V=50257, B=64, T=8192, ts=16, strong=True,
               workload="C3: INT8 decoder (MFMA i8 matmuls + fp16 paged attention), "
                        "24-layer/16-head/d=128, batch 64, KV context 8192, page 16"),
    # BASELINE.json configs[3]: beam=4 decode over forked prefixes (C3 model dims,
    # SURVEY §8 C4 build decision): 8 sequences x 4 beams; each sequence's first
    # 3840 tokens live in shared (forked) pages, each beam holds 256 private tokens
    "c4": dict(cls="INT8Decoder", L=24, H=16, D=128, V=50257, B=32, T=4096, ts=16,
               seqs=8, beams=4, shared=3840,
               workload="C4: beam=4 INT8 decode, 8 seqs x 4 beams (24-layer/16-head/d=128), "
                        "KV context 4096 = 3840 shared (page-table fork) + 256 per beam, "
                        "beam-aware attention schedule"),
    # BASELINE.json configs[4], per GPU: 64 of the 512 rows on each of 8 GPUs
    # (KV 275 GB per GPU at context 8192: the page pool fills the card)
    "c5": dict(cls="INT8Decoder", L=32, H=32, D=128, V=50257, B=64, T=8192, ts=16,
               workload="C5 (per GPU): INT8 decoder, 32-layer/32-head/d=128, 64 seqs/GPU "
                        "(512 over 8 GPUs), KV context 8192, page 16"),
    # BASELINE.json configs[0]: the reference's CPU-runnable case (INT8Decoder,
    # batch 1); its CPU baseline is timed end to end (whole steps)
    "c1": dict(cls="INT8Decoder", L=2, H=4, D=64, V=50257, B=1, T=128, ts=16, cpu_full=True,
               workload="C1: INT8 decoder, 2-layer/4-head/d=64, batch 1, KV context 128, "
                        "page 16"),
    # BASELINE.json configs[1]
    "c2": dict(cls="CUDADecoder", L=12, H=12, D=64, V=50257, B=16, T=2048, ts=16, strong=True,
               workload="C2: fp16 paged decode, 12-layer/12-head/d=64, batch 16, "
                        "KV context 2048, page 16"),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_weights(cfg, seed):
    rng = np.random.default_rng(seed)
    L, hid, V = cfg["L"], cfg["H"] * cfg["D"], cfg["V"]
    inter = 4 * hid
    w = {"emb": rng.standard_normal((V, hid), dtype=np.float32).astype(np.float16).view(np.uint16)}
    w["ln1_g"] = np.ones((L, hid), np.float32)
    w["ln2_g"] = np.ones((L, hid), np.float32)
    w["ln1_b"] = (0.1 * rng.standard_normal((L, hid), dtype=np.float32))
    w["ln2_b"] = (0.1 * rng.standard_normal((L, hid), dtype=np.float32))
    w["b1"] = (0.02 * rng.standard_normal((L, inter), dtype=np.float32))
    w["b2"] = (0.02 * rng.standard_normal((L, hid), dtype=np.float32))
    shapes = {"wqkv": (hid, 3 * hid), "wo": (hid, hid), "w1": (hid, inter), "w2": (inter, hid)}
    if cfg["cls"] == "INT8Decoder":
        for k, (K, N) in shapes.items():
            w[k] = rng.integers(-127, 128, size=(L, K, N), dtype=np.int8)
        scale = np.float32(0.02 * 3.0 / 127.0)
        w["sw_qkv"] = np.full((L, 3 * hid), scale, np.float32)
        w["sw_o"] = np.full((L, hid), scale, np.float32)
        w["sw1"] = np.full((L, inter), scale, np.float32)
        w["sw2"] = np.full((L, hid), scale, np.float32)
    else:
        for k, (K, N) in shapes.items():
            w[k] = (0.02 * rng.standard_normal((L, K, N), dtype=np.float32)).astype(np.float16).view(np.uint16)
    return w


def step_bytes(cfg, T_mean, B):
    """Algorithmic HBM bytes of one decode step: fp16 K+V of every
    row/head/token (shared beam prefixes once per sequence), page-table
    entries, int8 weights + fp32 scales, q/out, tied fp16 LM head.  Re-reads
    are not counted."""
    L, H, D, V, ts = cfg["L"], cfg["H"], cfg["D"], cfg["V"], cfg["ts"]
    hid, inter = H * D, 4 * H * D
    nt = (T_mean + ts - 1) / ts
    kv_tokens = B * T_mean
    if "beams" in cfg:
        kv_tokens = cfg["seqs"] * cfg["shared"] + B * (T_mean - cfg["shared"])
    attn = 2 * kv_tokens * H * D * 2 + B * H * nt * 4 + 2 * B * hid * 4
    wbytes = 1 if cfg["cls"] == "INT8Decoder" else 2
    gemm = hid * (3 * hid + hid + 2 * inter) * wbytes + 4 * (3 * hid + hid + inter + hid)
    return L * (attn + gemm) + V * hid * 2


def attention_launch_bytes(cfg, T, B, unique=False):
    """Algorithmic bytes of one attention launch: fp16 K+V of every (row, head,
    token) + page-table entries + q/out.  unique=True (beam configs) counts
    each shared prefix page once per sequence (what HBM must deliver)."""
    H, D, ts = cfg["H"], cfg["D"], cfg["ts"]
    nt = (T + ts - 1) // ts
    kv_tokens = B * T
    if unique and "beams" in cfg:
        kv_tokens = cfg["seqs"] * cfg["shared"] + B * (T - cfg["shared"])
    return 2 * kv_tokens * H * D * 2 + B * H * nt * 4 + 2 * B * H * D * 4


def time_attention(dec, layers, iters=24):
    """Live HIP-event timing of the decoder's own paged-attention launch
    (llm_decoder_run_attention: the step graph's kernels, grid and outputs --
    split + merge-and-quantise for INT8, the workgroup-merge form for FP16,
    the beam-group schedule for beams), enqueued on torch's current stream so
    the events bracket exactly those kernels.  The launches rotate over the
    `layers` layers, as in the step: relaunching one layer back to back lets
    the 256 MiB Infinity Cache re-serve a KV zone that fits it (C2: 101 MB per
    layer, 21.0 vs 22.3 us; scripts/attn_rotate.py)."""
    import torch
    st = torch.cuda.current_stream().cuda_stream
    for i in range(3):
        dec.run_attention(i % layers, st)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(iters):
        dec.run_attention(i % layers, st)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def time_attention_plain(dec, cfg, B, T, max_seq, iters=20):
    """The same attention as a plain pa_decode_grouped launch (row_group 1,
    fp32 output; beam configs: the schedule without beam awareness)."""
    import torch
    import llm_decoder
    H, D = cfg["H"], cfg["D"]
    q = torch.randn((B, H, D), device="cuda") * D ** -0.25
    out = torch.empty((B, H, D), device="cuda")
    ctx = torch.full((B,), T, dtype=torch.int32, device="cuda")
    max_tiles = (max_seq + cfg["ts"] - 1) // cfg["ts"]
    wsb = llm_decoder.workspace_bytes(B, H, D, max_tiles, 0)
    ws = torch.empty(max(wsb, 16), dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream().cuda_stream

    def run():
        llm_decoder.paged_attention(dec.kv_handle, 0, q.data_ptr(), out.data_ptr(), 0,
                                    ctx.data_ptr(), B, H, D, max_seq, 1.0, 0, 1.0,
                                    ws.data_ptr(), wsb, st, 1)
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        run()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


FORM_NAMES = {0: "direct (one split)", 1: "split + pa_merge_kernel",
              2: "split + pa_merge_row_kernel (merge + per-row int8 quantisation)",
              3: "split with workgroup merge"}
# what the launch writes, by decoder kind (the INT8 o_proj quantises fp32 rows in
# its prologue; the FP16 one reads packed fp16 rows)
FORM_OUT = {"INT8Decoder": {0: " (fp32 rows; the o_proj prologue quantises them)",
                            1: " (fp32 rows; the o_proj prologue quantises them)",
                            3: " (fp32 rows; the o_proj prologue quantises them, or a quantise "
                               "launch for rows wider than 2048)"},
            "CUDADecoder": {3: " (packed fp16 o_proj input)"}}
# form bit 32: the FP16 decoder's o_proj runs inside the workgroup merge
OPROJ_OUT = " (o_proj fused: each (row, head) workgroup adds o_h W_o[h] into int64 rows)"


def fused_weight_bytes(cfg, form):
    """Unique weight bytes the fused form of the FP16 attention launch reads
    besides the KV pages: W_o (o_proj fused, form bit 32), fp16, once per
    launch from HBM / the Infinity Cache."""
    hid = cfg["H"] * cfg["D"]
    return 2 * hid * hid if form & 32 else 0


TORCHRUN_CPU_SHARE = 16  # the GPU pool's OpenMP share of a 1-GPU job


def cpu_threads():
    """Threads of the CPU baseline: the job's OpenMP share (OMP_NUM_THREADS:
    the GPU pool gives each 1-GPU job 16 of the host's CPUs and sets it so;
    BASELINE.md's $(nproc) would take every CPU of a host shared by 8 GPUs'
    jobs), else every CPU this process may run on."""
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS", "")
    if env == "1" and "TORCHELASTIC_RUN_ID" in os.environ:
        # torch.distributed.run sets OMP_NUM_THREADS=1 in every worker it
        # starts; the baseline keeps the 1-GPU job's share instead, so it is
        # the same measurement at every N
        env = str(TORCHRUN_CPU_SHARE)
    n = int(env) if env.isdigit() and int(env) > 0 else avail
    return min(n, avail), avail


def cpu_baseline(cfg_name, budget_s=20.0):
    """The CPU baseline, run in a child process (no GPU in it) whose OpenMP
    runtime starts with OMP_PROC_BIND=close, OMP_PLACES=cores and
    OMP_NUM_THREADS = cpu_threads(): those are read when
    the OpenMP runtime starts, which in this process torch has already done."""
    import subprocess
    threads, avail = cpu_threads()
    env = dict(os.environ, OMP_NUM_THREADS=str(threads), OMP_PROC_BIND="close",
               OMP_PLACES="cores")
    r = subprocess.run([sys.executable, str(Path(__file__).resolve()), "--cpu-baseline-child",
                        "--config", cfg_name, "--cpu-budget", str(budget_s)],
                       env=env, capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        raise RuntimeError(f"cpu baseline child failed ({r.returncode}): {r.stderr[-2000:]}")
    res = json.loads(r.stdout.strip().splitlines()[-1])
    res["cpus_available"] = avail
    res["cpu"]["cpus_available"] = avail  # (the child's own affinity is one place once bound)
    res["omp"] = {"OMP_NUM_THREADS": threads, "OMP_PROC_BIND": "close", "OMP_PLACES": "cores"}
    env_omp = os.environ.get("OMP_NUM_THREADS", "")
    if env_omp == "1" and "TORCHELASTIC_RUN_ID" in os.environ:
        res["threads_reason"] = (
            f"torch.distributed.run set OMP_NUM_THREADS=1 in this worker; the baseline keeps a "
            f"1-GPU job's OpenMP share ({threads} of {avail} CPUs in the affinity mask)")
        return res
    res["threads_reason"] = (
        f"the job's OpenMP share: OMP_NUM_THREADS={env_omp} set by the GPU pool for a 1-GPU job "
        f"on a host shared by 8 GPUs' jobs ({avail} CPUs in the affinity mask); BASELINE.md asks "
        f"for $(nproc), which here would take the other jobs' CPUs"
        if env_omp.isdigit() and int(env_omp) > 0 and int(env_omp) < avail
        else f"every CPU in this process's affinity mask ({avail})")
    return res


def cpu_baseline_run(cfg, budget_s=20.0):
    """The oracle (restated INT8Decoder / CUDADecoder, C++/OpenMP, built with
    -march=native on this host) timed on this host's cores over a bounded
    sample of the same workload.  C1 (the reference's own CPU-runnable
    config) is timed end to end: whole decode steps, every layer and the LM
    head.  Larger configs: up to 16 of the rows through ONE layer at the full
    KV context (median of up to 5), scaled to all layers, plus the LM head."""
    from oracle.oracle import Oracle, OracleDecoder, host_cpu, native_build
    native = native_build()
    o = Oracle(bench="native" if native else True)
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if threads > 0:
        o.lib.oracle_set_num_threads(threads)
    L, H, D, V, T, B = cfg["L"], cfg["H"], cfg["D"], cfg["V"], cfg["T"], cfg["B"]
    hid = H * D
    full = cfg.get("cpu_full", False)
    rows = B if full else min(B, 16)
    layers = L if full else 1
    mcfg = dict(cfg, L=layers)
    w = make_weights(mcfg, 99)
    wd = {k: np.ascontiguousarray(v) for k, v in w.items()}
    wd["emb"] = w["emb"].view(np.float16)
    wd["cfg"] = dict(L=layers, H=H, D=D, hid=hid, inter=4 * hid, V=V, max_seq=T + 1)
    dec = OracleDecoder(o, wd, rows)
    rng = np.random.default_rng(0)
    for l in range(layers):
        for which in (0, 1):  # fill the context: positive fp16 values in [0.125, 1)
            kv = dec.kv(l, which)
            kv[:, :, :T].view(np.uint16)[...] = rng.integers(0x3000, 0x3C00, kv[:, :, :T].shape,
                                                              dtype=np.uint16)
    toks = np.arange(rows, dtype=np.int32)
    pos = np.full(rows, T, np.int32)
    t0 = time.perf_counter()
    times = []
    while True:
        a = time.perf_counter()
        dec.step(toks, pos, layers=-1 if full else 1, lm_head=full)
        times.append(time.perf_counter() - a)
        if time.perf_counter() - t0 > budget_s * 0.6 or len(times) >= (20 if full else 5):
            break
    if full:
        t_step = float(np.median(times))
        sample = (f"{rows} row(s), whole decode steps ({L} layers + LM head) at KV context {T} "
                  f"(median of {len(times)})")
    else:
        a = time.perf_counter()
        dec.step(toks, pos, layers=0, lm_head=True)
        t_lm = time.perf_counter() - a
        t_step = L * float(np.median(times)) + t_lm
        sample = (f"{rows} of {B} rows, 1 of {L} layers at KV context {T} (median of "
                  f"{len(times)}) x {L} layers + LM head")
    lib = "oracle/liboracle_native.so (-O3 -march=native, built on this host)" if native else \
        "oracle/liboracle_bench.so (-O3 -march=x86-64-v3: the native build failed)"
    return {"value": rows / t_step, "unit": "tokens/s", "cores": o.num_threads(), "kind": "port",
            "sample": f"{sample}, {lib}",
            "decoder": "restated " + ("INT8Decoder" if cfg["cls"] == "INT8Decoder" else "CUDADecoder"),
            "cpu": host_cpu()}


def load_traffic(cfg_name):
    """Measured HBM bytes / algorithmic bytes of the attention launch, from the
    committed rocprofv3 --pmc summary (profiles/pmc_attention_<cfg>.json:
    (2*FETCH_SIZE + WRITE_SIZE) KiB per launch, gfx950-corrected, over
    scripts/prof_attention.py at this config), or None."""
    p = ROOT / "profiles" / f"pmc_attention_{cfg_name}.json"
    if not p.exists():
        return None
    try:
        return float(json.loads(p.read_text())["traffic_over_algorithmic"])
    except Exception:
        return None


def spawn_ranks(n, argv):
    """`bench.py --gpus N` with no WORLD_SIZE in the environment: start N copies
    of this script as ranks 0..N-1 (RANK / LOCAL_RANK / WORLD_SIZE /
    LOCAL_WORLD_SIZE / MASTER_ADDR / MASTER_PORT in their environment, the
    same variables torch.distributed.run sets).  This process has not imported
    torch and never touches a GPU: it only waits.  When a rank fails, the
    others are terminated (a rank blocked in a collective would wait for its
    dead peer forever) and the launcher exits non-zero.  Rank 0 prints the one
    JSON line; the other ranks print nothing on stdout."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    script = str(Path(__file__).resolve())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, script] + list(argv), env=env))
    import signal

    def stop(signum, _frame):  # the launcher itself stopped (driver timeout, ^C): take the ranks along
        for q in procs:
            if q.poll() is None:
                q.terminate()
        t_end = time.time() + 10
        for q in procs:
            try:
                q.wait(timeout=max(0.1, t_end - time.time()))
            except subprocess.TimeoutExpired:
                q.kill()
        sys.exit(128 + signum)
    signal.signal(signal.SIGTERM, stop)
    signal.signal(signal.SIGINT, stop)
    rc, deadline = 0, None
    live = dict(enumerate(procs))
    while live:
        for r, p in list(live.items()):
            c = p.poll()
            if c is None:
                continue
            del live[r]
            if c != 0 and rc == 0:
                rc = c if c > 0 else 128 - c
                log(f"bench.py launcher: rank {r} exited with {c}; stopping ranks {sorted(live)}")
                for q in live.values():
                    q.terminate()
                deadline = time.time() + 30
        if deadline is not None and time.time() > deadline:
            for q in live.values():
                q.kill()
            deadline = None
        time.sleep(0.1)
    return rc


class StubStep:
    """`--stub-step` (CPU tests of the launcher and of the multi-rank line
    only): a deterministic host step in place of the HIP decoder.  logits[b, v]
    and the next ids are cheap integer functions of the row's token."""

    def __init__(self, rows, vocab):
        self.rows, self.V = rows, vocab
        self.next = np.zeros(rows, np.int64)

    def __call__(self, tokens, logits_out):
        import torch
        tok = np.asarray(tokens if tokens is not None else self.next, np.int64)
        if logits_out is not None:
            v = torch.arange(self.V, dtype=torch.int64)
            t = torch.from_numpy(tok)[:, None]
            logits_out.copy_(((t * 31 + v * 7) % 97).to(torch.float32))
        self.next = (tok * 31 + 7) % self.V

    def ids_into(self, out):
        import torch
        out.copy_(torch.from_numpy(self.next.astype(np.int32)))


def run_mode(cfg, args, world, rank, strong, backend, stub):
    """Build this rank's decoder for one scaling mode and time the sharded
    decode loop (dist_decode.ShardedDecode + timed_run).  strong: the global
    batch (args.global_batch or the config's batch) split over the ranks,
    first tokens one global draw, sharded; weak: the config's batch on every
    rank, first tokens drawn per rank.  Returns (stats, decoder or None)."""
    import dist_decode
    B, T = cfg["B"], cfg["T"]
    shard_rows, G = None, B * world
    if strong:
        G = args.global_batch or B
        if G < world:
            raise SystemExit(f"bench.py: a global batch of {G} rows needs >= {world} rows")
        shard_rows = dist_decode.shard_sizes(G, world)
        B = shard_rows[rank]
        lo, hi = dist_decode.shard_range(G, world, rank)
        tokens = np.random.default_rng(args.seed).integers(0, cfg["V"], G).astype(np.int32)[lo:hi]
    else:
        tokens = np.random.default_rng(args.seed + rank).integers(0, cfg["V"], B).astype(np.int32)
    host_gather = world > 1 and backend != "nccl" and not stub
    gather = args.gather if world > 1 else "none"
    t0 = time.time()
    dec = None
    if stub:
        step = StubStep(B, cfg["V"])
        device, sync, timer, step_times = "cpu", (lambda: None), "cpu", None
    else:
        import torch
        import llm_decoder  # noqa: F401  (fails loudly if the HIP build is missing)
        max_seq = T + 2 * (args.warmup + args.steps) + 16
        cls = getattr(llm_decoder, cfg["cls"])
        dec = cls(cfg["L"], cfg["H"], cfg["D"], cfg["H"] * cfg["D"], cfg["V"], max_seq,
                  max_batch=B, page_size=cfg["ts"])
        w = make_weights(cfg, args.seed)
        dec.set_weights(w)
        del w
        if "beams" in cfg:
            dec.begin_beams(cfg["seqs"], cfg["beams"], cfg["shared"], T - cfg["shared"],
                            args.seed + rank, not args.contiguous_pages)
        else:
            dec.begin_synthetic(B, T, args.seed + rank, not args.contiguous_pages)
        step = dist_decode.HipDecoderStep(dec)
        device, sync = "cuda", torch.cuda.synchronize
        timer = "cpu" if host_gather else "cuda"
        step_times = None if host_gather else []
    log(f"[rank {rank}] {'strong' if strong else 'weak'}: {B} rows, setup {time.time() - t0:.1f}s")
    # each step's logits (or greedy ids, --gather ids) go to rank 0, double-buffered
    # behind the next step; gloo rehearsals on GPUs stage them through host memory
    sd = dist_decode.ShardedDecode(step, B, cfg["V"], world=world, rank=rank,
                                   shard_rows=shard_rows, gather=gather, device=device,
                                   staging="host" if host_gather else "device")
    rank_times = []
    elapsed = dist_decode.timed_run(sd, args.warmup, args.steps, list(map(int, tokens)),
                                    sync=sync, timer_device=timer, step_times=step_times,
                                    rank_times=rank_times)
    t_step = elapsed / args.steps
    st = {"rows_this_rank": B, "global_rows": G, "t_step": t_step,
          "per_rank_ms_per_step": [round(t / args.steps * 1e3, 4) for t in rank_times],
          "step_times": step_times, "value": G / t_step}
    t_g = dist_decode.time_gather(sd, sync=sync, timer_device=timer) if world > 1 else None
    if t_g is not None:
        per_peer = sd.g.bufs[0].numel() * sd.g.bufs[0].element_size()
        st["gather"] = {"what": gather, "bytes_per_rank": per_peer,
                        "alone_ms": round(t_g * 1e3, 4),
                        "share_of_step": round(t_g / t_step, 4),
                        "note": "one step's gather timed on its own (max over ranks); in the "
                                "step it is double-buffered behind the next step's compute"}
    return st, dec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-baseline-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--scaling", default="auto", choices=["auto", "strong", "weak"],
                    help="auto: the metric's mode (C3 / C2 strong, C4 / C5 weak)")
    ap.add_argument("--global-batch", type=int, default=0,
                    help="strong scaling: this many rows in total, sharded over the ranks "
                         "(default: the config's batch)")
    ap.add_argument("--no-weak-extra", action="store_true",
                    help="N > 1, strong headline: skip the extra weak-scaling run")
    ap.add_argument("--gather", default="logits", choices=["logits", "ids"],
                    help="N > 1: what each step gathers to rank 0 (SURVEY §8e)")
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--contiguous-pages", action="store_true",
                    help="sensitivity runs only: pages in allocation order instead of the "
                         "shuffled pool SURVEY §8d measures on")
    ap.add_argument("--stub-step", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--stub-fail-rank", type=int, default=-1, help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.cpu_baseline_child:  # cpu_baseline()'s child: no torch, no GPU
        print(json.dumps(cpu_baseline_run(CONFIGS[args.config], args.cpu_budget)), flush=True)
        return
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    # stdout carries the one JSON line alone: whatever native code prints there
    # (gloo's connection notes, RCCL / HIP chatter) goes to stderr instead
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started {world} rank(s)")
    if rank == args.stub_fail_rank:
        raise SystemExit(3)
    cfg = CONFIGS[args.config]
    stub = args.stub_step
    # LLM_DIST_BACKEND=gloo: rehearsal of the N-rank path on fewer GPUs (ranks
    # share devices round-robin, logits gathered through host memory); the
    # real multi-GPU run is one rank per GPU over RCCL ("nccl").
    backend = "gloo" if stub else os.environ.get("LLM_DIST_BACKEND", "nccl")

    import torch
    import torch.distributed as dist
    if not stub:
        ndev = torch.cuda.device_count()  # (does not initialise the GPU on this image)
        if ndev < 1:
            raise SystemExit("bench.py: no GPU visible")
        lws = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
        if backend == "nccl" and world > 1 and (ndev < lws or local >= ndev):
            raise SystemExit(f"bench.py: --gpus {world} over RCCL needs one GPU per rank, "
                             f"{ndev} visible to local rank {local} of {lws} (RCCL refuses two "
                             f"ranks on one device; LLM_DIST_BACKEND=gloo rehearses N ranks "
                             f"on fewer GPUs)")
        local = local % ndev
        torch.cuda.set_device(local)
        # every step, staging copy, gather and timing event runs on ONE explicit
        # stream (torch's default stream has handle 0, which the C ABI reads as the
        # decoder's own non-blocking stream)
        torch.cuda.set_stream(torch.cuda.Stream())
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"bench.py: process group of {dist.get_world_size()} ranks, "
                             f"--gpus {args.gpus}")
    pg_size = dist.get_world_size() if world > 1 else 1

    mode = args.scaling
    if mode == "auto":
        mode = "strong" if (cfg.get("strong") or args.global_batch) else "weak"
    strong = mode == "strong" and "beams" not in cfg
    st, dec = run_mode(cfg, args, world, rank, strong, backend, stub)
    B, T, t_step = st["rows_this_rank"], cfg["T"], st["t_step"]
    T_mean = T + args.warmup + args.steps / 2.0
    host_gather = world > 1 and backend != "nccl"

    # roofline of the dominant kernel (paged attention): the step's own launch,
    # timed live on rank 0's decoder
    roof, step_b = None, step_bytes(cfg, T_mean, B)
    if dec is not None and rank == 0:
        T_now = dec.context_len(0)
        nsplit, form = dec.attention_plan()
        t_attn = time_attention(dec, cfg["L"])
        attn_b = attention_launch_bytes(cfg, T_now, B, unique=True) + fused_weight_bytes(cfg, form)
        achieved = attn_b / t_attn / 1e9
        ratio = load_traffic(args.config)
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                # PMC-measured HBM bytes per launch (ratio from profiles/pmc_attention_<cfg>.json
                # applied to this launch's algorithmic bytes)
                "traffic": int(ratio * attn_b) if ratio else None,
                "traffic_over_algorithmic": ratio,
                "traffic_source": (f"profiles/pmc_attention_{args.config}.json: rocprofv3 PMC "
                                   "(2*FETCH_SIZE + WRITE_SIZE) / algorithmic bytes, committed, "
                                   "times this launch's algorithmic bytes (not measured in this "
                                   "run)") if ratio else None,
                "kernel": f"pa_split_kernel<D={cfg['D']},TS={cfg['ts']}>"
                          + (" beam-group" if form & 16 else "") + ": " + FORM_NAMES[form & 15]
                          + (OPROJ_OUT if form & 32 else FORM_OUT.get(cfg["cls"], {}).get(form & 15, ""))
                          + f", {nsplit} splits, {B} rows (the step's own launch, "
                            "llm_decoder_run_attention)",
                "bytes_per_launch": attn_b, "launch_us": round(t_attn * 1e6, 2),
                "launch_timing": f"HIP events over 24 launches rotating over the {cfg['L']} layers"}
        if "beams" in cfg:  # logical bytes: every beam reads its whole context
            logical = attention_launch_bytes(cfg, T_now, B)
            roof["bytes_note"] = "achieved counts shared prefix pages once per sequence"
            roof["logical_bytes_per_launch"] = logical
            roof["logical_GBps"] = round(logical / t_attn / 1e9, 1)
            max_seq = T + 2 * (args.warmup + args.steps) + 16
            t_plain = time_attention_plain(dec, cfg, B, T_now, max_seq)
            roof["ungrouped_launch_us"] = round(t_plain * 1e6, 2)  # plain schedule, fp32 out

    weak = None
    if world > 1 and strong and not args.no_weak_extra:
        del dec  # the strong run's pools go before the weak run allocates its own
        import gc
        gc.collect()
        sw, dec = run_mode(cfg, args, world, rank, False, backend, stub)
        weak = {"value": round(sw["value"], 2), "unit": "tokens/s",
                "ms_per_step": round(sw["t_step"] * 1e3, 4), "batch_per_gpu": cfg["B"],
                "global_batch": sw["global_rows"],
                "per_rank_ms_per_step": sw["per_rank_ms_per_step"],
                "hbm_roofline_frac_step": round(step_bytes(cfg, T_mean, cfg["B"])
                                                / sw["t_step"] / 1e9 / HBM_PEAK_GBPS, 4),
                "gather": sw.get("gather"),
                "note": "the config's batch on every rank (weak scaling), same loop, run after "
                        "the headline in the same job"}
    del dec

    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(args.config, args.cpu_budget)
        except Exception as ex:  # the baseline never blocks the GPU number
            log(f"cpu baseline failed: {ex!r}")
    if rank == 0:
        G = st["global_rows"]
        step_times = st["step_times"]
        import dist_decode
        rows_all = dist_decode.shard_sizes(G, world) if strong else [B] * world
        res = {
            "metric": "decode tokens/sec at batch=64 seq_len=8192; % HBM-roofline (1/2/4/8 GPU)"
            if args.config == "c3" else f"decode tokens/sec ({args.config})",
            "value": round(st["value"], 2),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t_step * 1e3, 4),
            "ms_per_step_median_hip_events": round(float(np.median(step_times)) * 1e3, 4)
            if step_times else None,
            "per_rank_ms_per_step": st["per_rank_ms_per_step"],
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "int8 GEMM (i32 acc) + fp16 KV attention (fp32 acc)"
            if cfg["cls"] == "INT8Decoder" else "fp16 GEMM + fp16 KV attention (fp32 acc)",
            "data": "synthetic (random-init weights, random fp16 KV context, "
                    + ("pages in allocation order)" if args.contiguous_pages else "shuffled pages)")
                    + ("; STUB host step (launcher test, no decoder)" if stub else ""),
            "config": {"workload": cfg["workload"] + (f"; strong scaling: {G} rows over {world} "
                                                      f"GPU(s)" if strong else
                                                      f"; weak scaling: {B} rows per GPU"),
                       "global_batch": G, "batch_per_gpu": B, "seq_len": T,
                       "page_size": cfg["ts"],
                       "parallelism": "single GPU (no collective)" if world == 1
                       else f"batch-sharded x{world} (RCCL {args.gather} gather to rank 0)"
                       if not host_gather else f"batch-sharded x{world} ({backend} rehearsal)"},
            "rccl_ranks": pg_size if backend == "nccl" and world > 1 else 0,
            "process_group": {"backend": backend if world > 1 else None, "size": pg_size},
            "gather": st.get("gather"),
            # mean over the GPUs of each one's algorithmic step bytes / t_step / 8 TB/s
            "hbm_roofline_frac_step": round(sum(step_bytes(cfg, T_mean, r) for r in rows_all)
                                            / world / t_step / 1e9 / HBM_PEAK_GBPS, 4),
            "step_bytes": int(step_b),
            "roofline": roof,
            "weak_scaling": weak,
            "cpu_baseline": cpu,
        }
        print(json.dumps(res), file=json_out, flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
