"""Free-running greedy decode helpers shared by the CPU yardstick test
(test_generate_free_run.py: the oracle against itself with its reductions
reordered) and the GPU test (test_generate_free_run_gpu.py: the HIP decoder
against the oracle)."""
from __future__ import annotations

import numpy as np

from _util import rel_err

# C1 model dims (the reference's own CPU config) and C3's head shape / width
CASES = {
    "c1_dims": dict(L=2, H=4, D=64, V=1000, seed=2024),
    "h16_d128": dict(L=2, H=16, D=128, V=1000, seed=77),
}
ROWS, GEN = 8, 64


def case_model(oracle, case):
    """(weights, prompts) of a case: ROWS ragged prompts of 1..23 tokens."""
    from oracle.oracle import synthetic_int8_model
    p = CASES[case]
    rng = np.random.default_rng(p["seed"])
    prompts = [rng.integers(0, p["V"], int(n)).tolist() for n in rng.integers(1, 24, ROWS)]
    S = max(len(q) for q in prompts) + GEN
    w = synthetic_int8_model(oracle, L=p["L"], H=p["H"], D=p["D"], V=p["V"], max_seq=S,
                             seed=p["seed"])
    return w, prompts


def oracle_generate(oracle, w, prompts, gen):
    """The oracle INT8Decoder free running every row: each prompt token stepped
    at its position, then `gen` greedy ids per row, each fed back
    (INT8Decoder::generate, decoder/int8_decoder.cpp:106-119; argmax,
    decoder/cuda_decoder.cu:7-14).  Rows are independent (own positions, own
    KV); they step together so the oracle's GEMMs run one row per thread.
    Returns per row (ids [gen], logits of the step that produced each id
    [gen][V])."""
    from oracle.oracle import OracleDecoder
    B = len(prompts)
    od = OracleDecoder(oracle, w, B)
    ids = [[] for _ in range(B)]
    lg = [[] for _ in range(B)]
    nxt = [0] * B
    for i in range(max(len(p) for p in prompts) + gen - 1):
        tok = np.array([p[i] if i < len(p) else nxt[b] for b, p in enumerate(prompts)], np.int32)
        _, logits, n = od.step(tok, np.full(B, i, np.int32))
        nxt = [int(x) for x in n]
        for b, p in enumerate(prompts):
            if i >= len(p) - 1 and len(ids[b]) < gen:
                ids[b].append(nxt[b])
                lg[b].append(logits[b].copy())
    return [(ids[b], np.stack(lg[b])) for b in range(B)]


def compare_ids(got, ref, ref_logits):
    """First position where the generated ids differ (None: identical) and the
    gap there between the reference's top id and `got`'s id, relative to the
    reference row's logit scale."""
    j = next((i for i in range(len(ref)) if got[i] != ref[i]), None)
    if j is None:
        return None, None
    lg = ref_logits[j]
    return j, float((lg[ref[j]] - lg[got[j]]) / np.abs(lg).max())


def oracle_step_drift(oracle, w, seqs, reverse=False):
    """The oracle stepped over the given full sequences (no feedback) with its
    reductions in the reference order and, as `other`, reversed: worst
    tensor-normalised logit error per row.  With reverse=False `other` is the
    same order (zero drift: a self-check)."""
    from oracle.oracle import OracleDecoder
    B = len(seqs)
    n = min(len(s) for s in seqs)
    a, b = OracleDecoder(oracle, w, B), OracleDecoder(oracle, w, B)
    worst = np.zeros(B)
    for s in range(n - 1):
        tok = np.array([q[s] for q in seqs], np.int32)
        pos = np.full(B, s, np.int32)
        _, la, _ = a.step(tok, pos)
        with oracle.reduction_order(reverse):
            _, lb, _ = b.step(tok, pos)
        for r in range(B):
            worst[r] = max(worst[r], rel_err(lb[r], la[r]))
    return worst


def oracle_self_divergence(oracle, w, prompts, gen):
    """The oracle free running with reversed reductions against the reference
    order: per prompt (first divergence, gap), the reference order's
    (ids, logits) per row, and its full sequences (prompt + ids)."""
    ref = oracle_generate(oracle, w, prompts, gen)
    with oracle.reduction_order(True):
        rev = oracle_generate(oracle, w, prompts, gen)
    res = [compare_ids(rv[0], rf[0], rf[1]) for rv, rf in zip(rev, ref)]
    return res, ref, [list(p) + rf[0] for p, rf in zip(prompts, ref)]
