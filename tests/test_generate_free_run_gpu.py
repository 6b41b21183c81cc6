"""Free-running greedy generation against the oracle INT8Decoder.

`north_star`: "Outputs match attention_cpu/INT8Decoder on identical synthetic
weights+prompts".  The teacher-forced tests (test_decoder_gpu.py) hold every
step to 1e-3 with the int8 GEMM inputs forced; this file runs both decoders
FREE: the GPU's `generate_batch` (chunked prefill of the prompt, then greedy
decode steps; INT8Decoder::generate, decoder/int8_decoder.cpp:106-119, argmax
of sample_from_logits, decoder/cuda_decoder.cu:7-14) and the oracle decoder
stepping each prompt token by token, then feeding back its OWN argmax.

Free running, the two are not bit-identical and cannot be: an fp32 reduction
in another order (LayerNorm sums, attention dot products and softmax, split
merges) now and then moves one activation across an int8 rounding boundary
(one LSB = 1/127 of its row's absmax), and the KV cache carries that flip into
every later step.  How far that takes an INT8 decoder is a property of the
model, not of the GPU: the YARDSTICK is the oracle against ITSELF with only its
summation order reversed (oracle_set_reduction_order, tests/_freerun.py).
Measured on CPU with these prompts: at C1 dims 3 of 8 rows diverge (at ids 34,
44, 57; oracle gaps 0.26-0.92 % of the logit scale) and the logits drift up to
2.3 % of their scale; at 16 heads x d 128, 6 of 8 rows diverge (gaps 0.02-2.0 %)
with drift up to 7.0 % (tests/test_generate_free_run.py holds the C1 case).

The bar, per case, on the same weights and prompts:
  * generated ids identical to the oracle's up to each row's first divergence,
    and at that divergence the oracle's own logits show a near-tie: gap within
    twice the yardstick's logit drift (a flip cannot come from a wider gap than
    twice the logit error);
  * logit drift (both decoders fed the GPU's ids, no forcing): the GPU's worst
    row within 1.5x the yardstick's worst row on the SAME sequences, and below
    FREE_RUN_TOL[case] (the measured figure plus a margin);
  * a row where neither the GPU nor the yardstick flipped (drift < 1e-5) has
    identical ids all the way.
Measured figures go to gpurun_out/free_run.jsonl (profiles/r06/free_run_generate.jsonl)."""
import numpy as np
import pytest

from _freerun import CASES, GEN, ROWS, case_model, compare_ids, oracle_generate
from _util import record, rel_err

pytestmark = pytest.mark.gpu

# measured worst drift (profiles/r06/free_run_generate.jsonl) plus a margin
FREE_RUN_TOL = {"c1_dims": 3e-2, "h16_d128": 9e-2}
NO_FLIP_TOL = 1e-5


def _gpu_decoder(w, max_batch):
    import llm_decoder
    c = w["cfg"]
    dec = llm_decoder.INT8Decoder(c["L"], c["H"], c["D"], c["hid"], c["V"], c["max_seq"],
                                  max_batch=max_batch)
    d = {k: np.ascontiguousarray(v) for k, v in w.items() if k != "cfg"}
    d["emb"] = w["emb"].view(np.uint16)
    dec.set_weights(d)
    return dec


def _drift(dec, oracle, w, seqs):
    """GPU, oracle and reversed-order oracle stepped over the same sequences
    (no feedback, no forcing): worst logit error per row of the GPU and of the
    yardstick against the oracle."""
    import torch
    from oracle.oracle import OracleDecoder
    V = w["cfg"]["V"]
    B = len(seqs)
    n = min(len(s) for s in seqs)
    ref, rev = OracleDecoder(oracle, w, B), OracleDecoder(oracle, w, B)
    dec.begin_synthetic(B, 0, 0, False)
    logits = torch.empty((B, V), device="cuda")
    gpu, yard = np.zeros(B), np.zeros(B)
    for s in range(n - 1):
        tok = [q[s] for q in seqs]
        dec.step(tok, logits_ptr=logits.data_ptr())
        t, pos = np.array(tok, np.int32), np.full(B, s, np.int32)
        _, lr, _ = ref.step(t, pos)
        with oracle.reduction_order(True):
            _, lv, _ = rev.step(t, pos)
        torch.cuda.synchronize()
        gl = logits.cpu().numpy()
        for b in range(B):
            gpu[b] = max(gpu[b], rel_err(gl[b], lr[b]))
            yard[b] = max(yard[b], rel_err(lv[b], lr[b]))
    return gpu, yard


@pytest.mark.parametrize("case", sorted(CASES))
def test_generate_batch_free_running_vs_oracle(gpu, oracle, case):
    w, prompts = case_model(oracle, case)
    dec = _gpu_decoder(w, ROWS)
    out = dec.generate_batch(prompts, GEN)
    ref = oracle_generate(oracle, w, prompts, GEN)
    with oracle.reduction_order(True):
        rev = oracle_generate(oracle, w, prompts, GEN)
    gpu_div, yard_div = [], []
    for b, p in enumerate(prompts):
        assert out[b][:len(p)] == p and len(out[b]) == len(p) + GEN
        gpu_div.append(compare_ids(out[b][len(p):], ref[b][0], ref[b][1]))
        yard_div.append(compare_ids(rev[b][0], ref[b][0], ref[b][1]))
    gpu_drift, yard_drift = _drift(dec, oracle, w, out)
    agree = sum(GEN if j is None else j for j, _ in gpu_div)
    yagree = sum(GEN if j is None else j for j, _ in yard_div)
    record("free_run", test="generate_batch_free_running", case=case, rows=ROWS, gen=GEN,
           dims={k: CASES[case][k] for k in ("L", "H", "D", "V")},
           prompt_lens=[len(p) for p in prompts],
           gpu={"ids_identical_before_first_divergence": agree, "ids_total": ROWS * GEN,
                "first_divergence": [j for j, _ in gpu_div],
                "oracle_gap_at_divergence": [g for _, g in gpu_div],
                "logit_drift_per_row": gpu_drift.tolist()},
           yardstick_reversed_order_oracle={
               "ids_identical_before_first_divergence": yagree,
               "first_divergence": [j for j, _ in yard_div],
               "oracle_gap_at_divergence": [g for _, g in yard_div],
               "logit_drift_per_row": yard_drift.tolist()})
    print(f"{case}: GPU {agree}/{ROWS * GEN} ids before the first divergence "
          f"{[j for j, _ in gpu_div]}, drift {gpu_drift.max():.2e}; yardstick {yagree}, "
          f"{[j for j, _ in yard_div]}, drift {yard_drift.max():.2e}")
    bound = max(yard_drift.max(), 1e-3)
    for b, (j, gap) in enumerate(gpu_div):
        if j is not None:
            assert gap <= 2 * bound, (b, j, gap, bound)
    assert gpu_drift.max() <= 1.5 * yard_drift.max() + 1e-4, (gpu_drift, yard_drift)
    assert gpu_drift.max() < FREE_RUN_TOL[case], gpu_drift
    for b in range(ROWS):
        if gpu_drift[b] <= NO_FLIP_TOL and yard_drift[b] <= NO_FLIP_TOL:
            assert gpu_div[b][0] is None, (b, gpu_div[b])
