"""The decoder's OWN attention epilogue against the oracle at the split counts
the BASELINE configs run.

Inside a decode step the paged attention runs split-T: many splits per (row,
head).  INT8Decoder: up to 8 splits merge inside the split workgroup and more
in the fp32 merge launch, and the o_proj GEMM's prologue quantises each row
(all heads) into its int8 A; beam groups (C4) merge in pa_merge_row_kernel,
which quantises the rows itself.  CUDADecoder: merged inside the split
workgroup into the packed fp16 o_proj input (workgroup merge).  That merge is the reference's AV-and-store
(attention_cpu/cpu_attention_kernel.cpp:103-120) followed by the quantiser
(attention_cpu/int8_quant.cpp:5-13,59-64).

Each test starts the decoder at a long context (llm_decoder_begin_synthetic /
begin_beams: seeded random K/V in shuffled pages), reads every row's pages
back through the page table into the oracle's contiguous KV
(_util.decoder_kv_to_oracle), and steps GPU and oracle together:
  * INT8: teacher forced at the four int8 GEMM inputs (taps); stage 1 (the
    o_proj input = the merged, quantised attention rows) within one LSB of the
    oracle's own quantisation of its fp32 attention, < 1e-3 of the values
    flipped; logits at the north_star bar (1e-3, tensor and elementwise per
    row), tokens exact unless tied.
  * FP16: teacher forced at the four fp16 GEMM inputs and at the K / V the
    step appends (both within one fp16 ulp of the oracle's own); the tapped packed
    fp16 attention rows against the oracle's fp32 attention at 1e-3 (tensor
    and elementwise) and within one fp16 ulp of its own rounding, < 1e-2 of
    them differing; logits 1e-3 (tensor and elementwise per row).
The split count of the step's own launch is read from the decoder
(llm_decoder_attention_plan) and asserted, so the multi-split merge is what
is compared."""
import numpy as np
import pytest

from _util import assert_parity, decoder_kv_at, decoder_kv_to_oracle, rel_err

pytestmark = pytest.mark.gpu
LOGIT_TOL = 1e-3
TIE_TOL = 1e-5
FORM_DIRECT, FORM_SPLIT_MERGE, FORM_SPLIT_MERGE_ROW, FORM_WG_MERGE, FORM_BEAM = 0, 1, 2, 3, 16
FORM_STEAL = 64  # beam groups: tiles assigned to the splits while the launch runs
FORM_OPROJ = 32  # FP16 decoder: o_proj fused into the workgroup merge


def _torch():
    import torch
    return torch


class _Taps:
    """llm_decoder_set_taps buffers (INT8: int8 + scales; FP16: fp16 values)."""

    def __init__(self, dec, c, max_batch, f16=False):
        torch = _torch()
        self.L, self.hid, self.inter, self.f16 = c["L"], c["hid"], c["inter"], f16
        self.K = max(self.hid, self.inter)
        self.b16 = (max_batch + 15) // 16 * 16
        self.maxB = max_batch
        es = 2 if f16 else 1
        self.q = torch.zeros(self.L * 4 * self.b16 * self.K * es, dtype=torch.int8, device="cuda")
        self.s = torch.zeros(self.L * 4 * max_batch, dtype=torch.float32, device="cuda")
        dec.set_taps(self.q.data_ptr(), self.s.data_ptr())

    def read_i8(self, B):
        from oracle.oracle import unpack_a_i8
        q = self.q.cpu().numpy().reshape(self.L, 4, self.b16 * self.K)
        s = self.s.cpu().numpy().reshape(self.L, 4, self.maxB)
        fq = np.zeros((self.L, 4, B, self.K), np.int8)
        for l in range(self.L):
            for st in range(4):
                Kst = self.inter if st == 3 else self.hid
                fq[l, st, :, :Kst] = unpack_a_i8(q[l, st, :self.b16 * Kst], B, Kst)
        return fq, np.ascontiguousarray(s[:, :, :B])

    def read_f16(self, B):
        """The four fp16 GEMM inputs of every layer: [L][4][B][Kmax] fp16
        (stage 1 = the merged attention rows, the packed o_proj input)."""
        from oracle.oracle import unpack_a_f16
        q = self.q.cpu().numpy().view(np.uint16).reshape(self.L, 4, self.b16 * self.K)
        fh = np.zeros((self.L, 4, B, self.K), np.float16)
        for l in range(self.L):
            for st in range(4):
                Kst = self.inter if st == 3 else self.hid
                fh[l, st, :, :Kst] = unpack_a_f16(q[l, st, :self.b16 * Kst], B, Kst)
        return fh


def _check_tokens(g_next, o_next, o_logits):
    for b in range(len(g_next)):
        if g_next[b] != o_next[b]:
            gap = o_logits[b][o_next[b]] - o_logits[b][g_next[b]]
            assert gap <= TIE_TOL * np.abs(o_logits[b]).max(), (b, gap)


def _forced_steps_int8(dec, odec, taps, rows, T, steps, V, seed):
    """GPU and teacher-forced oracle in lockstep from context T; returns the
    stage-1 (attention) flip count, values compared, and the worst logit rel err."""
    torch = _torch()
    hid = odec.cfg["hid"]
    logits = torch.empty((rows, V), device="cuda")
    rng = np.random.default_rng(seed)
    tok = [int(t) for t in rng.integers(0, V, rows)]
    flips, vals, worst = 0, 0, 0.0
    for s in range(steps):
        g_next = dec.step(tok, logits_ptr=logits.data_ptr())
        torch.cuda.synchronize()
        fq, fs = taps.read_i8(rows)
        o_logits, o_next, stats, attn = odec.step_attn(np.array(tok, np.int32),
                                                       np.full(rows, T + s, np.int32), fq, fs)
        # every int8 GEMM input within one LSB, row scales equal
        assert stats[:, :, 1].max() <= 1, (s, stats)
        assert stats[:, :, 2].max() < 1e-5, (s, stats)
        assert np.isfinite(attn).all()
        flips += int(stats[:, 1, 0].sum())
        vals += odec.cfg["L"] * rows * hid
        gl = logits.cpu().numpy()
        assert_parity(gl, o_logits, LOGIT_TOL, axis=1, what=f"step {s} logits")
        worst = max(worst, rel_err(gl, o_logits))
        _check_tokens(g_next, o_next, o_logits)
        tok = list(g_next)
    return flips, vals, worst


def _int8_decoder(oracle, L, H, D, V, max_seq, rows, seed):
    import llm_decoder
    from oracle.oracle import synthetic_int8_model
    w = synthetic_int8_model(oracle, L=L, H=H, D=D, V=V, max_seq=max_seq, seed=seed)
    c = w["cfg"]
    dec = llm_decoder.INT8Decoder(c["L"], c["H"], c["D"], c["hid"], c["V"], c["max_seq"],
                                  max_batch=rows)
    d = {k: np.ascontiguousarray(v) for k, v in w.items() if k != "cfg"}
    d["emb"] = w["emb"].view(np.uint16)
    dec.set_weights(d)
    return w, dec


@pytest.mark.parametrize("rows,T,form", [(4, 2048, FORM_WG_MERGE), (8, 8192, FORM_SPLIT_MERGE)])
def test_int8_step_multi_split_attention_vs_oracle(gpu, oracle, rows, T, form):
    """C3 model dims (16 heads x 128), 2 layers, 4 rows at T 2048 and 8 rows at
    T 8192: the step's attention runs 8 splits, merged inside the split
    workgroup (T 2048) or by the fp32 merge launch (T 8192: one full resident
    round would be 16 splits of 33 pages; the launch halves it to 8 of 65,
    pa_decode.hip half_round), and the o_proj prologue quantises the fp32 rows
    (the tapped stage-1 A)."""
    from oracle.oracle import OracleDecoder
    w, dec = _int8_decoder(oracle, 2, 16, 128, 512, T + 8, rows, seed=51)
    taps = _Taps(dec, w["cfg"], rows)
    dec.begin_synthetic(rows, T, 77, True)
    ns, got = dec.attention_plan()
    assert got == form and ns == 8, (ns, got)
    odec = OracleDecoder(oracle, w, rows)
    decoder_kv_to_oracle(dec, odec, rows, T)
    flips, vals, worst = _forced_steps_int8(dec, odec, taps, rows, T, 2, 512, seed=T)
    assert flips < 1e-3 * vals, (flips, vals)
    print(f"INT8 rows {rows} T {T}: {ns} splits, attention int8 flips {flips}/{vals}, "
          f"logits rel err {worst:.2e}")


@pytest.mark.timeout(600)
def test_int8_c3_shipped_launch_vs_oracle(gpu, oracle):
    """C3's exact product launch: 64 rows x 16 heads x D 128 at T 8192 (the
    bench's row count and context), 2 layers.  The step's attention is the
    shipped workgroup-merge form with 8 splits of 65 pages (the split length
    is derived on device from each row's context: ceil(513 / 8)), the fp32
    rows quantised by the o_proj prologue -- against the oracle on every row,
    teacher forced, at the north_star bar."""
    from oracle.oracle import OracleDecoder
    rows, T = 64, 8192
    w, dec = _int8_decoder(oracle, 2, 16, 128, 512, T + 8, rows, seed=53)
    taps = _Taps(dec, w["cfg"], rows)
    dec.begin_synthetic(rows, T, 78, True)
    ns, form = dec.attention_plan()
    assert (ns, form) == (8, FORM_WG_MERGE), (ns, form)
    odec = OracleDecoder(oracle, w, rows)
    decoder_kv_to_oracle(dec, odec, rows, T)
    flips, vals, worst = _forced_steps_int8(dec, odec, taps, rows, T, 2, 512, seed=3)
    assert flips < 1e-3 * vals, (flips, vals)
    print(f"C3 shipped launch: {ns} splits (workgroup merge), attention int8 flips "
          f"{flips}/{vals}, logits rel err {worst:.2e}")


@pytest.mark.timeout(600)
@pytest.mark.parametrize("rows,T,form", [(16, 2048, FORM_WG_MERGE), (2, 8192, FORM_SPLIT_MERGE_ROW)])
def test_int8_c5_dims_step_vs_oracle(gpu, oracle, rows, T, form):
    """C5's per-GPU model dims: 32 heads x D 128 (hid 4096, inter 16384), 2
    layers.  hid 4096 is too wide for the o_proj quantising prologue (K <=
    2048), so at 16 rows x T 2048 the attention merges its splits in the
    workgroup into fp32 rows and a quantise launch writes each 4096-wide row
    into the o_proj's packed int8 A; at 2 rows x T 8192 the fp32-row plan
    needs more than 8 splits, so the launch falls back to split +
    pa_merge_row_kernel (merge and quantise in one launch).  The GEMMs run
    C5's shapes (qkv 4096x12288, o_proj 4096x4096, fc1 4096x16384, fc2
    16384x4096: 256 k-steps) -- against the oracle, teacher forced at the four
    int8 GEMM inputs (attention_cpu/cpu_attention_kernel.cpp:103-120,
    attention_cpu/int8_quant.cpp:5-13, decoder/mlp.hpp:23-41)."""
    from oracle.oracle import OracleDecoder
    w, dec = _int8_decoder(oracle, 2, 32, 128, 512, T + 8, rows, seed=54)
    assert w["cfg"]["hid"] == 4096 and w["cfg"]["inter"] == 16384
    taps = _Taps(dec, w["cfg"], rows)
    dec.begin_synthetic(rows, T, 79, True)
    ns, got = dec.attention_plan()
    assert got == form and ns >= 2, (ns, got)
    odec = OracleDecoder(oracle, w, rows)
    decoder_kv_to_oracle(dec, odec, rows, T)
    flips, vals, worst = _forced_steps_int8(dec, odec, taps, rows, T, 2, 512, seed=5)
    assert flips < 1e-3 * vals, (flips, vals)
    print(f"C5 dims, {rows} rows x T {T}: {ns} splits (form {got}), attention int8 flips "
          f"{flips}/{vals}, logits rel err {worst:.2e}")


@pytest.mark.timeout(900)
def test_int8_c5_shipped_launch_vs_oracle(gpu, oracle):
    """C5's exact per-GPU launch (bench.py --config c5 on each of the 8 GPUs):
    64 rows x 32 heads x D 128 at T 8192, one layer.  The plan is the one the
    bench runs -- 8 splits of ceil(513 / 8) = 65 pages (derived on device from
    each row's context) merged in the workgroup into fp32 rows, then one
    launch quantising each 4096-wide row -- and the GEMMs are C5's four shapes at 64 rows in
    the decoder's own packed-A form (qkv 4096x12288, o_proj 4096x4096, fc1
    4096x16384, fc2 16384x4096).  Every row's pages are read back into the
    oracle and the step is teacher forced at the four int8 GEMM inputs
    (attention_cpu/cpu_attention_kernel.cpp:103-120, attention_cpu/int8_quant.cpp:5-13,
    decoder/mlp.hpp:23-41): each within one LSB, < 1e-3 of the attention values
    flipped, logits at 1e-3 per row."""
    from oracle.oracle import OracleDecoder
    rows, T = 64, 8192
    w, dec = _int8_decoder(oracle, 1, 32, 128, 512, T + 8, rows, seed=55)
    c = w["cfg"]
    assert (c["hid"], c["inter"]) == (4096, 16384)
    taps = _Taps(dec, c, rows)
    dec.begin_synthetic(rows, T, 80, True)
    ns, form = dec.attention_plan()
    assert (ns, form) == (8, FORM_WG_MERGE), (ns, form)
    ntiles = (T + 1 + 15) // 16  # the step attends its own new token too: 513 tiles
    assert -(-ntiles // ns) == 65, ntiles  # pages per split, as the kernel derives them
    odec = OracleDecoder(oracle, w, rows)
    distinct = decoder_kv_to_oracle(dec, odec, rows, T)
    assert distinct[0] == rows * 32 * (T // 16), distinct  # every (row, head, tile) its own page
    flips, vals, worst = _forced_steps_int8(dec, odec, taps, rows, T, 2, 512, seed=6)
    assert flips < 1e-3 * vals, (flips, vals)
    print(f"C5 shipped launch: {ns} splits (workgroup merge + quantise), attention int8 flips "
          f"{flips}/{vals}, logits rel err {worst:.2e}")


def test_int8_c4_beam_state_attention_vs_oracle(gpu, oracle):
    """The C4 bench state (begin_beams(8, 4, 3840, 256): 240 shared tiles per
    sequence through page-table forks, 16 private per beam) at C3 head dims,
    2 layers: the beam-group launch with cost-balanced splits, merged and
    quantised by pa_merge_row_kernel, against the oracle on every row."""
    from oracle.oracle import OracleDecoder
    rows, T = 32, 4096
    w, dec = _int8_decoder(oracle, 2, 16, 128, 512, T + 8, rows, seed=52)
    taps = _Taps(dec, w["cfg"], rows)
    dec.begin_beams(8, 4, 3840, 256, 99, True)
    ns, form = dec.attention_plan()
    assert form == (FORM_SPLIT_MERGE_ROW | FORM_BEAM) and ns >= 8, (ns, form)
    odec = OracleDecoder(oracle, w, rows)
    distinct = decoder_kv_to_oracle(dec, odec, rows, T)
    # shared prefixes are read from shared pages: 8 x 16 x 240 + 32 x 16 x 16
    assert distinct[0] == 8 * 16 * 240 + 32 * 16 * 16, distinct
    flips, vals, worst = _forced_steps_int8(dec, odec, taps, rows, T, 2, 512, seed=4)
    assert flips < 1e-3 * vals, (flips, vals)
    print(f"C4 state: {ns} splits, attention int8 flips {flips}/{vals}, logits {worst:.2e}")


def test_f16_step_workgroup_merge_vs_oracle(gpu, oracle):
    """C2 dims (12 heads x 64, 16 rows, T 2048): the FP16 decoder's attention
    merges its splits inside the split workgroup (3 splits) and writes the
    packed fp16 o_proj input, compared with the oracle's fp32 attention, and
    adds its o_proj into the fused columns (LLM_PA_FORM_OPROJ).  The tapped
    LN1 rows and the appended K / V are held to the oracle's own within one
    fp16 ulp, like the GEMM inputs."""
    torch = _torch()
    import llm_decoder
    from oracle.oracle import OracleDecoder
    rows, T, L, H, D, V = 16, 2048, 2, 12, 64, 512
    rng = np.random.default_rng(61)
    hid, inter = H * D, 4 * H * D
    w = {"cfg": dict(L=L, H=H, D=D, hid=hid, inter=inter, V=V, max_seq=T + 8)}
    w["emb"] = rng.standard_normal((V, hid)).astype(np.float16)
    for k in ("ln1_g", "ln2_g"):
        w[k] = (1 + 0.1 * rng.standard_normal((L, hid))).astype(np.float32)
    for k in ("ln1_b", "ln2_b"):
        w[k] = (0.1 * rng.standard_normal((L, hid))).astype(np.float32)
    for k, shp in (("wqkv", (hid, 3 * hid)), ("wo", (hid, hid)), ("w1", (hid, inter)),
                   ("w2", (inter, hid))):
        w[k] = (0.02 * rng.standard_normal((L,) + shp)).astype(np.float16)
    w["b1"] = (0.02 * rng.standard_normal((L, inter))).astype(np.float32)
    w["b2"] = (0.02 * rng.standard_normal((L, hid))).astype(np.float32)
    dec = llm_decoder.CUDADecoder(L, H, D, hid, V, T + 8, max_batch=rows)
    d = {k: np.ascontiguousarray(v) for k, v in w.items() if k != "cfg"}
    for k in ("emb", "wqkv", "wo", "w1", "w2"):
        d[k] = d[k].view(np.uint16)
    dec.set_weights(d)
    taps = _Taps(dec, w["cfg"], rows, f16=True)
    dec.begin_synthetic(rows, T, 5, True)
    ns, form = dec.attention_plan()
    assert form == FORM_WG_MERGE | FORM_OPROJ and 2 <= ns <= 8, (ns, form)
    odec = OracleDecoder(oracle, w, rows)
    decoder_kv_to_oracle(dec, odec, rows, T)
    logits = torch.empty((rows, V), device="cuda")
    tok = [int(t) for t in rng.integers(0, V, rows)]
    flips, vals = 0, 0
    for s in range(2):
        g_next = dec.step(tok, logits_ptr=logits.data_ptr())
        torch.cuda.synchronize()
        fh = taps.read_f16(rows)
        # teacher forced at the four fp16 GEMM inputs (an fp32 reordering can
        # move a value across an fp16 rounding boundary; forcing keeps that
        # one-ulp flip from propagating)
        # ... and at the K / V the step appended (the qkv GEMM's fp32 order)
        fkv = decoder_kv_at(dec, rows, [T + s] * rows, L)
        o_logits, o_next, stats, attn = odec.step_attn(np.array(tok, np.int32),
                                                       np.full(rows, T + s, np.int32), fh,
                                                       forced_kv=fkv)
        assert stats[:, :, 1].max() <= 1, (s, stats)  # one fp16 ulp (or 1e-6 of the row max)
        assert odec.kv_stats[:, 1].max() <= 1, (s, odec.kv_stats)
        ga = fh[:, 1, :, :hid].astype(np.float32)       # the merged attention rows
        assert_parity(ga, attn, 1e-3, what=f"step {s} attention rows")
        flips += int(stats[:, 1, 0].sum())
        vals += L * rows * hid
        gl = logits.cpu().numpy()
        assert_parity(gl, o_logits, LOGIT_TOL, axis=1, what=f"step {s} logits")
        _check_tokens(g_next, o_next, o_logits)
        tok = list(g_next)
    # fp16 rounding boundaries are 2^-11 of the value apart (int8: 1/127 of the
    # row's absmax): ~1e-6 relative fp32 differences flip a few 1e-3 of them,
    # each within one ulp (asserted per step above)
    assert flips < 1e-2 * vals, (flips, vals)
    print(f"FP16 C2 dims: {ns} splits (workgroup merge), attention fp16 ulp flips {flips}/{vals}")
