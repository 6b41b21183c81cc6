"""Workgroup-merge form of the FP16 decoder's attention (pa_decode.hip WGM).

When the split count of a row-output launch is 2..8, the splits of one
(row, head) run as the waves of one workgroup and merge in LDS, replacing the
pa_merge_row_kernel launch.  The merge repeats that kernel's arithmetic, so a
decoder step must produce the SAME BITS either way.  The tuning build's
LLM_WG_MERGE=0 restores split + merge launches; both forms are stepped through
the C-ABI (llm_decoder_create / set_f16_weights / begin_synthetic / step) at
C2's width (12 heads x 64, 16 rows), at a long context (every split full) and
a short one (splits past the row's tiles are empty: ns < nsplit).
"""
import ctypes
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


class _Cfg(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("num_layers", "num_heads", "head_dim", "hidden_dim",
                                            "vocab_size", "max_seq_len", "inter_dim", "page_size",
                                            "weight_dtype", "max_batch")] + [
        ("attn_scale", ctypes.c_float), ("num_pages", ctypes.c_longlong)]


class _F16W(ctypes.Structure):
    _fields_ = [("emb", ctypes.c_void_p)] + [(n, ctypes.c_void_p) for n in (
        "ln1_g", "ln1_b", "ln2_g", "ln2_b", "wqkv", "wo", "w1", "w2", "b1", "b2")]


def _model(rng, L, H, D, V):
    hid, inter = H * D, 4 * H * D
    w = {"emb": rng.standard_normal((V, hid)).astype(np.float16)}
    for k in ("ln1_g", "ln2_g"):
        w[k] = (1 + 0.1 * rng.standard_normal((L, hid))).astype(np.float32)
    for k in ("ln1_b", "ln2_b"):
        w[k] = (0.1 * rng.standard_normal((L, hid))).astype(np.float32)
    w["wqkv"] = (0.02 * rng.standard_normal((L, hid, 3 * hid))).astype(np.float16)
    w["wo"] = (0.02 * rng.standard_normal((L, hid, hid))).astype(np.float16)
    w["w1"] = (0.02 * rng.standard_normal((L, hid, inter))).astype(np.float16)
    w["w2"] = (0.02 * rng.standard_normal((L, inter, hid))).astype(np.float16)
    w["b1"] = (0.02 * rng.standard_normal((L, inter))).astype(np.float32)
    w["b2"] = (0.02 * rng.standard_normal((L, hid))).astype(np.float32)
    return {k: np.ascontiguousarray(v) for k, v in w.items()}


def _run(lib, w, L, H, D, V, S, B, ctx, steps, wgm, splits=0, ts=16, fuse=True, taps=False):
    """Logits of `steps` decode steps of a fresh FP16 decoder of `lib`
    (tuning build: splits > 0 forces the split count, fuse=False keeps the
    o_proj GEMM launch instead of the workgroup merge's fused o_proj).
    taps=True: also the activation taps of the last step (llm_decoder_set_taps:
    per layer the four packed fp16 GEMM inputs), as uint16 [L][4][B16 * qa_ld]."""
    import torch
    import llm_capi
    os.environ["LLM_WG_MERGE"] = "1" if wgm else "0"
    os.environ["LLM_WGM_SPLITS"] = str(splits)
    os.environ["LLM_OPROJ_FUSE"] = "1" if fuse else "0"
    lib.llm_decoder_create.argtypes = [ctypes.POINTER(_Cfg), ctypes.POINTER(ctypes.c_void_p)]
    lib.llm_decoder_set_f16_weights.argtypes = [ctypes.c_void_p, ctypes.POINTER(_F16W)]
    lib.llm_decoder_begin_synthetic.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                                ctypes.c_uint64, ctypes.c_int]
    lib.llm_decoder_step.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_void_p]
    lib.llm_decoder_sync.argtypes = [ctypes.c_void_p]
    lib.llm_decoder_destroy.argtypes = [ctypes.c_void_p]
    lib.llm_decoder_destroy.restype = None
    cfg = _Cfg(L, H, D, H * D, V, S, 0, ts, llm_capi.LLM_F16, B, 1.0, 0)
    dec = ctypes.c_void_p()
    llm_capi.check(lib.llm_decoder_create(ctypes.byref(cfg), ctypes.byref(dec)), lib)
    try:
        ww = _F16W(*[w[k].ctypes.data for k in ("emb", "ln1_g", "ln1_b", "ln2_g", "ln2_b", "wqkv",
                                                 "wo", "w1", "w2", "b1", "b2")])
        llm_capi.check(lib.llm_decoder_set_f16_weights(dec, ctypes.byref(ww)), lib)
        llm_capi.check(lib.llm_decoder_begin_synthetic(dec, B, ctx, 77, 1), lib)
        b16, qa_ld = (B + 15) // 16 * 16, 4 * H * D
        if taps:
            tq = torch.zeros((L, 4, b16 * qa_ld), dtype=torch.int16, device="cuda")
            ts_ = torch.zeros((L * 4 * B,), dtype=torch.float32, device="cuda")
            lib.llm_decoder_set_taps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
            llm_capi.check(lib.llm_decoder_set_taps(dec, tq.data_ptr(), ts_.data_ptr()), lib)
        rng = np.random.default_rng(5)
        out = []
        logits = torch.empty((B, V), device="cuda")
        for _ in range(steps):
            tok = rng.integers(0, V, B).astype(np.int32)
            llm_capi.check(lib.llm_decoder_step(dec, tok.ctypes.data, logits.data_ptr(), None, None),
                           lib)
            llm_capi.check(lib.llm_decoder_sync(dec), lib)
            out.append(logits.cpu().numpy().copy())
        if taps:
            return np.stack(out), tq.cpu().numpy().view(np.uint16)
        return np.stack(out)
    finally:
        lib.llm_decoder_destroy(dec)
        os.environ.pop("LLM_WG_MERGE", None)
        os.environ.pop("LLM_WGM_SPLITS", None)
        os.environ.pop("LLM_OPROJ_FUSE", None)


@pytest.mark.parametrize("H,D,ts", [(12, 64, 16), (8, 128, 16), (4, 256, 16), (8, 128, 32)],
                         ids=["c2_width_d64", "d128", "d256", "d128_page32"])
@pytest.mark.parametrize("ctx", [1500, 40])
def test_wg_merge_bitwise(gpu, ctx, H, D, ts):
    """Same split count, with and without the workgroup merge: same bits (at
    ctx 40, 5 and 8 splits leave splits past the row's tiles empty); and the
    product build's own split choice equals the tuning build's.  C2's width
    (12 x 64) and the other head dims the FP16 decoder runs the merge form at
    (D 128 and 256, page 32), whose 512-thread workgroups halve the register
    budget of the 2-stage register staging."""
    import llm_capi
    tune = llm_capi.load_tune()
    L, V, S, B = 2, 512, 2100, 16
    w = _model(np.random.default_rng(3), L, H, D, V)
    for ns in ((3, 5, 8) if D == 64 else (3, 8)):
        on = _run(tune, w, L, H, D, V, S, B, ctx, 3, True, ns, ts, fuse=False)
        off = _run(tune, w, L, H, D, V, S, B, ctx, 3, False, ns, ts, fuse=False)
        assert np.isfinite(on).all()
        assert np.array_equal(on.view(np.uint32), off.view(np.uint32)), (ns, np.abs(on - off).max())
    auto = _run(tune, w, L, H, D, V, S, B, ctx, 3, True, 0, ts)
    prod = _run(llm_capi.load(), w, L, H, D, V, S, B, ctx, 3, True, 0, ts)
    assert np.array_equal(prod.view(np.uint32), auto.view(np.uint32))


@pytest.mark.parametrize("H,D,ts", [(12, 64, 16), (8, 128, 16), (8, 128, 32)],
                         ids=["c2_width_d64", "d128", "d128_page32"])
@pytest.mark.parametrize("ctx", [1500, 40])
def test_fused_oproj(gpu, ctx, H, D, ts):
    """The o_proj fused into the workgroup merge (each (row, head) workgroup
    adds o_h . W_o[h rows] into counted int64 fixed-point columns; the adder
    completing a column writes x and clears it) against the o_proj GEMM
    launch at the same split count: step-0 logits within 1e-3, tensor-
    normalised (fp32 sums in another order plus 2^-33 per head of fixed-point
    rounding, moved across the fp16 roundings of the next GEMM inputs now and
    then; the elementwise oracle bound is checked teacher-forced,
    test_decoder_gpu.py); bit-identical from run to run (the integer sum does
    not depend on the order the heads' atomics land in) over several steps
    (every layer's columns cleared for the next); and, through the taps, the
    same o_proj input and an fc1 input within one fp16 ulp."""
    import llm_capi
    from _util import rel_err
    tune = llm_capi.load_tune()
    L, V, S, B = 2, 512, 2100, 16
    w = _model(np.random.default_rng(4), L, H, D, V)
    for ns in (3, 8):
        fused = _run(tune, w, L, H, D, V, S, B, ctx, 4, True, ns, ts, fuse=True)
        again = _run(tune, w, L, H, D, V, S, B, ctx, 4, True, ns, ts, fuse=True)
        gemm = _run(tune, w, L, H, D, V, S, B, ctx, 4, True, ns, ts, fuse=False)
        assert np.isfinite(fused).all()
        assert np.array_equal(fused.view(np.uint32), again.view(np.uint32)), ns
        assert rel_err(fused[0], gemm[0]) < 1e-3, (ns, rel_err(fused[0], gemm[0]))
        assert not np.array_equal(fused.view(np.uint32), gemm.view(np.uint32))  # the fused form ran
        # one step with taps: layer 0's attention output (the o_proj input) is
        # the same bits, and fc1's input LN2(x) -- x the o_proj output, rounded
        # to fp16 -- differs in a few elements by one fp16 ulp (or, where
        # x - mean cancels, by 1e-5 of the tensor's largest value)
        _, tf = _run(tune, w, L, H, D, V, S, B, ctx, 1, True, ns, ts, fuse=True, taps=True)
        _, tg = _run(tune, w, L, H, D, V, S, B, ctx, 1, True, ns, ts, fuse=False, taps=True)
        hid = H * D
        n16 = (B + 15) // 16 * 16 * hid
        assert np.array_equal(tf[0, 1, :n16], tg[0, 1, :n16])
        fa = tf[0, 2, :n16].view(np.float16).astype(np.float64)
        fg = tg[0, 2, :n16].view(np.float16).astype(np.float64)
        bound = np.spacing(np.abs(fg).astype(np.float16)).astype(np.float64) + 1e-5 * np.abs(fg).max()
        assert np.all(np.abs(fa - fg) <= bound), np.max(np.abs(fa - fg) / bound)
        assert np.mean(fa != fg) < 0.05, np.mean(fa != fg)


def _guard_run(lib, w, L, H, D, V, B, steps, fuse, splits=3, after=None):
    """Fused-o_proj range guard runs (tuning build, forced split count, context
    0 so each row's attention output is exactly its new V row): per step the
    logits, llm_decoder_sync's status, then llm_decoder_oproj_status, and the
    step-0 taps (uint16 [L][4][B16 * qa_ld]).  Every step's sync is followed by
    a second one, whose status must be LLM_OK (a clamp is reported once).
    after(lib, dec): called on the decoder after the steps (its result is
    returned last)."""
    import torch
    import llm_capi
    os.environ["LLM_WGM_SPLITS"] = str(splits)
    os.environ["LLM_OPROJ_FUSE"] = "1" if fuse else "0"
    for name, args in (("llm_decoder_create", [ctypes.POINTER(_Cfg), ctypes.POINTER(ctypes.c_void_p)]),
                       ("llm_decoder_set_f16_weights", [ctypes.c_void_p, ctypes.POINTER(_F16W)]),
                       ("llm_decoder_begin_synthetic", [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                                        ctypes.c_uint64, ctypes.c_int]),
                       ("llm_decoder_step", [ctypes.c_void_p] * 5),
                       ("llm_decoder_sync", [ctypes.c_void_p]),
                       ("llm_decoder_set_taps", [ctypes.c_void_p] * 3),
                       ("llm_decoder_oproj_status", [ctypes.c_void_p] * 3),
                       ("llm_decoder_destroy", [ctypes.c_void_p])):
        getattr(lib, name).argtypes = args
    lib.llm_decoder_destroy.restype = None
    cfg = _Cfg(L, H, D, H * D, V, 64, 0, 16, llm_capi.LLM_F16, B, 1.0, 0)
    dec = ctypes.c_void_p()
    llm_capi.check(lib.llm_decoder_create(ctypes.byref(cfg), ctypes.byref(dec)), lib)
    try:
        ww = _F16W(*[w[k].ctypes.data for k in ("emb", "ln1_g", "ln1_b", "ln2_g", "ln2_b", "wqkv",
                                                 "wo", "w1", "w2", "b1", "b2")])
        llm_capi.check(lib.llm_decoder_set_f16_weights(dec, ctypes.byref(ww)), lib)
        llm_capi.check(lib.llm_decoder_begin_synthetic(dec, B, 0, 77, 1), lib)
        b16, qa_ld = (B + 15) // 16 * 16, 4 * H * D
        tq = torch.zeros((L, 4, b16 * qa_ld), dtype=torch.int16, device="cuda")
        ts_ = torch.zeros((L * 4 * B,), dtype=torch.float32, device="cuda")
        llm_capi.check(lib.llm_decoder_set_taps(dec, tq.data_ptr(), ts_.data_ptr()), lib)
        rng = np.random.default_rng(5)
        logits = torch.empty((B, V), device="cuda")
        out, rcs, taps = [], [], None
        for s in range(steps):
            tok = rng.integers(0, V, B).astype(np.int32)
            llm_capi.check(lib.llm_decoder_step(dec, tok.ctypes.data, logits.data_ptr(), None, None),
                           lib)
            rcs.append(lib.llm_decoder_sync(dec))
            assert lib.llm_decoder_sync(dec) == 0  # reported once, then cleared
            out.append(logits.cpu().numpy().copy())
            if s == 0:
                taps = tq.cpu().numpy().view(np.uint16).copy()
                llm_capi.check(lib.llm_decoder_set_taps(dec, None, None), lib)
        clamped, nz = ctypes.c_int(-1), ctypes.c_longlong(-1)
        llm_capi.check(lib.llm_decoder_oproj_status(dec, ctypes.byref(clamped), ctypes.byref(nz)), lib)
        res = (np.stack(out), rcs, (clamped.value, nz.value), taps)
        return res + (after(lib, dec),) if after else res
    finally:
        lib.llm_decoder_destroy(dec)
        os.environ.pop("LLM_WGM_SPLITS", None)
        os.environ.pop("LLM_OPROJ_FUSE", None)


def test_fused_oproj_range_guard(gpu):
    """The fused o_proj's counted int64 columns hold |sum| < 2^23 only; each
    head's term is clamped to (2^23 - 1) / H (common.hpp oacc_term), so the
    arrival count can never be corrupted, and a clamp raises LLM_ERR_RANGE at
    llm_decoder_sync.  Layer 0's V projection is made large and its W_o column
    n0 set to a constant s, so head h of row b adds s * sum(o[b, hD:(h+1)D]):
    s is chosen from the GEMM form's own tapped o_proj input so that the
    largest head term is just under the limit (0.97x: the fused form must
    match the o_proj GEMM, no error; one step) or over it (1.6x: LLM_ERR_RANGE
    on both steps, yet every accumulator column back at zero); a
    non-finite head (V overflowing fp16) trips it the same way."""
    import llm_capi
    from oracle.oracle import unpack_a_f16
    from _util import rel_err
    tune = llm_capi.load_tune()
    L, H, D, V, B = 2, 12, 64, 512, 16
    hid = H * D
    rng = np.random.default_rng(11)
    w = _model(rng, L, H, D, V)
    w["wqkv"][0, :, 2 * hid:] = rng.standard_normal((hid, hid)).astype(np.float16)
    n0 = 5
    w["wo"][0, :, n0] = np.float16(1.0)
    _, rcs, st, tg = _guard_run(tune, w, L, H, D, V, B, 1, fuse=False)
    assert rcs == [0] and st == (0, 0), (rcs, st)  # the GEMM form has no accumulator
    o = unpack_a_f16(tg[0, 1], B, hid).astype(np.float32)  # layer 0's o_proj input
    head_sums = o.reshape(B, H, D).sum(axis=2)
    lim = ((1 << 23) - 1) / H
    peak = float(np.abs(head_sums).max())
    for frac, trips in ((0.97, False), (1.6, True)):
        s = np.float16(frac * lim / peak)
        assert np.isfinite(s) and s > 0
        ws = dict(w)
        ws["wo"] = w["wo"].copy()
        ws["wo"][0, :, n0] = s
        ws = {k: np.ascontiguousarray(v) for k, v in ws.items()}
        # (one step just under: the step-0 heads set s; the next step's heads
        # attend two V rows and may be larger)
        steps = 2 if trips else 1
        gl, grc, gst, gt = _guard_run(tune, ws, L, H, D, V, B, steps, fuse=False)
        fl, frc, fst, ft = _guard_run(tune, ws, L, H, D, V, B, steps, fuse=True)
        assert grc == [0] * steps and gst == (0, 0)
        assert fst[1] == 0, fst  # every column completed and cleared
        if not trips:
            assert frc == [0] and fst == (0, 0), (frac, frc, fst)
            assert rel_err(fl[0], gl[0]) < 1e-3, rel_err(fl[0], gl[0])
            assert np.array_equal(ft[0, 1], gt[0, 1])  # same o_proj input
        else:
            assert frc == [llm_capi.LLM_ERR_RANGE] * 2 and fst == (1, 0), (frc, fst)
    # non-finite heads: V rows overflow fp16 (inf), the merged heads are inf / NaN
    wn = dict(w)
    wn["wqkv"] = w["wqkv"].copy()
    wn["wqkv"][0, :, 2 * hid:] = (3000 * rng.standard_normal((hid, hid))).astype(np.float16)
    wn = {k: np.ascontiguousarray(v) for k, v in wn.items()}
    _, frc, fst, _, (gen_rc, gen_out, st_after, run_rc) = _guard_run(
        tune, wn, L, H, D, V, B, 2, fuse=True, after=_generate_and_rerun)
    assert frc == [llm_capi.LLM_ERR_RANGE] * 2 and fst == (1, 0), (frc, fst)
    # generate over the clamping model: every step clamps, yet every
    # id is produced; the status comes back once, at the end
    assert gen_rc == llm_capi.LLM_ERR_RANGE, gen_rc
    assert gen_out.min() >= 0 and gen_out.max() < V, gen_out
    assert st_after == (0, 1, 0), st_after  # sync after generate: reported; status: clamped
    # a timing re-run of the clamping attention has its own flag: the sync
    # after it succeeds
    assert run_rc == (0, 0), run_rc


def _generate_and_rerun(lib, dec):
    """llm_decoder_generate on a clamping decoder (output pre-filled with -1),
    then sync / oproj_status, then llm_decoder_run_attention(layer 0) + sync."""
    lib.llm_decoder_generate.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                         ctypes.c_void_p]
    lib.llm_decoder_run_attention.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    B, n_gen, plen = 3, 4, 2
    prompts = np.arange(B * plen, dtype=np.int32).reshape(B, plen)
    lens = np.full(B, plen, np.int32)
    out = np.full((B, n_gen), -1, np.int32)
    rc = lib.llm_decoder_generate(dec, prompts.ctypes.data, lens.ctypes.data, plen, B, n_gen,
                                  ctypes.c_float(1.0), out.ctypes.data)
    sync_rc = lib.llm_decoder_sync(dec)
    clamped, nz = ctypes.c_int(-1), ctypes.c_longlong(-1)
    lib.llm_decoder_oproj_status(dec, ctypes.byref(clamped), ctypes.byref(nz))
    run = lib.llm_decoder_run_attention(dec, 0, None)
    return rc, out, (sync_rc, clamped.value, nz.value), (run, lib.llm_decoder_sync(dec))
