"""The INT8 decoder's last-arriver LayerNorm seam (tuning build, LLM_LNX=1).

The o_proj and fc2 GEMMs write their output rows with write-through stores,
count their workgroups per 16-row block with a returning atomic, and the last
workgroup of a block normalises and quantises its rows (LN2 for fc1, the next
layer's LN1 for its q/k/v GEMM), replacing two LayerNorm launches per layer
(gemm_impl.hpp LNX).  Same-box it lost C4 -10 % and C3 -1 % against those
launches, so the product keeps them; the form stays in the
tuning build, held here to the launch form: logits of 3 steps within 1e-3,
run to run bit-identical, and the product library equal to the tuning build
with the switch off.
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


class _I8W(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in (
        "emb", "ln1_g", "ln1_b", "ln2_g", "ln2_b", "wqkv", "sw_qkv", "wo", "sw_o",
        "w1", "sw1", "b1", "w2", "sw2", "b2")]


def _model(rng, L, hid, inter, V):
    w = {"emb": rng.standard_normal((V, hid)).astype(np.float16)}
    for k in ("ln1_g", "ln2_g"):
        w[k] = (1 + 0.1 * rng.standard_normal((L, hid))).astype(np.float32)
    for k in ("ln1_b", "ln2_b"):
        w[k] = (0.1 * rng.standard_normal((L, hid))).astype(np.float32)
    for k, s, (K, N) in (("wqkv", "sw_qkv", (hid, 3 * hid)), ("wo", "sw_o", (hid, hid)),
                         ("w1", "sw1", (hid, inter)), ("w2", "sw2", (inter, hid))):
        w[k] = rng.integers(-127, 128, (L, K, N)).astype(np.int8)
        w[s] = (0.6 / (127 * np.sqrt(K)) * (1 + 0.1 * rng.random((L, N)))).astype(np.float32)
    w["b1"] = (0.02 * rng.standard_normal((L, inter))).astype(np.float32)
    w["b2"] = (0.02 * rng.standard_normal((L, hid))).astype(np.float32)
    return {k: np.ascontiguousarray(v) for k, v in w.items()}


def _run(lib, w, L, H, D, V, S, B, ctx, steps, lnx):
    import torch
    import llm_capi
    os.environ["LLM_LNX"] = "1" if lnx else "0"
    lib.llm_decoder_create.argtypes = [ctypes.POINTER(_Cfg), ctypes.POINTER(ctypes.c_void_p)]
    lib.llm_decoder_set_int8_weights.argtypes = [ctypes.c_void_p, ctypes.POINTER(_I8W)]
    lib.llm_decoder_begin_synthetic.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                                ctypes.c_uint64, ctypes.c_int]
    lib.llm_decoder_step.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_void_p]
    lib.llm_decoder_sync.argtypes = [ctypes.c_void_p]
    lib.llm_decoder_destroy.argtypes = [ctypes.c_void_p]
    lib.llm_decoder_destroy.restype = None
    hid = H * D
    cfg = _Cfg(L, H, D, hid, V, S, 4 * hid, 16, llm_capi.LLM_I8, B, 1.0, 0)
    dec = ctypes.c_void_p()
    llm_capi.check(lib.llm_decoder_create(ctypes.byref(cfg), ctypes.byref(dec)), lib)
    try:
        ww = _I8W(*[w[k].ctypes.data for k, _ in _I8W._fields_])
        llm_capi.check(lib.llm_decoder_set_int8_weights(dec, ctypes.byref(ww)), lib)
        llm_capi.check(lib.llm_decoder_begin_synthetic(dec, B, ctx, 91, 1), lib)
        rng = np.random.default_rng(8)
        out = []
        logits = torch.empty((B, V), device="cuda")
        for _ in range(steps):
            tok = rng.integers(0, V, B).astype(np.int32)
            llm_capi.check(lib.llm_decoder_step(dec, tok.ctypes.data, logits.data_ptr(), None, None),
                           lib)
            llm_capi.check(lib.llm_decoder_sync(dec), lib)
            out.append(logits.cpu().numpy().copy())
        return np.stack(out)
    finally:
        lib.llm_decoder_destroy(dec)
        os.environ.pop("LLM_LNX", None)


@pytest.mark.parametrize("B", [16, 40, 64])
def test_ln_seam_vs_launches(gpu, B):
    """C3's width (16 heads x 128, hid 2048, inter 8192), 2 layers: 16 rows
    (one row block), 40 (a partial block) and 64 (C3's batch)."""
    import llm_capi
    from _util import rel_err
    tune = llm_capi.load_tune()
    L, H, D, V, S = 2, 16, 128, 512, 512
    w = _model(np.random.default_rng(4), L, H * D, 4 * H * D, V)
    seam = _run(tune, w, L, H, D, V, S, B, 300, 3, True)
    again = _run(tune, w, L, H, D, V, S, B, 300, 3, True)
    launch = _run(tune, w, L, H, D, V, S, B, 300, 3, False)
    assert np.isfinite(seam).all()
    assert np.array_equal(seam.view(np.uint32), again.view(np.uint32))
    for st in range(3):
        assert rel_err(seam[st], launch[st]) < 1e-3, (st, rel_err(seam[st], launch[st]))
    prod = _run(llm_capi.load(), w, L, H, D, V, S, B, 300, 3, False)
    assert np.array_equal(prod.view(np.uint32), launch.view(np.uint32))
