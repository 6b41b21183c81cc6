"""Persistent workgroup-merge attention (pa_decode.hip pa_wgm_persist_kernel).

The tuning build's LLM_WGM_PERSIST=1: when a workgroup-merge launch has
more (row, head) items than one resident round of workgroups (C3: 64 rows x
16 heads = 1024 items on 256 CUs), it launches the resident workgroup count
and each workgroup walks items blockIdx.x, + gridDim.x, ...: the waves of a
workgroup start their next item while wave 0 merges the current one.  Every
item runs the same body as the one-workgroup-per-item launch (the product's
form: the persistent one measured slower), so a decoder step must give the
SAME BITS either way.  Both forms are stepped through the C-ABI at 64 rows x 16 heads, for the
INT8 decoder (fp32 rows for the quantising o_proj prologue: C3's form) and the
FP16 decoder (packed fp16 rows, and the fused o_proj), at a long context
(every split full) and a short one (empty splits).
"""
import ctypes
import os

import numpy as np
import pytest

from test_wg_merge_gpu import _Cfg, _F16W, _model

pytestmark = pytest.mark.gpu


class _I8W(ctypes.Structure):
    _fields_ = [("emb", ctypes.c_void_p)] + [(n, ctypes.c_void_p) for n in (
        "ln1_g", "ln1_b", "ln2_g", "ln2_b", "wqkv", "sw_qkv", "wo", "sw_o", "w1", "sw1", "b1",
        "w2", "sw2", "b2")]


def _i8_model(rng, L, H, D, V):
    hid, inter = H * D, 4 * H * D
    w = {"emb": rng.standard_normal((V, hid)).astype(np.float16)}
    for k in ("ln1_g", "ln2_g"):
        w[k] = (1 + 0.1 * rng.standard_normal((L, hid))).astype(np.float32)
    for k in ("ln1_b", "ln2_b"):
        w[k] = (0.1 * rng.standard_normal((L, hid))).astype(np.float32)
    for k, (K, N) in {"wqkv": (hid, 3 * hid), "wo": (hid, hid), "w1": (hid, inter),
                      "w2": (inter, hid)}.items():
        w[k] = rng.integers(-127, 128, size=(L, K, N), dtype=np.int8)
    sc = np.float32(0.02 * 3.0 / 127.0)
    w["sw_qkv"] = np.full((L, 3 * hid), sc, np.float32)
    w["sw_o"] = np.full((L, hid), sc, np.float32)
    w["sw1"] = np.full((L, inter), sc, np.float32)
    w["sw2"] = np.full((L, hid), sc, np.float32)
    w["b1"] = (0.02 * rng.standard_normal((L, inter))).astype(np.float32)
    w["b2"] = (0.02 * rng.standard_normal((L, hid))).astype(np.float32)
    return {k: np.ascontiguousarray(v) for k, v in w.items()}


def _steps(lib, w, dtype, L, H, D, V, S, B, ctx, steps, persist, splits=0, fuse=True):
    """Logits of `steps` decode steps of a fresh decoder of `lib` (tuning build:
    persist=False keeps one workgroup per (row, head) item, splits > 0 forces
    the workgroup-merge split count, fuse=False the FP16 o_proj GEMM launch)."""
    import torch
    import llm_capi
    os.environ["LLM_WGM_PERSIST"] = "1" if persist else "0"
    os.environ["LLM_WGM_SPLITS"] = str(splits)
    os.environ["LLM_OPROJ_FUSE"] = "1" if fuse else "0"
    lib.llm_decoder_step.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_void_p]
    lib.llm_decoder_sync.argtypes = [ctypes.c_void_p]
    dec = _create(lib, w, dtype, L, H, D, V, S, B, ctx)
    try:
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
        for k in ("LLM_WGM_PERSIST", "LLM_WGM_SPLITS", "LLM_OPROJ_FUSE"):
            os.environ.pop(k, None)


def _create(lib, w, dtype, L, H, D, V, S, B, ctx):
    """A decoder of `lib` with weights `w`, `B` synthetic rows at context `ctx`."""
    import llm_capi
    lib.llm_decoder_create.argtypes = [ctypes.POINTER(_Cfg), ctypes.POINTER(ctypes.c_void_p)]
    lib.llm_decoder_set_f16_weights.argtypes = [ctypes.c_void_p, ctypes.POINTER(_F16W)]
    lib.llm_decoder_set_int8_weights.argtypes = [ctypes.c_void_p, ctypes.POINTER(_I8W)]
    lib.llm_decoder_begin_synthetic.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                                ctypes.c_uint64, ctypes.c_int]
    lib.llm_decoder_destroy.argtypes = [ctypes.c_void_p]
    lib.llm_decoder_destroy.restype = None
    cfg = _Cfg(L, H, D, H * D, V, S, 0, 16, dtype, B, 1.0, 0)
    dec = ctypes.c_void_p()
    llm_capi.check(lib.llm_decoder_create(ctypes.byref(cfg), ctypes.byref(dec)), lib)
    try:
        if dtype == llm_capi.LLM_F16:
            ww = _F16W(*[w[k].ctypes.data for k in ("emb", "ln1_g", "ln1_b", "ln2_g", "ln2_b",
                                                     "wqkv", "wo", "w1", "w2", "b1", "b2")])
            llm_capi.check(lib.llm_decoder_set_f16_weights(dec, ctypes.byref(ww)), lib)
        else:
            ww = _I8W(*[w[k].ctypes.data for k in ("emb", "ln1_g", "ln1_b", "ln2_g", "ln2_b",
                                                    "wqkv", "sw_qkv", "wo", "sw_o", "w1", "sw1",
                                                    "b1", "w2", "sw2", "b2")])
            llm_capi.check(lib.llm_decoder_set_int8_weights(dec, ctypes.byref(ww)), lib)
        llm_capi.check(lib.llm_decoder_begin_synthetic(dec, B, ctx, 91, 1), lib)
    except Exception:
        lib.llm_decoder_destroy(dec)
        raise
    return dec


def _plan(lib, w, dtype, L, H, D, V, S, B, ctx):
    """(split count, form) of the step's attention launch (llm_decoder_attention_plan)."""
    import llm_capi
    lib.llm_decoder_attention_plan.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                                               ctypes.POINTER(ctypes.c_int)]
    dec = _create(lib, w, dtype, L, H, D, V, S, B, ctx)
    try:
        ns, form = ctypes.c_int(), ctypes.c_int()
        llm_capi.check(lib.llm_decoder_attention_plan(dec, ctypes.byref(ns), ctypes.byref(form)), lib)
        return ns.value, form.value
    finally:
        lib.llm_decoder_destroy(dec)


@pytest.mark.parametrize("ctx", [4100, 8200])
def test_wgm_persistent_int8_bitwise(gpu, ctx):
    """INT8 decoder, 64 rows x 16 heads x D 128 (C3's head shape) at contexts
    that take 4 and 8 splits (512 / 256 resident workgroups for 1024 items):
    persistent and one-workgroup-per-item launches give the same logits bit
    for bit, and so does the product build (one workgroup per item)."""
    import llm_capi
    tune = llm_capi.load_tune()
    L, H, D, V, B = 2, 16, 128, 512, 64
    S = ctx + 64
    w = _i8_model(np.random.default_rng(11), L, H, D, V)
    ns, form = _plan(tune, w, llm_capi.LLM_I8, L, H, D, V, S, B, ctx)
    assert (form & 15) == 3 and ns in (4, 8), (ns, form)  # the workgroup-merge form
    on = _steps(tune, w, llm_capi.LLM_I8, L, H, D, V, S, B, ctx, 3, True)
    off = _steps(tune, w, llm_capi.LLM_I8, L, H, D, V, S, B, ctx, 3, False)
    assert np.isfinite(on).all()
    assert np.array_equal(on.view(np.uint32), off.view(np.uint32)), np.abs(on - off).max()
    prod = _steps(llm_capi.load(), w, llm_capi.LLM_I8, L, H, D, V, S, B, ctx, 3, True)
    assert np.array_equal(prod.view(np.uint32), on.view(np.uint32))


@pytest.mark.parametrize("fuse", [True, False], ids=["fused_oproj", "oproj_gemm"])
@pytest.mark.parametrize("ctx", [1500, 40])
def test_wgm_persistent_f16_bitwise(gpu, ctx, fuse):
    """FP16 decoder at 64 rows x 16 heads x D 128, 3 and 8 splits (1024 items:
    more than one resident round at either workgroup size), packed fp16 rows
    and the fused o_proj: persistent == one workgroup per item, bit for bit."""
    import llm_capi
    tune = llm_capi.load_tune()
    L, H, D, V, S, B = 2, 16, 128, 512, 1600, 64
    w = _model(np.random.default_rng(12), L, H, D, V)
    for ns in (3, 8):
        on = _steps(tune, w, llm_capi.LLM_F16, L, H, D, V, S, B, ctx, 3, True, ns, fuse)
        off = _steps(tune, w, llm_capi.LLM_F16, L, H, D, V, S, B, ctx, 3, False, ns, fuse)
        assert np.isfinite(on).all()
        assert np.array_equal(on.view(np.uint32), off.view(np.uint32)), (ns, np.abs(on - off).max())
