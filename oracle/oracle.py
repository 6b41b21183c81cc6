"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes front-end for ``oracle/liboracle.so`` (the C++/OpenMP restatement of the
reference's paged-attention decode path and INT8Decoder layer maths, see
``oracle.cpp``) plus small numpy helpers shared by the tests and bench.py's
``cpu_baseline`` leg.  Nothing in the product package imports this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent

_f32p = ctypes.POINTER(ctypes.c_float)
_i32p = ctypes.POINTER(ctypes.c_int32)
_i8p = ctypes.POINTER(ctypes.c_int8)
_u16p = ctypes.POINTER(ctypes.c_uint16)


def build(force: bool = False) -> None:
    """Compile oracle/liboracle*.so (gcc, no GPU needed)."""
    libs = [HERE / "liboracle.so", HERE / "liboracle_bench.so"]
    if force or not all(p.exists() for p in libs) or any(
        p.stat().st_mtime < (HERE / "oracle.cpp").stat().st_mtime for p in libs
    ):
        subprocess.run(["make", "-s", "-C", str(HERE)], check=True)


def native_build() -> bool:
    """Compile liboracle_native.so for the host this runs on (-O3
    -march=native); False if that fails (bench.py then times the portable
    build and says so)."""
    try:
        subprocess.run(["make", "-s", "-C", str(HERE), "liboracle_native.so"], check=True,
                       capture_output=True, timeout=300)
        return True
    except Exception:
        return False


def host_cpu() -> dict:
    """CPU model and the cores this process may use (the baseline's `cores`
    is the OpenMP thread count actually used)."""
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    return {"model": model, "cpus_available": avail, "cpus_machine": os.cpu_count()}


class OracleModel(ctypes.Structure):
    _fields_ = [
        ("L", ctypes.c_int), ("H", ctypes.c_int), ("D", ctypes.c_int), ("hid", ctypes.c_int),
        ("inter", ctypes.c_int), ("V", ctypes.c_int), ("max_seq", ctypes.c_int),
        ("emb", _u16p),
        ("ln1_g", _f32p), ("ln1_b", _f32p), ("ln2_g", _f32p), ("ln2_b", _f32p),
        ("wqkv", _i8p), ("sw_qkv", _f32p),
        ("wo", _i8p), ("sw_o", _f32p),
        ("w1", _i8p), ("sw1", _f32p), ("b1", _f32p),
        ("w2", _i8p), ("sw2", _f32p), ("b2", _f32p),
        ("hwqkv", _u16p), ("hwo", _u16p), ("hw1", _u16p), ("hw2", _u16p),
    ]


def _ptr(a: np.ndarray | None, typ):
    if a is None:
        return ctypes.cast(None, typ)
    assert a.flags["C_CONTIGUOUS"], "oracle arrays must be C-contiguous"
    return a.ctypes.data_as(typ)


class Oracle:
    def __init__(self, bench: bool | str = False):
        """bench=False: the checker build; True: the portable CPU-baseline
        build (x86-64-v3); "native": liboracle_native.so (-march=native, built
        on this host by native_build())."""
        build()
        name = ("liboracle_native.so" if bench == "native" else
                "liboracle_bench.so" if bench else "liboracle.so")
        self.lib = ctypes.CDLL(str(HERE / name))
        L = self.lib
        L.oracle_paged_attention.restype = ctypes.c_int
        L.oracle_paged_attention.argtypes = [
            _f32p, _f32p, _f32p, _i32p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
            _i32p, _i32p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
            ctypes.c_float, ctypes.c_int, ctypes.c_float, ctypes.c_int, ctypes.c_float,
            _f32p, _f32p, _f32p]
        L.oracle_page_lookup.restype = ctypes.c_int
        L.oracle_page_lookup.argtypes = [_i32p] + [ctypes.c_int] * 6
        L.oracle_minmax_scale.restype = ctypes.c_float
        L.oracle_minmax_scale.argtypes = [_f32p, ctypes.c_int64]
        L.oracle_quantize.argtypes = [_f32p, ctypes.c_int64, ctypes.c_float, _i8p]
        L.oracle_quantize_rows.argtypes = [_f32p, ctypes.c_int, ctypes.c_int, _i8p, _f32p]
        L.oracle_quantize_cols.argtypes = [_f32p, ctypes.c_int, ctypes.c_int, _i8p, _f32p]
        L.oracle_i8_gemm.argtypes = [_i8p, _i8p, _i32p, _f32p, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, _f32p, _f32p, _f32p, ctypes.c_int]
        L.oracle_layer_norm.argtypes = [_f32p, ctypes.c_int, ctypes.c_int, _f32p, _f32p,
                                        ctypes.c_float, _f32p]
        L.oracle_mlp_f32.argtypes = [_f32p, ctypes.c_int, ctypes.c_int, ctypes.c_int, _f32p,
                                     _f32p, _f32p, _f32p, _f32p]
        L.oracle_argmax_rows.argtypes = [_f32p, ctypes.c_int, ctypes.c_int, _i32p]
        L.oracle_half_to_float.argtypes = [_u16p, _f32p, ctypes.c_int64]
        L.oracle_float_to_half.argtypes = [_f32p, _u16p, ctypes.c_int64]
        L.oracle_set_reduction_order.argtypes = [ctypes.c_int]
        L.oracle_get_reduction_order.restype = ctypes.c_int
        L.oracle_decoder_create.restype = ctypes.c_void_p
        L.oracle_decoder_create.argtypes = [ctypes.POINTER(OracleModel), ctypes.c_int]
        L.oracle_decoder_destroy.argtypes = [ctypes.c_void_p]
        L.oracle_decoder_kv_ptr.restype = _u16p
        L.oracle_decoder_kv_ptr.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        L.oracle_decoder_step.restype = ctypes.c_int
        L.oracle_decoder_step.argtypes = [ctypes.c_void_p, _i32p, _i32p, ctypes.c_float,
                                          ctypes.c_int, ctypes.c_int, _f32p, _f32p, _i32p]
        L.oracle_decoder_step_forced.restype = ctypes.c_int
        L.oracle_decoder_step_forced.argtypes = [ctypes.c_void_p, _i32p, _i32p, ctypes.c_float,
                                                 _f32p, _i32p, _i8p, _f32p, _f32p]
        L.oracle_decoder_step_attn.restype = ctypes.c_int
        L.oracle_decoder_step_attn.argtypes = [ctypes.c_void_p, _i32p, _i32p, ctypes.c_float,
                                               _f32p, _i32p, _i8p, _f32p, _f32p, _f32p, _u16p,
                                               _f32p]
        L.oracle_num_threads.restype = ctypes.c_int
        L.oracle_set_num_threads.argtypes = [ctypes.c_int]

    # -- attention ---------------------------------------------------------
    def paged_attention(self, q, k_pool, v_pool, page_table, *, T, beam_ids=None,
                        context_lens=None, temperature=1.0, top_k=0, top_p=1.0, eos_token=-1,
                        eos_threshold=0.0, want_probs=False):
        q = np.ascontiguousarray(q, np.float32)
        B, H, D = q.shape
        num_pages, ts, D2 = k_pool.shape
        assert D2 == D
        k_pool = np.ascontiguousarray(k_pool, np.float32)
        v_pool = np.ascontiguousarray(v_pool, np.float32)
        pt = np.ascontiguousarray(page_table, np.int32)
        num_beams, H2, max_tiles = pt.shape
        assert H2 == H
        out = np.zeros((B, H, D), np.float32)
        probs = np.zeros((B, H, T), np.float32) if want_probs else None
        scores = np.zeros((B, H, T), np.float32) if want_probs else None
        bi = None if beam_ids is None else np.ascontiguousarray(beam_ids, np.int32)
        cl = None if context_lens is None else np.ascontiguousarray(context_lens, np.int32)
        rc = self.lib.oracle_paged_attention(
            _ptr(q, _f32p), _ptr(k_pool, _f32p), _ptr(v_pool, _f32p), _ptr(pt, _i32p),
            num_pages, ts, num_beams, max_tiles, _ptr(bi, _i32p), _ptr(cl, _i32p),
            B, H, D, T, temperature, top_k, top_p, eos_token, eos_threshold,
            _ptr(out, _f32p), _ptr(probs, _f32p), _ptr(scores, _f32p))
        assert rc == 0
        return (out, probs, scores) if want_probs else out

    # -- int8 ---------------------------------------------------------------
    def quantize_rows(self, x):
        x = np.ascontiguousarray(x, np.float32)
        rows, cols = x.shape
        q = np.empty((rows, cols), np.int8)
        s = np.empty(rows, np.float32)
        self.lib.oracle_quantize_rows(_ptr(x, _f32p), rows, cols, _ptr(q, _i8p), _ptr(s, _f32p))
        return q, s

    def quantize_cols(self, w):
        w = np.ascontiguousarray(w, np.float32)
        K, N = w.shape
        q = np.empty((K, N), np.int8)
        s = np.empty(N, np.float32)
        self.lib.oracle_quantize_cols(_ptr(w, _f32p), K, N, _ptr(q, _i8p), _ptr(s, _f32p))
        return q, s

    def i8_gemm(self, A, W, sa=None, sw=None, bias=None, act=0):
        A = np.ascontiguousarray(A, np.int8)
        W = np.ascontiguousarray(W, np.int8)
        M, K = A.shape
        K2, N = W.shape
        assert K == K2
        acc = np.empty((M, N), np.int32)
        C = np.empty((M, N), np.float32)
        f = lambda a: None if a is None else np.ascontiguousarray(a, np.float32)
        sa, sw, bias = f(sa), f(sw), f(bias)
        self.lib.oracle_i8_gemm(_ptr(A, _i8p), _ptr(W, _i8p), _ptr(acc, _i32p), _ptr(C, _f32p),
                                M, N, K, _ptr(sa, _f32p), _ptr(sw, _f32p), _ptr(bias, _f32p), act)
        return acc, C

    def layer_norm(self, x, gamma, beta, eps=1e-5):
        x = np.ascontiguousarray(x, np.float32)
        rows, cols = x.shape
        out = np.empty_like(x)
        self.lib.oracle_layer_norm(_ptr(x, _f32p), rows, cols,
                                   _ptr(np.ascontiguousarray(gamma, np.float32), _f32p),
                                   _ptr(np.ascontiguousarray(beta, np.float32), _f32p), eps,
                                   _ptr(out, _f32p))
        return out

    def mlp_f32(self, x, w1, b1, w2, b2):
        x = np.ascontiguousarray(x, np.float32)
        rows, hid = x.shape
        inter = w1.shape[1]
        out = np.empty((rows, hid), np.float32)
        c = lambda a: np.ascontiguousarray(a, np.float32)
        w1, b1, w2, b2 = c(w1), c(b1), c(w2), c(b2)
        self.lib.oracle_mlp_f32(_ptr(x, _f32p), rows, hid, inter, _ptr(w1, _f32p),
                                _ptr(b1, _f32p), _ptr(w2, _f32p), _ptr(b2, _f32p),
                                _ptr(out, _f32p))
        return out

    def argmax_rows(self, logits):
        logits = np.ascontiguousarray(logits, np.float32)
        rows, V = logits.shape
        out = np.empty(rows, np.int32)
        self.lib.oracle_argmax_rows(_ptr(logits, _f32p), rows, V, _ptr(out, _i32p))
        return out

    def reduction_order(self, reverse: bool):
        """Context manager (test-only control, oracle.cpp oracle_set_reduction_order):
        inside it the LayerNorm sums and the decoder's attention dot products
        run in reverse index order -- same maths, other fp32 roundings."""
        import contextlib

        @contextlib.contextmanager
        def cm():
            old = self.lib.oracle_get_reduction_order()
            self.lib.oracle_set_reduction_order(1 if reverse else 0)
            try:
                yield
            finally:
                self.lib.oracle_set_reduction_order(old)
        return cm()

    def num_threads(self) -> int:
        return int(self.lib.oracle_num_threads())


class OracleDecoder:
    """Restated INT8Decoder (contiguous fp16 KV) over host weights (see
    ``synthetic_int8_model``), or the restated CUDADecoder when the four
    projection matrices are fp16 (``wqkv`` etc. float16 / uint16 bits)."""

    def __init__(self, oracle: Oracle, w: dict, B: int):
        self.o = oracle
        self.w = w  # keep arrays alive
        cfg = w["cfg"]
        m = OracleModel()
        m.L, m.H, m.D, m.hid, m.inter, m.V, m.max_seq = (
            cfg["L"], cfg["H"], cfg["D"], cfg["hid"], cfg["inter"], cfg["V"], cfg["max_seq"])
        m.emb = _ptr(w["emb"].view(np.uint16), _u16p)
        f16 = w["wqkv"].dtype in (np.float16, np.uint16)  # CUDADecoder weights
        for name in ("ln1_g", "ln1_b", "ln2_g", "ln2_b", "b1", "b2"):
            setattr(m, name, _ptr(w[name], _f32p))
        if f16:
            for name in ("wqkv", "wo", "w1", "w2"):
                setattr(m, "h" + name, _ptr(np.ascontiguousarray(w[name]).view(np.uint16), _u16p))
        else:
            for name in ("sw_qkv", "sw_o", "sw1", "sw2"):
                setattr(m, name, _ptr(w[name], _f32p))
            for name in ("wqkv", "wo", "w1", "w2"):
                setattr(m, name, _ptr(w[name], _i8p))
        self.model = m
        self.B = B
        self.cfg = cfg
        self.h = oracle.lib.oracle_decoder_create(ctypes.byref(m), B)

    def __del__(self):
        if getattr(self, "h", None):
            self.o.lib.oracle_decoder_destroy(self.h)
            self.h = None

    def kv(self, layer: int, which: int) -> np.ndarray:
        """fp16 view [B][H][max_seq][D] of layer's K (which=0) or V (which=1)."""
        c = self.cfg
        p = self.o.lib.oracle_decoder_kv_ptr(self.h, layer, which)
        n = self.B * c["H"] * c["max_seq"] * c["D"]
        arr = np.ctypeslib.as_array(p, shape=(n,)).view(np.float16)
        return arr.reshape(self.B, c["H"], c["max_seq"], c["D"])

    def step_forced(self, tokens, pos, forced_q, forced_s, attn_scale=1.0):
        """One step teacher-forced at every int8 GEMM input (oracle.cpp
        oracle_decoder_step_forced): forced_q [L][4][B][max(hid, inter)] int8,
        forced_s [L][4][B] fp32.  Returns (logits, next, stats [L][4][3]: int8
        values that differed from the oracle's own quantisation, their max
        |difference|, max rel. difference of the row scales)."""
        c = self.cfg
        tokens = np.ascontiguousarray(tokens, np.int32)
        pos = np.ascontiguousarray(pos, np.int32)
        fq = np.ascontiguousarray(forced_q, np.int8)
        fs = np.ascontiguousarray(forced_s, np.float32)
        assert fq.shape == (c["L"], 4, self.B, max(c["hid"], c["inter"])), fq.shape
        assert fs.shape == (c["L"], 4, self.B), fs.shape
        logits = np.empty((self.B, c["V"]), np.float32)
        nxt = np.empty(self.B, np.int32)
        stats = np.zeros((c["L"], 4, 3), np.float32)
        rc = self.o.lib.oracle_decoder_step_forced(
            self.h, _ptr(tokens, _i32p), _ptr(pos, _i32p), attn_scale, _ptr(logits, _f32p),
            _ptr(nxt, _i32p), _ptr(fq, _i8p), _ptr(fs, _f32p), _ptr(stats, _f32p))
        assert rc == 0, rc
        return logits, nxt, stats

    def step_attn(self, tokens, pos, forced_q=None, forced_s=None, attn_scale=1.0,
                  forced_kv=None):
        """A step that also returns every layer's attention output before the
        o_proj input conversion: (logits, next, stats or None, attn [L][B][hid]
        fp32).  Teacher forced when forced_q is given: int8 [L][4][B][Kmax] +
        forced_s scales for INT8 weights, or fp16 [L][4][B][Kmax] (float16 /
        uint16 bits, forced_s unused) for the fp16 CUDADecoder restatement,
        whose stats are (fp16 values that differ, max |difference| / (one
        fp16 ulp + 1e-6 of the row's max), max |difference| / row max).
        forced_kv (fp16 [L][B][2][H][D]): the K / V the step appends, taken
        instead of the oracle's own rounding; self.kv_stats [L][2] then holds
        (values that differed, max |difference| / (one ulp + 1e-6 of the head's
        max))."""
        c = self.cfg
        tokens = np.ascontiguousarray(tokens, np.int32)
        pos = np.ascontiguousarray(pos, np.int32)
        logits = np.empty((self.B, c["V"]), np.float32)
        nxt = np.empty(self.B, np.int32)
        attn = np.empty((c["L"], self.B, c["hid"]), np.float32)
        stats = fq = fs = None
        if forced_q is not None:
            shape = (c["L"], 4, self.B, max(c["hid"], c["inter"]))
            if np.asarray(forced_q).dtype in (np.float16, np.uint16):
                fq = np.ascontiguousarray(np.asarray(forced_q).view(np.uint16)).view(np.int8)
                assert fq.shape[:3] == shape[:3] and fq.shape[3] == 2 * shape[3], fq.shape
            else:
                fq = np.ascontiguousarray(forced_q, np.int8)
                fs = np.ascontiguousarray(forced_s, np.float32)
                assert fq.shape == shape, fq.shape
                assert fs.shape == (c["L"], 4, self.B), fs.shape
            stats = np.zeros((c["L"], 4, 3), np.float32)
        fkv = None
        self.kv_stats = None
        if forced_kv is not None:
            fkv = np.ascontiguousarray(np.asarray(forced_kv).view(np.uint16))
            assert fkv.shape == (c["L"], self.B, 2, c["H"], c["D"]), fkv.shape
            self.kv_stats = np.zeros((c["L"], 2), np.float32)
        rc = self.o.lib.oracle_decoder_step_attn(
            self.h, _ptr(tokens, _i32p), _ptr(pos, _i32p), attn_scale, _ptr(logits, _f32p),
            _ptr(nxt, _i32p), _ptr(fq, _i8p), _ptr(fs, _f32p), _ptr(stats, _f32p),
            _ptr(attn, _f32p), _ptr(fkv, _u16p), _ptr(self.kv_stats, _f32p))
        assert rc == 0, rc
        return logits, nxt, stats, attn

    def step(self, tokens, pos, attn_scale=1.0, layers=-1, lm_head=True):
        c = self.cfg
        tokens = np.ascontiguousarray(tokens, np.int32)
        pos = np.ascontiguousarray(pos, np.int32)
        x = np.empty((self.B, c["hid"]), np.float32)
        logits = np.empty((self.B, c["V"]), np.float32) if lm_head else None
        nxt = np.empty(self.B, np.int32) if lm_head else None
        rc = self.o.lib.oracle_decoder_step(self.h, _ptr(tokens, _i32p), _ptr(pos, _i32p),
                                            attn_scale, layers, 1 if lm_head else 0,
                                            _ptr(x, _f32p), _ptr(logits, _f32p),
                                            _ptr(nxt, _i32p))
        assert rc == 0, rc
        return x, logits, nxt


# ---------------------------------------------------------------------------
# numpy helpers shared by tests / bench (host-side data preparation)
# ---------------------------------------------------------------------------

def unpack_a_i8(packed: np.ndarray, rows: int, K: int) -> np.ndarray:
    """[rows][K] int8 from the packed-A order of the GPU's GEMM inputs
    (csrc/common.hpp a_frag_off_i8: one 1 KiB block per (16-row tile, 64-k
    step); lane l = row l&15 + 16 * ((k&63) >> 4), 16 consecutive k per lane)."""
    KS = K // 64
    m = np.arange(rows)[:, None]
    k = np.arange(K)[None, :]
    off = ((((m >> 4) * KS + (k >> 6)) * 64 + (m & 15) + 16 * ((k & 63) >> 4)) * 16 + (k & 15))
    return np.asarray(packed).reshape(-1)[off]


def unpack_a_f16(packed: np.ndarray, rows: int, K: int) -> np.ndarray:
    """[rows][K] fp16 from the packed-A order of the FP16 decoder's GEMM inputs
    (csrc/common.hpp a_frag_off_f16: one 1 KiB block per (16-row tile, 32-k
    step); lane l = row l&15 + 16 * ((k&31) >> 3), 8 consecutive k per lane)."""
    KS = K // 32
    m = np.arange(rows)[:, None]
    k = np.arange(K)[None, :]
    off = ((((m >> 4) * KS + (k >> 5)) * 64 + (m & 15) + 16 * ((k & 31) >> 3)) * 8 + (k & 7))
    return np.asarray(packed).reshape(-1).view(np.float16)[off]


def dnnl_matmul_int8_np(A, B, scaleA, scaleB, scaleC=1.0, bias=None, activation=""):
    """Restatement of dnnl_matmul_int8 (attention_cpu/dnnl_matmul_int8.cpp:7-75):
    A s8 [BATCH][M][K] x B s8 [BATCH][K][N] -> C s8 [BATCH][M][N] with
    alpha = scaleA * scaleB / scaleC (:40) as the output scale, an optional f32
    bias [N] (:23, 34-37) and a relu / gelu_erf post-op (:43-50).  oneDNN is not
    in this image, so the order is oneDNN v2's reference matmul, restated:
    res = float(acc) (+ bias); res *= alpha; post-op; saturate to [-128, 127];
    round half to even (parity unpinned against oneDNN itself).  Every step is
    float32-rounded; gelu's erf is evaluated in float64 and rounded, so it can
    differ from a float32 erff by an ulp: returns (C, y) with y the value before
    rounding, for tests to skip ties at .5 boundaries."""
    A = np.asarray(A, np.int8)
    B = np.asarray(B, np.int8)
    acc = np.matmul(A.astype(np.int64), B.astype(np.int64))
    assert np.abs(acc).max(initial=0) < 2 ** 31
    f = np.float32
    alpha = f(f(f(scaleA) * f(scaleB)) / f(scaleC))
    y = acc.astype(np.int32).astype(f)
    if bias is not None:
        y = (y + np.asarray(bias, f)[None, None, :]).astype(f)
    y = (y * alpha).astype(f)
    if activation == "relu":
        y = np.maximum(y, f(0))
    elif activation == "gelu":
        import math
        t = (y * f(0.70710678118654752)).astype(f)
        erf = np.vectorize(math.erf, otypes=[np.float64])(t.astype(np.float64)).astype(f)
        y = ((f(0.5) * y).astype(f) * (f(1) + erf).astype(f)).astype(f)
    y = np.clip(y, f(-128), f(127))
    return np.rint(y).astype(np.int8), y


def quantize_rows_np(x: np.ndarray):
    """numpy mirror of int8_quant.cpp per-row quantisation (round half away)."""
    x = np.asarray(x, np.float32)
    absmax = np.maximum(np.abs(x.min(axis=1)), np.abs(x.max(axis=1)))
    scale = (np.float32(127.0) / (absmax + np.float32(1e-6))).astype(np.float32)
    y = (x * scale[:, None]).astype(np.float64)  # float32 product, exact in f64
    q = np.clip(np.sign(y) * np.floor(np.abs(y) + 0.5), -128, 127).astype(np.int8)
    return q, (np.float32(1.0) / scale).astype(np.float32)


def synthetic_int8_model(oracle: Oracle, *, L, H, D, V, max_seq, seed=1234, inter=None,
                         fast=False):
    """Seeded synthetic INT8Decoder weights: FP weights ~ N(0, 0.02),
    per-output-column int8 quantisation with int8_quant.cpp semantics; LN
    gamma ~ 1 + N(0, 0.1), beta ~ N(0, 0.1); biases ~ N(0, 0.02); embedding /
    tied LM head fp16 ~ N(0, 1).  ``fast=True`` draws the int8 weights and scales
    directly (bench-size models, same shapes, no fp32 staging)."""
    hid = H * D
    inter = inter or 4 * hid
    rng = np.random.default_rng(seed)
    w = {"cfg": dict(L=L, H=H, D=D, hid=hid, inter=inter, V=V, max_seq=max_seq)}
    w["emb"] = rng.standard_normal((V, hid), dtype=np.float32).astype(np.float16)
    w["ln1_g"] = (1 + 0.1 * rng.standard_normal((L, hid), dtype=np.float32)).astype(np.float32)
    w["ln1_b"] = (0.1 * rng.standard_normal((L, hid), dtype=np.float32)).astype(np.float32)
    w["ln2_g"] = (1 + 0.1 * rng.standard_normal((L, hid), dtype=np.float32)).astype(np.float32)
    w["ln2_b"] = (0.1 * rng.standard_normal((L, hid), dtype=np.float32)).astype(np.float32)
    shapes = {"wqkv": (hid, 3 * hid), "wo": (hid, hid), "w1": (hid, inter), "w2": (inter, hid)}
    scales = {"wqkv": "sw_qkv", "wo": "sw_o", "w1": "sw1", "w2": "sw2"}
    for name, (K, N) in shapes.items():
        qs = np.empty((L, K, N), np.int8)
        ss = np.empty((L, N), np.float32)
        for l in range(L):
            if fast:
                qs[l] = rng.integers(-127, 128, size=(K, N), dtype=np.int8)
                ss[l] = np.float32(0.02 * 3.5 / 127.0)
            else:
                wf = (0.02 * rng.standard_normal((K, N), dtype=np.float32)).astype(np.float32)
                qs[l], ss[l] = oracle.quantize_cols(wf)
        w[name] = qs
        w[scales[name]] = ss
    w["b1"] = (0.02 * rng.standard_normal((L, inter), dtype=np.float32)).astype(np.float32)
    w["b2"] = (0.02 * rng.standard_normal((L, hid), dtype=np.float32)).astype(np.float32)
    return w


def shuffled_page_table(rng, num_beams, H, max_tiles, ntiles, num_pages=None, missing=()):
    """Page table [num_beams][H][max_tiles] filled for the first ntiles tiles with a
    shuffled permutation of the page pool (non-contiguous gather);
    entries listed in ``missing`` (beam, head, tile) are -1."""
    need = num_beams * H * ntiles
    num_pages = num_pages or need
    perm = rng.permutation(num_pages)[:need].astype(np.int32)
    pt = np.full((num_beams, H, max_tiles), -1, np.int32)
    pt[:, :, :ntiles] = perm.reshape(num_beams, H, ntiles)
    for (b, h, t) in missing:
        pt[b, h, t] = -1
    return pt


# ---------------------------------------------------------------------------
# Token sampling: numpy restatement of the filter in
# top_k_top_p_filter (attention/top_k_top_p_filter.cuh:55-111) and
# apply_topk_topp_filter (attention_cpu/softmax_lut.cpp:233-256), with the
# build's defined draw (sample_uniform: splitmix64, 24 bits).
# ---------------------------------------------------------------------------
_M64 = (1 << 64) - 1


def sample_uniform(seed: int, row: int, counter: int) -> float:
    z = (seed ^ ((row & 0xFFFFFFFF) << 32) ^ (counter & 0xFFFFFFFF)) & _M64
    z = (z + 0x9E3779B97F4A7C15) & _M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    z ^= z >> 31
    return float(np.float32(z >> 40) * np.float32(1.0 / 16777216.0))


def sample_rows(logits, temperature=1.0, top_k=0, top_p=1.0, seed=0, counter=0):
    """Returns (tokens int32 [R], margin [R]): margin = relative distance of the
    draw from the nearest CDF boundary (small margins may legitimately differ
    from a device run whose float sums are ordered differently)."""
    logits = np.asarray(logits, np.float32)
    R, V = logits.shape
    toks = np.zeros(R, np.int32)
    margin = np.full(R, np.inf)
    for r in range(R):
        row = logits[r]
        if temperature <= 0 or top_k == 1:
            toks[r] = int(np.argmax(row))  # first maximum
            continue
        x = row / np.float32(temperature)
        e = np.exp((x - x.max()).astype(np.float32)).astype(np.float32)
        p = (e * np.float32(1.0 / (np.float64(e.sum(dtype=np.float64)) + 1e-6))).astype(np.float32)
        keep = np.ones(V, bool)
        if 0 < top_k < V:
            kth = np.sort(p)[-top_k]
            keep &= p >= kth
        if top_p < 1.0:
            order = np.argsort(-p, kind="stable")
            ps = p[order].astype(np.float64)
            cum_before = np.cumsum(ps) - ps
            # ties: the mass strictly above p_i (equal probabilities share it)
            uniq, first = np.unique(-ps, return_index=True)
            above = dict(zip(uniq, cum_before[first]))
            cb = np.array([above[-v] for v in ps])
            kp = np.zeros(V, bool)
            kp[order] = cb < top_p
            keep &= kp
        q = np.where(keep, p, 0).astype(np.float64)
        Z = q.sum()
        target = np.float32(sample_uniform(seed, r, counter)) * np.float32(Z)
        cdf = np.cumsum(q)
        i = int(np.searchsorted(cdf, target, side="right"))
        i = min(i, int(np.nonzero(q)[0][-1]))
        toks[r] = i
        bnd = np.abs(cdf[q > 0] - target)
        margin[r] = bnd.min() / max(Z, 1e-30)
    return toks, margin
