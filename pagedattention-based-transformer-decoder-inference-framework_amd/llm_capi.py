"""ctypes binding of the C ABI (include/llm_decoder.h) exported by
libllm_decoder_hip.so.

This is the thin Python face of the drop-in boundary used by the tests and
bench.py to call individual entry points (pa_decode, i8_gemm, ...) on device
buffers they own (torch tensors, via data_ptr()).  The decoder-level surface
of the reference (CUDADecoder / INT8Decoder / PageTable / KVTileCache) is the
pybind11 module ``llm_decoder`` built next to this file.

There is no fallback: if the HIP library is missing, load() raises.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "libllm_decoder_hip.so"
TUNE_LIB_PATH = HERE / "libllm_decoder_hip_tune.so"  # `make tune`: A/B hooks, never the product

(LLM_OK, LLM_ERR_INVALID, LLM_ERR_UNSUPPORTED, LLM_ERR_HIP, LLM_ERR_OOM, LLM_ERR_IO,
 LLM_ERR_RANGE) = range(7)
LLM_F16, LLM_I8, LLM_F32, LLM_BF16 = 0, 1, 2, 3
LLM_ACT_NONE, LLM_ACT_RELU, LLM_ACT_GELU = 0, 1, 2
LLM_EVICT_NONE, LLM_EVICT_LRU = 0, 1

c_int, c_float, c_void_p, c_size_t = ctypes.c_int, ctypes.c_float, ctypes.c_void_p, ctypes.c_size_t
c_ll = ctypes.c_longlong
c_i32p = ctypes.POINTER(ctypes.c_int32)


class PaKvView(ctypes.Structure):
    _fields_ = [("k_pool", c_void_p), ("v_pool", c_void_p), ("page_table", c_void_p),
                ("num_pages", ctypes.c_int32), ("page_size", ctypes.c_int32),
                ("head_dim", ctypes.c_int32), ("num_beams", ctypes.c_int32),
                ("num_heads", ctypes.c_int32), ("max_tiles", ctypes.c_int32),
                ("kv_dtype", ctypes.c_int32), ("page_stride", ctypes.c_int64)]


class PaDecodeOptions(ctypes.Structure):
    _fields_ = [("temperature", ctypes.c_float), ("top_k", ctypes.c_int),
                ("top_p", ctypes.c_float), ("eos_token", ctypes.c_int),
                ("eos_threshold", ctypes.c_float), ("probs_out", c_void_p),
                ("scores_out", c_void_p)]


class LlmError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"[llm status {status}] {msg}")
        self.status = status


# name -> (restype, argtypes)
_SIGS = {
    "llm_last_error": (ctypes.c_char_p, []),
    "llm_abi_version": (c_int, []),
    "pa_decode_workspace_bytes": (c_size_t, [c_int, c_int, c_int, c_int, c_int]),
    "pa_decode_pages_per_split": (c_int, [c_int, c_int, c_int, c_int, c_int]),
    "pa_decode_plan": (c_int, [ctypes.POINTER(PaKvView), c_int, c_int, c_int, c_int, c_int, c_int,
                               c_i32p, c_i32p]),
    "pa_decode": (c_int, [ctypes.POINTER(PaKvView), c_void_p, c_void_p, c_void_p, c_void_p,
                          c_int, c_int, c_int, c_int, c_float, c_int, c_void_p, c_size_t,
                          c_void_p]),
    "pa_decode_grouped": (c_int, [ctypes.POINTER(PaKvView), c_void_p, c_void_p, c_void_p,
                                  c_void_p, c_int, c_int, c_int, c_int, c_float, c_int, c_int,
                                  c_void_p, c_size_t, c_void_p]),
    "pa_decode_ex": (c_int, [ctypes.POINTER(PaKvView), c_void_p, c_void_p, c_void_p, c_void_p,
                             c_int, c_int, c_int, c_int, ctypes.POINTER(PaDecodeOptions),
                             c_void_p, c_size_t, c_void_p]),
    "pa_prefill_workspace_bytes": (c_size_t, [ctypes.POINTER(PaKvView), c_int, c_int]),
    "pa_decode_ex_workspace_bytes": (c_size_t, [c_int, c_int, c_int]),
    "pa_prefill": (c_int, [ctypes.POINTER(PaKvView), c_void_p, c_int, c_void_p, c_int, c_int,
                           c_int, c_int, c_float, c_void_p, c_size_t, c_void_p]),
    "gemm_packed_bytes": (c_size_t, [c_int, c_int, c_int]),
    "gemm_pack_weights": (c_int, [c_int, c_void_p, c_void_p, c_int, c_int, c_void_p]),
    "i8_gemm": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                        c_void_p, c_void_p, c_void_p, c_int, c_void_p]),
    "i8_matmul_s8": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_float,
                             c_float, c_float, c_void_p, c_int, c_void_p]),
    "f16_gemm": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p,
                         c_int, c_void_p]),
    "lm_head": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p]),
    "argmax_rows": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "sample_rows": (c_int, [c_void_p, c_int, c_int, c_float, c_int, c_float, ctypes.c_uint64,
                            c_int, c_void_p, c_void_p]),
    "sample_uniform_host": (c_float, [ctypes.c_uint64, c_int, c_int]),
    "quantize_rows": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "layernorm_quant": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_float, c_void_p,
                                c_void_p, c_void_p, c_void_p]),
    "kv_cache_create": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, c_ll,
                                ctypes.POINTER(c_void_p)]),
    "kv_cache_create_typed": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, c_ll, c_int,
                                      ctypes.POINTER(c_void_p)]),
    "kv_cache_destroy": (None, [c_void_p]),
    "kv_cache_view": (c_int, [c_void_p, c_int, ctypes.POINTER(PaKvView)]),
    "kv_cache_num_pages": (c_ll, [c_void_p]),
    "kv_cache_free_pages": (c_ll, [c_void_p]),
    "kv_cache_assign": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int]),
    "kv_cache_lookup": (c_int, [c_void_p, c_int, c_int, c_int, c_int]),
    "kv_cache_remove": (c_int, [c_void_p, c_int, c_int, c_int, c_int]),
    "kv_cache_register_tile": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_i32p]),
    "kv_cache_set_eviction": (c_int, [c_void_p, c_int]),
    "kv_cache_reserve": (c_int, [c_void_p, c_int, c_int]),
    "kv_cache_fork": (c_int, [c_void_p, c_int, c_int]),
    "kv_cache_release": (c_int, [c_void_p, c_int]),
    "kv_cache_clear": (c_int, [c_void_p]),
    "kv_cache_sync": (c_int, [c_void_p, c_void_p]),
    "kv_cache_write_tokens": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    "kv_cache_k_pool": (c_void_p, [c_void_p]),
    "kv_cache_v_pool": (c_void_p, [c_void_p]),
    "kv_cache_page_stride": (ctypes.c_longlong, [c_void_p]),
    "kv_cache_page_table": (c_void_p, [c_void_p, c_int]),
    "kv_cache_save": (c_int, [c_void_p, ctypes.c_char_p]),
    "kv_cache_load": (c_int, [c_void_p, ctypes.c_char_p]),
    "kv_cache_inspect": (c_int, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_longlong)]),
    "kv_cache_save_pools": (c_int, [c_void_p, ctypes.c_char_p]),
    "kv_cache_load_pools": (c_int, [c_void_p, ctypes.c_char_p]),
    "kv_cache_save_tiles": (c_int, [c_void_p, c_int, c_int, ctypes.c_char_p]),
    "kv_cache_load_tiles": (c_int, [c_void_p, c_int, c_int, ctypes.c_char_p]),
    "kv_tiles_inspect": (c_int, [ctypes.c_char_p, ctypes.c_longlong, ctypes.POINTER(c_int)]),
    "llm_decoder_oproj_status": (c_int, [c_void_p, ctypes.POINTER(c_int),
                                         ctypes.POINTER(ctypes.c_longlong)]),
}

_lib = None


def declared_symbols() -> list[str]:
    """Every function name declared in include/llm_decoder.h."""
    import re
    hdr = (HERE.parent / "include" / "llm_decoder.h").read_text()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    names = re.findall(r"\b([a-z_][a-z0-9_]*)\s*\(", hdr)
    skip = {"if", "for", "while", "sizeof", "return", "defined"}
    return sorted({n for n in names if n not in skip})


def load(path: str | Path | None = None) -> ctypes.CDLL:
    """Load the HIP C-ABI library (raises if it is missing: no fallback)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    # LLM_CAPI_LIB: another build of the same library (same-box A/B of build flags)
    p = Path(path) if path else Path(os.environ.get("LLM_CAPI_LIB", LIB_PATH))
    if not p.exists():
        raise FileNotFoundError(
            f"{p} not found: build it with `make -C {HERE}` (or __graft_entry__.build())")
    lib = ctypes.CDLL(str(p), mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in _SIGS.items():
        if not hasattr(lib, name):  # export completeness is asserted by tests/test_capi_symbols.py
            continue
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    if path is None:
        _lib = lib
    return lib


_tune = None


def load_tune() -> ctypes.CDLL:
    """The tuning build (pa_decode_tune, i8_gemm_tune, i8_gemm_stamps and the
    env overrides), loaded RTLD_LOCAL beside the product library; for scripts
    and the variant tests only."""
    global _tune
    if _tune is None:
        if not TUNE_LIB_PATH.exists():
            raise FileNotFoundError(f"{TUNE_LIB_PATH} not found: `make -C {HERE} tune`")
        _tune = ctypes.CDLL(str(TUNE_LIB_PATH), mode=ctypes.RTLD_LOCAL)
        for name, (res, args) in _SIGS.items():
            if hasattr(_tune, name):
                f = getattr(_tune, name)
                f.restype = res
                f.argtypes = args
    return _tune


def check(status: int, lib: ctypes.CDLL | None = None) -> None:
    if status != LLM_OK:
        msg = (lib or load()).llm_last_error()
        raise LlmError(status, msg.decode() if msg else "")


def stream_ptr(stream=None):
    """hipStream_t of a torch stream (current stream by default) as void*."""
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def ptr(t) -> ctypes.c_void_p:
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


def kv_dtype_of(t) -> int:
    """llm_dtype of a torch KV pool tensor (fp16, bf16, fp32 or int8)."""
    import torch
    m = {torch.float16: LLM_F16, torch.bfloat16: LLM_BF16, torch.float32: LLM_F32,
         torch.int8: LLM_I8}
    if t.dtype not in m:
        raise TypeError(f"KV pool dtype {t.dtype} is not one of fp16/bf16/fp32/int8")
    return m[t.dtype]


def kv_view(k_pool, v_pool, page_table, *, num_beams=None) -> PaKvView:
    """View over torch device tensors k/v [num_pages][ts][D] (fp16, bf16, fp32
    or int8, both the same) and page table int32 [num_beams][H][max_tiles].
    Pages may be strided (e.g. k = kv[:, 0], v = kv[:, 1] of one
    [num_pages][2][ts][D] tensor: K and V pages interleaved) as long as each
    page is contiguous; the view's page_stride is then the page-to-page step."""
    nb, H, mt = page_table.shape
    for t in (k_pool, v_pool):
        if t.dim() != 3 or t.stride(2) != 1 or t.stride(1) != t.shape[2]:
            raise ValueError("KV pools must be [num_pages][ts][D] with contiguous pages")
    if k_pool.stride(0) != v_pool.stride(0):
        raise ValueError("k_pool and v_pool must share one page stride")
    v = PaKvView()
    v.k_pool, v.v_pool, v.page_table = k_pool.data_ptr(), v_pool.data_ptr(), page_table.data_ptr()
    v.num_pages, v.page_size, v.head_dim = k_pool.shape[0], k_pool.shape[1], k_pool.shape[2]
    v.num_beams, v.num_heads, v.max_tiles = num_beams or nb, H, mt
    if k_pool.dtype != v_pool.dtype:
        raise TypeError("k_pool and v_pool must have the same dtype")
    v.kv_dtype = kv_dtype_of(k_pool)
    dense = k_pool.shape[1] * k_pool.shape[2]
    v.page_stride = 0 if k_pool.stride(0) == dense else k_pool.stride(0) * k_pool.element_size()
    return v


def pa_decode(q, k_pool, v_pool, page_table, *, T, beam_ids=None, context_lens=None,
              sm_scale=1.0, pages_per_split=0, out=None, stream=None, row_group=1, lib=None):
    """Paged decode attention on torch device tensors; returns out [B][H][D] fp32.
    row_group > 1 uses the beam-aware schedule (pa_decode_grouped).  lib: the
    library to call (default the product build; load_tune() for variant tests)."""
    import torch
    lib = lib or load()
    B, H, D = q.shape
    if out is None:
        out = torch.empty((B, H, D), dtype=torch.float32, device=q.device)
    view = kv_view(k_pool, v_pool, page_table)
    ws_bytes = lib.pa_decode_workspace_bytes(B, H, D, page_table.shape[2], pages_per_split)
    ws = torch.empty(max(ws_bytes, 4), dtype=torch.uint8, device=q.device)
    if row_group > 1:
        check(lib.pa_decode_grouped(ctypes.byref(view), ptr(q), ptr(out), ptr(beam_ids),
                                    ptr(context_lens), B, H, D, T, sm_scale, pages_per_split,
                                    row_group, ptr(ws), ws_bytes, stream_ptr(stream)))
    else:
        check(lib.pa_decode(ctypes.byref(view), ptr(q), ptr(out), ptr(beam_ids),
                            ptr(context_lens), B, H, D, T, sm_scale, pages_per_split, ptr(ws),
                            ws_bytes, stream_ptr(stream)))
    return out


def pa_decode_ex(q, k_pool, v_pool, page_table, *, T, beam_ids=None, context_lens=None,
                 temperature=1.0, top_k=0, top_p=1.0, eos_token=-1, eos_threshold=0.0,
                 want_probs=False, stream=None):
    """pa_decode_ex on torch device tensors.  Returns out [B][H][D] fp32, or
    (out, probs [B][H][T], scores [B][H][T]) when want_probs."""
    import torch
    lib = load()
    B, H, D = q.shape
    out = torch.empty((B, H, D), dtype=torch.float32, device=q.device)
    probs = torch.empty((B, H, T), dtype=torch.float32, device=q.device) if want_probs else None
    scores = torch.empty((B, H, T), dtype=torch.float32, device=q.device) if want_probs else None
    view = kv_view(k_pool, v_pool, page_table)
    opt = PaDecodeOptions(temperature=temperature, top_k=top_k, top_p=top_p, eos_token=eos_token,
                          eos_threshold=eos_threshold,
                          probs_out=None if probs is None else probs.data_ptr(),
                          scores_out=None if scores is None else scores.data_ptr())
    ws_bytes = max(lib.pa_decode_workspace_bytes(B, H, D, page_table.shape[2], 0),
                   lib.pa_decode_ex_workspace_bytes(B, H, T))
    ws = torch.empty(max(ws_bytes, 8), dtype=torch.uint8, device=q.device)
    check(lib.pa_decode_ex(ctypes.byref(view), ptr(q), ptr(out), ptr(beam_ids), ptr(context_lens),
                           B, H, D, T, ctypes.byref(opt), ptr(ws), ws_bytes, stream_ptr(stream)))
    return (out, probs, scores) if want_probs else out


def pa_prefill(q, k_pool, v_pool, page_table, *, row, p0, sm_scale=1.0, out=None,
               split=True, stream=None):
    """Causal attention of a prompt chunk (pa_prefill): q [m][H][D] (or a
    [m][stride] row view whose first H*D floats are the heads) at positions
    p0 .. p0+m-1 of page-table row `row`; returns out [m][H][D] fp32.
    split=False runs the one-pass form (no workspace)."""
    import torch
    lib = load()
    m = q.shape[0]
    H, D = page_table.shape[1], k_pool.shape[2]
    q_stride = q.stride(0)
    if q.stride(-1) != 1:
        raise ValueError("q rows must be contiguous")
    if out is None:
        out = torch.empty((m, H, D), dtype=torch.float32, device=q.device)
    view = kv_view(k_pool, v_pool, page_table)
    ws_bytes = lib.pa_prefill_workspace_bytes(ctypes.byref(view), p0, m) if split else 0
    ws = torch.empty(max(ws_bytes, 4), dtype=torch.uint8, device=q.device) if ws_bytes else None
    check(lib.pa_prefill(ctypes.byref(view), ptr(q), q_stride, ptr(out), out.stride(0), row, p0,
                         m, sm_scale, ptr(ws), ws_bytes, stream_ptr(stream)))
    return out


def pack_weights(W, dtype: int, stream=None):
    """Repack a device [K][N] int8 / fp16 weight into MFMA fragment order."""
    import torch
    lib = load()
    K, N = W.shape
    nbytes = lib.gemm_packed_bytes(dtype, K, N)
    P = torch.empty(nbytes, dtype=torch.uint8, device=W.device)
    check(lib.gemm_pack_weights(dtype, ptr(W), ptr(P), K, N, stream_ptr(stream)))
    return P


def i8_gemm(A, W_packed, N, *, sa=None, sw=None, bias=None, act=0, want_acc=True, stream=None):
    import torch
    lib = load()
    M, K = A.shape
    acc = torch.empty((M, N), dtype=torch.int32, device=A.device) if want_acc else None
    C = torch.empty((M, N), dtype=torch.float32, device=A.device)
    check(lib.i8_gemm(ptr(A), A.stride(0), ptr(W_packed), ptr(acc), ptr(C), M, N, K, ptr(sa),
                      ptr(sw), ptr(bias), act, stream_ptr(stream)))
    return acc, C


_ACT_NAMES = {"": LLM_ACT_NONE, "relu": LLM_ACT_RELU, "gelu": LLM_ACT_GELU}


def dnnl_matmul_int8(A, B, C, BATCH, M, N, K, scaleA, scaleB, scaleC=1.0, bias=None,
                     activation="", stream=None) -> bool:
    """dnnl_matmul_int8 (attention_cpu/dnnl_matmul_int8.hpp:5-13) over device tensors:
    A int8 [BATCH][M][K], B int8 [BATCH][K][N], C int8 [BATCH][M][N] (written),
    bias fp32 [N] or None, activation "" / "relu" / "gelu".  Like the reference it
    returns False on any failure (and an unknown activation string is ignored, as
    the reference's post-op chain ignores it, dnnl_matmul_int8.cpp:44-50)."""
    import torch
    lib = load()
    act = _ACT_NAMES.get(activation, LLM_ACT_NONE)
    for t, n in ((A, BATCH * M * K), (B, BATCH * K * N), (C, BATCH * M * N)):
        if t.dtype != torch.int8 or not t.is_contiguous() or t.numel() < n:
            return False
    if bias is not None and (bias.dtype != torch.float32 or bias.numel() < N):
        return False
    return lib.i8_matmul_s8(ptr(A), ptr(B), ptr(C), BATCH, M, N, K, scaleA, scaleB, scaleC,
                            ptr(bias), act, stream_ptr(stream)) == LLM_OK


def f16_gemm(A, W_packed, N, *, bias=None, act=0, stream=None):
    import torch
    lib = load()
    M, K = A.shape
    C = torch.empty((M, N), dtype=torch.float32, device=A.device)
    check(lib.f16_gemm(ptr(A), A.stride(0), ptr(W_packed), ptr(C), M, N, K, ptr(bias), act,
                       stream_ptr(stream)))
    return C


def lm_head(x, E, stream=None):
    import torch
    lib = load()
    M, K = x.shape
    V = E.shape[0]
    out = torch.empty((M, V), dtype=torch.float32, device=x.device)
    check(lib.lm_head(ptr(x), ptr(E), ptr(out), M, V, K, stream_ptr(stream)))
    return out


def argmax_rows(logits, stream=None):
    import torch
    lib = load()
    R, V = logits.shape
    out = torch.empty(R, dtype=torch.int32, device=logits.device)
    check(lib.argmax_rows(ptr(logits), R, V, ptr(out), stream_ptr(stream)))
    return out


def sample_rows(logits, temperature=1.0, top_k=0, top_p=1.0, seed=0, counter=0, stream=None):
    """Device sampling of one token per row of fp32 logits [R][V] -> int32 [R]."""
    import torch
    lib = load()
    R, V = logits.shape
    out = torch.empty(R, dtype=torch.int32, device=logits.device)
    check(lib.sample_rows(ptr(logits), R, V, temperature, top_k, top_p, seed, counter, ptr(out),
                          stream_ptr(stream)))
    return out


def quantize_rows(x, stream=None):
    import torch
    lib = load()
    R, C = x.shape
    q = torch.empty((R, C), dtype=torch.int8, device=x.device)
    s = torch.empty(R, dtype=torch.float32, device=x.device)
    check(lib.quantize_rows(ptr(x), R, C, ptr(q), ptr(s), stream_ptr(stream)))
    return q, s


def layernorm_quant(x, gamma, beta, eps=1e-5, quant=True, stream=None):
    import torch
    lib = load()
    R, C = x.shape
    out = torch.empty((R, C), dtype=torch.float32, device=x.device)
    q = torch.empty((R, C), dtype=torch.int8, device=x.device) if quant else None
    s = torch.empty(R, dtype=torch.float32, device=x.device) if quant else None
    check(lib.layernorm_quant(ptr(x), R, C, ptr(gamma), ptr(beta), eps, ptr(out), ptr(q), ptr(s),
                              stream_ptr(stream)))
    return out, q, s
