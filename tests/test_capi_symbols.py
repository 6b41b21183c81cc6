"""CPU checks of the drop-in boundary: the C-ABI library loads (no GPU needed)
and exports every function include/llm_decoder.h declares; the pybind11
`llm_decoder` module imports and mirrors the reference's class surface
(src/bindings.cpp:3-35).  No compute calls are made here."""
import ctypes
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "pagedattention-based-transformer-decoder-inference-framework_amd"


def test_library_exports_every_declared_symbol():
    import llm_capi
    lib = llm_capi.load()
    declared = llm_capi.declared_symbols()
    assert len(declared) > 40
    missing = [n for n in declared if not hasattr(lib, n)]
    assert not missing, f"declared in include/llm_decoder.h but not exported: {missing}"
    # and they are real dynamic exports with C linkage (no C++ mangling)
    out = subprocess.run(["nm", "-D", "--defined-only", str(llm_capi.LIB_PATH)],
                         capture_output=True, text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    assert not [n for n in declared if n not in exported]


def test_abi_version_and_pure_host_helpers():
    import llm_capi
    lib = llm_capi.load()
    assert lib.llm_abi_version() == 3
    # host-only sizing helpers (no device calls)
    assert lib.gemm_packed_bytes(llm_capi.LLM_I8, 2048, 6144) == 6144 // 16 * 2048 // 64 * 1024
    assert lib.gemm_packed_bytes(llm_capi.LLM_F16, 768, 2304) == 2304 // 16 * 768 // 32 * 1024
    # C3: 64x16 rows x 513 tiles -> 6 splits of <= 86 pages (two full rounds of
    # the host-side 3072 resident-wave estimate; <= 128 pages per split)
    assert lib.pa_decode_pages_per_split(64, 16, 8192, 16, 513) == 86
    # dynamic splits: bounded by ceil(513/128) + ceil(8192/1024) + 1 = 14 splits
    assert lib.pa_decode_workspace_bytes(64, 16, 128, 513, 0) == 64 * 16 * 14 * 130 * 4
    # small launches: fewer, longer splits (>= 32 pages) while >= 512 waves remain
    assert lib.pa_decode_pages_per_split(16, 12, 2048, 16, 128) == 32  # C2: 4 splits
    assert lib.pa_decode_pages_per_split(8, 16, 4096, 16, 256) == 32
    assert lib.pa_decode_pages_per_split(1, 16, 8192, 16, 512) == 16   # 512 waves
    assert lib.pa_decode_pages_per_split(4, 12, 1024, 16, 64) == 8     # too few waves
    assert lib.pa_decode_workspace_bytes(2, 2, 64, 16, 8) == 2 * 2 * 2 * (64 + 2) * 4
    assert lib.pa_decode_pages_per_split(-1, 1, 1, 16, 1) == -1
    # few (row, head) pairs over a long context: at most 128 splits (the merge's
    # two split-weight registers per lane)
    assert lib.pa_decode_workspace_bytes(1, 1, 64, 2500, 0) == 1 * 1 * 128 * 66 * 4


def test_invalid_arguments_rejected_before_any_launch():
    """Argument validation happens on the host: these return LLM_ERR_INVALID
    without touching a device (safe on a CPU-only machine)."""
    import llm_capi
    lib = llm_capi.load()
    v = llm_capi.PaKvView()
    assert lib.pa_decode(None, None, None, None, None, 1, 1, 64, 1, 1.0, 0, None, 0, None) == 1
    assert lib.pa_decode(ctypes.byref(v), None, None, None, None, 1, 1, 64, 1, 1.0, 0, None, 0,
                         None) == 1
    assert lib.i8_gemm(None, 64, None, None, None, 1, 16, 100, None, None, None, 0, None) == 1
    assert lib.i8_gemm(ctypes.c_void_p(1), 64, ctypes.c_void_p(1), None, None, 1, 16, 96, None,
                       None, None, 0, None) == 1  # K % 64
    assert b"K must be a multiple of 64" in lib.llm_last_error()
    assert lib.f16_gemm(None, 32, None, None, 1, 16, 32, None, 0, None) == 1
    assert lib.lm_head(None, None, None, 1, 10, 33, None) == 1
    assert lib.argmax_rows(None, 1, 10, None, None) == 1
    assert lib.kv_cache_create(0, 1, 1, 64, 16, 1, 1, ctypes.byref(ctypes.c_void_p())) == 1
    assert lib.kv_cache_create_typed(1, 1, 1, 64, 16, 1, 1, 9, ctypes.byref(ctypes.c_void_p())) == 1
    # KV element types: an unknown kv_dtype is invalid; a page outside 1..16 KiB
    # (int8, D 32, 16 tokens = 512 B) is unsupported (fake pointers: rejected
    # before anything is dereferenced)
    fake = llm_capi.PaKvView(k_pool=1, v_pool=1, page_table=1, num_pages=1, page_size=16,
                             head_dim=32, num_beams=1, num_heads=1, max_tiles=1,
                             kv_dtype=llm_capi.LLM_I8)
    args = (ctypes.c_void_p(1), ctypes.c_void_p(1), None, None, 1, 1, 32, 16, 1.0, 0, None, 0, None)
    assert lib.pa_decode(ctypes.byref(fake), *args) == llm_capi.LLM_ERR_UNSUPPORTED
    fake.kv_dtype = 9
    assert lib.pa_decode(ctypes.byref(fake), *args) == llm_capi.LLM_ERR_INVALID
    assert b"kv_dtype" in lib.llm_last_error()
    # pa_decode_ex: temperature must be positive; the filtered kernel keeps a
    # row of scores in LDS (T <= 8192), in the workspace beyond
    fake.kv_dtype = llm_capi.LLM_F16
    fake.head_dim = 64
    opt = llm_capi.PaDecodeOptions(temperature=0.0, top_k=0, top_p=1.0, eos_token=-1)
    exargs = (ctypes.c_void_p(1), ctypes.c_void_p(1), None, None, 1, 1, 64, 16)
    assert lib.pa_decode_ex(ctypes.byref(fake), *exargs, ctypes.byref(opt), None, 0, None) == 1
    opt.temperature, opt.top_k = 1.0, 5
    big = exargs[:7] + (8193,)
    assert lib.pa_decode_ex(ctypes.byref(fake), *big, ctypes.byref(opt), None, 0,
                            None) == llm_capi.LLM_ERR_INVALID
    assert b"pa_decode_ex_workspace_bytes" in lib.llm_last_error()
    assert lib.pa_decode_ex_workspace_bytes(1, 1, 8192) == 0
    assert lib.pa_decode_ex_workspace_bytes(1, 1, 8193) == 16384 * 12
    assert lib.pa_decode_ex_workspace_bytes(3, 2, 20000) == 3 * 2 * 32768 * 12
    assert lib.pa_decode_ex_workspace_bytes(0, 2, 20000) == 0
    # rows past 2^30 tokens are refused up front (the sort length would overflow
    # an int), never a hang in the power-of-two search
    assert lib.pa_decode_ex_workspace_bytes(1, 1, (1 << 30) + 1) == 0
    assert lib.pa_decode_ex_workspace_bytes(1, 1, 2**31 - 1) == 0
    assert lib.pa_decode_ex_workspace_bytes(1, 1, 1 << 30) == (1 << 30) * 12
    huge = exargs[:7] + (2**31 - 1,)
    assert lib.pa_decode_ex(ctypes.byref(fake), *huge, ctypes.byref(opt), ctypes.c_void_p(8),
                            1 << 62, None) == llm_capi.LLM_ERR_UNSUPPORTED
    assert b"T <= 2^30" in lib.llm_last_error()
    # pa_prefill: NULL view / q / out, unsupported pools (int8) and positions
    # past the page table are rejected on the host
    assert lib.pa_prefill(None, None, 0, None, 0, 0, 0, 1, 1.0, None, 0, None) == 1
    fake.kv_dtype, fake.head_dim, fake.max_tiles = llm_capi.LLM_I8, 128, 4
    pf = (ctypes.c_void_p(16), 0, ctypes.c_void_p(16), 0, 0, 0, 8, 1.0, None, 0, None)
    assert lib.pa_prefill(ctypes.byref(fake), *pf) == llm_capi.LLM_ERR_UNSUPPORTED
    fake.kv_dtype = llm_capi.LLM_F16
    pf_late = pf[:5] + (100,) + pf[6:]  # positions 100..107 need 7 tiles > max_tiles 4
    assert lib.pa_prefill(ctypes.byref(fake), *pf_late) == llm_capi.LLM_ERR_INVALID
    assert b"max_tiles" in lib.llm_last_error()
    assert lib.pa_prefill_workspace_bytes(ctypes.byref(fake), 0, 0) == 0
    # zero-size work is a successful no-op
    assert lib.pa_decode(ctypes.byref(v), None, None, None, None, 0, 1, 64, 1, 1.0, 0, None, 0,
                         None) == 0


def test_pybind_module_surface():
    import llm_decoder
    for cls in ("CUDADecoder", "INT8Decoder", "KVTileCache", "PageTable"):
        assert hasattr(llm_decoder, cls)
    for m in ("load_weights", "generate", "generate_batch", "set_weights", "step",
              "begin_synthetic"):
        assert hasattr(llm_decoder.CUDADecoder, m)
    for m in ("load_quantized_weights", "quantize_weights", "generate"):
        assert hasattr(llm_decoder.INT8Decoder, m)
    for m in ("init", "resize", "get_key_ptr", "get_value_ptr", "register_tile",
              "sync_page_table_to_gpu", "save_to_file", "load_from_file", "fork"):
        assert hasattr(llm_decoder.KVTileCache, m)
    for m in ("init", "clear", "assign", "lookup", "device_data", "sync_to_gpu", "remove"):
        assert hasattr(llm_decoder.PageTable, m)


def test_caller_import_shims():
    """`from decoder.cuda_decoder import CUDADecoder` (api/router.py:4,
    web/backend_router.py:2-3, cli/generate_cli.py:5) resolves."""
    import importlib
    m1 = importlib.import_module("decoder.cuda_decoder")
    m2 = importlib.import_module("decoder.int8_decoder")
    import llm_decoder
    assert m1.CUDADecoder is llm_decoder.CUDADecoder
    assert m2.INT8Decoder is llm_decoder.INT8Decoder


def test_no_oracle_in_product_path():
    """The product package never imports, loads or links the oracle."""
    import re
    pat = re.compile(r"(from\s+oracle|import\s+oracle|liboracle|oracle/)")
    for p in list(PKG.rglob("*.py")) + list((PKG / "csrc").glob("*")) + [PKG / "Makefile"]:
        if p.is_file():
            assert not pat.search(p.read_text(errors="ignore")), p
