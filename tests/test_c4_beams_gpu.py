"""BASELINE config C4 at its full size: 8 sequences x 4 beams, C3 model dims
(24 layers, 16 heads, head_dim 128), KV context 4096 of which the first 3840
tokens are shared through page-table forks (kv_cache_fork) and 256 per beam
are private -- the exact state bench.py --config c4 measures
(llm_decoder_begin_beams(8, 4, 3840, 256)).  The beam-aware attention launch
(pa_decode_grouped, row_group 4: shared prefix pages staged once per 4-beam
workgroup, cost-balanced split boundaries over 240 shared + 16 private tiles)
is held against the oracle on sampled (row, head) pairs read back from the
cache's own pages, and against the plain schedule; beam routing follows the
reference's beam_ids indirection (attention/paged_flash_attention_kernel_fused.cu:22)."""
import ctypes

import numpy as np
import pytest

from _util import rel_err

pytestmark = pytest.mark.gpu


def _read_row(lib, kvh, k_pool, stride, pb, layer, row, head, ntiles, D, ts):
    """K, V pages [ntiles][ts][D] (fp32) of (layer, row, head) and their ids."""
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    buf = np.empty((ntiles, 2, ts, D), np.float16)
    ids = []
    for t in range(ntiles):
        p = lib.kv_cache_lookup(kvh, layer, row, head, t)
        assert p >= 0
        ids.append(p)
        assert hip.hipMemcpy(buf[t].ctypes.data, ctypes.c_void_p(k_pool + p * stride),
                             2 * pb, 2) == 0
    return buf[:, 0].astype(np.float32), buf[:, 1].astype(np.float32), ids


@pytest.mark.parametrize("layer", [0, 23])
def test_c4_beam_group_attention_vs_oracle(gpu, oracle, layer):
    import torch
    import llm_capi
    import llm_decoder
    from bench import CONFIGS
    cfg = CONFIGS["c4"]
    L, H, D, B, T, ts = (cfg[k] for k in ("L", "H", "D", "B", "T", "ts"))
    seqs, W, shared = cfg["seqs"], cfg["beams"], cfg["shared"]
    dec = llm_decoder.INT8Decoder(L, H, D, H * D, 512, T + 8, max_batch=B, page_size=ts)
    dec.begin_beams(seqs, W, shared, T - shared, 1234, True)
    assert dec.context_len(0) == T and dec.context_len(B - 1) == T
    lib = llm_capi.load()
    kvh = ctypes.c_void_p(dec.kv_handle)
    view = llm_capi.PaKvView()
    llm_capi.check(lib.kv_cache_view(kvh, layer, ctypes.byref(view)))
    nt, ns = T // ts, shared // ts
    # the fork structure bench.py measures: 240 shared tiles per sequence, 16 private
    for sq in range(seqs):
        for h in (0, H - 1):
            p0 = [lib.kv_cache_lookup(kvh, layer, sq * W + w, h, ns - 1) for w in range(W)]
            p1 = [lib.kv_cache_lookup(kvh, layer, sq * W + w, h, ns) for w in range(W)]
            assert len(set(p0)) == 1 and len(set(p1)) == W
    g = torch.Generator(device="cuda").manual_seed(layer)
    q = torch.randn((B, H, D), generator=g, device="cuda") * D ** -0.25
    outs = {}
    for rg in (W, 1):
        out = torch.empty((B, H, D), device="cuda")
        wsb = llm_decoder.workspace_bytes(B, H, D, view.max_tiles, 0)
        ws = torch.empty(max(wsb, 16), dtype=torch.uint8, device="cuda")
        llm_decoder.paged_attention(dec.kv_handle, layer, q.data_ptr(), out.data_ptr(), B=B, H=H,
                                    D=D, T=T, workspace=ws.data_ptr(), workspace_bytes=wsb,
                                    row_group=rg)
        torch.cuda.synchronize()
        outs[rg] = out.cpu().numpy()
    assert np.isfinite(outs[W]).all()
    # beam-aware schedule vs plain: the same maths, split boundaries placed by
    # cost, so only the fp32 merge rounding differs
    assert rel_err(outs[W], outs[1]) < 1e-5
    # oracle on sampled (row, head): beams 0 and 3 of a sequence, first and last sequence
    qh = q.cpu().numpy()
    for row, head in [(0, 0), (3, 5), (13, 15), (B - 1, 7), (B - 4, 2), (17, 9)]:
        kk, vv, ids = _read_row(lib, kvh, view.k_pool, view.page_stride, view.page_stride // 2,
                                layer, row, head, nt, D, ts)
        sub_pt = np.arange(nt, dtype=np.int32).reshape(1, 1, nt)
        ref = oracle.paged_attention(qh[row:row + 1, head:head + 1], kk, vv, sub_pt, T=T)
        assert rel_err(outs[W][row, head], ref[0, 0]) < 1e-3, (row, head)
        assert rel_err(outs[1][row, head], ref[0, 0]) < 1e-3, (row, head)
