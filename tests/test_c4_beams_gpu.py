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

from _util import assert_parity, rel_err

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
        assert_parity(outs[W][row, head], ref[0, 0], 1e-3)
        assert_parity(outs[1][row, head], ref[0, 0], 1e-3)


@pytest.mark.parametrize("B,T,shared,equal", [
    (6, 700, 30, True),    # a full group and a 2-row group (no sharing in the second)
    (8, 5, 1, True),       # context inside the first page, most splits empty
    (12, 330, 20, False),  # ragged contexts: one wave per beam, own pages
    (8, 4096, 240, True),  # C4 shape per sequence, 2 sequences
])
def test_beam_group_kernel_edges(gpu, oracle, B, T, shared, equal, monkeypatch):
    """The beam-group attention launch (row_group 4, fp16, D 128, page 16) on
    the cases its schedule branches on: partial groups, sub-page contexts and
    empty splits, ragged contexts, beam_ids routing inside a group, a missing
    shared page, and never-written (NaN) token rows past every context in both
    shared and private pages.  Oracle 1e-3, plain schedule 1e-5.  The same
    cases run through the tuning build's MFMA beam kernel (LLM_BEAM_MFMA=1),
    its one-wave-per-group kernel (LLM_BEAM4=1), the shipped form fed by an
    LDS-DMA ring (LLM_BEAM_RING=3 / 4 / 8: the same bits), the group-major
    workgroup order (LLM_BEAM_SMAJ=0: the same bits), round 4's
    contiguous cost-balanced splits (LLM_BEAM_INTERLEAVE=0) and the
    dynamic-assignment form (LLM_BEAM_STEAL=1)."""
    import torch
    import llm_capi
    rng = np.random.default_rng(B * 7 + T)
    H, D, ts, W = 3, 128, 16, 4
    nt = (T + ts - 1) // ts
    shared = min(shared, nt)
    seqs = (B + W - 1) // W
    num_pages = seqs * H * shared + B * H * (nt - shared) + 2
    perm = rng.permutation(num_pages).astype(np.int32)
    pt = np.full((B, H, nt), -1, np.int32)
    i = 0
    for sq in range(seqs):
        blk = perm[i:i + H * shared].reshape(H, shared)
        i += H * shared
        for w in range(W):
            if sq * W + w < B:
                pt[sq * W + w, :, :shared] = blk
    for b in range(B):
        pt[b, :, shared:] = perm[i:i + H * (nt - shared)].reshape(H, nt - shared)
        i += H * (nt - shared)
    if shared > 2:
        pt[0:W, 1, 2] = -1  # a missing shared page
    if equal:
        lens = np.repeat(rng.integers(max(1, T - 40), T + 1, size=seqs), W)[:B].astype(np.int32)
    else:
        lens = rng.integers(1, T + 1, size=B).astype(np.int32)
    kp = (rng.standard_normal((num_pages, ts, D)) * D ** -0.25).astype(np.float16)
    vp = rng.standard_normal((num_pages, ts, D)).astype(np.float16)
    # never-written rows: NaN past each row's context in its last page (only
    # where no other row of the group reads those tokens: equal contexts, or a
    # private page)
    for b in range(B):
        t = int(lens[b])
        if t % ts and (equal or t // ts >= shared):
            for h in range(H):
                pg = pt[b, h, t // ts]
                if pg >= 0:
                    kp[pg, t % ts:] = np.nan
                    vp[pg, t % ts:] = np.nan
    # beam_ids: rows of a group read their page-table rows in a permuted order
    beam_ids = np.arange(B, dtype=np.int32)
    beam_ids[:W] = [1, 3, 0, 2][:min(W, B)]
    q = (rng.standard_normal((B, H, D)) * D ** -0.25).astype(np.float32)
    d = lambda a: torch.from_numpy(a).cuda()
    kf = np.nan_to_num(kp.astype(np.float32), nan=0.0)
    vf = np.nan_to_num(vp.astype(np.float32), nan=0.0)
    ref = oracle.paged_attention(q, kf, vf, pt, T=T, context_lens=lens, beam_ids=beam_ids)
    plain = llm_capi.pa_decode(d(q), d(kp), d(vp), d(pt), T=T, context_lens=d(lens),
                               beam_ids=d(beam_ids)).cpu().numpy()
    outg = llm_capi.pa_decode(d(q), d(kp), d(vp), d(pt), T=T, context_lens=d(lens),
                              beam_ids=d(beam_ids), row_group=4).cpu().numpy()
    assert np.isfinite(outg).all()
    assert_parity(plain, ref, 1e-3)
    assert_parity(outg, ref, 1e-3)
    assert rel_err(outg, plain) < 1e-5
    # the tuning build's MFMA beam kernel (not in the product library; its
    # switch is read per launch, and restored when the test ends)
    monkeypatch.setenv("LLM_BEAM_MFMA", "1")
    outm = llm_capi.pa_decode(d(q), d(kp), d(vp), d(pt), T=T, context_lens=d(lens),
                              beam_ids=d(beam_ids), row_group=4,
                              lib=llm_capi.load_tune()).cpu().numpy()
    assert np.isfinite(outm).all()
    assert_parity(outm, ref, 1e-3)
    assert rel_err(outm, plain) < 1e-5
    # ... and its one-wave-per-beam-group kernel (pa_beam4_kernel, LLM_BEAM4=1)
    monkeypatch.setenv("LLM_BEAM_MFMA", "0")
    monkeypatch.setenv("LLM_BEAM4", "1")
    out4 = llm_capi.pa_decode(d(q), d(kp), d(vp), d(pt), T=T, context_lens=d(lens),
                              beam_ids=d(beam_ids), row_group=4,
                              lib=llm_capi.load_tune()).cpu().numpy()
    assert np.isfinite(out4).all()
    assert_parity(out4, ref, 1e-3)
    assert rel_err(out4, plain) < 1e-5
    # ... and the shipped form with its shared chunks delivered by an LDS-DMA
    # ring (LLM_BEAM_RING): the same arithmetic over the same bytes, so the
    # same bits as the product launch
    monkeypatch.setenv("LLM_BEAM4", "0")
    for ring in (3, 4, 8):
        monkeypatch.setenv("LLM_BEAM_RING", str(ring))
        outr = llm_capi.pa_decode(d(q), d(kp), d(vp), d(pt), T=T, context_lens=d(lens),
                                  beam_ids=d(beam_ids), row_group=4,
                                  lib=llm_capi.load_tune()).cpu().numpy()
        assert np.array_equal(outr.view(np.uint32), outg.view(np.uint32)), (ring, rel_err(outr, outg))
    monkeypatch.delenv("LLM_BEAM_RING")
    # ... and the group-major workgroup order (LLM_BEAM_SMAJ=0, the order until
    # round 6; the product launches split-major): every workgroup does the same
    # work either way, so the same bits
    monkeypatch.setenv("LLM_BEAM_SMAJ", "0")
    outo = llm_capi.pa_decode(d(q), d(kp), d(vp), d(pt), T=T, context_lens=d(lens),
                              beam_ids=d(beam_ids), row_group=4,
                              lib=llm_capi.load_tune()).cpu().numpy()
    assert np.array_equal(outo.view(np.uint32), outg.view(np.uint32)), rel_err(outo, outg)
    monkeypatch.delenv("LLM_BEAM_SMAJ")
    # ... and round 4's contiguous, cost-balanced splits (a 512-tile prefix scan
    # in every workgroup) in place of the interleaved ones
    monkeypatch.setenv("LLM_BEAM_INTERLEAVE", "0")
    outc = llm_capi.pa_decode(d(q), d(kp), d(vp), d(pt), T=T, context_lens=d(lens),
                              beam_ids=d(beam_ids), row_group=4,
                              lib=llm_capi.load_tune()).cpu().numpy()
    assert np.isfinite(outc).all()
    assert_parity(outc, ref, 1e-3)
    assert rel_err(outc, plain) < 1e-5
    monkeypatch.delenv("LLM_BEAM_INTERLEAVE")
    # ... and the decoder's form: tiles assigned to the splits while the launch
    # runs (pa_beam_steal.hpp; standalone here on the tuning build's own
    # counters, LLM_BEAM_STEAL=1).  Run three times: the counters must come
    # back to zero after every launch (a stale counter skips tiles).  Which
    # split sums which tile varies run to run, so only fp32 merge rounding differs.
    monkeypatch.setenv("LLM_BEAM_STEAL", "1")
    for _ in range(3):
        outs = llm_capi.pa_decode(d(q), d(kp), d(vp), d(pt), T=T, context_lens=d(lens),
                                  beam_ids=d(beam_ids), row_group=4,
                                  lib=llm_capi.load_tune()).cpu().numpy()
        assert np.isfinite(outs).all()
        assert_parity(outs, ref, 1e-3)
        assert rel_err(outs, plain) < 1e-5
