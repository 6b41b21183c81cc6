"""Parity of the MFMA prefill attention (pa_prefill, via the C ABI): causal
paged attention of a prompt chunk, the reference's is_prefill pass
(attention/attention_cuda.hpp:21) with the maths of cpu_paged_attention_forward
(attention_cpu/cpu_attention_kernel.cpp:37-129) per query.

Oracle: the CPU restatement run as a decode batch of m rows with
beam_ids = row and context_lens = p0 + i + 1 — exactly the rows the decode
kernel computed per prompt token before this kernel existed.  Tolerance as
pa_decode: 1e-3 relative, tensor-normalised and elementwise.  The elementwise
floor is ATOL_FRAC = 4e-6 of the largest |output| (decode: 1e-6): q and p
enter the fp16 MFMAs as hi + lo halves, ~22 significant bits, so a score
carries ~2.4e-7 x sum|q_i k_i| of error and an output element ~1e-6 of the
output scale (measured 2e-7 .. 1.5e-6 of it, scripts/diag_prefill.py); an
element near zero is held to that floor, every other to 1e-3 of itself."""
import numpy as np
import pytest

from _util import assert_parity, rel_err

pytestmark = pytest.mark.gpu
RTOL = 1e-3
ATOL_FRAC = 4e-6


def _dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _case(rng, *, rows, H, D, T, ts, missing=0.0, nan_tail=False):
    nt = (T + ts - 1) // ts
    num_pages = rows * H * nt + 7
    scale = D ** -0.25
    k_pool = (rng.standard_normal((num_pages, ts, D)) * scale).astype(np.float16)
    v_pool = rng.standard_normal((num_pages, ts, D)).astype(np.float16)
    perm = rng.permutation(num_pages)[: rows * H * nt].astype(np.int32)
    pt = np.full((rows, H, nt + 2), -1, np.int32)
    pt[:, :, :nt] = perm.reshape(rows, H, nt)
    if missing:
        m = rng.random(pt[:, :, :nt].shape) < missing
        pt[:, :, :nt][m] = -1
    if nan_tail and T % ts:
        # tokens past the context in the last page were never written: NaN there
        # must not reach the output (masked keys stage V = 0)
        for r in range(rows):
            for h in range(H):
                p = pt[r, h, nt - 1]
                if p >= 0:
                    k_pool[p, T % ts:] = np.nan
                    v_pool[p, T % ts:] = np.nan
    return k_pool, v_pool, pt


def _oracle(oracle, q, kp, vp, pt, row, p0, sm_scale=1.0):
    m = q.shape[0]
    T = p0 + m
    return oracle.paged_attention(
        q, kp.astype(np.float32), vp.astype(np.float32), pt, T=T,
        beam_ids=np.full(m, row, np.int32), context_lens=np.arange(p0 + 1, T + 1, dtype=np.int32),
        temperature=sm_scale ** -0.5)


@pytest.mark.parametrize("H,D,ts,p0,m,row", [
    (4, 64, 16, 0, 1, 0),       # one token, one key
    (4, 64, 16, 0, 37, 1),      # ragged query block, first chunk
    (12, 64, 16, 100, 64, 0),   # C2 heads
    (3, 128, 16, 0, 33, 2),
    (2, 128, 16, 1000, 200, 1), # later chunk: long prefix, ragged tail page
    (2, 128, 32, 517, 96, 0),   # page 32
    (2, 64, 32, 31, 1, 1),
    (16, 128, 16, 7680, 512, 0),  # C3 heads, the last chunk of an 8192-token prompt
])
@pytest.mark.parametrize("split", [True, False])
def test_pa_prefill_vs_oracle(gpu, oracle, H, D, ts, p0, m, row, split):
    """split: key range over several workgroups + the decode merge; else one pass."""
    import llm_capi
    rng = np.random.default_rng(p0 * 7 + m + D)
    kp, vp, pt = _case(rng, rows=3, H=H, D=D, T=p0 + m, ts=ts, nan_tail=True)
    q = (rng.standard_normal((m, H, D)) * D ** -0.25).astype(np.float32)
    out = llm_capi.pa_prefill(_dev(q), _dev(kp), _dev(vp), _dev(pt), row=row, p0=p0,
                              split=split).cpu().numpy()
    ref = _oracle(oracle, q, kp, vp, pt, row, p0)
    assert np.isfinite(out).all()
    assert_parity(out, ref, RTOL, ATOL_FRAC)
    # and the decode kernel on the same rows agrees
    dec = llm_capi.pa_decode(_dev(q), _dev(kp), _dev(vp), _dev(pt), T=p0 + m,
                             beam_ids=_dev(np.full(m, row, np.int32)),
                             context_lens=_dev(np.arange(p0 + 1, p0 + m + 1, dtype=np.int32)))
    assert_parity(out, dec.cpu().numpy(), RTOL, ATOL_FRAC)


def test_pa_prefill_missing_pages_and_scale(gpu, oracle):
    import llm_capi
    rng = np.random.default_rng(11)
    H, D, ts, p0, m = 3, 128, 16, 300, 70
    kp, vp, pt = _case(rng, rows=2, H=H, D=D, T=p0 + m, ts=ts, missing=0.15)
    # spiky scores: a large sm_scale stresses the running-max rescale
    q = (rng.standard_normal((m, H, D)) * 2.0).astype(np.float32)
    out = llm_capi.pa_prefill(_dev(q), _dev(kp), _dev(vp), _dev(pt), row=1, p0=p0,
                              sm_scale=0.5).cpu().numpy()
    ref = _oracle(oracle, q, kp, vp, pt, 1, p0, sm_scale=0.5)
    assert_parity(out, ref, RTOL, ATOL_FRAC)


def test_pa_prefill_all_missing_is_zero(gpu):
    import llm_capi
    rng = np.random.default_rng(3)
    kp, vp, pt = _case(rng, rows=1, H=2, D=64, T=40, ts=16)
    pt[:] = -1
    q = rng.standard_normal((40, 2, 64)).astype(np.float32)
    out = llm_capi.pa_prefill(_dev(q), _dev(kp), _dev(vp), _dev(pt), row=0, p0=0).cpu().numpy()
    np.testing.assert_array_equal(out, np.zeros_like(out))


def test_pa_prefill_strided_q_interleaved_pools(gpu, oracle):
    """q read in place from a wider row (the decoder's qkv rows) and K/V pages
    interleaved in one allocation (kv_cache's own layout)."""
    import torch
    import llm_capi
    rng = np.random.default_rng(5)
    H, D, ts, p0, m = 4, 128, 16, 64, 48
    kp, vp, pt = _case(rng, rows=1, H=H, D=D, T=p0 + m, ts=ts)
    kv = torch.empty((kp.shape[0], 2, ts, D), dtype=torch.float16, device="cuda")
    kv[:, 0] = _dev(kp)
    kv[:, 1] = _dev(vp)
    q = (rng.standard_normal((m, H, D)) * D ** -0.25).astype(np.float32)
    wide = torch.zeros((m, 3 * H * D), dtype=torch.float32, device="cuda")
    wide[:, :H * D] = _dev(q.reshape(m, H * D))
    out = llm_capi.pa_prefill(wide, kv[:, 0], kv[:, 1], _dev(pt), row=0, p0=p0).cpu().numpy()
    ref = _oracle(oracle, q, kp, vp, pt, 0, p0)
    assert_parity(out, ref, RTOL, ATOL_FRAC)


def test_pa_prefill_rejects_unsupported(gpu):
    import llm_capi
    rng = np.random.default_rng(1)
    kp, vp, pt = _case(rng, rows=1, H=2, D=32, T=20, ts=16)
    q = rng.standard_normal((20, 2, 32)).astype(np.float32)
    with pytest.raises(llm_capi.LlmError) as ei:
        llm_capi.pa_prefill(_dev(q), _dev(kp), _dev(vp), _dev(pt), row=0, p0=0)
    assert ei.value.status == llm_capi.LLM_ERR_UNSUPPORTED
    with pytest.raises(llm_capi.LlmError):  # positions past max_tiles
        kp, vp, pt = _case(rng, rows=1, H=2, D=64, T=20, ts=16)
        q = rng.standard_normal((100, 2, 64)).astype(np.float32)
        llm_capi.pa_prefill(_dev(q), _dev(kp), _dev(vp), _dev(pt), row=0, p0=0)
