"""The paged attention launch at its size limits, and the empty batch.

The reference kernel has no bound of its own: it walks the page table for as
many tiles as the call asks (attention/paged_flash_attention_kernel_fused.cu:27,
`tile_id < T`).  This build's plan has one
(pa_decode.hip pa_decode_internal): at most 128 splits of at most 128 pages per
row, i.e. 16,384 pages = 262,144 tokens at page 16, the page ids of a split held
in two registers per lane (pa_split.hpp kMaxPps, kMaxSplits).  These tests hold
the longest context the plan accepts to the oracle at the north_star bar
(1e-3 tensor-wide and elementwise), with fixed splits of exactly 128 pages as
well, and check that one page more is refused with LLM_ERR_UNSUPPORTED and the
planner's message instead of being truncated."""
import numpy as np
import pytest

from _util import assert_parity

pytestmark = pytest.mark.gpu

MAX_PAGES = 128 * 128  # kMaxSplits x kMaxPps


def _case(rng, B, H, D, ts, pages):
    num_pages = B * H * pages
    perm = rng.permutation(num_pages).astype(np.int32)
    pt = perm.reshape(B, H, pages)
    kp = (rng.standard_normal((num_pages, ts, D), dtype=np.float32) * D ** -0.25).astype(np.float16)
    vp = rng.standard_normal((num_pages, ts, D), dtype=np.float32).astype(np.float16)
    q = (rng.standard_normal((B, H, D), dtype=np.float32) * D ** -0.25).astype(np.float32)
    return q, kp, vp, pt


@pytest.mark.parametrize("pps", [0, 128])
def test_longest_context_vs_oracle(gpu, oracle, pps):
    """16,384 pages per row (262,144 tokens): dynamic splits (the plan's own
    choice) and fixed 128-page splits (128 of them).  Row 1 ends 37 tokens
    short of the last page's end, so its last split holds a partial page."""
    import torch
    import llm_capi
    rng = np.random.default_rng(16384 + pps)
    B, H, D, ts = 2, 2, 128, 16
    T = MAX_PAGES * ts
    q, kp, vp, pt = _case(rng, B, H, D, ts, MAX_PAGES)
    lens = np.array([T, T - 37], np.int32)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    out = llm_capi.pa_decode(d(q), d(kp), d(vp), d(pt), T=T, context_lens=d(lens),
                             pages_per_split=pps).cpu().numpy()
    assert np.isfinite(out).all()
    ref = oracle.paged_attention(q, kp.astype(np.float32), vp.astype(np.float32), pt, T=T,
                                 context_lens=lens)
    # A head's output here averages 262,144 random-sign values: |out| ~ N^-1/2
    # of the terms' absolute sum, so an element near zero holds fp32 summation
    # noise of both sides (measured: a difference of 1.6e-8 at an element of
    # 1.5e-6, over a 1e-6-of-the-largest floor).  The elementwise floor is
    # therefore 1e-4 of the largest value (1e-6 in the shorter tests); the
    # 1e-3 bounds are unchanged.
    assert_parity(out, ref, 1e-3, atol_frac=1e-4, what=f"pages_per_split {pps}")


def test_one_page_past_the_limit_is_refused(gpu):
    """16,385 pages per row: no split plan holds them; the call fails with
    LLM_ERR_UNSUPPORTED and says why, before any launch."""
    import torch
    import llm_capi
    B, H, D, ts = 1, 1, 128, 16
    pages = MAX_PAGES + 1
    pt = torch.zeros((B, H, pages), dtype=torch.int32, device="cuda")
    kp = torch.zeros((4, ts, D), dtype=torch.float16, device="cuda")
    vp = torch.zeros_like(kp)
    q = torch.zeros((B, H, D), dtype=torch.float32, device="cuda")
    with pytest.raises(llm_capi.LlmError) as e:
        llm_capi.pa_decode(q, kp, vp, pt, T=pages * ts)
        torch.cuda.synchronize()
    assert e.value.status == llm_capi.LLM_ERR_UNSUPPORTED
    assert "128 splits" in str(e.value)
    # ... while a context that ends inside the last allowed page still plans
    out = llm_capi.pa_decode(q, kp, vp, pt, T=MAX_PAGES * ts - 5)
    torch.cuda.synchronize()
    assert torch.isfinite(out).all()


def test_empty_batch_is_a_no_op(gpu):
    """Zero rows (a decode step with no live sequence): attention (plain and
    beam-group), the INT8 and FP16 GEMM entries return LLM_OK without a launch,
    whatever their (NULL) operand pointers."""
    import torch
    import llm_capi
    kp = torch.zeros((4, 16, 128), dtype=torch.float16, device="cuda")
    pt = torch.zeros((1, 2, 4), dtype=torch.int32, device="cuda")
    q = torch.zeros((0, 2, 128), dtype=torch.float32, device="cuda")
    assert llm_capi.pa_decode(q, kp, kp, pt, T=64).shape == (0, 2, 128)
    assert llm_capi.pa_decode(q, kp, kp, pt, T=64, row_group=4).shape == (0, 2, 128)
    lib = llm_capi.load()
    assert lib.i8_gemm(None, 256, None, None, None, 0, 64, 256, None, None, None, 0,
                       llm_capi.stream_ptr()) == llm_capi.LLM_OK
    assert lib.f16_gemm(None, 256, None, None, 0, 64, 256, None, 0,
                        llm_capi.stream_ptr()) == llm_capi.LLM_OK
    torch.cuda.synchronize()
