"""Parity of the HIP paged decode attention (pa_decode, via the C ABI) against
the CPU oracle and the reference-built golden fixtures.

Tolerance (north_star): page-table indexing is bit-exact by construction (a
wrong page changes the output by O(1)); fp16-KV / fp32-accumulate outputs must
agree within 1e-3 relative (max-abs error / max-abs reference)."""
import numpy as np
import pytest

from _util import assert_parity, GOLDEN, load_attn_fixture, rel_err, tiles_to_pool

pytestmark = pytest.mark.gpu
RTOL = 1e-3

GPU_CASES = ["c1_base", "c1_missing", "beam_route", "temp07", "d128", "ragged_tail", "ts32",
             "all_missing"]


def _dev(a, dtype=None):
    import torch
    t = torch.from_numpy(np.ascontiguousarray(a))
    if dtype is not None:
        t = t.to(dtype)
    return t.cuda()


@pytest.mark.parametrize("name", GPU_CASES)
@pytest.mark.parametrize("pps", [0, 1, 3])
def test_pa_decode_matches_golden(gpu, oracle, name, pps):
    import llm_capi
    f = load_attn_fixture(name)
    assert f["top_k"] == 0 and f["top_p"] >= 1.0 and f["eos"] < 0
    k_pool, v_pool, pt = tiles_to_pool(f["k"], f["v"], f["present"])
    bi = None if f["beam_ids"] is None else _dev(f["beam_ids"])
    out = llm_capi.pa_decode(_dev(f["q"]), _dev(k_pool), _dev(v_pool), _dev(pt), T=f["T"],
                             beam_ids=bi, sm_scale=1.0 / f["temperature"] ** 2,
                             pages_per_split=pps).cpu().numpy()
    if name == "all_missing":
        np.testing.assert_array_equal(out, np.zeros_like(out))
    else:
        assert_parity(out, f["out"], RTOL)
    ref = oracle.paged_attention(f["q"], k_pool.astype(np.float32), v_pool.astype(np.float32), pt,
                                 T=f["T"], beam_ids=f["beam_ids"], temperature=f["temperature"])
    if name != "all_missing":
        assert_parity(out, ref, RTOL)


def _random_case(rng, B, H, D, T, ts, *, num_beams=None, max_tiles=None, missing_frac=0.0):
    num_beams = num_beams or B
    nt = (T + ts - 1) // ts
    max_tiles = max_tiles or nt
    num_pages = num_beams * H * nt + 5
    scale = D ** -0.25
    q = (rng.standard_normal((B, H, D)) * scale).astype(np.float32)
    k_pool = (rng.standard_normal((num_pages, ts, D)) * scale).astype(np.float16)
    v_pool = rng.standard_normal((num_pages, ts, D)).astype(np.float16)
    perm = rng.permutation(num_pages)[: num_beams * H * nt].astype(np.int32)
    pt = np.full((num_beams, H, max_tiles), -1, np.int32)
    pt[:, :, :nt] = perm.reshape(num_beams, H, nt)
    if missing_frac:
        mask = rng.random(pt[:, :, :nt].shape) < missing_frac
        pt[:, :, :nt][mask] = -1
    return q, k_pool, v_pool, pt


@pytest.mark.parametrize("B,H,D,T,ts", [
    (16, 12, 64, 2048, 16),   # C2 attention shape
    (3, 4, 128, 1000, 16),    # ragged tail, D=128
    (2, 2, 256, 300, 16),
    (5, 3, 32, 257, 32),
    (4, 2, 128, 4096, 32),
])
def test_pa_decode_random_vs_oracle(gpu, oracle, B, H, D, T, ts):
    import llm_capi
    rng = np.random.default_rng(B * 1000 + T)
    q, kp, vp, pt = _random_case(rng, B, H, D, T, ts, missing_frac=0.02)
    ref = oracle.paged_attention(q, kp.astype(np.float32), vp.astype(np.float32), pt, T=T)
    for pps in (0, 8, 64):
        out = llm_capi.pa_decode(_dev(q), _dev(kp), _dev(vp), _dev(pt), T=T,
                                 pages_per_split=pps).cpu().numpy()
        assert_parity(out, ref, RTOL)


def test_pa_decode_long_splits_second_page_register(gpu, oracle):
    """B*H large enough that the balanced split count is small and each split
    walks > 64 pages (page ids 64..127 come from the second per-lane register),
    with ragged per-row contexts so every row derives its own split length."""
    import llm_capi
    rng = np.random.default_rng(21)
    B, H, D, T, ts = 64, 32, 32, 16 * 300, 16
    q, kp, vp, pt = _random_case(rng, B, H, D, T, ts, missing_frac=0.01)
    lens = rng.integers(1, T + 1, size=B).astype(np.int32)
    lens[0], lens[1] = T, 16 * 257 + 3  # 4 splits: 300 tiles -> 75 per split; 258 -> 65
    ref = oracle.paged_attention(q, kp.astype(np.float32), vp.astype(np.float32), pt, T=T,
                                 context_lens=lens)
    lib = llm_capi.load()
    assert lib.pa_decode_pages_per_split(B, H, T, ts, pt.shape[2]) > 64
    for pps in (0, 100, 128):
        out = llm_capi.pa_decode(_dev(q), _dev(kp), _dev(vp), _dev(pt), T=T,
                                 context_lens=_dev(lens), pages_per_split=pps).cpu().numpy()
        assert_parity(out, ref, RTOL)


def test_pa_decode_ragged_context_and_beams(gpu, oracle):
    import llm_capi
    rng = np.random.default_rng(11)
    B, H, D, T, ts = 6, 4, 128, 700, 16
    q, kp, vp, pt = _random_case(rng, B, H, D, T, ts, num_beams=3, max_tiles=50)
    beam_ids = np.array([2, 0, 1, 1, 0, 2], np.int32)
    lens = np.array([700, 1, 0, 17, 512, 333], np.int32)
    ref = oracle.paged_attention(q, kp.astype(np.float32), vp.astype(np.float32), pt, T=T,
                                 beam_ids=beam_ids, context_lens=lens)
    for pps in (0, 4, 64):
        out = llm_capi.pa_decode(_dev(q), _dev(kp), _dev(vp), _dev(pt), T=T,
                                 beam_ids=_dev(beam_ids), context_lens=_dev(lens),
                                 pages_per_split=pps).cpu().numpy()
        assert_parity(out, ref, RTOL)
        np.testing.assert_array_equal(out[2], 0.0)  # empty context -> zeros


def test_pa_decode_softmax_spike(gpu, oracle):
    """Force the online-softmax rescale: a key in a late page dominates."""
    import llm_capi
    rng = np.random.default_rng(5)
    B, H, D, T, ts = 2, 2, 128, 1024, 16
    q, kp, vp, pt = _random_case(rng, B, H, D, T, ts)
    # put a strongly aligned key at token 900 of (0,0) and token 17 of (1,1)
    for (b, h, t) in [(0, 0, 900), (1, 1, 17)]:
        page = pt[b, h, t // ts]
        kp[page, t % ts] = (q[b, h] * 3.0).astype(np.float16)
    ref = oracle.paged_attention(q, kp.astype(np.float32), vp.astype(np.float32), pt, T=T)
    for pps in (0, 8, 64):
        out = llm_capi.pa_decode(_dev(q), _dev(kp), _dev(vp), _dev(pt), T=T,
                                 pages_per_split=pps).cpu().numpy()
        assert_parity(out, ref, RTOL)


@pytest.mark.parametrize("H", [16, 32], ids=["c3", "c5_per_gpu"])
def test_pa_decode_full_size_properties(gpu, oracle, H):
    """C3 attention shape (B64 H16 D128 T8192 ts16, shuffled pages) and the C5
    per-GPU shard (B64 H32: 64 of the 512 rows, 8.6 GB of KV per launch): exact
    oracle parity on sampled (b, h) rows plus size-independent identities."""
    import torch
    import llm_capi
    B, D, T, ts = 64, 128, 8192, 16
    nt = T // ts
    num_pages = B * H * nt
    g = torch.Generator(device="cuda").manual_seed(0)
    kp = (torch.randn((num_pages, ts, D), generator=g, device="cuda") * D ** -0.25).half()
    vp = torch.randn((num_pages, ts, D), generator=g, device="cuda").half()
    q = torch.randn((B, H, D), generator=g, device="cuda") * D ** -0.25
    perm = torch.randperm(num_pages, generator=g, device="cuda").to(torch.int32)
    pt = perm.reshape(B, H, nt).contiguous()
    out = llm_capi.pa_decode(q, kp, vp, pt, T=T)
    torch.cuda.synchronize()
    rng = np.random.default_rng(0)
    pt_h = pt.cpu().numpy()
    for _ in range(6):
        b, h = int(rng.integers(B)), int(rng.integers(H))
        pages = pt_h[b, h]
        kk = kp[torch.from_numpy(pages).long().cuda()].float().cpu().numpy()
        vv = vp[torch.from_numpy(pages).long().cuda()].float().cpu().numpy()
        sub_pt = np.arange(nt, dtype=np.int32).reshape(1, 1, nt)
        ref = oracle.paged_attention(q[b:b + 1, h:h + 1].cpu().numpy(), kk, vv, sub_pt, T=T)
        assert_parity(out[b, h].cpu().numpy(), ref[0, 0], RTOL)
    # identity 1: constant V rows -> out == that row (sum p / (sum p + 1e-6))
    c = torch.randn(D, device="cuda").half()
    vconst = c.expand(num_pages, ts, D).contiguous()
    o1 = llm_capi.pa_decode(q, kp, vconst, pt, T=T)
    assert torch.allclose(o1, c.float().expand(B, H, D), rtol=1e-3, atol=1e-3)
    # identity 2: K = 0 -> uniform softmax -> mean of V over the row's tokens
    o2 = llm_capi.pa_decode(q, torch.zeros_like(kp), vp, pt, T=T)
    mean = vp[pt.long()].float().mean(dim=(2, 3))  # [B][H][D]
    assert rel_err(o2.cpu().numpy(), mean.cpu().numpy()) < RTOL  # identity vs torch, not oracle


def test_pa_decode_rejects_bad_shapes(gpu):
    import ctypes
    import torch
    import llm_capi
    lib = llm_capi.load()
    kp = torch.zeros((4, 16, 64), dtype=torch.float16, device="cuda")
    pt = torch.zeros((1, 2, 4), dtype=torch.int32, device="cuda")
    view = llm_capi.kv_view(kp, kp, pt)
    q = torch.zeros((1, 2, 64), device="cuda")
    out = torch.zeros_like(q)
    # H mismatch
    rc = lib.pa_decode(ctypes.byref(view), llm_capi.ptr(q), llm_capi.ptr(out), None, None,
                       1, 3, 64, 16, 1.0, 0, None, 0, llm_capi.stream_ptr())
    assert rc == llm_capi.LLM_ERR_INVALID
    # unsupported D
    rc = lib.pa_decode(ctypes.byref(view), llm_capi.ptr(q), llm_capi.ptr(out), None, None,
                       1, 2, 48, 16, 1.0, 0, None, 0, llm_capi.stream_ptr())
    assert rc == llm_capi.LLM_ERR_INVALID


def test_pa_decode_stale_nan_rows_ignored(gpu, oracle):
    """Rows of a page past the context hold whatever was there before (a fresh
    hipMalloc can hold NaN/Inf bit patterns); they must not leak into out."""
    import llm_capi
    rng = np.random.default_rng(17)
    B, H, D, T, ts = 3, 2, 128, 200, 16  # 200 = 12 full pages + 8 rows
    q, kp, vp, pt = _random_case(rng, B, H, D, T, ts)
    ref = oracle.paged_attention(q, kp.astype(np.float32), vp.astype(np.float32), pt, T=T)
    last = pt[:, :, T // ts]
    kp[last, T % ts:] = np.nan
    vp[last, T % ts:] = np.inf
    unused = np.setdiff1d(np.arange(kp.shape[0]), pt.ravel())
    kp[unused] = np.nan
    vp[unused] = np.nan
    for pps in (0, 4):
        out = llm_capi.pa_decode(_dev(q), _dev(kp), _dev(vp), _dev(pt), T=T,
                                 pages_per_split=pps).cpu().numpy()
        assert np.isfinite(out).all()
        assert_parity(out, ref, RTOL)


def _kv_elems(rng, dtype, shape, scale):
    """Random KV pool values exactly representable in `dtype`; returns (device
    tensor, fp32 numpy copy the oracle reads)."""
    import torch
    if dtype == torch.int8:  # raw int8 values (KVTileCache<int8_t>, no scale)
        a = rng.integers(-4, 5, size=shape).astype(np.int8)
        return torch.from_numpy(a).cuda(), a.astype(np.float32)
    t = torch.from_numpy((rng.standard_normal(shape) * scale).astype(np.float32)).to(dtype)
    return t.cuda(), t.float().numpy()


@pytest.mark.parametrize("kv_dtype", ["bfloat16", "float32", "int8", "float16"])
@pytest.mark.parametrize("B,H,D,T,ts", [
    (3, 4, 128, 1000, 16),
    (2, 2, 64, 300, 32),
    (2, 3, 256, 200, 16),
    (5, 3, 32, 257, 32),
])
def test_pa_decode_kv_dtypes_vs_oracle(gpu, oracle, kv_dtype, B, H, D, T, ts):
    """AttentionCUDA::forward's element types (attention/attention_cuda.cu:58-94:
    __half, bf16, int8_t, float): pools of each type, every page 1..16 KiB.
    The kernel widens each element to fp32 exactly, so the oracle reads the
    same values as fp32 and the 1e-3 bound applies unchanged."""
    import torch
    import llm_capi
    dt = getattr(torch, kv_dtype)
    es = torch.empty(0, dtype=dt).element_size()
    if not (1024 <= ts * D * es <= 16384):
        pytest.skip("page size outside 1..16 KiB")
    rng = np.random.default_rng(D * 7 + T + es)
    nt = (T + ts - 1) // ts
    num_pages = B * H * nt + 3
    qs = 0.1 if dt == torch.int8 else D ** -0.25
    q = (rng.standard_normal((B, H, D)) * qs).astype(np.float32)
    kd, kf = _kv_elems(rng, dt, (num_pages, ts, D), D ** -0.25)
    vd, vf = _kv_elems(rng, dt, (num_pages, ts, D), 1.0)
    pt = rng.permutation(num_pages)[: B * H * nt].astype(np.int32).reshape(B, H, nt)
    pt[0, 0, 1] = -1  # one missing page
    lens = rng.integers(1, T + 1, size=B).astype(np.int32)
    ref = oracle.paged_attention(q, kf, vf, pt, T=T, context_lens=lens)
    for pps in (0, 4):
        out = llm_capi.pa_decode(_dev(q), kd, vd, _dev(pt), T=T, context_lens=_dev(lens),
                                 pages_per_split=pps).cpu().numpy()
        assert_parity(out, ref, RTOL)


@pytest.mark.parametrize("kv_dtype", ["float16", "bfloat16", "float32", "int8"])
def test_pa_decode_interleaved_pools_bitwise(gpu, oracle, kv_dtype):
    """Pools whose K and V pages interleave in one allocation
    ([num_pages][K page | V page], the kv_cache layout; pa_kv_view.page_stride
    = 2 pages) give bit-identical outputs to dense copies of the same pools,
    on the split kernel (one and several splits), the beam-aware schedule and
    the filter path (pa_decode_ex)."""
    import torch
    import llm_capi
    dt = getattr(torch, kv_dtype)
    B, H, D, T, ts = 4, 3, 128, 700, 16
    rng = np.random.default_rng(11)
    nt = (T + ts - 1) // ts
    num_pages = B * H * nt + 5
    qs = 0.1 if dt == torch.int8 else D ** -0.25
    q = _dev((rng.standard_normal((B, H, D)) * qs).astype(np.float32))
    kd, kf = _kv_elems(rng, dt, (num_pages, ts, D), D ** -0.25)
    vd, vf = _kv_elems(rng, dt, (num_pages, ts, D), 1.0)
    both = torch.stack([kd, vd], dim=1).contiguous()  # [P][2][ts][D]
    ki, vi = both[:, 0], both[:, 1]
    assert llm_capi.kv_view(ki, vi, _dev(np.zeros((1, H, nt), np.int32))).page_stride == \
        2 * ts * D * both.element_size()
    pt = _dev(rng.permutation(num_pages)[: B * H * nt].astype(np.int32).reshape(B, H, nt))
    lens = _dev(rng.integers(1, T + 1, size=B).astype(np.int32))
    ref = oracle.paged_attention(q.cpu().numpy(), kf, vf, pt.cpu().numpy(), T=T,
                                 context_lens=lens.cpu().numpy())
    for pps in (0, 4, 64):
        dense = llm_capi.pa_decode(q, kd, vd, pt, T=T, context_lens=lens, pages_per_split=pps)
        inter = llm_capi.pa_decode(q, ki, vi, pt, T=T, context_lens=lens, pages_per_split=pps)
        assert torch.equal(dense, inter), (kv_dtype, pps)
        assert_parity(inter.cpu().numpy(), ref, RTOL)
    if dt == torch.float16:  # beam-aware prefetch form (fp16 pools, groups of 4)
        dense = llm_capi.pa_decode(q, kd, vd, pt, T=T, context_lens=lens, row_group=4)
        inter = llm_capi.pa_decode(q, ki, vi, pt, T=T, context_lens=lens, row_group=4)
        assert torch.equal(dense, inter)
    dense = llm_capi.pa_decode_ex(q, kd, vd, pt, T=T, context_lens=lens, top_k=5)
    inter = llm_capi.pa_decode_ex(q, ki, vi, pt, T=T, context_lens=lens, top_k=5)
    assert torch.equal(dense, inter)


FILTER_CASES = ["topk5", "topp09", "eos", "c1_base", "c1_missing", "beam_route", "temp07",
                "ragged_tail", "ts32", "all_missing"]


def _check_scores(got, want):
    missing = want <= -1e8
    np.testing.assert_array_equal(got[missing], np.full(missing.sum(), -1e9, np.float32))
    if (~missing).any():
        assert_parity(got[~missing], want[~missing], RTOL)


@pytest.mark.parametrize("name", FILTER_CASES)
def test_pa_decode_ex_matches_golden(gpu, oracle, name):
    """The reference's optional attention stages (top-k, top-p, EOS threshold,
    attention-weight and score outputs; CPUAttentionInput / Output,
    attention_cpu/attention_cpu.hpp:8-43) against the reference-built golden
    fixtures, which hold out, probs (after the filter) and scores."""
    import llm_capi
    f = load_attn_fixture(name)
    k_pool, v_pool, pt = tiles_to_pool(f["k"], f["v"], f["present"])
    bi = None if f["beam_ids"] is None else _dev(f["beam_ids"])
    out, probs, scores = llm_capi.pa_decode_ex(
        _dev(f["q"]), _dev(k_pool), _dev(v_pool), _dev(pt), T=f["T"], beam_ids=bi,
        temperature=f["temperature"], top_k=f["top_k"], top_p=f["top_p"], eos_token=f["eos"],
        eos_threshold=f["eos_thr"], want_probs=True)
    out, probs, scores = (x.cpu().numpy() for x in (out, probs, scores))
    if name == "all_missing":
        np.testing.assert_array_equal(out, np.zeros_like(out))
    else:
        assert_parity(out, f["out"], RTOL)
    assert_parity(probs, f["probs"], RTOL)
    # the filter keeps exactly the reference's set of positions
    np.testing.assert_array_equal(probs > 0, f["probs"] > 0)
    _check_scores(scores, f["scores"])


@pytest.mark.parametrize("kv_dtype", ["float16", "bfloat16", "float32", "int8"])
@pytest.mark.parametrize("top_k,top_p,eos", [(0, 1.0, -1), (7, 1.0, -1), (0, 0.6, -1),
                                             (20, 0.8, -1), (0, 1.0, 3)])
def test_pa_decode_ex_random_vs_oracle(gpu, oracle, kv_dtype, top_k, top_p, eos):
    """Filters on ragged rows with beam routing and missing pages, every KV
    element type, against the oracle's restatement of apply_topk_topp_filter."""
    import torch
    import llm_capi
    dt = getattr(torch, kv_dtype)
    rng = np.random.default_rng(top_k * 31 + eos + 5)
    B, H, D, T, ts, beams = 4, 3, 64, 700, 16, 3
    nt = (T + ts - 1) // ts
    num_pages = beams * H * nt + 2
    temp = 0.8
    q = (rng.standard_normal((B, H, D)) * (0.1 if dt == torch.int8 else 0.5)).astype(np.float32)
    kd, kf = _kv_elems(rng, dt, (num_pages, ts, D), 0.5)
    vd, vf = _kv_elems(rng, dt, (num_pages, ts, D), 1.0)
    pt = rng.permutation(num_pages)[: beams * H * nt].astype(np.int32).reshape(beams, H, nt)
    pt[1, 2, 3] = -1
    beam_ids = np.array([2, 0, 1, 2], np.int32)
    lens = np.array([700, 1, 333, 650], np.int32)
    ref, rp, rs = oracle.paged_attention(q, kf, vf, pt, T=T, beam_ids=beam_ids, context_lens=lens,
                                         temperature=temp, top_k=top_k, top_p=top_p,
                                         eos_token=eos, eos_threshold=0.0, want_probs=True)
    out, probs, scores = llm_capi.pa_decode_ex(
        _dev(q), kd, vd, _dev(pt), T=T, beam_ids=_dev(beam_ids), context_lens=_dev(lens),
        temperature=temp, top_k=top_k, top_p=top_p, eos_token=eos, eos_threshold=0.0,
        want_probs=True)
    out, probs, scores = (x.cpu().numpy() for x in (out, probs, scores))
    assert_parity(out, ref, RTOL)
    assert_parity(probs, rp, RTOL)
    np.testing.assert_array_equal(probs > 0, rp > 0)
    _check_scores(scores, rs)
    if top_k == 0 and top_p >= 1.0 and eos < 0:  # no stage active: same as the hot path
        hot = llm_capi.pa_decode(_dev(q), kd, vd, _dev(pt), T=T, beam_ids=_dev(beam_ids),
                                 context_lens=_dev(lens), sm_scale=1.0 / temp ** 2).cpu().numpy()
        assert_parity(hot, out, RTOL)


@pytest.mark.parametrize("kv_dtype", ["float16", "int8"])
@pytest.mark.parametrize("top_k,top_p,eos", [(0, 1.0, -1), (64, 1.0, -1), (0, 0.5, -1),
                                             (300, 0.9, -1), (0, 1.0, 12000)])
def test_pa_decode_ex_long_rows_vs_oracle(gpu, oracle, kv_dtype, top_k, top_p, eos):
    """Rows past the LDS form's 8192 tokens: the filtered kernel keeps each
    row's scores and sort keys in the workspace (pa_decode_ex_workspace_bytes),
    as cpu_paged_attention_forward has no context bound
    (attention_cpu/cpu_attention_kernel.cpp:61).  Ragged rows up to 20000
    tokens, beam routing, a missing page, against the oracle."""
    import torch
    import llm_capi
    dt = getattr(torch, kv_dtype)
    rng = np.random.default_rng(top_k + 7 * eos + 11)
    B, H, D, T, ts, beams = 3, 2, 64, 20000, 16, 2
    nt = (T + ts - 1) // ts
    num_pages = beams * H * nt + 2
    q = (rng.standard_normal((B, H, D)) * (0.1 if dt == torch.int8 else 0.5)).astype(np.float32)
    kd, kf = _kv_elems(rng, dt, (num_pages, ts, D), 0.5)
    vd, vf = _kv_elems(rng, dt, (num_pages, ts, D), 1.0)
    pt = rng.permutation(num_pages)[: beams * H * nt].astype(np.int32).reshape(beams, H, nt)
    pt[0, 1, 600] = -1
    beam_ids = np.array([1, 0, 1], np.int32)
    lens = np.array([20000, 8193, 13001], np.int32)
    ref, rp, rs = oracle.paged_attention(q, kf, vf, pt, T=T, beam_ids=beam_ids, context_lens=lens,
                                         temperature=0.9, top_k=top_k, top_p=top_p,
                                         eos_token=eos, eos_threshold=0.0, want_probs=True)
    out, probs, scores = llm_capi.pa_decode_ex(
        _dev(q), kd, vd, _dev(pt), T=T, beam_ids=_dev(beam_ids), context_lens=_dev(lens),
        temperature=0.9, top_k=top_k, top_p=top_p, eos_token=eos, eos_threshold=0.0,
        want_probs=True)
    out, probs, scores = (x.cpu().numpy() for x in (out, probs, scores))
    assert_parity(out, ref, RTOL)
    assert_parity(probs, rp, RTOL)
    np.testing.assert_array_equal(probs > 0, rp > 0)
    _check_scores(scores, rs)


def test_pa_decode_ex_workspace_form_equals_lds_form(gpu):
    """The same rows (<= 8192 tokens) through the LDS form (T 8192) and the
    workspace form (T 8193, the rows' context_lens unchanged): the same
    arithmetic in the same order, so out and probs are bit-identical."""
    import torch
    import llm_capi
    rng = np.random.default_rng(5)
    B, H, D, ts = 2, 3, 128, 16
    nt = 8208 // ts
    num_pages = H * nt + 1
    q = (rng.standard_normal((B, H, D)) * 0.3).astype(np.float32)
    kd, _ = _kv_elems(rng, torch.float16, (num_pages, ts, D), 0.5)
    vd, _ = _kv_elems(rng, torch.float16, (num_pages, ts, D), 1.0)
    pt = rng.permutation(num_pages)[: H * nt].astype(np.int32).reshape(1, H, nt)
    lens = _dev(np.array([8192, 5000], np.int32))
    res = []
    for T in (8192, 8193):
        out, probs, _ = llm_capi.pa_decode_ex(_dev(q), kd, vd, _dev(pt), T=T, context_lens=lens,
                                              top_k=100, top_p=0.8, want_probs=True)
        res.append((out.cpu().numpy(), probs[:, :, :8192].cpu().numpy()))
    assert np.array_equal(res[0][0].view(np.uint32), res[1][0].view(np.uint32))
    assert np.array_equal(res[0][1].view(np.uint32), res[1][1].view(np.uint32))


def test_paged_attention_binding_filters(gpu, oracle):
    """llm_decoder.paged_attention (AttentionCUDA::forward surface) with top_k /
    top_p now runs the filtered kernel instead of refusing."""
    import torch
    import llm_decoder
    rng = np.random.default_rng(2)
    H, D, TS, T = 2, 64, 16, 90
    kv = llm_decoder.KVTileCache()
    kv.init(num_pages=32, tile_size=TS, head_dim=D, num_layers=1, num_beams=1, num_heads=H,
            max_tiles=8)
    k = (rng.standard_normal((T, H, D)) * 0.4).astype(np.float16)
    v = rng.standard_normal((T, H, D)).astype(np.float16)
    kv.write_tokens(0, 0, 0, k.view(np.uint16), v.view(np.uint16))
    kv.sync_page_table_to_gpu()
    q = (rng.standard_normal((1, H, D)) * 0.5).astype(np.float32)
    qd = torch.from_numpy(q).cuda()
    out = torch.empty((1, H, D), device="cuda")
    probs = torch.empty((1, H, T), device="cuda")
    llm_decoder.paged_attention(kv.handle, 0, qd.data_ptr(), out.data_ptr(), B=1, H=H, D=D, T=T,
                                top_k=10, top_p=0.9, probs_out=probs.data_ptr())
    torch.cuda.synchronize()
    nt = (T + TS - 1) // TS
    pt = np.arange(H * nt, dtype=np.int32).reshape(1, H, nt)
    kp = np.zeros((H * nt, TS, D), np.float32)
    vp = np.zeros_like(kp)
    for h in range(H):
        for t in range(T):
            kp[pt[0, h, t // TS], t % TS] = k[t, h]
            vp[pt[0, h, t // TS], t % TS] = v[t, h]
    ref, rp, _ = oracle.paged_attention(q, kp, vp, pt, T=T, top_k=10, top_p=0.9, want_probs=True)
    assert_parity(out.cpu().numpy(), ref, RTOL)
    np.testing.assert_array_equal(probs.cpu().numpy() > 0, rp > 0)


@pytest.mark.parametrize("B,H", [(1, 1), (1, 8)])
def test_pa_decode_long_context_few_rows(gpu, oracle, B, H):
    """A long context on few (row, head) pairs wants many splits: they are
    capped at 128 (the merge keeps 128 split weights per lane) with pages per
    split raised to match.  T = 40000 is 2500 pages: 128 splits of <= 20.
    A fixed pages_per_split that would need more than 128 splits is rejected."""
    import llm_capi
    rng = np.random.default_rng(B * 10 + H)
    D, ts, T = 64, 16, 40000
    nt = (T + ts - 1) // ts
    num_pages = B * H * nt
    kp = (rng.standard_normal((num_pages, ts, D)) * D ** -0.25).astype(np.float16)
    vp = rng.standard_normal((num_pages, ts, D)).astype(np.float16)
    pt = rng.permutation(num_pages).astype(np.int32).reshape(B, H, nt)
    q = (rng.standard_normal((B, H, D)) * D ** -0.25).astype(np.float32)
    ref = oracle.paged_attention(q, kp.astype(np.float32), vp.astype(np.float32), pt, T=T)
    out = llm_capi.pa_decode(_dev(q), _dev(kp), _dev(vp), _dev(pt), T=T).cpu().numpy()
    assert_parity(out, ref, RTOL)
    with pytest.raises(llm_capi.LlmError, match="128 splits"):
        llm_capi.pa_decode(_dev(q), _dev(kp), _dev(vp), _dev(pt), T=T, pages_per_split=8)
