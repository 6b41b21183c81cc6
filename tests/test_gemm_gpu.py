"""Parity of the MFMA GEMMs and row kernels (via the C ABI) against the oracle.

INT8: int32 accumulators bit-exact (north_star); the fp32 epilogue uses the
same float operations as the oracle (mul, then add, round-to-nearest, not
contracted) and is compared bit-exactly for act none/relu, 1e-6 rel for GELU.
FP16 GEMM / LM head: fp32 reference, 1e-3 / 1e-5 rel."""
import numpy as np
import pytest

from _util import rel_err

pytestmark = pytest.mark.gpu


def _dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


@pytest.mark.parametrize("M,K,N", [
    (1, 256, 1024), (16, 768, 2304), (64, 2048, 6144), (64, 8192, 2048), (37, 256, 48),
    (130, 512, 256), (64, 256, 16), (5, 64, 32),
    # prefill-chunk row counts (M up to 512)
    (512, 2048, 2048), (300, 512, 256), (256, 8192, 512), (513, 1024, 96),
    # 17..32 rows: the 16-row tile forms (narrow_decode_tile), every output class
    (17, 2048, 2048), (24, 2048, 6144), (32, 8192, 2048), (32, 2048, 8192), (20, 768, 768),
    # 33..64 rows, under 256 column tiles: 2 column tiles x 16-row workgroups
    (33, 2048, 2048), (48, 8192, 2048), (64, 2048, 2048), (40, 768, 2304),
    # C5's per-GPU shapes (hid 4096, inter 16384): qkv, o_proj, fc1, fc2 (256 k-steps)
    (64, 4096, 12288), (64, 4096, 4096), (64, 4096, 16384), (64, 16384, 4096),
])
def test_i8_gemm_exact(gpu, oracle, M, K, N):
    import llm_capi
    rng = np.random.default_rng(M * 7 + K + N)
    A = rng.integers(-128, 128, (M, K), dtype=np.int8)
    W = rng.integers(-128, 128, (K, N), dtype=np.int8)
    sa = rng.uniform(1e-3, 1e-2, M).astype(np.float32)
    sw = rng.uniform(1e-3, 1e-2, N).astype(np.float32)
    bias = rng.standard_normal(N).astype(np.float32)
    Wp = llm_capi.pack_weights(_dev(W), llm_capi.LLM_I8)
    for act in (0, 1, 2):
        acc, C = llm_capi.i8_gemm(_dev(A), Wp, N, sa=_dev(sa), sw=_dev(sw), bias=_dev(bias), act=act)
        ref_acc, ref_C = oracle.i8_gemm(A, W, sa, sw, bias, act)
        np.testing.assert_array_equal(acc.cpu().numpy(), ref_acc)
        if act < 2:
            np.testing.assert_array_equal(C.cpu().numpy(), ref_C)
        else:
            np.testing.assert_allclose(C.cpu().numpy(), ref_C, rtol=1e-6, atol=1e-6)


def test_i8_gemm_no_scales(gpu, oracle):
    import llm_capi
    rng = np.random.default_rng(3)
    A = rng.integers(-128, 128, (8, 128), dtype=np.int8)
    W = rng.integers(-128, 128, (128, 64), dtype=np.int8)
    Wp = llm_capi.pack_weights(_dev(W), llm_capi.LLM_I8)
    acc, C = llm_capi.i8_gemm(_dev(A), Wp, 64)
    ref = A.astype(np.int64) @ W.astype(np.int64)
    np.testing.assert_array_equal(acc.cpu().numpy(), ref)
    np.testing.assert_array_equal(C.cpu().numpy(), ref.astype(np.float32))


@pytest.mark.parametrize("M,K,N,nt,waves", [
    (64, 2048, 6144, 2, 8), (64, 8192, 2048, 1, 8), (64, 2048, 2048, 1, 16), (37, 512, 96, 2, 8),
    (16, 256, 64, 1, 8), (100, 1024, 512, 2, 16), (64, 8192, 2048, 4, 4), (48, 2048, 2048, 4, 8),
    (64, 2048, 6144, 3, 8), (40, 2048, 6144, 3, 8),  # C3's qkv form: 3 column tiles
    (512, 1024, 768, 0, 0), (300, 512, 4096, 0, 0),  # prefill-chunk row counts
    # C5's per-GPU shapes in the decoder's automatic form (packed A)
    (64, 4096, 12288, 0, 0), (64, 4096, 4096, 0, 0), (64, 4096, 16384, 0, 0),
    (64, 16384, 4096, 0, 0),
])
def test_i8_gemm_packed_a_variants_exact(gpu, oracle, M, K, N, nt, waves):
    """The decoder's GEMM form: A in packed-A (MFMA fragment) order, forced
    column-tile count / waves per workgroup (i8_gemm_tune of the tuning build,
    `make tune`: the same kernels): bit-exact against the oracle like the
    row-major C ABI."""
    import ctypes
    import torch
    import llm_capi
    lib = llm_capi.load_tune()
    lib.i8_gemm_tune.restype = ctypes.c_int
    lib.i8_gemm_tune.argtypes = [ctypes.c_int] * 4 + [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                                      ctypes.c_void_p] + [ctypes.c_int] * 3 + \
        [ctypes.c_void_p] * 3
    rng = np.random.default_rng(M + K + N + nt)
    A = rng.integers(-128, 128, (M, K), dtype=np.int8)
    W = rng.integers(-128, 128, (K, N), dtype=np.int8)
    sa = rng.uniform(1e-3, 1e-2, M).astype(np.float32)
    sw = rng.uniform(1e-3, 1e-2, N).astype(np.float32)
    Wp = llm_capi.pack_weights(_dev(W), llm_capi.LLM_I8)
    Ap = llm_capi.pack_weights(_dev(np.ascontiguousarray(A.T)), llm_capi.LLM_I8)  # A-fragment order
    _, ref_C = oracle.i8_gemm(A, W, sa, sw, None, 0)
    dsa, dsw, dA = _dev(sa), _dev(sw), _dev(A)
    for packed, a_t in ((1, Ap), (0, dA)):
        for mrows in (0, 16, 32, 64):
            C = torch.full((M, N), float("nan"), device="cuda")
            llm_capi.check(lib.i8_gemm_tune(nt, waves, mrows, packed, a_t.data_ptr(), K,
                                            Wp.data_ptr(), C.data_ptr(), M, N, K, dsa.data_ptr(),
                                            dsw.data_ptr(), None), lib)
            np.testing.assert_array_equal(C.cpu().numpy(), ref_C)


@pytest.mark.parametrize("M,K,N", [(64, 2048, 2048), (32, 8192, 2048), (45, 1024, 256)])
def test_i8_gemm_split_k_forms_exact(gpu, oracle, M, K, N):
    """The tuning build's split-K forms (i8_gemm_tune_sk: 1-8 k slices of
    exact int32 partials, 1/2/4 column tiles, with and without the XCD-aware
    slice placement): the slices sum to the oracle's int32 product exactly."""
    import ctypes
    import torch
    import llm_capi
    lib = llm_capi.load_tune()
    lib.i8_gemm_tune_sk.restype = ctypes.c_int
    lib.i8_gemm_tune_sk.argtypes = [ctypes.c_int] * 5 + [ctypes.c_void_p] * 3 + \
        [ctypes.c_int] * 3 + [ctypes.c_void_p]
    rng = np.random.default_rng(M + K + N)
    A = rng.integers(-128, 128, (M, K), dtype=np.int8)
    W = rng.integers(-128, 128, (K, N), dtype=np.int8)
    Wp = llm_capi.pack_weights(_dev(W), llm_capi.LLM_I8)
    Ap = llm_capi.pack_weights(_dev(np.ascontiguousarray(A.T)), llm_capi.LLM_I8)
    ref = A.astype(np.int64) @ W.astype(np.int64)
    part = torch.empty((8, M, N), dtype=torch.int32, device="cuda")
    for nt, waves, mrows, ks, xcd in ((1, 8, 64, 2, 0), (1, 8, 64, 2, 1), (2, 8, 16, 4, 1),
                                      (4, 4, 32, 8, 1), (2, 4, 16, 1, 0), (1, 8, 32, 8, 0)):
        part.fill_(-7)
        llm_capi.check(lib.i8_gemm_tune_sk(nt, waves, mrows, ks, xcd, Ap.data_ptr(), Wp.data_ptr(),
                                           part.data_ptr(), M, N, K, None), lib)
        got = part[:ks].to(torch.int64).sum(0).cpu().numpy()
        np.testing.assert_array_equal(got, ref, err_msg=str((nt, waves, mrows, ks, xcd)))


@pytest.mark.parametrize("M,K,N", [(16, 768, 2304), (64, 2048, 512), (3, 96, 48), (80, 256, 64),
                                   (512, 768, 2304), (300, 256, 64)])
def test_f16_gemm(gpu, M, K, N):
    import llm_capi
    rng = np.random.default_rng(K + N)
    A = rng.standard_normal((M, K)).astype(np.float16)
    W = (0.05 * rng.standard_normal((K, N))).astype(np.float16)
    bias = rng.standard_normal(N).astype(np.float32)
    Wp = llm_capi.pack_weights(_dev(W), llm_capi.LLM_F16)
    for act in (0, 1, 2):
        C = llm_capi.f16_gemm(_dev(A), Wp, N, bias=_dev(bias), act=act).cpu().numpy()
        ref = A.astype(np.float64) @ W.astype(np.float64) + bias
        if act == 1:
            ref = np.maximum(ref, 0)
        elif act == 2:
            from scipy.special import erf
            ref = 0.5 * ref * (1 + erf(ref / np.sqrt(2)))
        assert rel_err(C, ref) < 1e-3


@pytest.mark.parametrize("M,V,K", [(64, 50257, 2048), (1, 1000, 256), (16, 50257, 768), (70, 333, 64),
                                   (17, 4099, 512), (32, 50257, 2048), (24, 257, 128)])
def test_lm_head(gpu, M, V, K):
    import llm_capi
    rng = np.random.default_rng(V + K)
    x = rng.standard_normal((M, K)).astype(np.float32)
    E = rng.standard_normal((V, K)).astype(np.float16)
    out = llm_capi.lm_head(_dev(x), _dev(E)).cpu().numpy()
    ref = x.astype(np.float64) @ E.astype(np.float64).T
    assert rel_err(out, ref) < 2e-6


def test_argmax_first_wins(gpu):
    import llm_capi
    rng = np.random.default_rng(0)
    L = rng.standard_normal((9, 50257)).astype(np.float32)
    L[1, 10] = L[1, 20] = 100.0  # tie: first index wins
    L[2, :] = 0.0
    L[3, 50256] = 1e9
    out = llm_capi.argmax_rows(_dev(L)).cpu().numpy()
    np.testing.assert_array_equal(out, np.argmax(L, axis=1))
    assert out[1] == 10 and out[2] == 0


def test_quantize_rows_exact(gpu, oracle):
    import llm_capi
    rng = np.random.default_rng(2)
    x = (rng.standard_normal((33, 2048)) * 3).astype(np.float32)
    x[0] = 0.0
    x[1, :4] = [0.5, -0.5, 1.5, 127.0]
    q, s = llm_capi.quantize_rows(_dev(x))
    qr, sr = oracle.quantize_rows(x)
    np.testing.assert_array_equal(q.cpu().numpy(), qr)
    np.testing.assert_array_equal(s.cpu().numpy(), sr)


def test_layernorm_quant(gpu, oracle):
    import llm_capi
    rng = np.random.default_rng(4)
    x = (rng.standard_normal((20, 2048)) * 2 + 0.5).astype(np.float32)
    g = (1 + 0.1 * rng.standard_normal(2048)).astype(np.float32)
    b = (0.1 * rng.standard_normal(2048)).astype(np.float32)
    out, q, s = llm_capi.layernorm_quant(_dev(x), _dev(g), _dev(b))
    ref = oracle.layer_norm(x, g, b)
    np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=1e-5, atol=1e-5)
    qr, sr = oracle.quantize_rows(ref)
    dq = np.abs(q.cpu().numpy().astype(np.int32) - qr.astype(np.int32))
    assert dq.max() <= 1 and (dq > 0).mean() < 1e-3
    np.testing.assert_allclose(s.cpu().numpy(), sr, rtol=1e-5)


@pytest.mark.parametrize("V", [1000, 50257])
@pytest.mark.parametrize("T,k,p", [(0.0, 0, 1.0), (1.0, 1, 1.0), (1.0, 0, 1.0), (0.7, 50, 1.0),
                                   (1.2, 0, 0.9), (1.0, 20, 0.8), (0.5, 0, 0.5)])
def test_sample_rows_vs_oracle(gpu, oracle, V, T, k, p):
    """Device sampling (temperature / top-k / top-p) against
    the oracle's restatement with the same counter-based draw: same token per
    row, except where the draw lands within 1e-4 of a CDF boundary."""
    import llm_capi
    from oracle.oracle import sample_rows, sample_uniform
    lib = llm_capi.load()
    assert abs(lib.sample_uniform_host(7, 3, 11) - sample_uniform(7, 3, 11)) == 0.0
    rng = np.random.default_rng(V + int(T * 10) + k)
    logits = (rng.standard_normal((6, V)) * 3).astype(np.float32)
    for counter in (0, 1, 17):
        got = llm_capi.sample_rows(_dev(logits), T, k, p, seed=5, counter=counter).cpu().numpy()
        ref, margin = sample_rows(logits, T, k, p, seed=5, counter=counter)
        ok = (got == ref) | (margin < 1e-4)
        assert ok.all(), (counter, got, ref, margin)
        if T > 0 and k > 1:  # the token is within the top-k
            for r in range(6):
                assert logits[r, got[r]] >= np.sort(logits[r])[-k]


def test_sample_rows_distribution(gpu):
    """Frequencies of 4000 draws (counters 0..3999) of an 8-token distribution
    match softmax(logits / T) within 5 sigma; top-k keeps only the top tokens."""
    import torch
    import llm_capi
    logits = np.array([[2.0, 1.0, 0.5, 0.0, -0.5, -1.0, 1.5, 0.2]], np.float32)
    T = 0.9
    pr = np.exp(logits[0] / T - (logits[0] / T).max())
    pr /= pr.sum()
    d = _dev(logits)
    n = 4000
    toks = torch.stack([llm_capi.sample_rows(d, T, 0, 1.0, seed=123, counter=c) for c in range(n)])
    cnt = np.bincount(toks.cpu().numpy().ravel(), minlength=8)
    sigma = np.sqrt(n * pr * (1 - pr))
    assert np.all(np.abs(cnt - n * pr) < 5 * sigma + 1), (cnt, n * pr)
    tk = torch.stack([llm_capi.sample_rows(d, T, 3, 1.0, seed=9, counter=c) for c in range(300)])
    assert set(tk.cpu().numpy().ravel().tolist()) <= {0, 6, 1}


@pytest.mark.parametrize("batch,M,N,K", [
    (1, 1, 1, 1), (1, 64, 64, 64), (3, 17, 33, 70), (2, 130, 70, 200), (1, 5, 1000, 2048),
    (4, 64, 256, 4096),
])
@pytest.mark.parametrize("activation", ["", "relu", "gelu"])
def test_dnnl_matmul_int8_s8_batch(gpu, batch, M, N, K, activation):
    """i8_matmul_s8 (the s8-output, BATCH form of dnnl_matmul_int8,
    attention_cpu/dnnl_matmul_int8.cpp:7-75) vs the oracle restatement: exact
    int8 outputs; for gelu only values within 1e-3 of a .5 rounding boundary may
    differ, by one (erff vs the oracle's rounded float64 erf)."""
    import torch
    import llm_capi
    from oracle.oracle import dnnl_matmul_int8_np
    rng = np.random.default_rng(batch * 1000 + M + N + K)
    A = rng.integers(-128, 128, (batch, M, K), dtype=np.int8)
    B = rng.integers(-128, 128, (batch, K, N), dtype=np.int8)
    bias = (rng.standard_normal(N) * 500).astype(np.float32)
    # output scale sized so the results straddle the int8 range
    sA, sB = 0.02, 0.05
    sC = float(sA * sB * 128 * 128 * np.sqrt(K) / 180)
    for b in (None, bias):
        want, y = dnnl_matmul_int8_np(A, B, sA, sB, sC, b, activation)
        C = torch.zeros((batch, M, N), dtype=torch.int8, device="cuda")
        ok = llm_capi.dnnl_matmul_int8(_dev(A), _dev(B), C, batch, M, N, K, sA, sB, sC,
                                       None if b is None else _dev(b), activation)
        assert ok
        got = C.cpu().numpy()
        if activation == "gelu":
            tie = np.abs(np.abs(y - np.trunc(y)) - 0.5) < 1e-3
            assert np.all(np.abs(got.astype(int) - want.astype(int)) <= tie.astype(int))
        else:
            np.testing.assert_array_equal(got, want)
        assert (got == 127).any() or (got == -128).any() or M * N < 64  # saturation exercised


def test_dnnl_matmul_int8_refusals(gpu):
    """False on a bad call, as the reference's catch (...) (dnnl_matmul_int8.cpp:73-74),
    through both the ctypes mirror and the pybind module; C untouched."""
    import torch
    import llm_capi
    import llm_decoder
    A = torch.ones((1, 4, 8), dtype=torch.int8, device="cuda")
    B = torch.ones((1, 8, 4), dtype=torch.int8, device="cuda")
    C = torch.full((1, 4, 4), 7, dtype=torch.int8, device="cuda")
    assert not llm_capi.dnnl_matmul_int8(A, B, C, 1, 4, 4, 8, 1.0, 1.0, 0.0)  # scaleC 0
    assert not llm_capi.dnnl_matmul_int8(A, B, C, 1, 4, 4, 200000, 1.0, 1.0)  # K too large
    assert not llm_capi.dnnl_matmul_int8(A.float(), B, C, 1, 4, 4, 8, 1.0, 1.0)
    assert (C == 7).all()
    assert llm_decoder.dnnl_matmul_int8(A.data_ptr(), B.data_ptr(), C.data_ptr(), 1, 4, 4, 8,
                                        1.0, 1.0, 2.0, 0, "relu")
    torch.cuda.synchronize()
    assert (C == 4).all()  # 8 / 2
    assert not llm_decoder.dnnl_matmul_int8(A.data_ptr(), B.data_ptr(), C.data_ptr(), 1, 4, 4, 8,
                                            1.0, 1.0, 0.0)
