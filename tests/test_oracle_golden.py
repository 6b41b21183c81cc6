"""Pin the CPU oracle against the golden vectors produced by the reference's own
compilable sources (tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest

from _util import GOLDEN, load_attn_fixture, rel_err, tiles_to_pool
from oracle.oracle import quantize_rows_np

ATTN_CASES = sorted(p.stem[len("attn_"):] for p in GOLDEN.glob("attn_*.npz"))


@pytest.mark.parametrize("name", ATTN_CASES)
def test_oracle_attention_matches_reference(oracle, name):
    f = load_attn_fixture(name)
    k_pool, v_pool, pt = tiles_to_pool(f["k"], f["v"], f["present"])
    out, probs, scores = oracle.paged_attention(
        f["q"], k_pool.astype(np.float32), v_pool.astype(np.float32), pt, T=f["T"],
        beam_ids=f["beam_ids"], temperature=f["temperature"], top_k=f["top_k"],
        top_p=f["top_p"], eos_token=f["eos"], eos_threshold=f["eos_thr"], want_probs=True)
    # Same float operations in the same order as the reference loop: bit-exact
    # scores; probabilities / outputs within float rounding of exp().
    np.testing.assert_array_equal(scores, f["scores"])
    np.testing.assert_allclose(probs, f["probs"], rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(out, f["out"], rtol=1e-5, atol=1e-6)


def test_oracle_attention_independent_float64(oracle):
    """Cross-check against an independent float64 numpy attention."""
    f = load_attn_fixture("c1_base")
    k = f["k"].astype(np.float64)
    v = f["v"].astype(np.float64)
    q = f["q"].astype(np.float64)
    T, ts = f["T"], f["ts"]
    kk = k.reshape(1, f["H"], -1, f["D"])[:, :, :T]
    vv = v.reshape(1, f["H"], -1, f["D"])[:, :, :T]
    s = np.einsum("bhd,bhtd->bht", q, kk)
    p = np.exp(s - s.max(-1, keepdims=True))
    p /= p.sum(-1, keepdims=True) + 1e-6
    ref = np.einsum("bht,bhtd->bhd", p, vv)
    k_pool, v_pool, pt = tiles_to_pool(f["k"], f["v"], f["present"])
    out = oracle.paged_attention(f["q"], k_pool.astype(np.float32), v_pool.astype(np.float32),
                                 pt, T=T)
    assert rel_err(out, ref) < 1e-5


def test_oracle_page_lookup(oracle):
    import ctypes
    pt = np.arange(2 * 3 * 4, dtype=np.int32).reshape(2, 3, 4)
    p = pt.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
    for b in range(2):
        for h in range(3):
            for t in range(4):
                assert oracle.lib.oracle_page_lookup(p, 2, 3, 4, b, h, t) == b * 12 + h * 4 + t
    assert oracle.lib.oracle_page_lookup(p, 2, 3, 4, 2, 0, 0) == -1
    assert oracle.lib.oracle_page_lookup(p, 2, 3, 4, 0, 0, -1) == -1


@pytest.mark.parametrize("name", ["t1", "t05"])
def test_oracle_softmax_matches_reference(oracle, name):
    z = np.load(GOLDEN / f"softmax_{name}.npz")
    # softmax is exercised through attention; re-derive via the T-length path
    s = z["scores"]
    t = float(z["temperature"])
    m = max(-1e9, float(s.max()))
    e = np.exp(((s - np.float32(m)) / np.float32(t)).astype(np.float32))
    ref = z["out"]
    np.testing.assert_allclose(e / (e.sum() + 1e-6), ref, rtol=2e-6, atol=1e-12)


def test_oracle_quantizer_matches_reference(oracle):
    z = np.load(GOLDEN / "quant_v1024.npz")
    x = z["x"]
    rows = int(z["rows"])
    scale = oracle.lib.oracle_minmax_scale(
        x.ctypes.data_as(__import__("ctypes").POINTER(__import__("ctypes").c_float)), x.size)
    assert np.float32(scale) == z["scale"]
    q, inv = oracle.quantize_rows(x.reshape(1, -1))
    np.testing.assert_array_equal(q.ravel(), z["q"])
    np.testing.assert_array_equal(np.float32(1.0) / inv, np.float32(1.0) / (np.float32(1.0) / z["scale"]))
    qr, invr = oracle.quantize_rows(x.reshape(rows, -1))
    np.testing.assert_array_equal(qr.ravel(), z["qr"])
    # numpy mirror agrees bit-exactly too
    qn, _ = quantize_rows_np(x.reshape(rows, -1))
    np.testing.assert_array_equal(qn.ravel(), z["qr"])
    # dequant = q / scale (int8_quant.cpp:38-44)
    np.testing.assert_array_equal(z["q"].astype(np.float32) / z["scale"], z["dq"])


def test_oracle_layernorm_matches_reference(oracle):
    z = np.load(GOLDEN / "layernorm_r3c256.npz")
    out = oracle.layer_norm(z["x"], z["gamma"], z["beta"])
    np.testing.assert_array_equal(out, z["out"])


def test_oracle_mlp_matches_reference(oracle):
    z = np.load(GOLDEN / "mlp_r2h64.npz")
    out = oracle.mlp_f32(z["x"], z["w1"], z["b1"], z["w2"], z["b2"])
    np.testing.assert_array_equal(out, z["out"])


def test_oracle_i8_gemm_exact_int32(oracle):
    """int32 accumulators are exact: cross-check with torch._int_mm (CPU)."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(0)
    for (M, K, N) in [(64, 256, 1024), (64, 1024, 256), (17, 128, 48)]:
        A = rng.integers(-128, 128, (M, K), dtype=np.int8)
        W = rng.integers(-128, 128, (K, N), dtype=np.int8)
        acc, _ = oracle.i8_gemm(A, W)
        ref = (A.astype(np.int64) @ W.astype(np.int64)).astype(np.int32)
        np.testing.assert_array_equal(acc, ref)
        if M >= 17 and K % 8 == 0 and N % 8 == 0:
            try:
                t = torch._int_mm(torch.from_numpy(A), torch.from_numpy(W)).numpy()
                np.testing.assert_array_equal(acc, t)
            except RuntimeError:
                pass


def test_oracle_i8_gemm_epilogue(oracle):
    rng = np.random.default_rng(1)
    M, K, N = 8, 128, 64
    A = rng.integers(-128, 128, (M, K), dtype=np.int8)
    W = rng.integers(-128, 128, (K, N), dtype=np.int8)
    sa = rng.uniform(0.001, 0.01, M).astype(np.float32)
    sw = rng.uniform(0.001, 0.01, N).astype(np.float32)
    bias = rng.standard_normal(N).astype(np.float32)
    acc, C0 = oracle.i8_gemm(A, W, sa, sw, bias, act=0)
    ref = acc.astype(np.float32) * (sa[:, None] * sw[None, :]) + bias
    np.testing.assert_array_equal(C0, ref.astype(np.float32))
    _, C1 = oracle.i8_gemm(A, W, sa, sw, bias, act=1)
    np.testing.assert_array_equal(C1, np.maximum(ref, 0))
    _, C2 = oracle.i8_gemm(A, W, sa, sw, bias, act=2)
    from math import erf
    g = np.array([0.5 * y * (1 + erf(y / np.sqrt(2))) for y in ref.ravel()]).reshape(ref.shape)
    np.testing.assert_allclose(C2, g, rtol=1e-5, atol=1e-5)


def test_oracle_dnnl_matmul_int8_known_answers():
    """dnnl_matmul_int8 restatement (s8 output, BATCH): hand-computed values for
    the bias-then-scale order, round half to even, saturation and the post-ops;
    batches are independent.  Parity unpinned against oneDNN (absent here)."""
    from oracle.oracle import dnnl_matmul_int8_np
    A = np.array([[[1, 2], [-3, 1]], [[100, 100], [-100, 100]]], np.int8)  # [2][2][2]
    B = np.array([[[3, 0], [4, 1]], [[127, -128], [127, 0]]], np.int8)     # [2][2][2]
    # batch 0 acc = [[11, 2], [-5, 1]]; bias [0.5, -0.5]; alpha = 1 * 2 / 4
    C, _ = dnnl_matmul_int8_np(A, B, 1.0, 2.0, 4.0, np.array([0.5, -0.5], np.float32))
    # (11.5) * 0.5 = 5.75 -> 6; (1.5) * .5 = .75 -> 1; (-4.5) * .5 = -2.25 -> -2; (.5) * .5 -> 0
    np.testing.assert_array_equal(C[0], [[6, 1], [-2, 0]])
    # batch 1 acc = [[25400, -12800], [0, 12800]]: saturates; (0 + .5) * .5 -> 0
    np.testing.assert_array_equal(C[1], [[127, -128], [0, 127]])
    C, _ = dnnl_matmul_int8_np(A[:1], B[:1], 1.0, 1.0, 2.0)   # halves: 5.5 -> 6 (even), 1 -> 1, -2.5 -> -2, .5 -> 0
    np.testing.assert_array_equal(C[0], [[6, 1], [-2, 0]])
    C, _ = dnnl_matmul_int8_np(A[:1], B[:1], 1.0, 1.0, 1.0, activation="relu")
    np.testing.assert_array_equal(C[0], [[11, 2], [0, 1]])
    C, _ = dnnl_matmul_int8_np(A[:1], B[:1], 1.0, 1.0, 1.0, activation="gelu")
    from math import erf
    g = lambda x: 0.5 * x * (1 + erf(x / np.sqrt(2)))
    np.testing.assert_array_equal(C[0], np.rint([[g(11), g(2)], [g(-5), g(1)]]).astype(np.int8))


def test_oracle_embedding_matches_reference():
    z = np.load(GOLDEN / "embed_v50.npz")
    np.testing.assert_array_equal(z["emb"][z["ids"]], z["out"])


def test_oracle_decoder_step_consistent(oracle):
    """The restated INT8Decoder step, recomputed layer by layer from the
    pinned pieces (LN, quantiser, int32 GEMM, attention) in numpy."""
    from oracle.oracle import OracleDecoder, synthetic_int8_model
    L, H, D, V, S = 2, 4, 64, 512, 32
    w = synthetic_int8_model(oracle, L=L, H=H, D=D, V=V, max_seq=S, seed=3)
    B = 2
    dec = OracleDecoder(oracle, w, B)
    toks = [np.array([5, 9], np.int32), np.array([7, 1], np.int32)]
    for p in range(2):
        x, logits, nxt = dec.step(toks[p], np.array([p, p], np.int32))
    # numpy recompute of the last step (position 1) with the KV the oracle kept
    hid = H * D
    xx = w["emb"][toks[1]].astype(np.float32)
    for l in range(L):
        a = oracle.layer_norm(xx, w["ln1_g"][l], w["ln1_b"][l])
        qa, sa = oracle.quantize_rows(a)
        _, qkv = oracle.i8_gemm(qa, w["wqkv"][l], sa, w["sw_qkv"][l])
        kc = dec.kv(l, 0)[:, :, :2].astype(np.float32)
        vc = dec.kv(l, 1)[:, :, :2].astype(np.float32)
        np.testing.assert_array_equal(dec.kv(l, 0)[:, :, 1].reshape(B, hid),
                                      qkv[:, hid:2 * hid].astype(np.float16))
        q = qkv[:, :hid].reshape(B, H, D)
        s = np.einsum("bhd,bhtd->bht", q.astype(np.float64), kc)
        pr = np.exp(s - s.max(-1, keepdims=True))
        pr /= pr.sum(-1, keepdims=True) + 1e-6
        o = np.einsum("bht,bhtd->bhd", pr, vc).reshape(B, hid).astype(np.float32)
        qo, so = oracle.quantize_rows(o)
        _, xx = oracle.i8_gemm(qo, w["wo"][l], so, w["sw_o"][l])
        a2 = oracle.layer_norm(xx, w["ln2_g"][l], w["ln2_b"][l])
        q2, s2 = oracle.quantize_rows(a2)
        _, h1 = oracle.i8_gemm(q2, w["w1"][l], s2, w["sw1"][l], w["b1"][l], act=1)
        q3, s3 = oracle.quantize_rows(h1)
        _, xx = oracle.i8_gemm(q3, w["w2"][l], s3, w["sw2"][l], w["b2"][l])
    assert rel_err(x, xx) < 1e-4
    ref_logits = xx.astype(np.float64) @ w["emb"].astype(np.float64).T
    assert rel_err(logits, ref_logits) < 1e-4
    np.testing.assert_array_equal(nxt, np.argmax(logits, axis=1))


def test_oracle_under_address_sanitizer():
    """The checker itself is memory-clean: oracle.cpp built with
    -fsanitize=address,undefined and driven over ragged shapes, missing and
    out-of-pool pages, filters and the (teacher-forced) decoder step
    (oracle/asan_check.cpp, `make -C oracle asan`)."""
    import shutil
    import subprocess
    from pathlib import Path
    if shutil.which("g++") is None:
        pytest.skip("no host compiler")
    root = Path(__file__).resolve().parents[1]
    r = subprocess.run(["make", "-s", "-C", str(root / "oracle"), "asan"], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0 and "asan_check: ok" in r.stdout, r.stdout + r.stderr
