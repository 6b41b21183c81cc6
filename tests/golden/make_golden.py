"""Regenerate the committed golden fixtures in tests/golden/*.npz.

Container-only (needs /root/reference): builds oracle/_ref/gen_golden from the
reference's own compilable sources (oracle/ref_golden/Makefile) and runs it on
seeded inputs.  Each fixture holds the inputs AND the reference outputs; the
reference source itself never enters the repository.

    python tests/golden/make_golden.py            # every fixture
    python tests/golden/make_golden.py kvtiles    # only the KV record files
"""
from __future__ import annotations

import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
GOLDEN = Path(__file__).resolve().parent
GEN = ROOT / "oracle" / "_ref" / "gen_golden"


def build_generator():
    subprocess.run(["make", "-s", "-C", str(ROOT / "oracle" / "ref_golden")], check=True)


def run(*args):
    subprocess.run([str(GEN), *map(str, args)], check=True)


def attn_case(name, *, B, H, D, T, ts, beams=None, beam_ids=None, temperature=1.0, top_k=0,
              top_p=1.0, eos=-1, eos_thr=0.0, missing=(), seed=0):
    rng = np.random.default_rng(seed)
    beams = beams or B
    nt = (T + ts - 1) // ts
    scale = D ** -0.25
    q = (rng.standard_normal((B, H, D)) * scale).astype(np.float32)
    # K/V are fp16-representable so the same fixture drives the fp16 HIP path.
    k = (rng.standard_normal((beams, H, nt, ts, D)) * scale).astype(np.float16)
    v = rng.standard_normal((beams, H, nt, ts, D)).astype(np.float16)
    present = np.ones((beams, H, nt), np.int32)
    for (r, h, t) in missing:
        present[r, h, t] = 0
    with tempfile.TemporaryDirectory() as d:
        d = Path(d)
        q.tofile(d / "q.f32")
        k.astype(np.float32).tofile(d / "k.f32")
        v.astype(np.float32).tofile(d / "v.f32")
        present.tofile(d / "present.i32")
        has_bi = beam_ids is not None
        if has_bi:
            np.asarray(beam_ids, np.int32).tofile(d / "beam_ids.i32")
        run("attn", d, B, H, D, T, ts, beams, repr(float(temperature)), top_k, repr(float(top_p)),
            eos, repr(float(eos_thr)), int(has_bi))
        out = np.fromfile(d / "out.f32", np.float32).reshape(B, H, D)
        probs = np.fromfile(d / "probs.f32", np.float32).reshape(B, H, T)
        scores = np.fromfile(d / "scores.f32", np.float32).reshape(B, H, T)
    np.savez_compressed(
        GOLDEN / f"attn_{name}.npz", q=q, k=k, v=v, present=present,
        beam_ids=np.asarray(beam_ids if has_bi else [], np.int32),
        params=np.array([B, H, D, T, ts, beams, top_k, eos], np.int32),
        fparams=np.array([temperature, top_p, eos_thr], np.float32),
        out=out, probs=probs, scores=scores)


def softmax_case(name, length, temperature, seed):
    rng = np.random.default_rng(seed)
    s = (rng.standard_normal(length) * 3).astype(np.float32)
    s[::7] = -1e9  # masked entries as the attention kernel writes them
    with tempfile.TemporaryDirectory() as d:
        d = Path(d)
        s.tofile(d / "scores.f32")
        run("softmax", d, length, repr(float(temperature)))
        out = np.fromfile(d / "out.f32", np.float32)
    np.savez_compressed(GOLDEN / f"softmax_{name}.npz", scores=s,
                        temperature=np.float32(temperature), out=out)


def quant_case(name, n, rows, seed):
    rng = np.random.default_rng(seed)
    x = (rng.standard_normal(n) * 2.5).astype(np.float32)
    # exact half-way products and zeros / extremes
    x[:8] = np.array([0.0, 0.5, -0.5, 1.5, -2.5, 3.0, -3.0, 0.0], np.float32)
    x[8:12] = 0.0
    with tempfile.TemporaryDirectory() as d:
        d = Path(d)
        x.tofile(d / "x.f32")
        run("quant", d, n, rows)
        res = dict(
            x=x, rows=np.int32(rows),
            scale=np.fromfile(d / "scale.f32", np.float32)[0],
            absmax=np.fromfile(d / "absmax.f32", np.float32)[0],
            q=np.fromfile(d / "q.i8", np.int8), dq=np.fromfile(d / "dq.f32", np.float32),
            row_scales=np.fromfile(d / "row_scales.f32", np.float32),
            qr=np.fromfile(d / "qr.i8", np.int8), dqr=np.fromfile(d / "dqr.f32", np.float32))
    np.savez_compressed(GOLDEN / f"quant_{name}.npz", **res)


def ln_case(name, rows, cols, seed):
    rng = np.random.default_rng(seed)
    x = (rng.standard_normal((rows, cols)) * 1.7 + 0.3).astype(np.float32)
    gamma = (1 + 0.1 * rng.standard_normal(cols)).astype(np.float32)
    beta = (0.1 * rng.standard_normal(cols)).astype(np.float32)
    with tempfile.TemporaryDirectory() as d:
        d = Path(d)
        x.tofile(d / "x.f32")
        np.concatenate([gamma, beta]).tofile(d / "gamma_beta.f32")
        run("ln", d, rows, cols)
        out = np.fromfile(d / "out.f32", np.float32).reshape(rows, cols)
    np.savez_compressed(GOLDEN / f"layernorm_{name}.npz", x=x, gamma=gamma, beta=beta, out=out)


def mlp_case(name, rows, hid, inter, seed):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((rows, hid)).astype(np.float32)
    w1 = (0.05 * rng.standard_normal((hid, inter))).astype(np.float32)
    b1 = (0.05 * rng.standard_normal(inter)).astype(np.float32)
    w2 = (0.05 * rng.standard_normal((inter, hid))).astype(np.float32)
    b2 = (0.05 * rng.standard_normal(hid)).astype(np.float32)
    with tempfile.TemporaryDirectory() as d:
        d = Path(d)
        x.tofile(d / "x.f32")
        np.concatenate([w1.ravel(), b1, w2.ravel(), b2]).tofile(d / "mlp.f32")
        run("mlp", d, rows, hid, inter)
        out = np.fromfile(d / "out.f32", np.float32).reshape(rows, hid)
    np.savez_compressed(GOLDEN / f"mlp_{name}.npz", x=x, w1=w1, b1=b1, w2=w2, b2=b2, out=out)


def embed_case(name, vocab, hid, n, seed):
    rng = np.random.default_rng(seed)
    emb = rng.standard_normal((vocab, hid)).astype(np.float32)
    ids = rng.integers(0, vocab, n).astype(np.int32)
    with tempfile.TemporaryDirectory() as d:
        d = Path(d)
        emb.tofile(d / "emb.f32")
        ids.tofile(d / "ids.i32")
        run("embed", d, vocab, hid, n)
        out = np.fromfile(d / "out.f32", np.float32).reshape(n, hid)
    np.savez_compressed(GOLDEN / f"embed_{name}.npz", emb=emb, ids=ids, out=out)


def kvtiles_case(name, *, ts, D, dtype, idx, seed):
    """KVTileCacheCPU<T>::save / load (kv_cache/kv_tile_cache_cpu.cpp:89-123): the
    reference writes the record file for these tiles, then reads it back."""
    rng = np.random.default_rng(seed)
    idx = np.asarray(idx, np.int32).reshape(-1, 3)
    n, te = len(idx), ts * D
    if dtype == np.int8:
        data = rng.integers(-128, 128, (n, ts, D)).astype(np.int8)
    else:
        data = rng.standard_normal((n, ts, D)).astype(dtype)
    es = data.dtype.itemsize
    with tempfile.TemporaryDirectory() as d:
        d = Path(d)
        idx.tofile(d / "idx.i32")
        data.tofile(d / "data.bin")
        run("kvtiles", d, n, te, es)
        file_bytes = np.fromfile(d / "tiles.bin", np.uint8)
        back = np.fromfile(d / "back.bin", data.dtype).reshape(n, ts, D)
    np.savez_compressed(GOLDEN / f"kvtiles_{name}.npz", idx=idx, data=data, ts=np.int32(ts),
                        D=np.int32(D), file_bytes=file_bytes, back=back)


def kvtiles_cases():
    # fp16 pools are KVTileCacheCPU<uint16_t> (kv_tile_cache_cpu.cpp:138); a
    # beam/head/tile spread with gaps, a repeated beam and tile 0.
    kvtiles_case("f16_ts16_d64", ts=16, D=64, dtype=np.float16, seed=70,
                 idx=[(0, 0, 0), (0, 0, 1), (0, 1, 0), (1, 0, 3), (2, 1, 2), (1, 1, 0)])
    kvtiles_case("f32_ts16_d32", ts=16, D=32, dtype=np.float32, seed=71,
                 idx=[(0, 1, 1), (1, 0, 0), (0, 0, 2), (1, 1, 1)])
    kvtiles_case("i8_ts32_d64", ts=32, D=64, dtype=np.int8, seed=72,
                 idx=[(0, 0, 0), (1, 1, 1), (0, 1, 0)])


def main():
    if not Path("/root/reference").exists():
        sys.exit("make_golden.py needs /root/reference (build container only)")
    build_generator()
    if sys.argv[1:] == ["kvtiles"]:  # only the KV record-file fixtures
        kvtiles_cases()
        return
    # C1 attention shapes (B1/H4/D64/T128/ts16) and the edge cases the
    # reference's code paths have: missing tiles, beam routing, temperature,
    # top-k / top-p / EOS filters, ragged last tile, other tile sizes, D=128.
    attn_case("c1_base", B=1, H=4, D=64, T=128, ts=16, seed=1)
    attn_case("c1_missing", B=1, H=4, D=64, T=128, ts=16, seed=2,
              missing=[(0, 0, 3), (0, 2, 0), (0, 3, 7)])
    attn_case("beam_route", B=4, H=2, D=64, T=64, ts=16, beams=2, beam_ids=[1, 0, 1, 0], seed=3)
    attn_case("temp07", B=2, H=2, D=64, T=64, ts=16, temperature=0.7, seed=4)
    attn_case("topk5", B=1, H=2, D=64, T=64, ts=16, top_k=5, seed=5)
    attn_case("topp09", B=1, H=2, D=64, T=64, ts=16, top_p=0.9, seed=6)
    attn_case("eos", B=1, H=2, D=64, T=64, ts=16, eos=3, eos_thr=0.001, seed=7)
    attn_case("d128", B=2, H=2, D=128, T=96, ts=16, seed=8)
    attn_case("ragged_tail", B=2, H=3, D=64, T=120, ts=16, seed=9)
    attn_case("ts32", B=2, H=2, D=64, T=128, ts=32, seed=10)
    attn_case("all_missing", B=1, H=1, D=64, T=32, ts=16, seed=11, missing=[(0, 0, 0), (0, 0, 1)])
    softmax_case("t1", 128, 1.0, 20)
    softmax_case("t05", 64, 0.5, 21)
    quant_case("v1024", 1024, 4, 30)
    ln_case("r3c256", 3, 256, 40)
    mlp_case("r2h64", 2, 64, 256, 50)
    embed_case("v50", 50, 16, 7, 60)
    kvtiles_cases()
    print("golden fixtures written to", GOLDEN)


if __name__ == "__main__":
    main()
