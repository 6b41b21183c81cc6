"""Per-wave timeline of the C4 beam-group attention launch (tuning build).

Run with the tuning library in front of the product one, e.g.
  LD_LIBRARY_PATH=$PWD/ab_tune python scripts/beam_stamps.py [--layers 1]
It builds bench.py's C4 state (begin_beams: 8 sequences x 4 beams, 3840
shared + 256 private tokens, shuffled pages), times the decoder's own
attention launch of layer 0, then launches it once with LLM_BEAM_STAMPS=1
(pa_split_kernel STAMPS: s_memrealtime at entry, first KV load, end of the
shared-prefix chunks, exit, and HW_ID per wave) and prints where the launch's
time goes: the dispatch ramp, the start-up before the first KV load, the
shared and private phases, and the tail of the last waves.
"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "pagedattention-based-transformer-decoder-inference-framework_amd"))


def pct(x, qs=(0, 10, 50, 90, 99, 100)):
    return " ".join(f"p{q}={np.percentile(x, q):7.2f}" for q in qs)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=1)
    ap.add_argument("--config", default="c4")
    ap.add_argument("--tag", default="", help="suffix of the saved .npy")
    args = ap.parse_args()
    import torch
    import bench
    import llm_decoder
    torch.cuda.set_device(0)
    torch.cuda.set_stream(torch.cuda.Stream())
    cfg = dict(bench.CONFIGS[args.config])
    cfg["L"] = args.layers
    T, B = cfg["T"], cfg["B"]
    hid = cfg["H"] * cfg["D"]
    dec = getattr(llm_decoder, cfg["cls"])(cfg["L"], cfg["H"], cfg["D"], hid, cfg["V"], T + 16,
                                            max_batch=B, page_size=cfg["ts"])
    dec.set_weights(bench.make_weights(cfg, 1234))
    dec.begin_beams(cfg["seqs"], cfg["beams"], cfg["shared"], T - cfg["shared"], 1234, True)
    us = bench.time_attention(dec, cfg["L"], iters=20) * 1e6
    ns, form = dec.attention_plan()
    print(f"{args.config} attention launch (split + merge) {us:.2f} us, {ns} splits, form {form}")

    lib_path = None
    with open("/proc/self/maps") as f:
        for line in f:
            if line.rstrip().endswith("libllm_decoder_hip.so"):
                lib_path = line.split()[-1]
                break
    lib = ctypes.CDLL(lib_path)
    if not hasattr(lib, "pa_tune_stamps"):
        raise SystemExit(f"{lib_path} is not the tuning build (no pa_tune_stamps)")
    lib.pa_tune_stamps.argtypes = [ctypes.c_void_p, ctypes.c_longlong]
    lib.pa_tune_stamps.restype = ctypes.c_longlong
    st = torch.cuda.current_stream().cuda_stream
    os.environ["LLM_BEAM_STAMPS"] = "1"
    for _ in range(3):  # the last one is recorded
        dec.run_attention(0, st)
    torch.cuda.synchronize()
    os.environ.pop("LLM_BEAM_STAMPS")
    if form & 64:  # the steal form: 8 stamps per wave
        steal_report(lib, args)
        return
    buf = np.zeros((1 << 16, 5), np.uint64)
    n = lib.pa_tune_stamps(buf.ctypes.data, buf.shape[0])
    if n <= 0:
        raise SystemExit("no stamps recorded (not a beam launch?)")
    s = buf[:n]
    live = s[:, 3] > 0
    wid = np.nonzero(live)[0]
    s = s[live].astype(np.int64)
    t0 = s[:, 0].min()
    ent, ld, sh, ex = [(s[:, i] - t0) / 100.0 for i in range(4)]  # 100 MHz -> us
    hw = s[:, 4]
    xcc = (hw >> 32) & 0xF
    cu = (hw >> 8) & 0xF
    se = (hw >> 13) & 0x7
    print(f"waves recorded {len(s)} of {n} (the rest held no pages); kernel span {ex.max():.2f} us")
    print("entry      ", pct(ent))
    print("first load ", pct(ld))
    print("start-up   ", pct(ld - ent))
    print("shared     ", pct(sh - ld))
    print("private    ", pct(ex - sh))
    print("exit       ", pct(ex))
    print("wave life  ", pct(ex - ent))
    # streaming waves over time (how many are between first load and exit)
    grid = np.arange(0, ex.max() + 1, 1.0)
    active = [(np.sum((ld <= t) & (ex > t))) for t in grid]
    print("waves streaming per us:", " ".join(str(a) for a in active))
    print("waves per XCC:", np.bincount(xcc, minlength=8).tolist())
    print("exit p90 per XCC:", [round(float(np.percentile(ex[xcc == x], 90)), 2)
                                for x in range(8) if np.any(xcc == x)])
    # where the late waves are: by split, head, sequence (the grid's
    # decomposition: wid = blk * 4 + beam, blk split-major unless LLM_BEAM_SMAJ=0), and
    # by how many waves their CU held
    H = cfg["H"]
    blk = wid // 4
    if os.environ.get("LLM_BEAM_SMAJ", "1") != "0":  # split-major order (PaSplitArgs::smaj): blk = split * GH + seq * H + head
        GH = ((B + 3) // 4) * H
        split, rest = blk // GH, blk % GH
    else:
        split, rest = blk % ns, blk // ns
    head, seq = rest % H, rest // H
    nblk = ((B + 3) // 4) * H * ns
    slot = blk * 4 // nblk  # dispatch slot: the CU's 1st..4th resident workgroup
    for name, key, k in (("split", split, ns), ("head", head, H), ("seq", seq, rest.max() + 1),
                         ("dispatch slot", slot, 4)):
        print(f"exit p50 / p90 by {name}:", " ".join(
            f"{int(i)}:{np.percentile(ex[key == i], 50):.1f}/{np.percentile(ex[key == i], 90):.1f}"
            for i in range(int(k)) if np.any(key == i)))
    cu_id = (xcc << 8) | ((hw >> 8) & 0xFF)  # CU, SH, SE within the XCC
    _, inv, cnt = np.unique(cu_id, return_inverse=True, return_counts=True)
    per = cnt[inv]
    print("waves per CU (count of CUs):", dict(zip(*np.unique(cnt, return_counts=True))))
    for c in sorted(set(per.tolist())):
        print(f"  waves whose CU held {c}: exit p50 {np.percentile(ex[per == c], 50):.1f} "
              f"p90 {np.percentile(ex[per == c], 90):.1f}")
    np.save(os.path.join(ROOT, "gpurun_out", f"beam_stamps_{args.config}{args.tag}.npy"),
            np.concatenate([wid[:, None], s], axis=1))


def steal_report(lib, args):
    """pa_beam_steal_kernel STAMPS: entry, first tile, after the last tile,
    exit, tiles, shared tiles, mid-batch barrier ticks, HW_ID per wave."""
    lib.pa_tune_stamps8.argtypes = [ctypes.c_void_p, ctypes.c_longlong]
    lib.pa_tune_stamps8.restype = ctypes.c_longlong
    buf = np.zeros((1 << 16, 8), np.uint64)
    n = lib.pa_tune_stamps8(buf.ctypes.data, buf.shape[0])
    if n <= 0:
        raise SystemExit("no steal stamps recorded")
    s = buf[:n].astype(np.int64)
    live = s[:, 3] > 0
    s = s[live]
    t0 = s[:, 0].min()
    ent, fst, lst, ex = [(s[:, i] - t0) / 100.0 for i in range(4)]
    items, shared, mid = s[:, 4], s[:, 5], s[:, 6] / 100.0
    xcc = (s[:, 7] >> 32) & 0xF
    print(f"steal form: waves {len(s)} of {n}; kernel span {ex.max():.2f} us")
    print("entry      ", pct(ent))
    print("first tile ", pct(fst))
    print("start-up   ", pct(fst - ent))
    print("tiles span ", pct(lst - fst))
    print("exit       ", pct(ex))
    print("tiles/wave ", pct(items))
    print("shared/wave", pct(shared))
    print("mid-barrier", pct(mid))
    print("us per tile", pct((lst - fst) / np.maximum(items, 1)))
    grid = np.arange(0, ex.max() + 1, 1.0)
    active = [(np.sum((fst <= t) & (lst > t))) for t in grid]
    print("waves on tiles per us:", " ".join(str(a) for a in active))
    print("exit p90 per XCC:", [round(float(np.percentile(ex[xcc == x], 90)), 2)
                                for x in range(8) if np.any(xcc == x)])
    np.save(os.path.join(ROOT, "gpurun_out", f"steal_stamps_{args.config}.npy"), s)


if __name__ == "__main__":
    main()
