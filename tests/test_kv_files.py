"""KV-cache file formats on the CPU (no device needed).

* The oracle's restatement of KVTileCacheCPU::save / load
  (kv_cache/kv_tile_cache_cpu.cpp:89-123) against the reference-built fixtures
  tests/golden/kvtiles_*.npz (tests/golden/make_golden.py kvtiles).
* The C-ABI's host-side validation of tile-record files and snapshots
  (kv_tiles_inspect, kv_cache_inspect): the same parser kv_cache_load_tiles /
  kv_cache_load run before they change a cache, so corrupt, truncated and
  out-of-range files are refused here exactly as they are on the GPU box.
"""
import ctypes
import struct

import numpy as np
import pytest

from oracle import kv_formats
from _util import GOLDEN

FIXTURES = ["f16_ts16_d64", "f32_ts16_d32", "i8_ts32_d64"]
MAGIC_V2 = 0x32564B4D49505041


def _fixture(name):
    f = np.load(GOLDEN / f"kvtiles_{name}.npz")
    return {k: f[k] for k in f.files}


@pytest.mark.parametrize("name", FIXTURES)
def test_oracle_tile_format_matches_reference_file(name):
    f = _fixture(name)
    data, idx = f["data"], f["idx"]
    te = int(f["ts"]) * int(f["D"])
    raw = f["file_bytes"].tobytes()
    recs = kv_formats.read_tiles(raw, te, data.dtype)
    # the reference wrote every tile once, in its hash map's order
    got = kv_formats.tiles_dict(recs)
    want = {tuple(int(x) for x in i): d.ravel() for i, d in zip(idx, data)}
    assert set(got) == set(want) and len(recs) == len(want)
    for k in want:
        assert got[k].tobytes() == want[k].tobytes()
    # re-writing the records in the file's order gives the file byte for byte
    assert kv_formats.write_tiles(recs) == raw
    # the reference's own load() returned the data bit for bit
    assert f["back"].tobytes() == data.tobytes()


def _lib():
    import llm_capi
    return llm_capi.load()


def _inspect_tiles(lib, path, tile_bytes):
    n = ctypes.c_int(-1)
    rc = lib.kv_tiles_inspect(str(path).encode(), tile_bytes, ctypes.byref(n))
    return rc, n.value


@pytest.mark.parametrize("name", FIXTURES)
def test_capi_inspects_reference_tile_files(tmp_path, name):
    import llm_capi
    lib = _lib()
    f = _fixture(name)
    raw = f["file_bytes"].tobytes()
    tb = int(f["ts"]) * int(f["D"]) * f["data"].dtype.itemsize
    p = tmp_path / "t.bin"
    p.write_bytes(raw)
    assert _inspect_tiles(lib, p, tb) == (0, len(f["idx"]))
    # another tile size cannot describe the same file
    assert _inspect_tiles(lib, p, tb * 2)[0] == llm_capi.LLM_ERR_IO
    # truncated, one byte too long, a negative count, a negative index
    for bad in (raw[:-1], raw + b"\0", struct.pack("<i", -1) + raw[4:],
                raw[:4] + struct.pack("<i", -3) + raw[8:]):
        p.write_bytes(bad)
        assert _inspect_tiles(lib, p, tb)[0] == llm_capi.LLM_ERR_IO
    # an empty cache saves as a bare zero count (kv_tile_cache_cpu.cpp:96-97)
    p.write_bytes(kv_formats.write_tiles([]))
    assert _inspect_tiles(lib, p, tb) == (0, 0)
    assert _inspect_tiles(lib, tmp_path / "missing.bin", tb)[0] == llm_capi.LLM_ERR_IO


def _snapshot(L=1, beams=2, H=2, D=8, TS=4, mt=3, pages=6, dtype=0, table=None, used=None,
              pages_data=None, magic=MAGIC_V2):
    """An APPIMKV2 snapshot as kv_cache_save writes it (csrc/kv_io.cpp)."""
    entries = L * beams * H * mt
    if table is None:
        table = np.full(entries, -1, np.int32)
        table[:3] = [4, 1, 4]
    table = np.asarray(table, np.int32)
    if used is None:
        used = sorted({int(t) for t in table if t >= 0})
    used = np.asarray(used, np.int32)
    es = {0: 2, 1: 1, 2: 4, 3: 2}.get(dtype, 2)
    pb = TS * D * es
    if pages_data is None:
        pages_data = np.arange(len(used) * 2 * pb, dtype=np.uint8).tobytes()
    hdr = struct.pack("<9q", magic, L, beams, H, D, TS, mt, pages, dtype)
    return hdr + table.tobytes() + struct.pack("<q", len(used)) + used.tobytes() + pages_data


def test_capi_inspects_snapshots(tmp_path):
    import llm_capi
    lib = _lib()
    geo = (ctypes.c_longlong * 9)()
    p = tmp_path / "s.bin"

    def inspect(blob):
        p.write_bytes(blob)
        return lib.kv_cache_inspect(str(p).encode(), geo)

    assert inspect(_snapshot()) == 0
    assert list(geo) == [1, 2, 2, 8, 4, 3, 6, 0, 2]
    E = llm_capi.LLM_ERR_IO
    good = _snapshot()
    bad_cases = {
        "bad magic": _snapshot(magic=0x1234),
        "truncated page data": good[:-1],
        "trailing bytes": good + b"\0",
        "truncated table": good[:72 + 5],
        "table entry past the pool": _snapshot(table=[6] + [-1] * 11, used=[5]),
        "table entry below -1": _snapshot(table=[-2] + [-1] * 11, used=[]),
        "table names an unsaved page": _snapshot(table=[4, 1] + [-1] * 10, used=[1]),
        "used id past the pool": _snapshot(table=[-1] * 12, used=[6]),
        "negative used id": _snapshot(table=[-1] * 12, used=[-1]),
        "duplicate used ids": _snapshot(table=[1] + [-1] * 11, used=[1, 1]),
        "more used pages than the pool": _snapshot(pages=1, table=[-1] * 12, used=[0, 1]),
        "zero heads": _snapshot(H=0, table=[], used=[]),
        "unknown kv dtype": _snapshot(dtype=9),
        "absurd geometry": struct.pack("<9q", MAGIC_V2, 1 << 40, 1 << 40, 1, 8, 4, 3, 6, 0),
    }
    for what, blob in bad_cases.items():
        assert inspect(blob) == E, what
    assert lib.kv_cache_inspect(str(tmp_path / "none.bin").encode(), geo) == E
