import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "pagedattention-based-transformer-decoder-inference-framework_amd"
for p in (str(ROOT), str(PKG), str(Path(__file__).resolve().parent)):
    if p not in sys.path:
        sys.path.insert(0, p)

os.environ.setdefault("OMP_NUM_THREADS", str(min(8, os.cpu_count() or 1)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs under gpurun)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def oracle():
    from oracle.oracle import Oracle
    return Oracle()


def _gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    """The HIP C-ABI library on cuda:0.  Fails loudly (never skips) when a GPU
    test runs without the native library: a GPU test that silently fell back
    would void every parity claim."""
    if not _gpu_available():
        pytest.skip("no GPU in this container (run with -m gpu under gpurun)")
    import torch
    import llm_capi
    lib = llm_capi.load()  # raises if libllm_decoder_hip.so is missing
    torch.cuda.init()
    return lib
