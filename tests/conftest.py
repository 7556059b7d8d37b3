import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libtgpu.so)")


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.fixture(params=["interp", "jit"])
def codec(request, monkeypatch):
    """Runs a GPU test through both program paths of libtgpu: the library's
    interpreting kernels (TGPU_JIT=0) and the per-schema kernels the schema
    compiler generates (TGPU_JIT=1, tgpu_jit.cpp)."""
    monkeypatch.setenv("TGPU_JIT", "1" if request.param == "jit" else "0")
    return request.param
