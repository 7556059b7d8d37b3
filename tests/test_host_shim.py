"""The C++ host mirror (include/thrift_gpu/GpuBatchSerializer.h): builds and
links against libtgpu.so on CPU; on the GPU it round-trips a codegen-layout
struct and rethrows the reference's exception types."""
import os
import subprocess

import pytest

import helpers

CPP = os.path.join(helpers.ROOT, "tests", "cpp")
BIN = os.path.join(CPP, "build", "test_host_shim")


def test_host_shim_builds():
    subprocess.run(["make", "-s", "-C", CPP], check=True)
    out = subprocess.run(["ldd", BIN], capture_output=True, text=True).stdout
    assert "libtgpu.so" in out and "not found" not in out.split("libtgpu.so")[1].split("\n")[0]


@pytest.mark.gpu
def test_host_shim_runs(gpu):
    subprocess.run(["make", "-s", "-C", CPP], check=True)
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "host shim ok" in r.stdout
