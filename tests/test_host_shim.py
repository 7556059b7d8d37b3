"""The C++ host mirror (include/thrift_gpu/GpuBatchSerializer.h): builds and
links against libtgpu.so on CPU; on the GPU it round-trips a codegen-layout
struct and rethrows the reference's exception types; the IOBuf batch API
(serializeBatch / deserializeBatch) round-trips codegen'd objects with
std::string / std::vector / std::map / std::set / nested struct members and
matches a plain Binary writer byte for byte (tests/cpp/test_host_objects.cpp)."""
import os
import subprocess

import pytest

import helpers

CPP = os.path.join(helpers.ROOT, "tests", "cpp")
BIN = os.path.join(CPP, "build", "test_host_shim")
BIN2 = os.path.join(CPP, "build", "test_host_objects")


def test_host_shim_builds():
    subprocess.run(["make", "-s", "-C", CPP], check=True)
    out = subprocess.run(["ldd", BIN], capture_output=True, text=True).stdout
    assert os.path.exists(BIN2)
    assert "libtgpu.so" in out and "not found" not in out.split("libtgpu.so")[1].split("\n")[0]


@pytest.mark.gpu
def test_host_shim_runs(gpu):
    subprocess.run(["make", "-s", "-C", CPP], check=True)
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "host shim ok" in r.stdout


@pytest.mark.gpu
def test_host_objects_runs(gpu):
    subprocess.run(["make", "-s", "-C", CPP], check=True)
    r = subprocess.run([BIN2], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "host objects ok" in r.stdout


BIN3 = os.path.join(CPP, "build", "test_host_recursive")


@pytest.mark.gpu
def test_host_recursive_runs(gpu):
    """Boxed (std::unique_ptr) recursive members and struct map keys through
    serializeBatch / deserializeBatch (tests/cpp/test_host_recursive.cpp)."""
    subprocess.run(["make", "-s", "-C", CPP], check=True)
    r = subprocess.run([BIN3], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "host recursive ok" in r.stdout


BIN4 = os.path.join(CPP, "build", "test_binding_width")


def test_binding_list_width_guard():
    """HostBinding.h without a GPU: a list<i16> bound to std::vector<int32_t>
    takes the per-element path (sign-extended) both ways; a width-matched
    binding keeps the one-copy path (tests/cpp/test_binding_width.cpp)."""
    subprocess.run(["make", "-s", "-C", CPP, "build/test_binding_width"], check=True)
    r = subprocess.run([BIN4], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert "binding width ok" in r.stdout
