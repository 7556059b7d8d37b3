"""The device record generators bench.py uses for configs 3 and 4
(tools/datagen.hip) reproduce tests/golden/datagen.py's spec exactly."""
import ctypes
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import datagen  # noqa: E402

from fbthrift_amd.schema import Schema  # noqa: E402

LIB = os.path.join(ROOT, "tools", "build", "libtgpu_datagen.so")


def _gen(kind, first, n, packed=False):
    import torch

    schema = Schema.from_table(datagen.SCHEMAS[kind])
    rs = schema.record_size
    recs = torch.zeros(n * rs, dtype=torch.uint8, device="cuda")
    side = torch.zeros(n * 64, dtype=torch.uint8, device="cuda")
    lib = ctypes.CDLL(LIB)
    fn = getattr(lib, "tgpu_gen_%s%s" % (kind, "_packed" if packed else ""))
    assert fn(ctypes.c_uint64(datagen.SEED), ctypes.c_uint64(first), ctypes.c_uint64(n),
              ctypes.c_void_p(recs.data_ptr()), ctypes.c_void_p(side.data_ptr()), None) == 0
    torch.cuda.synchronize()
    return schema, recs.cpu().numpy().view(schema.dtype()), side.cpu().numpy()


@pytest.mark.gpu
@pytest.mark.parametrize("packed", [False, True])
def test_mixed_generator_matches_spec(gpu, packed):
    first, n = 123456, 3000
    _, r, side = _gen("mixed", first, n, packed)
    for t in range(n):
        exp = datagen.gen_mixed(first + t)
        assert [int(r["f%d" % (k + 1)][t]) for k in range(4)] == exp[:4]
        for k in range(2):
            sp = r["f%d" % (k + 5)][t]
            got = bytes(side[sp["offset"]: sp["offset"] + sp["length"]])
            assert got == exp[4 + k]
        assert list(r["__isset"][t]) == [1] * 6


@pytest.mark.gpu
@pytest.mark.parametrize("packed", [False, True])
def test_nested_generator_matches_spec(gpu, packed):
    first, n = 98765, 3000
    _, r, side = _gen("nested", first, n, packed)
    elems = side.view(np.int32)
    for t in range(n):
        i64, lst, inner = datagen.gen_nested(first + t)
        assert int(r["f1"][t]) == i64
        sp = r["f2"][t]
        assert list(elems[sp["offset"] // 4: sp["offset"] // 4 + sp["length"]]) == lst
        assert [float(r["f3"][t]["f%d" % (k + 1)]) for k in range(3)] == inner
        assert list(r["f3"][t]["__isset"]) == [1] * 3 and list(r["__isset"][t]) == [1] * 3


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["mixed", "nested"])
def test_packed_payloads_are_contiguous(gpu, kind):
    """The packed generators leave no gaps: payload k starts where k-1 ends."""
    _, r, side = _gen(kind, 7, 5000, True)
    spans = ([r["f5"], r["f6"]] if kind == "mixed" else [r["f2"]])
    off = np.stack([s["offset"] for s in spans], 1).reshape(-1).astype(np.int64)
    ln = np.stack([s["length"] for s in spans], 1).reshape(-1).astype(np.int64)
    if kind == "nested":
        ln = ln * 4
    assert off[0] == 0 and np.array_equal(off[1:], np.cumsum(ln)[:-1])
