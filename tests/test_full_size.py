"""Config 2 at its full size (64 Mi flat {8 x i64} records, 5.97 GB of Binary
wire: the stream crosses 2^32 bytes at record 48,258,059) against the oracle:
the GPU's encode of the whole batch, compared byte for byte with the oracle's
encode of the same record indices in three windows — the first 10,000
records, 200 records straddling the 4 GiB boundary, the last 10,000 — and the
GPU's decode of the whole stream compared with the oracle's records in the
same windows (plus the whole-batch round trip on the device). A 32-bit offset
bug that is symmetric in the two kernels would pass a round trip but not
this."""
import os
import sys

import numpy as np
import pytest

import datagen
from fbthrift_amd.schema import Schema
from oracle import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

pytestmark = pytest.mark.gpu

N = 1 << 26
L = 89


def _windows():
    cross = (1 << 32) // L
    assert cross == 48_258_059
    return [(0, 10_000), (cross - 100, cross + 100), (N - 10_000, N)]


def test_config2_full_size_windows(gpu):
    import torch

    import bench
    from fbthrift_amd.serializer import BinarySerializer as S, GpuSchema

    gs = GpuSchema(Schema.from_table(datagen.SCHEMAS["flat8"]))
    S.context().reserve(N)
    recs = bench.gen_flat8_device(N, 0, gpu)
    wire = torch.empty(N * L, dtype=torch.uint8, device=gpu)
    S.serialize(gs, recs, N, out=wire, offsets=None, sync=True)
    back = torch.empty(N * 72, dtype=torch.uint8, device=gpu)
    _, _, consumed = S.deserialize(gs, wire, N, records=back)
    assert consumed == N * L
    lib = oracle.lib()
    for a, b in _windows():
        n = b - a
        want_rec = np.zeros(n * 72, np.uint8)
        lib.oracle_gen_flat8(datagen.SEED, a, n, want_rec.ctypes.data)
        want_wire = np.zeros(n * L, np.uint8)
        lib.oracle_flat8_binary_encode(want_rec.ctypes.data, n, want_wire.ctypes.data, 1)
        got_wire = wire[a * L: b * L].cpu().numpy()
        assert np.array_equal(got_wire, want_wire), "wire differs in records [%d, %d)" % (a, b)
        got_rec = back[a * 72: b * 72].cpu().numpy()
        assert np.array_equal(got_rec, want_rec), "records differ in [%d, %d)" % (a, b)
        # the device generator itself matches the oracle's spec in the window
        assert np.array_equal(recs[a * 72: b * 72].cpu().numpy(), want_rec)
    assert torch.equal(back, recs)
