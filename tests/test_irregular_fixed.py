"""Fixed-layout Binary streams (config 2's schema) that leave the canonical
form: the reference reads them record by record like any other stream
(reordered fields, unknown fields skipped, deserialize_struct.whisker:128-159),
so the device must too. The plan kernel decodes every record at its stride
and lists the ones it cannot take; the general reader reads those at their
stride position (k_general.hip fixed_exception_kernel). From the first one
that is not exactly the stride long (or fails) the stream is indexed and
decoded in parallel (tgpu_api.cpp fixed_tail); a stream whose record 0 is
already off the stride is indexed directly. Stream-ordered calls (no host
status) re-read from the first misfit at its own length with the tolerant
program (tgpu_jit_decode_tail) and walk from the first record off that
stride (k_general.hip fixed_stream_finish_kernel). Records, offsets and status
are compared with the oracle at 1M records."""
import numpy as np
import pytest

import datagen
from fbthrift_amd.schema import Schema
from oracle import oracle

pytestmark = pytest.mark.gpu

N = 1 << 20


def canonical(n, first=0):
    recs = np.zeros(n * 72, np.uint8)
    oracle.lib().oracle_gen_flat8(datagen.SEED, first, n, recs.ctypes.data)
    wire = np.zeros(n * 89, np.uint8)
    oracle.lib().oracle_flat8_binary_encode(recs.ctypes.data, n, wire.ctypes.data, 8)
    return recs, wire


def with_extra_field(wire89):
    """Every record gets an unknown i32 field (id 20) before its STOP: what a
    writer with a newer schema produces (96 bytes per record)."""
    n = wire89.size // 89
    a = wire89.reshape(n, 89)
    out = np.zeros((n, 96), np.uint8)
    out[:, :88] = a[:, :88]
    out[:, 88:91] = (8, 0, 20)
    out[:, 91:95] = a[:, 3:7]  # some value bytes
    out[:, 95] = 0
    return out.reshape(-1)


def reordered(rec89):
    """Fields 2 and 1 swapped (legal, read by the switch path)."""
    r = rec89.copy()
    r[0:11], r[11:22] = rec89[11:22], rec89[0:11]
    return r


def run(gpu, wire, n, sync=True):
    import torch

    from fbthrift_amd.serializer import BinarySerializer, GpuSchema

    schema = Schema.from_table(datagen.SCHEMAS["flat8"])
    gs = GpuSchema(schema)
    w = torch.from_numpy(np.ascontiguousarray(wire)).to(gpu)
    if sync:
        rec, _, st, nd, cons = BinarySerializer.deserialize_status(gs, w, n)
    else:
        rec = torch.zeros(n * 72, dtype=torch.uint8, device=gpu)
        BinarySerializer.deserialize(gs, w, n, records=rec, sync=False)
        st, nd, cons = BinarySerializer.context().wait()
    ost, orec, _, ond, ocons = oracle.decode(schema, 0, wire.tobytes(), n)
    assert st.as_tuple() == ost.as_tuple()
    assert (nd, cons) == (ond, ocons)
    k = (nd + (1 if st.code else 0)) * 72
    assert np.array_equal(rec.cpu().numpy()[:k], orec[:k])
    return st, nd


@pytest.mark.parametrize("sync", [True, False])
def test_first_record_irregular(gpu, sync):
    recs, wire = canonical(N)
    w = np.concatenate([reordered(wire[:89]), wire[89:]])
    st, nd = run(gpu, w, N, sync)
    assert st.code == 0 and nd == N


@pytest.mark.parametrize("sync,tail", [(True, "1"), (False, "1"), (False, "0")])
def test_every_record_has_an_unknown_field(gpu, sync, tail, monkeypatch):
    """Stream-ordered: the strided tail decode takes every record at 96 bytes
    (TGPU_STREAM_TAIL=0: the finish kernel's lane walks them all)."""
    monkeypatch.setenv("TGPU_STREAM_TAIL", tail)
    _, wire = canonical(N if tail == "1" else 1 << 16)
    n = wire.size // 89
    st, nd = run(gpu, with_extra_field(wire), n, sync)
    assert st.code == 0 and nd == n


@pytest.mark.parametrize("sync", [True, False])
def test_irregular_in_the_middle_then_error(gpu, sync):
    _, wire = canonical(N)
    k = 700_001
    w = wire.copy()
    w[89 * k: 89 * (k + 1)] = reordered(wire[89 * k: 89 * (k + 1)])
    # a bool-typed unknown field with byte 7 far after the irregular record:
    # Binary readBool throws... only for known bool fields; an i64 field id 5
    # sent as T_STRING with a huge length is a reader error (truncated)
    j = 900_000
    w[89 * j + 33] = 11  # field 4's header type byte: T_STRING, length from the value bytes
    run(gpu, w, N, sync)


@pytest.mark.parametrize("sync", [True, False])
def test_tail_shorter_than_n(gpu, sync):
    """The stream ends before n records: UNDERFLOW at the first missing one."""
    _, wire = canonical(4096)
    w = np.concatenate([reordered(wire[:89]), wire[89:]])
    st, nd = run(gpu, w, 5000, sync)
    assert st.code == 1 and nd == 4096


@pytest.mark.parametrize("where", [0, 1, 1234, 9999])
def test_async_call_matches(gpu, where):
    """The asynchronous form (no host status) gives the same result."""
    n = 10_000
    _, wire = canonical(n)
    w = wire.copy()
    w[89 * where: 89 * (where + 1)] = reordered(wire[89 * where: 89 * (where + 1)])
    run(gpu, w, n, sync=False)


def _reorder_at(wire, idx):
    w = wire.copy()
    for i in idx:
        w[89 * i: 89 * (i + 1)] = reordered(wire[89 * i: 89 * (i + 1)])
    return w


@pytest.mark.parametrize("sync", [True, False])
def test_many_exceptions_same_length(gpu, sync):
    """Every 1000th record reordered (same length): the plan kernel lists them,
    the general reader reads each at its stride position (no re-index)."""
    _, wire = canonical(N)
    st, nd = run(gpu, _reorder_at(wire, range(3, N, 1000)), N, sync)
    assert st.code == 0 and nd == N


def test_every_record_reordered(gpu):
    """An exception list of exactly its capacity (2^20 records)."""
    _, wire = canonical(N)
    w = wire.reshape(N, 89).copy()
    w[:, 0:11], w[:, 11:22] = wire.reshape(N, 89)[:, 11:22], wire.reshape(N, 89)[:, 0:11]
    st, nd = run(gpu, w.reshape(-1), N)
    assert st.code == 0 and nd == N


@pytest.mark.parametrize("sync", [True, False])
def test_exception_list_overflow(gpu, sync):
    """More exceptions than the list holds: the stream is indexed from the
    first one (stream-ordered: re-read at record 0's length, 89)."""
    n = N + 4096
    _, wire = canonical(n)
    w = wire.reshape(n, 89).copy()
    w[:, 0:11], w[:, 11:22] = wire.reshape(n, 89)[:, 11:22], wire.reshape(n, 89)[:, 0:11]
    st, nd = run(gpu, w.reshape(-1), n, sync)
    assert st.code == 0 and nd == n


@pytest.mark.parametrize("sync", [True, False])
def test_exception_then_length_change(gpu, sync):
    """Reordered records around a record one field longer: from the longer
    record on the stride is wrong, so the stream is re-read from it."""
    n = 100_000
    _, wire = canonical(n)
    w = _reorder_at(wire, [10, 500, 70_000])
    extra = with_extra_field(w[89 * 5000: 89 * 5001])
    w = np.concatenate([w[: 89 * 5000], extra, w[89 * 5001:]])
    st, nd = run(gpu, w, n, sync)
    assert st.code == 0 and nd == n


@pytest.mark.parametrize("sync", [True, False])
def test_every_record_extra_field_then_change(gpu, sync):
    """A stream at a second stride (every record + one appended field) whose
    records change shape again at 600k (an appended string instead): the
    tolerant program decodes at the second stride up to there, the stream is
    indexed from the first record off it."""
    _, wire = canonical(N)
    w = with_extra_field(wire).reshape(N, 96).copy()
    k = 600_000
    tail = wire.reshape(N, 89)[k:]
    extra = np.zeros((N - k, 89 + 3 + 4 + 5), np.uint8)
    extra[:, :88] = tail[:, :88]
    extra[:, 88:91] = (11, 0, 21)          # field 21: string
    extra[:, 91:95] = (0, 0, 0, 5)         # length 5
    extra[:, 95:100] = tail[:, 3:8]
    extra[:, 100] = 0
    s = np.concatenate([w[:k].reshape(-1), extra.reshape(-1)])
    st, nd = run(gpu, s, N, sync)
    assert st.code == 0 and nd == N


@pytest.mark.parametrize("sync", [True, False])
def test_second_stride_with_error(gpu, sync):
    """A bad record (an unknown field type) deep in a second-stride stream:
    the reference status at that record."""
    _, wire = canonical(200_000)
    w = with_extra_field(wire).copy()
    j = 150_001
    w[96 * j + 88] = 0x7F
    run(gpu, w, 200_000, sync)
