"""Containers of structs and of containers (list<Struct>, set<Struct>,
map<i32, Struct>, list<list<i32>>, map<string, list<string>>,
list<map<i32, string>>, map<i32, map<i32, Struct>>, set<list<list<i64>>>),
both protocols.

Reference semantics: protocol_methods.h:358-503 (lists of any element class:
reserve + emplace_back_default + read per element), EncodeHelpers.h:188-260
(maps / sets insert an element once it is read), TableBasedSerializerImpl.h:
300-460 (the table-driven reader's recursion through TypeInfo). Pinned by
golden streams the reference's own Python protocols wrote from nested values
(tests/golden/make_golden.py, nestgen.py): the oracle and the GPU must decode
them to those values and encode the values back to the same bytes; on
malformed input the GPU must report the oracle's status and leave the same
partial record (the failing list element present, a failing set element or
map pair absent)."""
import numpy as np
import pytest

import nested_helpers as nh
from oracle import oracle

CASES = nh.case_names()


def test_golden_cases_exist():
    assert len(CASES) == 10


@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("indexed", [False, True])
def test_oracle_decodes_golden(name, indexed):
    c = nh.NestedCase(name)
    st, rec, arena, nd, cons = oracle.decode(c.schema, c.protocol, c.wire, c.n,
                                             offsets=c.offsets if indexed else None)
    assert st.code == 0 and nd == c.n and cons == len(c.wire), st.as_tuple()
    assert nh.materialize_batch(c, rec, arena) == c.values


@pytest.mark.parametrize("name", CASES)
def test_oracle_encodes_golden(name):
    c = nh.NestedCase(name)
    rec, sb, lb = nh.pack(c)
    st, wire, offs = oracle.encode(c.schema, c.protocol, rec, c.n, sb, lb)
    assert st.code == 0 and wire == c.wire
    assert np.array_equal(offs, c.offsets)


@pytest.mark.parametrize("name", CASES)
def test_oracle_arena_bound(name):
    """Records read into regions of scale x their wire bytes: the documented
    arena (tgpu_schema_arena_scale x in_len) always suffices, and a record's
    containers stay inside its own region."""
    c = nh.NestedCase(name)
    scale = oracle.arena_scale(c.schema, c.protocol)
    assert scale % 8 == 0 and scale >= 8
    st, rec, arena, nd, _ = oracle.decode(c.schema, c.protocol, c.wire, c.n,
                                          arena_cap=scale * len(c.wire))
    assert st.code == 0 and nd == c.n


def cut_cases(c, k=6):
    """Records truncated at every byte (each its own one-record stream)."""
    out = []
    for i in range(k):
        b, e = int(c.offsets[i * 7]), int(c.offsets[i * 7 + 1])
        rec = c.wire[b:e]
        for cut in range(0, len(rec), max(1, len(rec) // 40)):
            out.append(rec[:cut])
    return out


@pytest.mark.parametrize("name", CASES)
def test_oracle_truncation_is_an_error(name):
    c = nh.NestedCase(name)
    for w in cut_cases(c):
        st = oracle.decode(c.schema, c.protocol, w, 1)[0]
        assert st.code in (1, 5), st.as_tuple()  # out_of_range or TProtocolException


# ---- GPU ----------------------------------------------------------------------
def _ser(protocol):
    from fbthrift_amd import serializer as S

    return {0: S.BinarySerializer, 2: S.CompactSerializer}[protocol]


def _t(b, dev):
    import torch

    a = np.frombuffer(bytes(b), np.uint8) if not isinstance(b, np.ndarray) else b
    if a.size == 0:
        a = np.zeros(1, np.uint8)
    return torch.from_numpy(a.copy()).to(dev)


def _gpu_decode(c, wire, n, offsets, gpu, limits=None):
    from fbthrift_amd.serializer import GpuSchema

    import torch

    gs = GpuSchema(c.schema)
    w = _t(wire, gpu) if len(wire) else torch.zeros(0, dtype=torch.uint8, device=gpu)
    o = None if offsets is None else torch.from_numpy(offsets.astype(np.int64)).to(gpu)
    rec, arena, st, nd, cons = _ser(c.protocol).deserialize_status(gs, w, n, o, limits)
    return st, rec.cpu().numpy(), arena.cpu().numpy(), nd, cons


@pytest.fixture(params=["general", "compiled"])
def jit(request, monkeypatch):
    """general: the AOT kernels; compiled: TGPU_JIT=1, so the schemas with a
    nested record program (lists / sets of structs or scalar lists) decode
    through it (tgpu_nested.h) and the rest through the general reader."""
    monkeypatch.setenv("TGPU_JIT", "1" if request.param == "compiled" else "0")
    return request.param


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("indexed", [False, True])
def test_gpu_decode_golden(gpu, name, indexed, jit):
    c = nh.NestedCase(name)
    offs = c.offsets if indexed else None
    st, rec, arena, nd, cons = _gpu_decode(c, c.wire, c.n, offs, gpu)
    assert st.code == 0 and nd == c.n and cons == len(c.wire), st.as_tuple()
    assert nh.materialize_batch(c, rec, arena) == c.values
    ost, orec, oarena, _, _ = oracle.decode(c.schema, c.protocol, c.wire, c.n, offsets=offs)
    S = c.layout.size[0]
    assert np.array_equal(rec[: c.n * S], orec[: c.n * S])  # same spans: same regions
    assert np.array_equal(arena[: oarena.size], oarena)


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_gpu_encode_golden(gpu, name, jit):
    c = nh.NestedCase(name)
    rec, sb, lb = nh.pack(c)
    from fbthrift_amd.serializer import GpuSchema

    gs = GpuSchema(c.schema)
    S = _ser(c.protocol)
    out, offs = S.serialize(gs, _t(rec, gpu), c.n, _t(sb, gpu), _t(lb, gpu))
    assert bytes(out.cpu().numpy()) == c.wire
    assert np.array_equal(offs.cpu().numpy().astype(np.uint64), c.offsets)
    sz, total = S.encoded_size(gs, _t(rec, gpu), c.n, list_base=_t(lb, gpu))
    assert total == len(c.wire)


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_gpu_arena_scale_matches(gpu, name):
    from fbthrift_amd.serializer import GpuSchema

    c = nh.NestedCase(name)
    gs = GpuSchema(c.schema)
    assert _ser(c.protocol).arena_bytes(gs, 1) == oracle.arena_scale(c.schema, c.protocol)


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_gpu_truncation_parity(gpu, name, jit):
    """Every cut of a record: the oracle's status and the same partial record
    (failing list element present, set element / map pair absent)."""
    c = nh.NestedCase(name)
    S = c.layout.size[0]
    for w in cut_cases(c, 3):
        st, rec, arena, nd, cons = _gpu_decode(c, w, 1, None, gpu)
        ost, orec, oarena, ond, ocons = oracle.decode(c.schema, c.protocol, w, 1)
        assert st.as_tuple() == ost.as_tuple(), (len(w), st.as_tuple(), ost.as_tuple())
        assert np.array_equal(rec[:S], orec[:S]), len(w)
        m = min(arena.size, oarena.size)
        assert np.array_equal(arena[:m], oarena[:m]), len(w)


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_gpu_transcode_golden(gpu, name, jit):
    """Binary <-> Compact of nested records == the reference's stream of the
    same values in the other protocol."""
    src = nh.NestedCase(name)
    other = name.replace("binary", "X").replace("compact", "binary").replace("X", "compact")
    dst = nh.NestedCase(other)
    from fbthrift_amd.serializer import GpuSchema

    out, offs, st, n_done, size = _ser(src.protocol).transcode(
        GpuSchema(src.schema), _t(src.wire, gpu), src.n, dst.protocol)
    assert st.code == 0 and n_done == src.n
    assert bytes(out.cpu().numpy()[:size]) == dst.wire


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["structlist_compact", "deepcont_binary"])
def test_gpu_container_limit_nested(gpu, name, jit):
    """container_limit applies to every nested container (checkContainerSize
    on each readListBegin / readMapBegin)."""
    c = nh.NestedCase(name)
    for lim in (3, 15):
        st, rec, arena, nd, cons = _gpu_decode(c, c.wire, c.n, None, gpu, limits=(0, lim, 12000, 0))
        ost, orec, oarena, ond, ocons = oracle.decode(c.schema, c.protocol, c.wire, c.n,
                                                      limits=(0, lim, 12000, 0))
        assert st.as_tuple() == ost.as_tuple() and (nd, cons) == (ond, ocons)
        S = c.layout.size[0]
        k = (nd + 1) * S
        assert np.array_equal(rec[:k], orec[:k])
