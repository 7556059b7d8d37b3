"""Nested-field skim (tgpu_skim_batch_ex): the schemaless field tables of
tgpu_skim_batch, descending into struct-valued fields the way
protocol::parseObject recurses (parseValue -> parseObjectInplace,
thrift/lib/cpp2/protocol/detail/Object.h:416-432) — entries in pre-order, a
descended struct's entry (its whole encoded value) before its fields', the
nesting level in flags bits 2-5; depth and height checked as
apache::thrift::skip checks the same struct (Protocol.h:187-283).

Pinned by the golden streams the reference's Python protocols wrote
(tests/golden/make_golden.py, nestgen.py): the level-0 entries are the flat
skim's, every descended struct's entries tile its bytes up to its STOP, and
the nested scalars' bytes decode to the golden values. The GPU matches the
oracle entry for entry and status for status (golden, recursive chains and
trees, the reference tests' corpus, depth limits)."""
import numpy as np
import pytest

import corpus
import helpers
import nested_helpers as nh
from oracle import oracle

from test_skim import _scalar

T_STRUCT = 12
LEVEL_SHIFT, LEVEL_MASK = 2, 0x3C


def _level(e):
    return (int(e["flags"]) & LEVEL_MASK) >> LEVEL_SHIFT


def _check_tiling(wire, offsets, fields, counts, nest, protocol):
    """Pre-order entries of each record: levels step by at most one down, a
    descended struct's children start after its first byte and the last one
    ends one byte (its STOP) before the struct does; every top-level entry
    follows the previous one."""
    for i in range(len(counts)):
        stack = []  # (level, end) of open descended structs
        prev_end = int(offsets[i])
        for j in range(int(counts[i])):
            e = fields[i, j]
            lv = _level(e)
            off, end = int(e["offset"]), int(e["offset"]) + int(e["length"])
            while stack and stack[-1][0] >= lv:
                lvl, s_end = stack.pop()
                assert prev_end + 1 == s_end, (i, j)  # the struct's STOP
                prev_end = s_end
            assert lv == len(stack), (i, j)
            assert off > prev_end, (i, j)  # a field header precedes every value
            if int(e["ttype"]) == T_STRUCT and lv < nest:
                stack.append((lv, end))
                prev_end = off  # its first field header starts here
            else:
                prev_end = end
            assert end <= int(offsets[i + 1])
        while stack:
            lvl, s_end = stack.pop()
            assert prev_end + 1 == s_end, i
            prev_end = s_end
        assert prev_end + 1 == int(offsets[i + 1]), i  # the record's STOP


@pytest.mark.parametrize("name", helpers.case_names())
@pytest.mark.parametrize("nest", [1, 3])
def test_oracle_nested_skim_golden(name, nest):
    c = helpers.Case(name)
    st0, flat, counts0, _ = oracle.skim(c.protocol, c.wire, c.offsets, c.n, max_fields=64)
    st, fields, counts, done = oracle.skim(c.protocol, c.wire, c.offsets, c.n, max_fields=64,
                                           nest=nest)
    assert st.code == 0 and done == c.n
    _check_tiling(c.wire, c.offsets, fields, counts, nest, c.protocol)
    for i in range(c.n):  # the level-0 entries are the flat skim's
        top = [fields[i, j] for j in range(int(counts[i])) if _level(fields[i, j]) == 0]
        flat_i = flat[i, : int(counts0[i])]
        assert len(top) == len(flat_i)
        for a, b in zip(top, flat_i):
            assert (a["id"], a["ttype"], a["length"], a["offset"]) == \
                   (b["id"], b["ttype"], b["length"], b["offset"])


@pytest.mark.parametrize("name", ["nested_binary", "nested_compact", "nested_compact_v1"])
def test_oracle_nested_skim_values(name):
    """Config 4's Inner {3 x double} (field 2): with one level of nesting its
    three doubles are entries of level 1 whose bytes are the golden values."""
    c = helpers.Case(name)
    st, fields, counts, _ = oracle.skim(c.protocol, c.wire, c.offsets, c.n, max_fields=16, nest=1)
    assert st.code == 0
    inner = c.schema.structs[1]
    for i in range(c.n):
        row = [fields[i, j] for j in range(int(counts[i]))]
        k = [e["id"] for e in row].index(3)  # the struct field (id 3)
        assert row[k]["ttype"] == T_STRUCT and _level(row[k]) == 0
        kids = row[k + 1: k + 1 + len(inner.fields)]
        for m, (e, f) in enumerate(zip(kids, inner.fields)):
            assert _level(e) == 1 and e["id"] == f.id
            raw = c.wire[e["offset"]: e["offset"] + e["length"]]
            assert _scalar(c.protocol, int(e["ttype"]), raw, int(e["flags"])) == \
                   int(c.values["2/%d.val" % m][i])


@pytest.mark.parametrize("name", ["chain_binary", "chain_compact", "tree_binary",
                                  "keyed_compact"])
def test_oracle_nested_skim_recursive(name):
    """Boxed chains (Node {next: Node}) descend level by level up to nest;
    deeper structs are one entry each, as flat skims see them."""
    c = nh.NestedCase(name)
    for nest in (0, 2, 8):
        st, fields, counts, _ = oracle.skim(c.protocol, c.wire, c.offsets, c.n, max_fields=256,
                                            nest=nest)
        assert st.code == 0
        _check_tiling(c.wire, c.offsets, fields, counts, nest, c.protocol)
        levels = [_level(fields[i, j]) for i in range(c.n)
                  for j in range(min(int(counts[i]), 256))]
        assert max(levels) <= nest
        if nest and name.startswith("chain"):
            assert max(levels) == nest


def test_oracle_nested_skim_depth_limit():
    """A chain deeper than max_depth: DEPTH_LIMIT where skip(T_STRUCT) would
    raise it for the same struct — the flat skim of the same bytes raises it
    inside its skip at the same record and byte."""
    c = nh.NestedCase("chain_binary")
    lim = (0, 0, 3, 0)  # string_limit, container_limit, max_depth, height
    st, _, _, done = oracle.skim(c.protocol, c.wire, c.offsets, c.n, max_fields=64, nest=8,
                                 limits=lim)
    st0, _, _, done0 = oracle.skim(c.protocol, c.wire, c.offsets, c.n, max_fields=64, limits=lim)
    assert st.code == 8 and st.as_tuple() == st0.as_tuple() and done == done0  # DEPTH_LIMIT


def _skim_both(gpu, protocol, wire, offsets, n, max_fields, nest, limits=None):
    import torch

    from fbthrift_amd import serializer as S

    ser = {0: S.BinarySerializer, 2: S.CompactSerializer, 0x102: S.CompactV1Serializer}[protocol]
    w = torch.from_numpy(np.frombuffer(bytes(wire) or b"\0", np.uint8).copy()).to(gpu)[: len(wire)]
    o = torch.from_numpy(np.asarray(offsets, np.uint64).astype(np.int64)).to(gpu)
    fields, counts, done, st = ser.skim(w, o, n, max_fields=max_fields, limits=limits, check=False,
                                        nest=nest)
    ost, ofields, ocounts, odone = oracle.skim(protocol, wire, offsets, n, max_fields, limits,
                                               nest=nest)
    assert st.as_tuple() == ost.as_tuple() and done == odone
    got = S.skim_records(fields, n, max_fields)
    cnt = counts.cpu().numpy()
    for i in range(done):
        assert cnt[i] == ocounts[i]
        k = min(int(cnt[i]), max_fields)
        assert np.array_equal(got[i, :k], ofields[i, :k]), i
    return st


@pytest.mark.gpu
@pytest.mark.parametrize("name", helpers.case_names())
@pytest.mark.parametrize("nest,max_fields", [(1, 4), (3, 64)])
def test_gpu_nested_skim_golden(gpu, name, nest, max_fields):
    c = helpers.Case(name)
    assert _skim_both(gpu, c.protocol, c.wire, c.offsets, c.n, max_fields, nest).code == 0


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(nh.manifest()["nested_cases"]))
@pytest.mark.parametrize("nest", [2, 8])
def test_gpu_nested_skim_recursive(gpu, name, nest):
    c = nh.NestedCase(name)
    assert _skim_both(gpu, c.protocol, c.wire, c.offsets, c.n, 64, nest).code == 0


@pytest.mark.gpu
@pytest.mark.parametrize("max_depth", [1, 2, 3, 5])
def test_gpu_nested_skim_depth_limit(gpu, max_depth):
    for name in ("chain_binary", "chain_compact"):
        c = nh.NestedCase(name)
        _skim_both(gpu, c.protocol, c.wire, c.offsets, c.n, 64, 8, (0, 0, max_depth, 0))


@pytest.mark.gpu
@pytest.mark.parametrize("case", [c for c in corpus.cases() if c[4] == 1], ids=lambda c: c[0])
def test_gpu_nested_skim_corpus(gpu, case):
    """The reference tests' damaged and edge-case records, descended into."""
    name, protocol, _table, wire, n, limits, _code = case
    _skim_both(gpu, protocol, wire, [0, len(wire)], 1, 8, 8, limits)
