"""The nested record program (tgpu_nested.h, tgpu_jit.cpp gen_nested_source):
schemas whose lists / sets hold structs or scalar lists decode through one
compiled kernel with a loop per container level instead of the general
reader's frame machine. It must give the general reader's records, spans and
arena bytes exactly (same record regions, same allocation order), and leave
every record off the canonical form to the general decoder.

CPU: the nested programs of the bench schema (tests/../bench.py NESTED_TABLE:
{i64, list<Item>, list<list<i32>>}) and of maps / string elements compile for
gfx950 in both protocols; recursive schemas an unrolled one. GPU: 40 Ki
records of that schema against the oracle's decode of the same stream, and the nested kernel against the general decoder
(TGPU_NESTED=0) bit for bit, incl. records and arena bytes; the golden nested
cases under TGPU_JIT=1 are in test_nested_containers.py."""
import os

import numpy as np
import pytest

import bench
from fbthrift_amd.schema import Schema
from fbthrift_amd.serializer import compile_check
from oracle import oracle

T_BOOL, T_I32, T_STRING, T_LIST, T_STRUCT, T_MAP = 2, 8, 11, 15, 12, 13


@pytest.mark.parametrize("protocol", [0, 2])
def test_nested_program_compiles(protocol):
    rc, log = compile_check(Schema.from_table(bench.NESTED_TABLE), protocol)
    assert rc == 0, log


def test_nested_program_scope():
    """Which shapes get a nested program (generated only: compiling is
    test_nested_program_compiles' and the GPU tests' job)."""
    # map<Item, i32> (a struct key) and list<map<i32, bool>> (bools inside
    # maps): one each since round 4 (tests/test_nested_shapes.py)
    skey = [[[1, T_MAP, T_STRUCT, 0, -1, T_I32, None, [T_STRUCT, 0, 0, 1]]],
            [[1, T_I32, 0, 0, -1]]]
    rc, log = compile_check(Schema.from_table(skey), 0, arch="")
    assert rc == 0, log
    mbool = [[[1, T_LIST, T_MAP, 0, -1, 0, [T_MAP, T_I32, T_BOOL, -1]]]]
    rc, log = compile_check(Schema.from_table(mbool), 2, arch="")
    assert rc == 0, log
    # struct Tree {1: list<Tree> kids} (recursive): unrolled (deeper records:
    # the general reader); none with TGPU_NESTED_UNROLL=0
    tree = [[[1, T_LIST, T_STRUCT, 0, 0]]]
    rc, log = compile_check(Schema.from_table(tree), 0, arch="")
    assert rc == 0, log
    os.environ["TGPU_NESTED_UNROLL"] = "0"
    try:
        rc, _ = compile_check(Schema.from_table(tree), 0, arch="")
    finally:
        del os.environ["TGPU_NESTED_UNROLL"]
    assert rc == 22
    # map<i32, Item>, map<string, list<string>>, list<map<i32, string>>: one each
    for t in ([[[1, T_MAP, T_I32, 0, 1, T_STRUCT]], [[1, T_I32, 0, 0, -1]]],
              [[[1, T_MAP, T_STRING, 0, -1, T_LIST, [T_LIST, T_STRING, 0, -1]]]],
              [[[1, T_LIST, T_MAP, 0, -1, 0, [T_MAP, T_I32, T_STRING, -1]]]]):
        for protocol in (0, 2):
            rc, log = compile_check(Schema.from_table(t), protocol, arch="")
            assert rc == 0, log
    # list<Item> with a union Item: one (at most one member a record)
    un = [[[1, T_LIST, T_STRUCT, 0, 1]],
          {"union": True, "fields": [[1, T_I32, 0, 0, -1], [2, T_STRING, 0, 0, -1]]}]
    rc, log = compile_check(Schema.from_table(un), 0, arch="")
    assert rc == 0, log
    # list<Item> with an optional member in Item: one (headers checked at run time)
    opt = [[[1, T_LIST, T_STRUCT, 0, 1]], [[1, T_I32, 0, 1, -1], [2, T_I32, 0, 0, -1]]]
    rc, log = compile_check(Schema.from_table(opt), 2, arch="")
    assert rc == 0, log
    # list<Item>: one
    ok = [[[1, T_LIST, T_STRUCT, 0, 1]], [[1, T_I32, 0, 0, -1], [2, T_STRING, 0, 0, -1]]]
    rc, log = compile_check(Schema.from_table(ok), 2, arch="")
    assert rc == 0, log


def _encode(gpu, protocol, n, seed, monkeypatch=None, nested=False, batch=None):
    import torch

    from fbthrift_amd import serializer as SZ

    if monkeypatch is not None:
        monkeypatch.setenv("TGPU_JIT", "1")
        monkeypatch.setenv("TGPU_NESTED", "1" if nested else "0")
    schema, recs, lbase, *_ = batch or bench.nested_batch(gpu, n, seed)
    gs = SZ.GpuSchema(schema)
    Ser = {0: SZ.BinarySerializer, 2: SZ.CompactSerializer}[protocol]
    wire, offs = Ser.serialize(gs, recs, n, list_base=lbase)
    torch.cuda.synchronize()
    return schema, gs, Ser, wire, offs


def _decode(Ser, gs, wire, n, offs, monkeypatch, nested):
    monkeypatch.setenv("TGPU_JIT", "1")
    monkeypatch.setenv("TGPU_NESTED", "1" if nested else "0")
    rec, arena, st, nd, cons = Ser.deserialize_status(gs, wire, n, offs)
    return st, rec.cpu().numpy(), arena.cpu().numpy(), nd, cons


@pytest.mark.gpu
@pytest.mark.parametrize("protocol", [0, 2])
def test_nested_program_parity(gpu, protocol, monkeypatch):
    monkeypatch.setenv("TGPU_JIT", "1")  # (the compile policy, whatever the run's)
    n = 40 * 1024
    schema, gs, Ser, wire, offs = _encode(gpu, protocol, n, 0x5eed + protocol)
    assert gs.compile(protocol)  # the nested program exists and compiles here
    st, rec, arena, nd, cons = _decode(Ser, gs, wire, n, offs, monkeypatch, True)
    assert st.code == 0 and nd == n and cons == wire.numel(), st.as_tuple()
    gst, grec, garena, gnd, gcons = _decode(Ser, gs, wire, n, offs, monkeypatch, False)
    assert gst.code == 0 and gnd == n
    assert np.array_equal(rec, grec)
    assert np.array_equal(arena, garena)
    w = wire.cpu().numpy().tobytes()
    ost, orec, oarena, ond, ocons = oracle.decode(schema, protocol, w, n,
                                                  offsets=offs.cpu().numpy().astype(np.uint64))
    assert ost.code == 0 and ond == n
    S = schema.size[0]
    assert np.array_equal(rec[: n * S], orec[: n * S])
    assert np.array_equal(arena[: oarena.size], oarena)


@pytest.mark.gpu
@pytest.mark.parametrize("protocol", [0, 2])
def test_nested_program_irregular_records(gpu, protocol, monkeypatch):
    """Records off the canonical form go to the general decoder: same status,
    records and arena as with the nested kernel off."""
    import torch

    n = 8 * 1024
    schema, gs, Ser, wire, offs = _encode(gpu, protocol, n, 0xbad + protocol)
    w = wire.cpu().numpy().copy()
    o = offs.cpu().numpy()
    # every 97th record: Binary — the items field's id turned into an unknown
    # one (header 0f 00 02 at +11 -> 0f 00 7f: the reader skips the list);
    # Compact — field 1's header 0x16 (i64) turned into 0x15 (i32: a type
    # mismatch, the varint skipped). Both stay valid streams.
    for i in range(0, n, 97):
        b = int(o[i])
        if protocol == 0:
            assert w[b + 11] == T_LIST and w[b + 13] == 2
            w[b + 13] = 0x7f
        else:
            assert w[b] == 0x16
            w[b] = 0x15
    t = torch.from_numpy(w).to(gpu)
    st, rec, arena, nd, cons = _decode(Ser, gs, t, n, offs, monkeypatch, True)
    gst, grec, garena, gnd, gcons = _decode(Ser, gs, t, n, offs, monkeypatch, False)
    assert st.as_tuple() == gst.as_tuple() and (nd, cons) == (gnd, gcons)
    assert np.array_equal(rec, grec)
    assert np.array_equal(arena, garena)


@pytest.mark.gpu
@pytest.mark.parametrize("protocol", [0, 2])
@pytest.mark.parametrize("outcap", ["default", "4096"])
def test_nested_program_encode_parity(gpu, protocol, outcap, monkeypatch):
    """The nested program's size / write passes: the general writer's bytes
    and offsets, and the oracle's encode of the same records. outcap 4096:
    the LDS output tile too small for any tile, every record written
    straight to the stream."""
    import torch

    if outcap != "default":
        monkeypatch.setenv("TGPU_NESTED_OUTCAP", outcap)

    n = 40 * 1024
    batch = bench.nested_batch(gpu, n, 0xe0c + protocol)
    schema, gs, Ser, wire, offs = _encode(gpu, protocol, n, 0, monkeypatch, True, batch)
    _, _, _, gwire, goffs = _encode(gpu, protocol, n, 0, monkeypatch, False, batch)
    assert torch.equal(wire, gwire) and torch.equal(offs, goffs)
    monkeypatch.setenv("TGPU_NESTED", "1")
    sz, total = Ser.encoded_size(gs, batch[1], n, list_base=batch[2])
    assert total == wire.numel()
    assert torch.equal(sz.to(offs.dtype)[: n + 1], offs[: n + 1])
    rec = batch[1].cpu().numpy()
    lb = batch[2].cpu().numpy()
    ost, owire, ooffs = oracle.encode(schema, protocol, rec, n, np.zeros(1, np.uint8), lb)
    assert ost.code == 0 and owire == wire.cpu().numpy().tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("protocol", [0, 2])
def test_nested_program_encode_size_limit(gpu, protocol, monkeypatch):
    """A list length above INT32_MAX (checked_container_size): the same
    WRITE_SIZE_LIMIT status, record and offset as the general writer."""
    from fbthrift_amd import serializer as SZ

    n = 1000
    schema, recs, lbase, *_ = bench.nested_batch(gpu, n, 0x51)
    m = schema.member[(0, 1)]
    recs.view(-1, schema.size[0])[613, m + 8: m + 12] = torch_u8([0, 0, 0, 0x80], gpu)
    gs = SZ.GpuSchema(schema)
    Ser = {0: SZ.BinarySerializer, 2: SZ.CompactSerializer}[protocol]
    import torch

    buf = torch.empty(1 << 20, dtype=torch.uint8, device=gpu)
    out = []
    for nested in ("1", "0"):
        monkeypatch.setenv("TGPU_JIT", "1")
        monkeypatch.setenv("TGPU_NESTED", nested)
        with pytest.raises(SZ.TProtocolException) as ei:
            Ser.serialize(gs, recs, n, list_base=lbase, out=buf, offsets=None)
        out.append(str(ei.value))
    assert out[0] == out[1] and "WRITE_SIZE_LIMIT" in out[0] and "613" in out[0], out


def torch_u8(v, dev):
    import torch

    return torch.tensor(v, dtype=torch.uint8, device=dev)


# ---- maps, sets and string elements: the golden nested schemas with every
# field unqualified (Item's optional double made unqualified), values from
# the same generators, the oracle's stream as the reference ------------------
def _unqualified_case(name, protocol, n):
    import copy
    import types

    import nested_helpers as nh
    import nestgen

    table = copy.deepcopy(nh.manifest()["nested_schemas"][name])
    for row in table[1]:
        row[3] = 0
    schema = Schema.from_table(table)
    gen = nestgen.NESTED_GENERATORS[name]
    values = [nestgen.to_json((T_STRUCT, 0), gen(i), table) for i in range(n)]
    c = types.SimpleNamespace(n=n, values=values, schema=schema, protocol=protocol,
                              layout=nh.Layout(schema, table))
    return c, nh.pack(c)


@pytest.mark.parametrize("name", ["structlist", "deepcont"])
def test_unqualified_nested_schemas_compile(name):
    c, _ = _unqualified_case(name, 0, 1)
    for protocol in (0, 2):  # compiled in one protocol, generated in the other
        rc, log = compile_check(c.schema, protocol, arch="gfx950" if protocol == 0 else "")
        assert rc == 0, log


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["structlist", "deepcont"])
@pytest.mark.parametrize("protocol", [0, 2])
def test_nested_program_maps_strings(gpu, name, protocol, monkeypatch):
    """list / set / map of structs, map<string, list<string>>,
    list<map<i32, string>>, map<i32, map<i32, Item>>, set<list<list<i64>>>,
    strings and list<i16> inside Items: the nested program's encode gives the
    oracle's bytes, its decode (indexed and unindexed) the oracle's records
    and arena."""
    import torch

    from fbthrift_amd import serializer as SZ

    monkeypatch.setenv("TGPU_JIT", "1")
    monkeypatch.setenv("TGPU_NESTED", "1")
    n = 3000
    c, (rec, sb, lb) = _unqualified_case(name, protocol, n)
    ost, owire, ooffs = oracle.encode(c.schema, protocol, rec, n, sb, lb)
    assert ost.code == 0
    gs = SZ.GpuSchema(c.schema)
    assert gs.compile(protocol)
    Ser = {0: SZ.BinarySerializer, 2: SZ.CompactSerializer}[protocol]
    t = lambda a: torch.from_numpy(np.array(a, copy=True)).to(gpu)
    wire, offs = Ser.serialize(gs, t(rec), n, t(sb), t(lb))
    assert wire.cpu().numpy().tobytes() == owire
    assert np.array_equal(offs.cpu().numpy().astype(np.uint64), ooffs)
    S = c.layout.size[0]
    w = np.frombuffer(owire, np.uint8)
    for indexed in (True, False):
        o = offs if indexed else None
        grec, garena, st, nd, cons = Ser.deserialize_status(gs, t(w), n, o)
        dst, drec, darena, dnd, dcons = oracle.decode(c.schema, protocol, owire, n,
                                                      offsets=ooffs if indexed else None)
        assert st.code == 0 and nd == n and cons == len(owire), st.as_tuple()
        assert np.array_equal(grec.cpu().numpy()[: n * S], drec[: n * S])
        assert np.array_equal(garena.cpu().numpy()[: darena.size], darena)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["sparse", "strcont", "unions"])
def test_nested_program_compiles_on_device(gpu, name, monkeypatch):
    """Schemas without a canonical record program — optional fields
    ('sparse'), strings inside containers ('strcont') — get the nested record
    program on the device: the golden parity runs with TGPU_JIT=1
    (test_gpu_parity.py, codec fixture) decode and encode them through it."""
    import helpers

    from fbthrift_amd.serializer import GpuSchema

    monkeypatch.setenv("TGPU_JIT", "1")  # (the compile policy, whatever the run's)
    gs = GpuSchema(Schema.from_table(helpers.manifest()["schemas"][name]))
    assert gs.compile(0) and gs.compile(2)


@pytest.mark.gpu
@pytest.mark.parametrize("protocol", [0, 2])
def test_nested_program_large_root_record(gpu, protocol, monkeypatch):
    """A flat schema of 44 optional string fields (a 720-byte root record:
    44 spans + 44 isset bytes) has a nested program but no canonical one; at
    64 Ki records (the compile threshold) its decode must not ask for a record
    tile beyond the LDS: the record tile is dropped and records go straight to
    HBM. Same records as the oracle, indexed and unindexed."""
    import torch

    import helpers
    from fbthrift_amd import serializer as SZ

    monkeypatch.setenv("TGPU_JIT", "1")
    monkeypatch.setenv("TGPU_NESTED", "1")
    nf, n = 44, 1 << 16
    schema = Schema.from_table([[[k, T_STRING, 0, 1, -1] for k in range(1, nf + 1)]])
    assert schema.size[0] >= 700
    rng = np.random.default_rng(0x1a7e + protocol)
    vals = {}
    for k in range(nf):
        present = rng.random(n) < 0.5
        lens = np.where(present, rng.integers(0, 5, n), 0)
        vals["%d.set" % k] = present.astype(np.uint8)
        vals["%d.len" % k] = lens
        vals["%d.data" % k] = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
    rec, sarena, _ = helpers.pack(schema, vals, n)
    rec = rec.view(np.uint8).reshape(-1)
    ost, owire, ooffs = oracle.encode(schema, protocol, rec, n, sarena)
    assert ost.code == 0
    gs = SZ.GpuSchema(schema)
    Ser = {0: SZ.BinarySerializer, 2: SZ.CompactSerializer}[protocol]
    t = lambda a: torch.from_numpy(np.array(a, copy=True)).to(gpu)
    wire, offs = Ser.serialize(gs, t(rec), n, t(sarena))
    assert wire.cpu().numpy().tobytes() == owire
    w = np.frombuffer(owire, np.uint8)
    S = schema.size[0]
    for indexed in (True, False):
        grec, _, st, nd, cons = Ser.deserialize_status(gs, t(w), n, offs if indexed else None)
        dst, drec, _, dnd, _ = oracle.decode(schema, protocol, owire, n,
                                             offsets=ooffs if indexed else None)
        assert st.code == 0 and nd == n and cons == len(owire), st.as_tuple()
        assert np.array_equal(grec.cpu().numpy()[: n * S], drec[: n * S])
