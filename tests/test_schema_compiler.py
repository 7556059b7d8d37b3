"""The schema compiler (tgpu_jit.cpp) on a GPU-less host: the kernels it
generates for a schema compile for gfx950 with hipRTC (all three kernel
groups: decode, encode, index); schemas without one (optional fields,
containers of structs, unions, bools inside maps) compile a nested record
program instead; recursive schemas an unrolled one (reader and writer).
GPU parity of
the compiled kernels is in test_gpu_parity.py (TGPU_JIT=1 runs). Compiles
cost seconds each, so the CPU suite covers the three BASELINE config schemas
in their benchmarked protocol plus the bool/long-form-id heavy 'scalars'."""
import pytest

import helpers
from fbthrift_amd.schema import Schema
from fbthrift_amd.serializer import compile_check

M = helpers.manifest()["schemas"]


@pytest.mark.parametrize("name,protocol", [("flat8", 0), ("mixed", 2), ("nested", 0),
                                           ("scalars", 2)])
def test_schema_kernels_compile(name, protocol):
    rc, log = compile_check(Schema.from_table(M[name]), protocol)
    assert rc == 0, log


def test_optional_fields_compile_nested_program():
    # optional fields: no canonical record program, but a nested record
    # program (field headers checked at run time, tgpu_nested.h)
    rc, log = compile_check(Schema.from_table(M["sparse"]), 2)
    assert rc == 0, log


def test_unions_compile_nested_program():
    rc, log = compile_check(Schema.from_table(M["unions"]), 2)
    assert rc == 0, log


@pytest.mark.parametrize("protocol", [0, 2])
def test_bool_map_keys_compile(protocol):
    """Bools inside maps are nested-program leaves since round 4 (Compact's
    container bool byte 1 / 2, Binary's 0 / 1, CompactProtocol-inl.h:692-701)."""
    rc, log = compile_check(Schema.from_table(M["maps"]), protocol,
                            arch="gfx950" if protocol == 2 else "")
    assert rc == 0, log


@pytest.mark.parametrize("name,src,dst", [("mixed", 2, 0), ("nested", 0, 2)])
def test_transcoding_pair_compiles(name, src, dst):
    """The transcoder's program pair (JIT_XCODE: size, write and single-pass
    tiles, tgpu_xcode.h) for BASELINE configs 3 and 4 in their transcoding
    direction."""
    from fbthrift_amd.serializer import transcode_compile_check

    rc, log = transcode_compile_check(Schema.from_table(M[name]), src, dst)
    assert rc == 0, log


@pytest.mark.parametrize("protocol", [0, 2])
def test_recursive_program_compiles_with_its_writer(protocol, monkeypatch):
    """struct Tree {1: i32 v, 2: list<Tree> kids}, unrolled 4 levels: since
    round 5 the nested program of a recursive schema carries its writer too
    (size / write passes deferring the records nesting deeper to the general
    writer's deep pass, TGPU_NESTED_DEFER)."""
    monkeypatch.setenv("TGPU_NESTED_UNROLL", "4")
    tree = [[[1, 8, 0, 0, -1], [2, 15, 12, 0, 0]]]
    rc, log = compile_check(Schema.from_table(tree), protocol)
    assert rc == 0, log


@pytest.mark.parametrize("define", [
    "#define TGPU_SETTLE_WAIT_ONLY 1",
    "#define TGPU_SETTLE_VMLGKM 1",
    '#define TGPU_STAGE_BARRIER "s_waitcnt vmcnt(0) lgkmcnt(0)\\n\\ts_barrier"',
])
def test_settle_diagnostic_variants_compile(define, monkeypatch):
    """The LDS-DMA settle's diagnostic variants (DESIGN.md §4.2, round 5:
    the staging's wait and barrier forms A/B'd on config 5 through
    TGPU_JIT_DEFINES) stay buildable: config 5's schema, all kernel groups."""
    monkeypatch.setenv("TGPU_JIT_DEFINES", define)
    rc, log = compile_check(Schema.from_table(M["mixed"]), 2)
    assert rc == 0, log
