"""Adversarial index sweep: 1 Mi CompactV1 records
of the nested schema, first-byte filter off (TGPU_INDEX_HMASK=0); with the
V1 program, then program-less (field 1 optional, TGPU_NESTED=0) under the
default sizing and forced chunk / reach settings (TGPU_INDEX_CHUNK,
TGPU_INDEX_SPEC_REACH). Records are compared with the oracle's. GPU only."""
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import datagen  # noqa: E402
from fbthrift_amd.schema import Schema  # noqa: E402
from fbthrift_amd.serializer import CompactV1Serializer as S, GpuSchema  # noqa: E402

n = 1 << 20
lib = ctypes.CDLL(os.path.join(ROOT, "tools", "build", "libtgpu_datagen.so"))


def stream(optional):
    table = [[list(r) for r in t] for t in datagen.SCHEMAS["nested"]]
    if optional:
        table[0][0][3] = 1
    schema = Schema.from_table(table)
    rs = schema.record_size
    recs = torch.empty(n * rs, dtype=torch.uint8, device="cuda")
    side = torch.empty(n * 64, dtype=torch.uint8, device="cuda")
    assert lib.tgpu_gen_nested_packed(ctypes.c_uint64(datagen.SEED), ctypes.c_uint64(0),
                                      ctypes.c_uint64(n), ctypes.c_void_p(recs.data_ptr()),
                                      ctypes.c_void_p(side.data_ptr()), None) == 0
    gs = GpuSchema(schema)
    wire, _ = S.serialize(gs, recs, n, list_base=side)
    torch.cuda.synchronize()
    return schema, gs, recs, wire


def run(gs, wire, ref, env):
    for k in ("TGPU_INDEX_SPEC_REACH", "TGPU_INDEX_XREACH", "TGPU_INDEX_CHUNK"):
        os.environ.pop(k, None)
    os.environ.update(env)
    S.deserialize_status(gs, wire, n)
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(2):
        t0 = time.perf_counter()
        grec, garena, gst, gnd, gcons = S.deserialize_status(gs, wire, n)
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    ok = gst.code == 0 and gnd == n and (ref is None or torch.equal(grec[: ref.numel()], ref))
    print("%-60s %9.2f ms ok=%s %s" % (env, best * 1e3, ok, S.context().index_stats()), flush=True)


os.environ["TGPU_INDEX_HMASK"] = "0"
schema, gs, recs, wire = stream(False)
print("program stream: %d bytes" % wire.numel(), flush=True)
ref = S.deserialize_status(gs, wire, n)[0].clone()
run(gs, wire, ref, {})
os.environ["TGPU_NESTED"] = "0"
schema, gs, recs, wire = stream(True)
print("programless stream: %d bytes" % wire.numel(), flush=True)
os.environ["TGPU_INDEX_EXHAUSTIVE"] = "0"
from oracle import oracle  # noqa: E402
ost, orec, _, ond, _ = oracle.decode(schema, 0x102, wire.cpu().numpy().tobytes(), n)
assert ost.code == 0 and ond == n
ref = torch.from_numpy(np.ascontiguousarray(orec[: n * schema.record_size])).cuda()
for env in ({},
            {"TGPU_INDEX_SPEC_REACH": "1024"},
            {"TGPU_INDEX_SPEC_REACH": "256"},
            {"TGPU_INDEX_SPEC_REACH": "1024", "TGPU_INDEX_CHUNK": "1024"},
            {"TGPU_INDEX_SPEC_REACH": "256", "TGPU_INDEX_CHUNK": "1024"},
            {"TGPU_INDEX_SPEC_REACH": "512", "TGPU_INDEX_CHUNK": "512"},
            {"TGPU_INDEX_SPEC_REACH": "256", "TGPU_INDEX_CHUNK": "512"},
            {"TGPU_INDEX_SPEC_REACH": "256", "TGPU_INDEX_CHUNK": "256"},
            {"TGPU_INDEX_SPEC_REACH": "128", "TGPU_INDEX_CHUNK": "256"},
            ):
    run(gs, wire, ref, env)
