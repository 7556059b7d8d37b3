"""`required` fields (TGPU_REQUIRED): written always, like unqualified fields
(serialize_field.whisker), read like them, and — in structs built with the
deprecated_enforce_required option (TGPU_STRUCT_ENFORCE_REQUIRED) — checked
after the struct's read (deserialize_struct.whisker:116-124). Decode
semantics are pinned by tests/corpus.py required_cases (oracle and GPU status
parity run over the whole corpus); here the writer."""
import numpy as np
import pytest

from fbthrift_amd.schema import Schema
from oracle import oracle

REQ_TABLE = [{"fields": [[1, 10, 0, 3, -1], [2, 8, 0, 1, -1], [3, 11, 0, 3, -1]],
              "enforce_required": True}]
PLAIN_TABLE = [[[1, 10, 0, 0, -1], [2, 8, 0, 1, -1], [3, 11, 0, 0, -1]]]


def records(schema, n):
    rec = np.zeros((n, schema.record_size), np.uint8)
    d = schema.dtype()
    v = rec.view(d).reshape(n)
    v["f1"] = np.arange(n) * 7 - 3
    v["f2"] = np.arange(n)
    v["f3"]["offset"] = 0
    v["f3"]["length"] = np.arange(n) % 5
    isset = v["__isset"]
    isset[:, 0] = 1
    isset[:, 1] = np.arange(n) % 2  # optional field 2 set on odd records
    isset[:, 2] = 1
    return rec.reshape(-1), np.frombuffer(b"abcdefgh", np.uint8).copy()


@pytest.mark.parametrize("proto", [0, 2])
def test_oracle_required_written_like_unqualified(proto):
    req, plain = Schema.from_table(REQ_TABLE), Schema.from_table(PLAIN_TABLE)
    rec, sb = records(req, 50)
    st, w1, _ = oracle.encode(req, proto, rec, 50, sb)
    st2, w2, _ = oracle.encode(plain, proto, rec, 50, sb)
    assert st.code == st2.code == 0 and w1 == w2
    # and it reads back with the enforcement satisfied
    st3, back, _, nd, _ = oracle.decode(req, proto, w1, 50)
    assert st3.code == 0 and nd == 50


@pytest.mark.gpu
@pytest.mark.parametrize("proto", [0, 2])
def test_gpu_required_roundtrip(gpu, codec, proto):
    import torch

    from fbthrift_amd import serializer as S

    ser = S.BinarySerializer if proto == 0 else S.CompactSerializer
    req = Schema.from_table(REQ_TABLE)
    n = 5000
    rec, sb = records(req, n)
    st, want, woffs = oracle.encode(req, proto, rec, n, sb)
    gs = S.GpuSchema(req)
    out, offs = ser.serialize(gs, torch.from_numpy(rec).to(gpu), n, torch.from_numpy(sb).to(gpu))
    assert bytes(out.cpu().numpy()) == want
    back, _, st2, nd, cons = ser.deserialize_status(gs, out, n)
    assert st2.code == 0 and nd == n and cons == len(want)
    ost, orec, _, _, _ = oracle.decode(req, proto, want, n)
    assert np.array_equal(back.cpu().numpy()[: n * req.record_size], orec[: n * req.record_size])
