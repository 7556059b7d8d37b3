"""Debug: index + unindexed decode of one golden case through the compiled
kernels (TGPU_JIT=1), printing the status and its HIP error."""
import os
import sys

sys.path.insert(0, os.getcwd())
sys.path.insert(0, "tests")
sys.path.insert(0, "tests/golden")
os.environ.setdefault("TGPU_JIT", "1")
os.environ.setdefault("TGPU_JIT_VERBOSE", "1")
import torch  # noqa: E402

import helpers  # noqa: E402
from fbthrift_amd.serializer import BinarySerializer, CompactSerializer, GpuSchema  # noqa: E402

for name in sys.argv[1:]:
    c = helpers.Case(name)
    ser = CompactSerializer if c.protocol == 2 else BinarySerializer
    gs = GpuSchema(c.schema)
    import numpy as np
    w = torch.from_numpy(np.frombuffer(c.wire, np.uint8).copy()).to("cuda:0")
    try:
        offs, n, first, last, st = ser.index_stream(gs, w)
        print(name, "index", st.as_tuple(), "hip", st.reserved, n, first, last, flush=True)
    except Exception as e:  # noqa: BLE001
        print(name, "index raised", e, getattr(getattr(e, "status", None), "reserved", None),
              flush=True)
    try:
        rec, arena, st, nd, cons = ser.deserialize_status(gs, w, c.n)
        print(name, "decode", st.as_tuple(), "hip", st.reserved, nd, cons, flush=True)
    except Exception as e:  # noqa: BLE001
        print(name, "decode raised", e, flush=True)
