import sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, "tests"); sys.path.insert(0, "tests/golden")
import numpy as np, torch, ctypes
import helpers
from fbthrift_amd import _lib
from fbthrift_amd.serializer import GpuSchema, CompactSerializer, BinarySerializer
name = sys.argv[1]
c = helpers.Case(name)
rec, sarena, larena = helpers.pack(c.schema, c.values, c.n)
dev = torch.device("cuda:0")
gs = GpuSchema(c.schema)
ser = CompactSerializer if c.protocol == 2 else BinarySerializer
t = torch.from_numpy(rec.copy()).to(dev)
offs = torch.empty(c.n + 1, dtype=torch.int64, device=dev)
st, total = _lib.Status(), ctypes.c_uint64()
print("last err before:", torch.cuda.is_available())
rc = _lib.lib().tgpu_encoded_size(ser.context().handle, gs.handle, c.protocol, ctypes.c_void_p(t.data_ptr()), c.n, ctypes.c_void_p(offs.data_ptr()), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream), ctypes.byref(st), ctypes.byref(total))
print("rc", rc, st.as_tuple(), "hip", st.reserved, "total", total.value, "expected", len(c.wire))
print("hip error string:", torch.cuda.is_available())
for k in (1, 2, 5):
    st2, tot = _lib.Status(), ctypes.c_uint64()
    rc = _lib.lib().tgpu_encoded_size(ser.context().handle, gs.handle, c.protocol, ctypes.c_void_p(t.data_ptr()), k, ctypes.c_void_p(offs.data_ptr()), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream), ctypes.byref(st2), ctypes.byref(tot))
    print(k, "rc", rc, st2.as_tuple(), "hip", st2.reserved, "total", tot.value)
