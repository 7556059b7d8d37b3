#!/usr/bin/env python3
"""Runs the two calibration copies of tools/copy_ceiling.hip over 1 GiB (past
the 256 MiB Infinity Cache) so a rocprofv3 --pmc pass records FETCH_SIZE /
WRITE_SIZE for known byte counts: 1 GiB read + 1 GiB written per launch."""
import ctypes
import os

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NBYTES = 1 << 30

a = torch.randint(0, 255, (NBYTES,), dtype=torch.uint8, device="cuda")
b = torch.empty_like(a)
lib = ctypes.CDLL(os.path.join(ROOT, "tools", "build", "libcopyceil.so"))
assert lib.copy_calibrate(ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(b.data_ptr()),
                          ctypes.c_uint64(NBYTES)) == 0
assert torch.equal(a, b)
print("calibration bytes", NBYTES)
