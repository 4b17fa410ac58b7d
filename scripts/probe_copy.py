"""Run the dev bandwidth probes (scripts/probe_copy.hip) and print a table.
TB/s counts bytes moved: read+write for copies, read or write for the
one-sided patterns."""
import ctypes
import json
import os

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L = ctypes.CDLL(os.path.join(REPO, "build", "libsqprobe.so"))
L.probe_run.argtypes = [ctypes.c_int] * 4 + [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                             ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]

nbytes = 1426063360  # = 1M * 1360
src = torch.randint(0, 256, (nbytes + 64,), dtype=torch.uint8, device="cuda")
dst = torch.empty(nbytes + 64, dtype=torch.uint8, device="cuda")
s = torch.cuda.current_stream().cuda_stream
cases = []
L.probe_set_lds.argtypes = [ctypes.c_uint32]
import sys
mode = sys.argv[1] if len(sys.argv) > 1 else "sweep"
if mode == "groups":
    for lds in (0, 53000, 80000):
        cases.append((1, 8, 3, 8, 21760, 0, lds))
        cases.append((1, 16, 3, 8, 21760, 0, lds))
        cases.append((6, 6, 3, 8, 21760, 0, lds))
        cases.append((6, 6, 3, 8, 87040, 0, lds))
elif mode == "holes":
    for lds in (0, 80000):
        for u in (8, 16):
            for pat in (1, 4, 5):
                cases.append((pat, u, 3, 8, 21760, 0, lds))
            cases.append((4, u, 1, 8, 21760, 0, lds))
            cases.append((5, u, 1, 8, 21760, 0, lds))
elif mode == "occ":
    for lds in (0, 20480, 27000, 40000, 53000, 80000):
        for u in (8, 16):
            cases.append((1, u, 3, 8, 87040, 0, lds))
            cases.append((1, u, 3, 8, 21760, 0, lds))
        cases.append((0, 4, 3, 0, 0, 8192, lds))
else:
    for pol in (0, 1, 2, 3):
        for g in (1024, 2048, 8192):
            cases.append((0, 4, pol, 0, 0, g, 0))
        cases.append((0, 8, pol, 0, 0, 2048, 0))
        cases.append((0, 16, pol, 0, 0, 1024, 0))
        cases.append((0, 4, pol, 8, 0, 2048, 0))
        for u in (4, 8, 16):
            for reg in (87040, 21760):
                cases.append((1, u, pol, 8, reg, 0, 0))
        cases.append((2, 4, pol, 0, 0, 2048, 0))
        cases.append((2, 8, pol, 0, 0, 2048, 0))
        cases.append((3, 4, pol, 0, 0, 2048, 0))
        cases.append((3, 8, pol, 0, 0, 2048, 0))
for pat, u, pol, off, reg, grid, lds in cases:
    L.probe_set_lds(lds)
    rc = L.probe_run(pat, u, pol, off, src.data_ptr(), dst.data_ptr(), nbytes, reg, grid, s)
    if rc != 0:
        print("skip", pat, u, pol, off, rc)
        continue
    for _ in range(2):
        L.probe_run(pat, u, pol, off, src.data_ptr(), dst.data_ptr(), nbytes, reg, grid, s)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        L.probe_run(pat, u, pol, off, src.data_ptr(), dst.data_ptr(), nbytes, reg, grid, s)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 10 * 1e3
    moved = nbytes * (2 if pat in (0, 1, 4, 5, 6) else 1)
    print(json.dumps(dict(pat=pat, U=u, pol=pol, off=off, region=reg, grid=grid, lds=lds,
                          us=round(us, 1), TBps=round(moved / us / 1e6, 3))), flush=True)
