"""Dev probe (GPU box): does a persistent grid (waves loop over units) copy
faster than one wave per unit?  Dense 1M x 1360-byte copy (scripts/probe_slots.hip),
16 packets per unit, the resident waves capped at 3 per SIMD with dynamic LDS
like the obfuscation kernel.  Interleaved rounds, median."""
import ctypes
import json
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L = ctypes.CDLL(os.path.join(REPO, "build", "libsqslots.so"))
L.slots_run.argtypes = [ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_uint32] * 5 + [
    ctypes.c_int, ctypes.c_void_p]
L.slots_persist_run.argtypes = [ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_uint32] * 6 + [
    ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
L.slots_set_lds.argtypes = [ctypes.c_uint32]

n = 1 << 20
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
src = torch.randint(0, 256, (n * 1360 + 4096,), dtype=torch.uint8, device="cuda")
dst = torch.empty(n * 1360 + 4096, dtype=torch.uint8, device="cuda")
ctr = torch.zeros(64, dtype=torch.int32, device="cuda")
s = torch.cuda.current_stream().cuda_stream
CUS = 256
# (name, lds per group, mode, waves per SIMD for the persistent grid)
cases = [("grid, 3/SIMD", 24 * 1024, 0, 0), ("persistent static, 3/SIMD", 24 * 1024, 1, 3),
         ("persistent dynamic, 3/SIMD", 24 * 1024, 2, 3),
         ("grid, 2/SIMD", 36 * 1024, 0, 0), ("persistent dynamic, 2/SIMD", 36 * 1024, 2, 2),
         ("grid, uncapped", 0, 0, 0), ("persistent dynamic, 4/SIMD", 0, 2, 4)]


def launch(c):
    _, lds, mode, w = c
    L.slots_set_lds(lds)
    if mode == 0:
        return L.slots_run(src.data_ptr(), dst.data_ptr(), n, 1360, 85, 85, 16, 4, s)
    return L.slots_persist_run(src.data_ptr(), dst.data_ptr(), n, 1360, 85, 85, 16,
                               CUS * 4 * w, mode, ctr.data_ptr(), s)


def run(c, steps=10):
    for _ in range(3):
        assert launch(c) == 0
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(steps):
        launch(c)
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / steps * 1e3


# correctness of the persistent loops: every unit copied
ref = None
for c in cases:
    dst.zero_()
    assert launch(c) == 0
    torch.cuda.synchronize()
    if ref is None:
        ref = dst.clone()
    elif not torch.equal(ref, dst):
        print("MISMATCH", c[0], flush=True)
        sys.exit(1)
res = {c[0]: [] for c in cases}
for r in range(rounds):
    for c in cases:
        res[c[0]].append(run(c))
for c in cases:
    us = statistics.median(res[c[0]])
    print(json.dumps(dict(case=c[0], us=round(us, 1), TBps=round(2 * n * 1360 / us / 1e6, 3),
                          all=[round(x, 1) for x in res[c[0]]])), flush=True)
