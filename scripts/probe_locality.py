"""Run the dev locality probes (scripts/probe_locality.hip): copy-XOR of the
configs[1] byte volume with per-wave vs per-block-interleaved walk orders.
TB/s counts read + write bytes."""
import ctypes
import json
import os

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L = ctypes.CDLL(os.path.join(REPO, "build", "libsqprobe2.so"))
L.probe2_run.argtypes = [ctypes.c_int] * 3 + [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                              ctypes.c_uint64, ctypes.c_void_p]

nbytes = 1424000000 // 16 * 16
src = torch.randint(0, 256, (nbytes + 64,), dtype=torch.uint8, device="cuda")
dst = torch.empty(nbytes + 64, dtype=torch.uint8, device="cuda")
s = torch.cuda.current_stream().cuda_stream
import sys
L.probe_pers_run.argtypes = [ctypes.c_int] * 4 + [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                                  ctypes.c_void_p]
cases = []
pers = sys.argv[1:2] == ["pers"]
glds = sys.argv[1:2] == ["glds"]
L.probe_glds_run.argtypes = [ctypes.c_int] * 2 + [ctypes.c_void_p, ctypes.c_void_p,
                                                  ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p]
for reg in (() if pers or glds else (4352, 10880, 21760, 43520, 87040)):
    for mode in (0, 1, 2):
        for u, bs in ((4, 256), (6, 256), (8, 256), (4, 512), (6, 512), (4, 1024)):
            if mode == 0 and bs != 256:
                continue
            cases.append((mode, u, bs, reg))
res = []


def timeit(fn):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 10 * 1e3


if glds:
    for reg in (4352, 21760, 43520, 87040):
        for u, aux in ((4, 0), (4, 2), (6, 2), (8, 0), (8, 2)):
            us = timeit(lambda: L.probe_glds_run(u, aux, src.data_ptr(), dst.data_ptr(), nbytes,
                                                 reg, s))
            r = dict(kind="glds", U=u, aux=aux, region=reg, us=round(us, 1),
                     TBps=round(2 * nbytes / us / 1e6, 3))
            res.append(r)
            print(json.dumps(r), flush=True)
        for u in (4, 8):
            us = timeit(lambda: L.probe2_run(0, u, 256, src.data_ptr(), dst.data_ptr(), nbytes,
                                             reg, s))
            r = dict(kind="vgpr", U=u, region=reg, us=round(us, 1),
                     TBps=round(2 * nbytes / us / 1e6, 3))
            res.append(r)
            print(json.dumps(r), flush=True)
if pers:
    for nb in (512, 1024, 2048, 4096):
        for mode, u, d in ((3, 6, 0), (4, 6, 0), (3, 6, 200), (4, 6, 200), (3, 4, 0), (3, 8, 0)):
            args = (mode, u, d, nb, src.data_ptr(), dst.data_ptr(), nbytes, s)
            assert L.probe_pers_run(*args) == 0
            for _ in range(3):
                L.probe_pers_run(*args)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                L.probe_pers_run(*args)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / 10 * 1e3
            moved = 2 * (nbytes // 1360 * 1360)
            r = dict(mode=mode, U=u, dummy=d, nb=nb, us=round(us, 1), TBps=round(moved / us / 1e6, 3))
            res.append(r)
            print(json.dumps(r), flush=True)
for mode, u, bs, reg in cases:
    args = (mode, u, bs, src.data_ptr(), dst.data_ptr(), nbytes, reg, s)
    if L.probe2_run(*args) != 0:
        print("skip", mode, u, bs, reg)
        continue
    for _ in range(3):
        L.probe2_run(*args)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        L.probe2_run(*args)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 10 * 1e3
    r = dict(mode=mode, U=u, bs=bs, region=reg, us=round(us, 1), TBps=round(2 * nbytes / us / 1e6, 3))
    res.append(r)
    print(json.dumps(r), flush=True)
print("best:", json.dumps(sorted(res, key=lambda r: r["us"])[:8]))
