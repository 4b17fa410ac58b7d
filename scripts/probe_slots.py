"""Dev probe (GPU box): HBM rate of a slotted copy (scripts/probe_slots.hip).
1M slots; per case the slot stride, blocks read and blocks written per slot.
`useful` counts 1360 B read + 1360 B written per slot (what the obfuscation
kernel's algorithmic bytes count for a 1358-byte datagram); `moved` counts
the blocks the case touches.  Interleaved rounds, median."""
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

n = 1 << 20
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
src = torch.randint(0, 256, (n * 2048 + 4096,), dtype=torch.uint8, device="cuda")
dst = torch.empty(n * 2048 + 4096, dtype=torch.uint8, device="cuda")
s = torch.cuda.current_stream().cuda_stream
# (name, stride, blocks read, blocks written, slots per wave, U)
cases = [
    ("dense 1360", 1360, 85, 85, 16, 4),
    ("slot2048 w1344 (64-B sectors)", 2048, 84, 84, 16, 4),
    ("slot2048 w1280 (128-B lines)", 2048, 80, 80, 16, 4),
    ("slot2048 w1360", 2048, 85, 85, 16, 4),
    ("slot2048 w1408 (lines)", 2048, 85, 88, 16, 4),
    ("slot2048 r1408 w1408", 2048, 88, 88, 16, 4),
    ("slot2048 w1536", 2048, 85, 96, 16, 4),
    ("slot2048 w2048", 2048, 85, 128, 16, 4),
    ("slot2048 r2048 w2048", 2048, 128, 128, 16, 4),
    ("slot1408 w1360", 1408, 85, 85, 16, 4),
    ("slot1408 w1408", 1408, 85, 88, 16, 4),
    ("slot1536 w1360", 1536, 85, 85, 16, 4),
    ("slot1536 w1408", 1536, 85, 88, 16, 4),
    ("slot2048 w1360 U8", 2048, 85, 85, 16, 8),
    ("slot2048 w1408 U8", 2048, 85, 88, 16, 8),
    ("dense 1360 U8", 1360, 85, 85, 16, 8),
    ("slot2048 w1360 per24", 2048, 85, 85, 24, 4),
    ("slot2048 w1408 per24", 2048, 85, 88, 24, 4),
]


def run(c, steps=10):
    _, stride, nbr, nbw, per, u = c
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for _ in range(2):
        assert L.slots_run(src.data_ptr(), dst.data_ptr(), n, stride, nbr, nbw, per, u, s) == 0
    ev[0].record()
    for _ in range(steps):
        L.slots_run(src.data_ptr(), dst.data_ptr(), n, stride, nbr, nbw, per, u, s)
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / steps * 1e3


res = {c[0]: [] for c in cases}
for r in range(rounds):
    for c in cases:
        res[c[0]].append(run(c))
for c in cases:
    us = statistics.median(res[c[0]])
    name, stride, nbr, nbw, per, u = c
    useful = n * 2 * 1360
    moved = n * 16 * (nbr + nbw)
    print(json.dumps(dict(case=name, us=round(us, 1), useful_TBps=round(useful / us / 1e6, 3),
                          moved_TBps=round(moved / us / 1e6, 3),
                          all=[round(x, 1) for x in res[name]])), flush=True)
