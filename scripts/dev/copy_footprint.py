"""Dev probe (GPU box): the copy control of VERDICT r5 item 2 -- a plain dense
dwordx4 copy (scripts/probe_copy.hip, nontemporal loads and stores) over the
same footprint as one obfuscation case of scripts/dev/case_run.py, launched
a few times in a process of its own, so a trace or a `--pmc` pass of this
process sees the copy alone.  The copy moves n x 1358 B (or 766 B) each way:
read + write = the case's algorithmic bytes (payload in, salt + payload out).
usage: copy_footprint.py CASE [LAUNCHES [PAT]]
PAT 1: per-wave contiguous 21,760-B regions (the kernel's unit shape), U 16;
PAT 0: grid-stride, 8,192 workgroups, U 4."""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))

import torch  # noqa: E402

CASES = {"F16": (1 << 20, 1358), "F4M": (1 << 22, 1358), "FB16": (2372000, 1358),
         "P28": (1 << 20, 766), "C28": (1 << 22, 766), "R28": (1 << 22, 766),
         "F16M": (1 << 24, 1358)}
case = sys.argv[1]
launches = int(sys.argv[2]) if len(sys.argv) > 2 else 12
pat = int(sys.argv[3]) if len(sys.argv) > 3 else 1
n, L = CASES[case]
nbytes = (n * L + 21759) // 21760 * 21760
lib = ctypes.CDLL(os.path.join(REPO, "build", "libsqprobe.so"))
lib.probe_run.argtypes = [ctypes.c_int] * 4 + [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                               ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]
lib.probe_set_lds.argtypes = [ctypes.c_uint32]
lib.probe_set_lds(0)
src = torch.randint(0, 256, (nbytes + 64,), dtype=torch.uint8, device="cuda")
dst = torch.empty(nbytes + 64, dtype=torch.uint8, device="cuda")
s = torch.cuda.current_stream().cuda_stream
u, off, reg, grid = (16, 8, 21760, 0) if pat == 1 else (4, 0, 0, 8192)
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * launches)]
for i in range(launches):
    ev[2 * i].record()
    rc = lib.probe_run(pat, u, 3, off, src.data_ptr(), dst.data_ptr(), nbytes, reg, grid, s)
    ev[2 * i + 1].record()
    if rc != 0:
        raise SystemExit(f"probe_run {rc}")
torch.cuda.synchronize()
us = sorted(ev[2 * i].elapsed_time(ev[2 * i + 1]) * 1e3 for i in range(launches // 2, launches))
med = us[len(us) // 2]
print(f"copy {case} pat {pat} bytes_each_way {nbytes} median_us {med:.1f} "
      f"TBps {2 * nbytes / med / 1e6:.3f} frac {2 * nbytes / med / 8e6:.4f}", flush=True)
