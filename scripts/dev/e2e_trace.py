"""Dev probe (GPU box): one host-staged batch shape (bench.e2e_all_ranks':
256K x 1,350 B in page-locked slots, SQOBFS_FLAG_OUT_UNINIT), run `reps`
times with a wall clock around each sqobfs_run_host, for a rocprofv3
--hip-trace --memory-copy-trace --kernel-trace run: where the wall time goes
(host work before the first copy, the copies, the drain).  Prints one JSON
line per call.  usage: e2e_trace.py [reps [packets]]"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
for p in (REPO, os.path.join(REPO, "sing-quic_amd")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401
import sqobfs  # noqa: E402
import bench  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 18
L, S = 1350, 8
ctx = sqobfs.Context(0)
kr = sqobfs.Keyring(ctx, sqobfs.SALAMANDER, [bench.PSK])
rng = np.random.Generator(np.random.PCG64(11))
nin, nout = n * bench.slot(L), n * bench.slot(L + S)
pd, po = sqobfs.PinnedArray(ctx, nin), sqobfs.PinnedArray(ctx, nout)
pd.array[:] = np.frombuffer(rng.bytes(nin), np.uint8)
in_off = np.arange(n, dtype=np.uint64) * bench.slot(L)
out_off = np.arange(n, dtype=np.uint64) * bench.slot(L + S)
salt = np.frombuffer(rng.bytes(n * S), np.uint8).copy()
hb = sqobfs.HostBatch(pd.array, in_off, np.full(n, L, np.uint32), po.array, out_off,
                      np.zeros(n, np.uint32), salt, flags=sqobfs.FLAG_OUT_UNINIT)
b = hb.as_batch()
for i in range(reps + 2):
    t0 = time.perf_counter_ns()
    sqobfs.run_host(ctx, kr, sqobfs.OBFUSCATE, b)
    t1 = time.perf_counter_ns()
    print(json.dumps({"call": i, "wall_us": (t1 - t0) / 1e3,
                      "GiB_s": n * L / ((t1 - t0) / 1e9) / 2**30}), flush=True)
assert int(hb.out_len[0]) == L + S and int(hb.out_len[-1]) == L + S
pd.free()
po.free()
