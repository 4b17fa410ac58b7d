"""Dev probe (GPU box): sqobfs_run_host end-to-end rate of several library
builds in one process, interleaved (bench.e2e_rate's three host-buffer modes).
usage: e2e_ab.py ROUNDS PACKETS lib1.so lib2.so ..."""
import os
import statistics
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
for p in (REPO, os.path.join(REPO, "sing-quic_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402
import sqobfs  # noqa: E402
import bench  # noqa: E402

rounds, n = int(sys.argv[1]), int(sys.argv[2])
libs = []
for path in sys.argv[3:]:
    sqobfs._lib = sqobfs.load(path)
    ctx = sqobfs.Context(0)
    kr = sqobfs.Keyring(ctx, sqobfs.SALAMANDER, [bench.PSK])
    libs.append((os.path.basename(os.path.dirname(path)) or os.path.basename(path), sqobfs._lib, ctx, kr))
res = {}
for r in range(rounds):
    for name, lib, ctx, kr in libs:
        sqobfs._lib = lib
        out = bench.e2e_rate(torch, sqobfs, ctx, kr, 0, n, 1350)
        for mode in ("pageable", "pinned", "pinned_out_uninit", "slots2048"):
            res.setdefault((name, mode), []).append(out[mode]["GiB_s_payload"])
for (name, mode), v in res.items():
    print(f"{name:20s} {mode:18s} median {statistics.median(v):7.2f} GiB/s  all {v}", flush=True)
