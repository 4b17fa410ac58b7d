"""Dev probe (GPU box): the engine's launch on page-locked, GPU-mapped
blocks (zero copy: the kernel reads and writes the datagrams over PCIe),
by batch size -- what bounds the GPU route of the packet conn engine
(DESIGN.md 9.5).  Datagrams of 1,350 B in 2,048-B slots, in place behind
8 bytes of salt headroom, SQOBFS_FLAG_OUT_BLOCKS | SQOBFS_FLAG_DEVICE_SALT,
descriptor arrays in page-locked memory too (the engine's layout); each
size timed by HIP events over `reps` back-to-back launches, and the same
batch in device memory beside it.  Prints one JSON line per size."""
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "sing-quic_amd"))
import sqobfs  # noqa: E402

L, SLOT, S = 1350, 2048, 8
dev = torch.device("cuda", 0)
torch.cuda.init()
ctx = sqobfs.Context(0)
ctx.salt_key(bytes(range(32)), 0)
kr = sqobfs.Keyring(ctx, 0, [b"sing-quic-mi355x-bench-psk"])
stream = torch.cuda.current_stream(dev)
s = stream.cuda_stream
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
flags = sqobfs.FLAG_OUT_BLOCKS | sqobfs.FLAG_DEVICE_SALT
for n in (256, 1024, 4096, 16384, 65536):
    ctx.unit_packets = sqobfs.unit_packets_for(n * L, n)
    blk = sqobfs.PinnedArray(ctx, n * SLOT + n * 24)
    a = blk.array
    a[: n * SLOT] = 7
    meta = a[n * SLOT:]
    in_off = np.frombuffer(meta[: 8 * n].data, np.uint64)
    out_off = np.frombuffer(meta[8 * n: 16 * n].data, np.uint64)
    ln = np.frombuffer(meta[16 * n: 20 * n].data, np.uint32)
    olen = np.frombuffer(meta[20 * n: 24 * n].data, np.uint32)
    slots = a[: n * SLOT]
    in_off[:] = np.arange(n, dtype=np.uint64) * SLOT + S
    out_off[:] = np.arange(n, dtype=np.uint64) * SLOT
    ln[:] = L
    hb = sqobfs.make_batch(n, slots, in_off, ln, slots, out_off, olen, None, None, flags=flags)
    # the same in device memory
    d = torch.full((n * SLOT,), 7, dtype=torch.uint8, device=dev)
    di = torch.from_numpy(in_off.astype(np.int64)).to(dev)
    do = torch.from_numpy(out_off.astype(np.int64)).to(dev)
    dl = torch.full((n,), L, dtype=torch.int32, device=dev)
    dol = torch.zeros(n, dtype=torch.int32, device=dev)
    db = sqobfs.make_batch(n, d, di, dl, d, do, dol, None, None, flags=flags)
    res = {"packets": n, "payload_MB": round(n * L / 1e6, 3)}
    for name, b in (("mapped", hb), ("device", db)):
        for _ in range(3):
            sqobfs.launch(ctx, kr, sqobfs.OBFUSCATE, b, s)
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            sqobfs.launch(ctx, kr, sqobfs.OBFUSCATE, b, s)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        us = e0.elapsed_time(e1) * 1e3 / reps
        res[name + "_us"] = round(us, 1)
        res[name + "_payload_GBps"] = round(n * L / us / 1e3, 2)
    res["mapped_ok"] = bool((olen == L + S).all())
    print(json.dumps(res), flush=True)
    del d, di, do, dl, dol
    blk.free()
kr.close()
ctx.close()
