"""Per-wave phase timeline of obfs_kernel (dev tool; GPU box).

Needs a library built with -DSQ_TIMELINE=1 (scripts/variants.sh
tl:"-DSQ_TIMELINE=1"), selected with SQOBFS_LIB.  Runs one configuration a
few times and prints, for the last launch: phase durations per wave, the
number of waves in each phase over time, and the launch's tail (from the last
wave start to the end).  Stamps: 0 start, 1 descriptor, 2 plan, 3 contents
(key, images, byte-exact stores), 4 stream issued, 5 stores complete.
"""
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "sing-quic_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
import sqobfs  # noqa: E402

NST = 6


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "salamander-1m"
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if cfg.startswith("const:"):  # const:N:L -- N Salamander packets of L bytes
        _, n_s, l_s = cfg.split(":")
        kind, n, L, n_psk = 0, int(n_s), int(l_s), 1
    else:
        kind, n, L, n_psk = bench.CONFIGS[cfg]
    sh = bench.build_shard(torch, dev, kind, n, L, n_psk, 0, 1, cfg, "dense", 0)
    ctx = sqobfs.Context(0)
    kr = sqobfs.Keyring(ctx, kind, sh["psks"])
    s = torch.cuda.current_stream(dev).cuda_stream
    b = sqobfs.make_batch(n, sh["data"], sh["in_off"], sh["lens"], sh["out"], sh["out_off"],
                          sh["out_len"], sh["salt"], sh["psk_id"])
    d = sqobfs.OBFUSCATE
    per_pkt_salt = 2 * sh["S"]
    if len(sys.argv) > 3 and sys.argv[3] == "deobfuscate":
        # decode the obfuscated shard into a compact buffer, as bench.py does
        sqobfs.launch(ctx, kr, sqobfs.OBFUSCATE, b, s)
        wl = (sh["lens"] + sh["S"]).to(torch.int32)
        lens64 = sh["lens"].to(torch.int64)
        back_off = torch.cumsum(lens64, 0) - lens64 + 64
        back = torch.zeros(int(sh["payload_bytes"]) + 128, device=dev, dtype=torch.uint8)
        b = sqobfs.make_batch(n, sh["out"], sh["out_off"], wl, back, back_off, sh["out_len"],
                              None, sh["psk_id"])
        d = sqobfs.DEOBFUSCATE
        per_pkt_salt = sh["S"]
    lib = sqobfs.lib()
    lib.sqobfs_build_info.restype = ctypes.c_char_p
    info = lib.sqobfs_build_info().decode()
    # unit size: argv[2], else sized by bytes as bench.py does
    ctx.unit_packets = (int(sys.argv[2]) if len(sys.argv) > 2 and int(sys.argv[2]) else
                        sqobfs.unit_packets_for(sh["payload_bytes"], n, n_psk > 1))
    ppw = ctx.unit_packets
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(60):  # past the first-launch ramp
        sqobfs.launch(ctx, kr, d, b, s)
    e0.record()
    sqobfs.launch(ctx, kr, d, b, s)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3
    units = (n + ppw - 1) // ppw
    buf = np.zeros(units * NST, np.uint64)
    f = lib.sqobfs_debug_timeline
    f.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    assert f(buf.ctypes.data, buf.size) == 0
    t = buf.reshape(units, NST).astype(np.float64)
    t0 = t[:, 0].min()
    span_ticks = t[:, 5].max() - t0
    tick_us = us / span_ticks  # calibrate the clock against the event time
    t = (t - t0) * tick_us
    ph = np.diff(t, axis=1)
    names = ["desc", "plan", "contents", "stream", "drain"]
    out = {"build": info, "config": cfg, "direction": "deobfuscate" if d else "obfuscate", "unit_packets": ppw, "kernel_us": round(us, 1),
           "tick_ns": round(tick_us * 1e3, 3), "waves": units}
    out["phase_us"] = {nm: {"p10": round(float(np.percentile(ph[:, i], 10)), 2),
                            "median": round(float(np.median(ph[:, i])), 2),
                            "p90": round(float(np.percentile(ph[:, i], 90)), 2)}
                       for i, nm in enumerate(names)}
    life = t[:, 5] - t[:, 0]
    out["life_us"] = {"median": round(float(np.median(life)), 1),
                      "mean": round(float(life.mean()), 2),
                      "p90": round(float(np.percentile(life, 90)), 1)}
    # resident waves on average (Little: sum of lives / span), and the gaps
    # between a slot's waves are not visible here
    out["mean_resident_waves"] = round(float(life.sum() / (t[:, 5].max())), 1)
    out["last_start_us"] = round(float(t[:, 0].max()), 1)
    out["first_end_us"] = round(float(t[:, 5].min()), 1)
    out["tail_us"] = round(float(t[:, 5].max() - t[:, 0].max()), 1)
    # waves per phase over time, and the streaming share of the bytes
    bins = np.arange(0.0, float(t[:, 5].max()) + 10.0, 10.0)
    rows = []
    per_wave = (2 * sh["payload_bytes"] + per_pkt_salt * n) / units
    for lo in bins:
        hi = lo + 10.0
        pro = int(((t[:, 0] < hi) & (t[:, 3] > lo)).sum())
        strm = int(((t[:, 3] < hi) & (t[:, 5] > lo)).sum())
        # bytes: each wave's bytes spread evenly over its stream phase
        a = np.clip(np.minimum(t[:, 5], hi) - np.maximum(t[:, 3], lo), 0, None)
        dur = np.maximum(t[:, 5] - t[:, 3], 1e-3)
        tbps = float((a / dur).sum() * per_wave / 10e-6 / 1e12)
        rows.append((round(float(lo)), pro, strm, round(tbps, 2)))
    out["timeline_10us"] = rows
    print(json.dumps(out))
    ctx.close()


if __name__ == "__main__":
    main()
