#!/usr/bin/env python3
"""Benchmark: GiB/s payload obfuscated, device-resident, 1M x 1350 B Salamander.

One process per GPU (torchrun for N > 1).  Each rank owns an independent
shard of 1,048,576 packets x 1350 B (BASELINE.json configs[1]) already
resident in HBM; a step is one launch of the fused Salamander-obfuscate
kernel over the shard (key derivation for every packet + XOR stream + salt
prefix + out_len).  Packets are independent, so there is no data-path
collective: per-GPU work is fixed as N grows ("weak").  The timed region is
bracketed by a barrier + device sync on both sides, and the max over ranks is
taken.

Rank 0 prints ONE JSON line (bench contract) with two extra objects:
  roofline      the dominant kernel's achieved algorithmic HBM bandwidth
                (2L + 2S bytes per packet / avg kernel duration from HIP
                events on the launch stream) vs 8 TB/s; `traffic` = HBM bytes
                per launch from the rocprofv3 PMC pass committed under
                profiles/ (FETCH_SIZE x 2 + WRITE_SIZE, gfx950 correction), or
                null when absent.
  cpu_baseline  the CPU restatement (oracle/, "port": the Go reference cannot
                be built here) on BASELINE configs[0]: 65,536 x 1200 B
                Salamander obfuscate + deobfuscate round trips on the host
                cores, rank 0 at N = 1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "sing-quic_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

METRIC = "GiB/s payload obfuscated, device-resident, 1M×1350B Salamander @1/2/4/8 GPU"
PEAK_HBM_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
PSK = b"sing-quic-mi355x-bench-psk"  # SURVEY.md 8(d) default PSK (26 B)
SALT_KEY = bytes(range(32))  # --device-salt: fixed ChaCha20 key so the run is checkable

CONFIGS = {
    # name: (kind, packets per rank, payload len (None = ragged), n_psk)
    "salamander-1m": (0, 1 << 20, 1350, 1),         # configs[1]  (the metric)
    "xplus-1m": (1, 1 << 20, 1200, 1),              # configs[2]
    "salamander-ragged-4m": (0, 1 << 22, None, 1),  # configs[3]
    "salamander-16m-256psk": (0, 1 << 24, 1350, 256),  # configs[4], sharded over ranks
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="salamander-1m", choices=sorted(CONFIGS))
    ap.add_argument("--direction", default="obfuscate", choices=["obfuscate", "deobfuscate"])
    ap.add_argument("--cpu-seconds", type=float, default=2.0,
                    help="wall seconds of CPU-baseline sampling (x threads = CPU work)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--inproc", type=int, default=0,
                    help="in-process sharding: one process, K contexts over the visible GPUs "
                         "(context k on GPU k mod count), the config's batch cut by bytes "
                         "(sqobfs_shard_cuts) and launched with sqobfs_shard_launch")
    ap.add_argument("--inflight", type=int, default=2,
                    help="--inproc: shard steps in flight (1 = sqobfs_shard_run, a host round "
                         "trip per step)")
    ap.add_argument("--unit-packets", type=int, default=0,
                    help="obfuscation kernel unit size, packets per wavefront (0 = sized "
                         "from the batch's bytes by sqobfs_unit_packets_for_kind, as a caller "
                         "that built the batch does)")
    ap.add_argument("--warmup-s", type=float, default=0.15,
                    help="keep warming up (untimed) until this much wall time has passed "
                         "and at least --warmup launches ran: a fresh process's first "
                         "~25 launches run up to 10 %% slower (scripts/dev/warm_curve.py)")
    ap.add_argument("--packets", type=int, default=0,
                    help="dev: override the config's packet count (scaling probes; not a "
                         "BASELINE configuration)")
    ap.add_argument("--layout", default="dense",
                    choices=["dense", "slot16", "slot2048", "inplace"],
                    help="dense: wire-dense outputs, wire-sized input slots (default); "
                         "slot16: every packet in its own 16-byte-aligned slot (inputs and "
                         "outputs), launched with SQOBFS_FLAG_OUT_BLOCKS; slot2048: fixed "
                         "2048-byte slots on 128-byte lines (the Go Slots geometry), launched "
                         "with SQOBFS_FLAG_OUT_LINES (--slot-flag); "
                         "inplace: obfuscate in the input buffer (headroom layout, "
                         "vectorised WriteTo semantics)")
    ap.add_argument("--slot-bytes", type=int, default=2048,
                    help="slot stride of --layout slot2048 (a multiple of 16)")
    ap.add_argument("--slot-flag", default="lines", choices=["lines", "blocks"],
                    help="--layout slot2048: SQOBFS_FLAG_OUT_LINES (every output written "
                         "through to the end of its last 128-byte line; default) or "
                         "SQOBFS_FLAG_OUT_BLOCKS only (whole 16-byte blocks)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL) for the timing barrier/max; gloo lets several "
                         "ranks share one GPU in tests")
    ap.add_argument("--device-salt", action="store_true",
                    help="obfuscate with SQOBFS_FLAG_DEVICE_SALT (salts from the GPU's "
                         "ChaCha20 generator; 2L+S bytes per packet)")
    ap.add_argument("--quic", action="store_true",
                    help="also time QUIC ChaCha20-Poly1305 packet protection (seal/open of "
                         "1M short-header packets, SURVEY.md 8(f) rank 4)")
    ap.add_argument("--udp", action="store_true",
                    help="also time loopback UDP end to end through the batched socket "
                         "layer (sqobfs_udp_conn: sendmmsg/recvmmsg + GPU)")
    ap.add_argument("--latency", action="store_true",
                    help="also run sing-quic_amd/bin/lat_bench: per-datagram p50/p99 latency of "
                         "run_host, a mapped launch, the UDP endpoint and the packet conn "
                         "engine at batches of 1/16/64/256, and the engine's loopback rate")
    ap.add_argument("--e2e", action="store_true",
                    help="also time every mode of the host-staged path on rank 0 (pageable, "
                         "pinned, OUT_UNINIT, 2,048-B slots: e2e.modes)")
    ap.add_argument("--no-e2e", action="store_true",
                    help="skip the all-ranks host-staged batch after the timed region "
                         "(e2e.aggregate_gib_s / e2e.per_rank)")
    return ap.parse_args()


def slot(n: int, a: int = 16) -> int:
    return (n + a - 1) // a * a


def shard(config, n_total, world, rank):
    """(packets on this rank, global index of its first packet).  configs[4]
    is ONE 16M-packet batch split in contiguous shards over the ranks (strong
    scaling); every other config gives each GPU its own full batch (weak)."""
    if config == "salamander-16m-256psk":
        lo = n_total * rank // world
        hi = n_total * (rank + 1) // world
        return hi - lo, lo
    return n_total, rank * n_total


def build_shard(torch, dev, kind, n, L, n_psk, rank, world, config, layout, first=0,
                slot_bytes=2048):
    """Synthetic shard in HBM: payload/salt bytes from torch's Philox RNG
    seeded per rank; 16-byte-aligned slots for inputs and outputs."""
    import numpy as np
    S = 8 if kind == 0 else 16
    g = torch.Generator(device=dev)
    g.manual_seed(1 + 1000 * rank)
    if L is None:  # configs[3]: U[64, 1452], seed 4
        lens = torch.randint(64, 1453, (n,), generator=g, device=dev, dtype=torch.int64)
    else:
        lens = torch.full((n,), L, device=dev, dtype=torch.int64)
    # buffers start with 64 spare bytes (dev probe SQ_BENCH_LEAD: slot phase
    # within the 128-byte line); 2048-byte slots start
    # on 128-byte lines, as the Go Slots' page-aligned memory
    lead = int(os.environ.get("SQ_BENCH_LEAD", "128" if layout == "slot2048" else "64"))
    if layout in ("slot16", "slot2048"):
        # every packet in its own 16-byte-aligned slot (16 B-
        # aligned input offsets), or in fixed 2048-byte slots
        if layout == "slot16":
            in_slot = (lens + 15) // 16 * 16
            out_slot = (lens + S + 15) // 16 * 16
        else:
            in_slot = torch.full_like(lens, slot_bytes)
            out_slot = torch.full_like(lens, slot_bytes)
        in_off = torch.cumsum(in_slot, 0) - in_slot + lead
        out_off = torch.cumsum(out_slot, 0) - out_slot + lead
        if layout == "slot2048":
            # payload position in its slot (dev probe SQ_BENCH_SLOT_PHASE; S =
            # the engine's geometry: payload behind the salt headroom, so the
            # payload sits at the same 16-byte phase as in the wire slot)
            phase = int(os.environ.get("SQ_BENCH_SLOT_PHASE", "0"))
            assert 0 <= phase and phase % 4 == 0 and int(lens.max().item()) + phase <= slot_bytes
            in_off = in_off + phase
    else:
        # wire-dense: datagrams back to back (every output byte written);
        # each payload sits behind S bytes of headroom in a wire-sized input
        # slot, like a socket buffer reserved for the salt
        out_slot = lens + S
        out_off = torch.cumsum(out_slot, 0) - out_slot + lead
        in_slot = out_slot
        in_off = out_off + S
    # (+ 16: the slot phase probe shifts the last slot's gap past the end)
    in_bytes = int(in_slot.sum().item()) + 2 * lead + 16
    # dev probe of output placement (no effect measured)
    shift = int(os.environ.get("SQ_BENCH_OUT_SHIFT", "0")) if layout != "inplace" else 0
    out_off = out_off + shift
    out_bytes = int(out_slot.sum().item()) + 2 * lead + shift
    data = torch.randint(0, 256, (in_bytes,), generator=g, device=dev, dtype=torch.uint8)
    # non-payload input bytes (lead, headroom / slot padding) are zero, so a
    # decoded batch can be compared with `data` as a whole buffer
    gap = in_slot - lens
    slotted = layout in ("slot16", "slot2048")
    gstart = (in_off - S) if not slotted else (in_off + lens)
    gidx = torch.repeat_interleave(gstart, gap) + (
        torch.arange(int(gap.sum().item()), device=dev)
        - torch.repeat_interleave(torch.cumsum(gap, 0) - gap, gap))
    # host-side bounds check before the indexed write (an out-of-range index
    # faults the GPU)
    assert gidx.numel() == 0 or int(gidx.max().item()) < in_bytes
    data[gidx] = 0
    data[:lead] = 0
    data[int((in_off[-1] + lens[-1]).item()):] = 0
    salt = torch.randint(0, 256, (n * S,), generator=g, device=dev, dtype=torch.uint8)
    out = data if layout == "inplace" else torch.zeros(out_bytes, device=dev, dtype=torch.uint8)
    # packet index shard: global ids rank*n .. for psk_id = i mod 256
    psk_id = None
    if n_psk > 1:
        gid = torch.arange(first, first + n, device=dev, dtype=torch.int64)
        psk_id = (gid % n_psk).to(torch.int16)
    rng = np.random.Generator(np.random.PCG64(3))
    psks = [PSK] if n_psk == 1 else [
        rng.integers(0, 256, int(k), dtype=np.uint8).tobytes() for k in rng.integers(8, 65, n_psk)]
    return dict(lens=lens.to(torch.int32), in_off=in_off, out_off=out_off, data=data, salt=salt,
                out=out, out_len=torch.zeros(n, device=dev, dtype=torch.int32), psk_id=psk_id,
                psks=psks, S=S, payload_bytes=int(lens.sum().item()),
                inplace=layout == "inplace", slotted=slotted)


def sample_idx(n):
    return sorted(set([0, n - 1] + list(range(0, n, 4099))))[:400]


def save_samples(sh, n):
    """Host copies of the sampled input payloads (before any launch)."""
    lens = sh["lens"].cpu().numpy()
    in_off = sh["in_off"].cpu().numpy()
    return {i: sh["data"][int(in_off[i]):int(in_off[i]) + int(lens[i])].cpu().numpy().tobytes()
            for i in sample_idx(n)}


def spot_check(torch, sh, kind, n, direction_out, saved, launches):
    """Parity spot check vs the oracle on sampled packets (outside timing).
    In place, an even number of launches XORs the payload back to itself."""
    import numpy as np
    import oracle_lib as ol
    idx = sample_idx(n)
    S = sh["S"]
    lens = sh["lens"].cpu().numpy()
    in_off = sh["in_off"].cpu().numpy()
    out_off = sh["out_off"].cpu().numpy()
    data, salt, out = sh["data"], sh["salt"], direction_out
    ids = sh["psk_id"].cpu().numpy() if sh["psk_id"] is not None else None
    write = ol.salamander_write if kind == 0 else ol.xplus_write
    for i in idx:
        L = int(lens[i])
        p = saved[i]
        s = salt[i * S:(i + 1) * S].cpu().numpy().tobytes()
        psk = sh["psks"][int(ids[i]) if ids is not None else 0]
        w, _ = write(psk, s, p)
        if sh["inplace"] and launches % 2 == 0:
            w = s + p
        got = out[int(out_off[i]):int(out_off[i]) + L + S].cpu().numpy().tobytes()
        if got != w:
            return False
    return bool((sh["out_len"].cpu().numpy() == lens + S).all())


def kernel_name(kind: int, direction: int, multi: bool, ppw: int) -> str:
    """The dispatched template, obfs_kernel<KIND, DIR, MULTI, U, WPB>
    (sq_kernels.hip: U and waves per workgroup from the build), and the unit
    the launch used."""
    import re
    import sqobfs
    info = sqobfs.build_info()
    u = re.search(r"\bU=(\d+)", info)
    w = re.search(r"\bwpb=(\d+)", info)
    return (f"obfs_kernel<{kind}, {direction}, {'true' if multi else 'false'}, "
            f"{u.group(1) if u else '?'}, {w.group(1) if w else '?'}> at {ppw} packets per wave")


def max_over_ranks(torch, dist, x: float, dev) -> float:
    t = torch.tensor([x], device=dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(torch, dist, x: float, dev) -> float:
    t = torch.tensor([x], device=dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def cpu_baseline(seconds: float):
    """Oracle (CPU restatement, byte-at-a-time like salamander.go:51-53,62-64)
    on configs[0]: 65,536 x 1200 B obfuscate -> deobfuscate round trips."""
    import numpy as np
    import sqobfs
    import oracle_lib as ol
    n, L, S = 65536, 1200, 8
    threads = cpu_share()
    rng = np.random.Generator(np.random.PCG64(1))
    data = rng.integers(0, 256, n * L, dtype=np.uint8)
    salt = np.random.Generator(np.random.PCG64(2)).integers(0, 256, n * S, dtype=np.uint8)
    in_off = (np.arange(n, dtype=np.uint64) * L)
    lens = np.full(n, L, np.uint32)
    wire = np.zeros(n * (L + S), np.uint8)
    w_off = np.arange(n, dtype=np.uint64) * (L + S)
    w_len = np.zeros(n, np.uint32)
    back = np.zeros(n * L, np.uint8)
    b_len = np.zeros(n, np.uint32)
    obf = sqobfs.HostBatch(data, in_off, lens, wire, w_off, w_len, salt)
    deo = sqobfs.HostBatch(wire, w_off, np.full(n, L + S, np.uint32), back, in_off, b_len)
    def timed(nthreads, secs):
        t_ob = t_de = 0.0
        passes = 0
        t_end = time.perf_counter() + secs
        while passes < 2 or time.perf_counter() < t_end:
            t0 = time.perf_counter()
            ol.batch_run(0, 0, [PSK], obf, nthreads=nthreads)
            t1 = time.perf_counter()
            ol.batch_run(0, 1, [PSK], deo, nthreads=nthreads)
            t2 = time.perf_counter()
            t_ob += t1 - t0
            t_de += t2 - t1
            passes += 1
        gib = n * L * passes / 2**30
        return gib / t_ob, gib / t_de, gib / (t_ob + t_de), passes, t_ob + t_de

    ob, de, rt, passes, wall = timed(threads, seconds)
    ok = bool(np.array_equal(back, data))
    ob1, de1, rt1, _, wall1 = timed(1, min(seconds, 2.0))  # one core: the per-core rate
    host = os.cpu_count() or threads
    share = {}
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and 0 < int(omp) < threads:
        # the pool's per-job share (OMP_NUM_THREADS), as a secondary figure
        o_ob, o_de, o_rt, _, o_wall = timed(int(omp), min(seconds, 2.0))
        wall1 += o_wall * int(omp)
        share = {"threads": int(omp), "obfuscate": round(o_ob, 3), "deobfuscate": round(o_de, 3),
                 "round_trip": round(o_rt, 3), "why": "OMP_NUM_THREADS (the pool's per-job "
                 "share, not enforced by the cgroup quota when that allows more)"}
    quota = cgroup_cpu_quota()
    return {"value": ob, "unit": "GiB/s", "cores": threads, "kind": "port",
            "sample": f"configs[0]: {passes} x (65,536 x 1200 B Salamander obfuscate + "
                      f"deobfuscate), one PSK, C restatement (oracle/oracle.c, byte loops as "
                      f"salamander.go:51-53,62-64) on {threads} threads (every CPU this "
                      f"process may run on: affinity {len(os.sched_getaffinity(0))}, cgroup "
                      f"quota {quota if quota is not None else 'none'}; host {host} CPUs); "
                      f"value = obfuscate direction; deobfuscate {de:.3f} GiB/s, round trip "
                      f"{rt:.3f} GiB/s; round-trip identity {ok}; Go reference unbuildable "
                      f"(no Go toolchain)",
            "cgroup_cpu_quota": quota,
            "omp_num_threads": int(omp) if omp and omp.isdigit() else None,
            "job_share": share or None,
            "per_direction": {"obfuscate": round(ob, 3), "deobfuscate": round(de, 3),
                              "round_trip": round(rt, 3)},
            "per_core": {"obfuscate": round(ob1, 3), "deobfuscate": round(de1, 3),
                         "round_trip": round(rt1, 3)},
            "host_cpus": host,
            "host_cpus_extrapolated": {
                "obfuscate": round(ob1 * host, 1), "deobfuscate": round(de1 * host, 1),
                "round_trip": round(rt1 * host, 1),
                "note": "per-core rate x host CPUs: a linear upper bound, NOT measured (the "
                        "GPU pool gives one job a 16-CPU share; SMT siblings and memory "
                        "bandwidth would cut it)"},
            "cpu_seconds": round(wall * threads + wall1, 2)}


def cpu_path_rate(seconds: float = 1.5):
    """The PRODUCT's CPU path (sqobfs_cpu_run: host/sq_cpu.cpp, AVX2 BLAKE2b,
    word XOR; what the packet conn engine runs without a GPU and for small
    batches) on configs[0]'s workload, one contiguous shard per thread (ctypes
    releases the GIL).  Not the baseline: that is the reference's byte loops
    (cpu_baseline)."""
    import threading
    import numpy as np
    import sqobfs
    n, L, S = 65536, 1200, 8
    threads = cpu_share()
    rng = np.random.Generator(np.random.PCG64(1))
    data = rng.integers(0, 256, n * L, dtype=np.uint8)
    salt = np.random.Generator(np.random.PCG64(2)).integers(0, 256, n * S, dtype=np.uint8)
    wire = np.ones(n * (L + S), np.uint8)  # (pages touched: no first-write faults timed)
    back = np.ones(n * L, np.uint8)
    cut = [n * t // threads for t in range(threads + 1)]
    kr = sqobfs.Keyring(None, sqobfs.SALAMANDER, [PSK])

    def shard(t, direction):
        a, b = cut[t], cut[t + 1]
        m = b - a
        if direction == sqobfs.OBFUSCATE:
            hb = sqobfs.HostBatch(data[a * L:b * L], np.arange(m, dtype=np.uint64) * L,
                                  np.full(m, L, np.uint32), wire[a * (L + S):b * (L + S)],
                                  np.arange(m, dtype=np.uint64) * (L + S), np.zeros(m, np.uint32),
                                  salt[a * S:b * S])
        else:
            hb = sqobfs.HostBatch(wire[a * (L + S):b * (L + S)],
                                  np.arange(m, dtype=np.uint64) * (L + S),
                                  np.full(m, L + S, np.uint32), back[a * L:b * L],
                                  np.arange(m, dtype=np.uint64) * L, np.zeros(m, np.uint32))
        return hb.as_batch(), hb

    def run(direction, nthreads):
        batches = [shard(t, direction) for t in range(nthreads)] if nthreads == threads else \
            [shard(0, direction)]
        ths = [threading.Thread(target=sqobfs.cpu_run, args=(kr, direction, b)) for b, _ in batches]
        t0 = time.perf_counter()
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        return time.perf_counter() - t0, sum(int(h.in_len.sum()) if direction == 0 else
                                             int(h.in_len.sum()) - S * h.n for _, h in batches)

    res = {}
    run(sqobfs.OBFUSCATE, threads)  # warm
    for name, direction in (("obfuscate", sqobfs.OBFUSCATE), ("deobfuscate", sqobfs.DEOBFUSCATE)):
        tot = byt = 0.0
        t_end = time.perf_counter() + seconds / 2
        while tot == 0 or time.perf_counter() < t_end:
            dt, b = run(direction, threads)
            tot += dt
            byt += b
        res[name] = round(byt / tot / 2**30, 3)
    ok = bool(np.array_equal(back, data))
    dt1, b1 = run(sqobfs.OBFUSCATE, 1)
    kr.close()
    return {"value": res["obfuscate"], "unit": "GiB/s", "threads": threads,
            "per_direction": res, "per_thread_obfuscate": round(b1 / dt1 / 2**30, 3),
            "round_trip_identity": ok,
            "what": "sqobfs_cpu_run (the product CPU path, no GPU) on configs[0]'s 65,536 x "
                    "1200 B, one shard per thread"}


def cgroup_cpu_quota():
    """CPUs the cgroup's CPU quota allows (cgroup v2 cpu.max "quota period",
    v1 cfs_quota_us / cfs_period_us), or None when unlimited / unreadable."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return round(q / per, 2) if q > 0 else None
    except (OSError, ValueError):
        return None


def cpu_share() -> int:
    """CPUs this process may use: its affinity, capped by the cgroup CPU quota
    when there is one (the CPU baseline runs on the host's
    cores).  OMP_NUM_THREADS, the pool's advisory per-job share, is timed as a
    secondary figure."""
    import math
    n = len(os.sched_getaffinity(0))
    q = cgroup_cpu_quota()
    if q is not None:
        n = min(n, max(1, math.ceil(q)))
    return max(1, n)


def host_info(torch, dev) -> dict:
    """Where the line was measured (nproc, CPU model, ROCm)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    rocm = None
    for path in ("/opt/rocm/.info/version", "/opt/rocm/.info/version-dev"):
        if os.path.exists(path):
            rocm = open(path).read().strip()
            break
    return {"gpu": torch.cuda.get_device_name(dev), "cpu_model": model,
            "nproc": os.cpu_count(), "cpu_affinity": len(os.sched_getaffinity(0)),
            "rocm": rocm, "torch": torch.__version__}


def load_traffic(config: str, kernel_bytes: float):
    """HBM bytes per launch from the committed PMC pass (the latest round's
    profiles/rNN/pmc_<config>.json)."""
    path = None
    for rnd in ("r06", "r05", "r04", "r03", "r02"):
        p = os.path.join(REPO, "profiles", rnd, f"pmc_{config}.json")
        if os.path.exists(p):
            path = p
            break
    if path is None:
        return None, None
    with open(path) as f:
        d = json.load(f)
    return d.get("hbm_bytes_per_launch"), d


def copy_at_footprint(config: str):
    """The best plain copy's fraction of 8 TB/s at this config's footprint,
    measured in a process of its own (profiles/r06/ragged/copy_at_footprint.json,
    scripts/dev/footprint.sh), or None: the ceiling a streaming kernel of that
    size reaches on this hardware ("The copy control")."""
    path = os.path.join(REPO, "profiles", "r06", "ragged", "copy_at_footprint.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    c = d.get("configs", {}).get(config)
    if not c:
        return None
    return {"copy_frac": c["copy_best_frac"], "case": c["case"],
            "kernel_frac_isolated": c["kernel_frac_isolated"],
            "source": "profiles/r06/ragged/copy_at_footprint.json (" + c["box"] + ")"}


def inproc_bench(args):
    """K contexts in one process (the Go service's multi-GPU path), steps of
    sqobfs_shard_launch kept --inflight deep (each waited through its ticket;
    --inflight 1: sqobfs_shard_run, a host round trip per step); one JSON
    line."""
    import torch
    import sqobfs
    ndev = torch.cuda.device_count()
    assert ndev > 0, "bench.py needs a GPU"
    kind, n_total, L, n_psk = CONFIGS[args.config]
    if args.packets:
        n_total = args.packets
    K = args.inproc
    # shard sizes by bytes (fixed-length configs split evenly)
    lens_all = (torch.randint(64, 1453, (n_total,), generator=torch.Generator().manual_seed(4))
                if L is None else torch.full((n_total,), L))
    cut = sqobfs.shard_cuts(lens_all.numpy().astype("uint32"), K)
    ctxs, krs, bs, shs, devs = [], [], [], [], []
    payload = 0
    for k in range(K):
        g = k % ndev
        dev = torch.device("cuda", g)
        n_k = int(cut[k + 1] - cut[k])
        sh = build_shard(torch, dev, kind, n_k, L, n_psk, k, K, args.config, "dense", int(cut[k]))
        c = sqobfs.Context(g)
        # synchronous shard steps: poll the streams rather than pay the
        # blocking wake-up (~80 us) after every step
        c.set_sync_spin(4000)
        c.unit_packets = args.unit_packets or sqobfs.unit_packets_for(
            sh["payload_bytes"], n_k, n_psk > 1, kind)
        kr = sqobfs.Keyring(c, kind, sh["psks"])
        ctxs.append(c)
        krs.append(kr)
        shs.append(sh)
        devs.append(dev)
        bs.append(sqobfs.make_batch(n_k, sh["data"], sh["in_off"], sh["lens"], sh["out"],
                                    sh["out_off"], sh["out_len"], sh["salt"], sh["psk_id"]))
        payload += sh["payload_bytes"]
    for d in set(devs):
        torch.cuda.synchronize(d)
    depth = max(1, args.inflight)

    def steps(k):
        pending = []
        for _ in range(k):
            pending.append(sqobfs.shard_launch(ctxs, krs, sqobfs.OBFUSCATE, bs))
            if len(pending) >= depth:
                pending.pop(0).wait()
        for t in pending:
            t.wait()
    # warm-up as the queued mode's: at least --warmup steps and --warmup-s of
    # wall time (a fresh process's first ~25 launches run up to 10 % slower)
    warm, wt0 = 0, time.perf_counter()
    while warm < args.warmup or time.perf_counter() - wt0 < args.warmup_s:
        steps(1)
        warm += 1
    t0 = time.perf_counter()
    steps(args.steps)
    el = time.perf_counter() - t0
    out = {"metric": f"GiB/s payload obfuscated, device-resident, {args.config}, "
                     f"{K} in-process shards (sqobfs_shard_launch, {depth} steps in flight)",
           "value": round(payload * args.steps / el / 2**30, 3), "unit": "GiB/s",
           "n_gpus": len(set(devs)), "contexts": K, "steps": args.steps,
           "warmup": args.warmup, "warmup_steps": warm,
           "ms_per_step": round(el * 1e3 / args.steps, 4),
           "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u8",
           "data": "synthetic", "shard_packets": [int(cut[k + 1] - cut[k]) for k in range(K)],
           "config": {"workload": args.config, "inproc": K, "inflight": depth}}
    print(json.dumps(out), flush=True)
    for kr in krs:
        kr.close()
    for c in ctxs:
        c.close()


# Measured integer VALU ceiling (scripts/probe_valu.hip,
# profiles/r03/valu/probe_valu.txt): v_add_u32 / v_xor_b32 / v_alignbit_b32
# chains issue 0.633 T wave-instructions/s on the whole chip at 8 waves per
# SIMD: 3.9 cycles per wave64 instruction per SIMD at the nominal 2.4 GHz
# (the clock under load is not measured; packed f32 FMAs ran 4.8), about half
# the rate of the 2-cycle figure the spec-based peak assumes.
VALU_INT_MEASURED = 0.633e12


def quic_valu_roofline(suite_name: str, op: str, kernel_us: float):
    """VALU roofline of a QUIC kernel from the committed PMC pass
    (profiles/r0N/quic/quic_pmc_summary.json, scripts/quic_pmc.sh): VALU
    wave-instructions per launch (SQ_INSTS_VALU) over this run's kernel time,
    against 256 CUs x 4 SIMDs x 2.4 GHz / 2 cycles per wave64 instruction
    (`frac`) and against the measured integer issue rate
    (`frac_of_measured_int_rate`)."""
    for rnd in ("r06", "r05", "r04", "r03", "r02"):  # the newest committed pass
        f = os.path.join(REPO, "profiles", rnd, "quic", "quic_pmc_summary.json")
        if os.path.exists(f):
            break
    else:
        return None
    d = json.load(open(f))
    name = {"chacha20_poly1305": "quic_kernel", "aes_128_gcm": "quic_gcm_kernel"}[suite_name]
    tmpl = {"seal": "<false, false, false>", "open": "<true, false, false>",
            "fused_seal": "<false, false, true>", "fused_open": "<true, false, true>"}[op]
    for k, e in d["kernels"].items():
        if f"sq::{name}{tmpl}" in k:
            valu = e["counters"]["SQ_INSTS_VALU"]
            peak = d["peak_valu_wave_instr_per_s"]
            ach = valu / (kernel_us * 1e-6)
            return {"bound": "valu", "valu_wave_instr_per_launch": round(valu),
                    "valu_wave_instr_per_packet": round(valu / (1 << 20), 1),
                    "achieved": round(ach / 1e12, 4), "peak": round(peak / 1e12, 4),
                    "unit": "T wave-instr/s", "frac": round(ach / peak, 4),
                    "measured_int_rate": VALU_INT_MEASURED / 1e12,
                    "frac_of_measured_int_rate": round(ach / VALU_INT_MEASURED, 4),
                    "measured_int_rate_source": "scripts/probe_valu.hip, "
                                                "profiles/r03/valu/probe_valu.txt",
                    "source": os.path.relpath(f, REPO) + " (SQ_INSTS_VALU)"}
    return None


def free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args) -> int:
    """`bench.py --gpus N` (N > 1) run as a bare command: start the N rank
    processes here, one per GPU, as children of this one, each with the
    torch.distributed.run environment (RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_ADDR 127.0.0.1 / MASTER_PORT).  This process never touches the GPU
    (torch.cuda.device_count() does not initialise HIP on this image) and
    never re-execs: it waits for the ranks, relays rank 0's one JSON line to
    stdout and every rank's stderr to stderr, and exits non-zero when any rank
    fails (the others are stopped, so a rank stuck in a barrier cannot hang
    the job).  The torchrun form (WORLD_SIZE set) does not come here."""
    import signal
    import subprocess
    import tempfile
    import torch
    ndev = torch.cuda.device_count()
    if args.gpus > ndev and args.dist_backend != "gloo":
        print(f"bench.py: --gpus {args.gpus} but {ndev} GPU(s) visible; one rank per GPU "
              f"(--dist-backend gloo lets ranks share a GPU, tests only)", file=sys.stderr)
        return 2
    port = free_port()
    procs, outs = [], []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        out = tempfile.TemporaryFile(mode="w+")
        outs.append(out)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env, stdout=out, start_new_session=True))
    failed = None
    try:
        while any(p.poll() is None for p in procs):
            bad = [i for i, p in enumerate(procs) if p.returncode not in (None, 0)]
            if bad:
                failed = bad[0]
                break
            time.sleep(0.05)
    finally:
        if failed is not None or any(p.poll() is None for p in procs):
            # a failed rank leaves the others in a collective: give them a
            # moment, then stop their process groups
            deadline = time.time() + 15
            while time.time() < deadline and any(p.poll() is None for p in procs):
                time.sleep(0.1)
            for p in procs:
                if p.poll() is None:
                    os.killpg(p.pid, signal.SIGTERM)
            for p in procs:
                try:
                    p.wait(timeout=10)
                except subprocess.TimeoutExpired:
                    os.killpg(p.pid, signal.SIGKILL)
                    p.wait()
    rcs = [p.returncode for p in procs]
    for r, out in enumerate(outs):
        out.seek(0)
        text = out.read()
        if r == 0:
            for line in text.splitlines():
                if line.startswith("{"):
                    print(line, flush=True)
                else:
                    print(line, file=sys.stderr)
        elif text.strip():
            print(f"[rank {r} stdout]\n{text}", file=sys.stderr)
    if any(rc != 0 for rc in rcs):
        print(f"bench.py: rank exit codes {rcs}", file=sys.stderr)
        rc = next(rc for rc in rcs if rc != 0)
        return rc if rc > 0 else 1  # a rank killed by a signal
    return 0


def main():
    args = parse()
    if args.inproc:
        return inproc_bench(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args)
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}")
    import torch
    import sqobfs

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    ndev = torch.cuda.device_count()
    assert ndev > 0, "bench.py needs a GPU"
    gpu = local % ndev  # several gloo ranks may share a GPU (tests only)
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(gpu)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group("gloo")
    dev = torch.device("cuda", gpu)
    torch.cuda.set_device(dev)

    kind, n_total, L, n_psk = CONFIGS[args.config]
    if args.packets:
        n_total = args.packets
    n, first = shard(args.config, n_total, world, rank)
    direction = sqobfs.OBFUSCATE if args.direction == "obfuscate" else sqobfs.DEOBFUSCATE
    sh = build_shard(torch, dev, kind, n, L, n_psk, rank, world, args.config, args.layout, first,
                     args.slot_bytes)
    S = sh["S"]
    ctx = sqobfs.Context(gpu)
    kr = sqobfs.Keyring(ctx, kind, sh["psks"])
    ctx.unit_packets = args.unit_packets or sqobfs.unit_packets_for(
        sh["payload_bytes"], n, n_psk > 1, kind)
    stream = torch.cuda.current_stream(dev)
    s = stream.cuda_stream

    if direction == sqobfs.DEOBFUSCATE and sh["inplace"]:
        raise SystemExit("--layout inplace is for obfuscate")
    if args.device_salt and (direction != sqobfs.OBFUSCATE or sh["inplace"]):
        raise SystemExit("--device-salt is for obfuscate, not in place")
    # slotted layouts: every output owns its 16-byte blocks; 2048-byte slots
    # also the rest of its last 128-byte line (slot padding)
    ob = sqobfs.FLAG_OUT_BLOCKS if sh["slotted"] else 0
    if args.layout == "slot2048" and args.slot_flag == "lines":
        # every output's last line, padding included, inside its slot
        lead = int(os.environ.get("SQ_BENCH_LEAD", "128")) % 128
        assert args.slot_bytes % 128 == 0 and (lead + S + (L or 1452) + 127) // 128 * 128 <= \
            args.slot_bytes, "--slot-flag lines needs slots holding the outputs' last lines"
        ob = sqobfs.FLAG_OUT_LINES
    if direction == sqobfs.OBFUSCATE and args.device_salt:
        ctx.salt_key(SALT_KEY, 0)
        b = sqobfs.make_batch(n, sh["data"], sh["in_off"], sh["lens"], sh["out"], sh["out_off"],
                              sh["out_len"], None, sh["psk_id"],
                              flags=sqobfs.FLAG_DEVICE_SALT | ob)
        alg_bytes = 2 * sh["payload_bytes"] + S * n  # no salt array read
    elif direction == sqobfs.OBFUSCATE:
        b = sqobfs.make_batch(n, sh["data"], sh["in_off"], sh["lens"], sh["out"], sh["out_off"],
                              sh["out_len"], sh["salt"], sh["psk_id"], flags=ob)
        alg_bytes = 2 * sh["payload_bytes"] + 2 * S * n
    else:
        # decode the obfuscated shard (made once, untimed)
        b0 = sqobfs.make_batch(n, sh["data"], sh["in_off"], sh["lens"], sh["out"],
                               sh["out_off"], sh["out_len"], sh["salt"], sh["psk_id"], flags=ob)
        sqobfs.launch(ctx, kr, sqobfs.OBFUSCATE, b0, s)
        wire_len = (sh["lens"] + S).to(torch.int32)
        if sh["slotted"]:
            # decoded payloads into slots like the input's (16-byte aligned)
            back_off = sh["in_off"]
            back = torch.zeros_like(sh["data"])
        else:
            # decoded payloads back to back (a compact receive buffer)
            back_off = torch.cumsum(sh["lens"].to(torch.int64), 0) - sh["lens"].to(torch.int64) + 64
            back = torch.zeros(int(sh["payload_bytes"]) + 128, device=dev, dtype=torch.uint8)
        b = sqobfs.make_batch(n, sh["out"], sh["out_off"], wire_len, back, back_off,
                              sh["out_len"], None, sh["psk_id"], flags=ob)
        alg_bytes = 2 * sh["payload_bytes"] + S * n

    saved = save_samples(sh, n) if direction == sqobfs.OBFUSCATE else None
    warm, wt0 = 0, time.perf_counter()
    while warm < args.warmup or time.perf_counter() - wt0 < args.warmup_s:
        sqobfs.launch(ctx, kr, direction, b, s)
        warm += 1
        if warm % 8 == 0:
            torch.cuda.synchronize(dev)  # wall time follows the GPU
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)

    # The timed region holds the launches only: one HIP event pair on the
    # launch stream spans it, so the kernel average is the span / steps
    # (back-to-back kernels, their dispatch gaps included).  An event pair
    # around every launch put two marker packets between kernels and cost
    # 7-9 us per step (scripts/dev/timing_probe.py).
    e_beg, e_end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e_beg.record(stream)
    for _ in range(args.steps):
        sqobfs.launch(ctx, kr, direction, b, s)
    e_end.record(stream)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    kern_avg_ms = e_beg.elapsed_time(e_end) / args.steps
    # per-launch spread, after the timed region (not in `value`): each
    # kernel's own dispatch records its event pair
    n_each = min(args.steps, 20)
    dev_ev = sqobfs.DispatchEvents(n_each)
    for i in range(n_each):
        dev_ev.arm(i)
        sqobfs.launch(ctx, kr, direction, b, s)
    torch.cuda.synchronize(dev)
    kern_ms = sorted(dev_ev.elapsed_ms(i) for i in range(n_each))
    dev_ev.close()

    tdev = dev if args.dist_backend == "nccl" else torch.device("cpu")
    if dist:
        elapsed = max_over_ranks(torch, dist, elapsed, tdev)
        kern_avg_ms = max_over_ranks(torch, dist, kern_avg_ms, tdev)

    parity = None
    if args.device_salt:
        # the last launch's salts, from the oracle's ChaCha20 (checker only)
        import numpy as np
        import oracle_lib as ol
        last = ctx.salt_seq - 1
        salts = np.frombuffer(ol.device_salts(SALT_KEY, last, n, S), np.uint8)
        sh["salt"] = torch.from_numpy(salts.copy()).to(dev)
    if direction == sqobfs.OBFUSCATE:
        parity = spot_check(torch, sh, kind, n, sh["out"], saved, warm + args.steps + n_each)
    else:
        lens = sh["lens"].cpu().numpy()
        offs = sh["in_off"].cpu().numpy()
        boffs = back_off.cpu().numpy()
        parity = all(torch.equal(back[int(boffs[i]):int(boffs[i]) + int(lens[i])],
                                 sh["data"][int(offs[i]):int(offs[i]) + int(lens[i])])
                     for i in sorted(set([0, n - 1] + list(range(0, n, 4099)))))
    if dist:
        parity = -max_over_ranks(torch, dist, -1.0 if parity else 0.0, tdev) > 0

    total_payload = sh["payload_bytes"] * args.steps
    if dist:
        total_payload = sum_over_ranks(torch, dist, total_payload, tdev)
    value = total_payload / elapsed / 2**30
    achieved = alg_bytes / (kern_avg_ms * 1e-3) / 1e9
    # the committed PMC passes are for host salts on the dense layout
    traffic, pmc = (None, None)
    if not args.device_salt and args.layout == "dense":
        key = args.config if direction == sqobfs.OBFUSCATE else f"{args.config}-deobfuscate"
        traffic, pmc = load_traffic(key, alg_bytes)
    out = {
        "metric": METRIC if args.config == "salamander-1m" and direction == 0
        and not args.device_salt else
        f"GiB/s payload {'obfuscated' if direction == 0 else 'deobfuscated'}"
        f"{' (device salts)' if args.device_salt else ''}, device-resident, {args.config}",
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "warmup_launches": warm,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak" if args.config != "salamander-16m-256psk" else "strong",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (torch Philox random payloads/salts, seeded per rank)",
        "config": {
            "workload": {"salamander-1m": "configs[1]: Salamander obfuscate, 1,048,576 x 1350 B "
                                          "per GPU, one 26-byte PSK",
                         "xplus-1m": "configs[2]: XPlus, 1,048,576 x 1200 B per GPU, one PSK",
                         "salamander-ragged-4m": "configs[3]: Salamander, 4,194,304 packets "
                                                 "U[64,1452] per GPU, one PSK",
                         "salamander-16m-256psk": "configs[4]: Salamander, 16,777,216 x 1350 B, "
                                                  "256 PSKs round-robin, sharded over ranks"}[args.config],
            "direction": args.direction,
            "salts": "device ChaCha20 (SQOBFS_FLAG_DEVICE_SALT)" if args.device_salt else "host array",
            "packets_per_gpu": n,
            "payload_bytes_per_gpu": sh["payload_bytes"],
            "layout": args.layout + (f" ({args.slot_bytes}-byte slots)"
                                     if args.layout == "slot2048" else ""),
            "batch_flags": {0: "none", sqobfs.FLAG_OUT_BLOCKS: "SQOBFS_FLAG_OUT_BLOCKS",
                            sqobfs.FLAG_OUT_LINES: "SQOBFS_FLAG_OUT_LINES"}[ob],
            "unit_packets": ctx.unit_packets,
            # sq_kernels.hip kXcdMinUnits: launches of >= 2^18 units remap
            # workgroups so each XCD walks a contiguous eighth of the batch
            "unit_order": ("XCD-contiguous" if -(-n // ctx.unit_packets) >= 1 << 18
                           else "dispatch order"),
            "unit_rule": ("--unit-packets" if args.unit_packets else
                          "sqobfs_unit_packets_for_kind(kind, payload bytes, n): ~21.7 KB per "
                          "wavefront (XPlus 19.5 KB; 31.5 KB with a multi-PSK keyring; at least "
                          "2,048 wavefronts)"),
            "parallelism": f"shard{world} (independent packets, no collective)",
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": PEAK_HBM_GBS,
            "unit": "GB/s",
            "frac": round(achieved / PEAK_HBM_GBS, 4),
            "traffic": traffic,
            "kernel": kernel_name(kind, direction, n_psk > 1, ctx.unit_packets),
            "build": sqobfs.build_info(),
            "kernel_avg_us": round(kern_avg_ms * 1e3, 2),
            "kernel_avg_rule": "HIP events spanning the timed region's back-to-back "
                               "launches / steps (dispatch gaps included)",
            "kernel_min_us": round(kern_ms[0] * 1e3, 2),
            "kernel_median_us": round(kern_ms[len(kern_ms) // 2] * 1e3, 2),
            "kernel_each_rule": f"{n_each} launches after the timed region, each timed by "
                                "its own dispatch (sqobfs_debug_time_next_launch)",
            "algorithmic_bytes_per_launch": alg_bytes,
            "bytes_rule": "obfuscate 2L+2S per packet (2L+S with device salts), "
                          "deobfuscate 2L+S (SURVEY.md 8(d))",
        },
        "parity_spot_check": parity,
    }
    if pmc:
        out["roofline"]["traffic_source"] = pmc.get("source")
    cf = copy_at_footprint(args.config) if args.layout == "dense" and not args.packets else None
    if cf:
        out["roofline"]["copy_at_footprint"] = cf
        out["roofline"]["frac_of_copy_at_footprint"] = round(achieved / PEAK_HBM_GBS / cf["copy_frac"], 4)
    if args.latency and rank == 0:
        out["latency"] = latency_bench()
    if not args.no_e2e:
        # every rank at once, behind a barrier, after the timed region (not in
        # `value`): the host-staged rate of the whole job
        out["e2e"] = e2e_all_ranks(torch, sqobfs, ctx, kr, kind, dist, tdev, world)
    if args.e2e and rank == 0:
        out.setdefault("e2e", {})["modes"] = e2e_rate(torch, sqobfs, ctx, kr, kind,
                                                      min(n, 1 << 18), L or 758)
    if args.quic and rank == 0:
        out["quic"] = {
            "chacha20_poly1305": quic_rate(torch, sqobfs, ctx, dev, max(5, args.steps), suite=0),
            "aes_128_gcm": quic_rate(torch, sqobfs, ctx, dev, max(5, args.steps), suite=1)}
    if args.udp and rank == 0:
        out["udp_e2e"] = [udp_rate(sqobfs, ctx, kr, kind, L or 758, batch=bt)
                          for bt in (64, 256, 1024)] + \
                         [udp_rate(sqobfs, ctx, kr, kind, L or 758, batch=bt,
                                   offload=sqobfs.UDP_TX_GSO | sqobfs.UDP_RX_GRO)
                          for bt in (256, 1024)]
        if kind == 0:
            out["udp_quic_e2e"] = [udp_quic_rate(sqobfs, ctx, kr, (L or 758) + 11, batch=bt,
                                                 suite=su)
                                   for su in (0, 1) for bt in (256, 1024)]
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
        out["cpu_path"] = cpu_path_rate()
    if rank == 0:
        out["host"] = host_info(torch, dev)
    if rank == 0:
        print(json.dumps(out), flush=True)
    kr.close()
    ctx.close()
    if dist:
        dist.destroy_process_group()


def latency_bench():
    """sing-quic_amd/bin/lat_bench (built by `make -C sing-quic_amd tools`):
    DESIGN.md section 9.5."""
    import subprocess
    exe = os.path.join(REPO, "sing-quic_amd", "bin", "lat_bench")
    if not os.path.exists(exe):
        return {"error": f"{exe} missing: make -C sing-quic_amd tools"}
    r = subprocess.run([exe], capture_output=True, text=True, timeout=240)
    if r.returncode != 0:
        return {"error": r.stderr[-500:]}
    return json.loads(r.stdout)


def e2e_all_ranks(torch, sqobfs, ctx, kr, kind, dist, tdev, world, n=1 << 18, L=1350, reps=3):
    """The host-staged batch on every rank at once: each
    rank runs sqobfs_run_host -- chunked H2D | kernel | D2H on its own GPU and
    PCIe link -- over n x L page-locked caller slots with
    SQOBFS_FLAG_OUT_UNINIT, `reps` times, all ranks released by one barrier.
    aggregate_gib_s = the payload of every rank / the max-over-ranks wall
    time; per_rank = each rank's own rate.  Bounded (~0.4 GB per rank).
    One packet per rank is checked against the device path's contract (its
    out_len); the bytes' parity is tests/test_gpu_*'s.  A rank whose part
    fails (e.g. page-locked memory refused) still joins every collective, so
    no rank waits forever; the result then names the failed ranks instead of
    an aggregate, and the bench line is printed as usual."""
    import numpy as np
    S = 8 if kind == 0 else 16
    rng = np.random.Generator(np.random.PCG64(11 + (dist.get_rank() if dist else 0)))
    nin, nout = n * slot(L), n * slot(L + S)
    pins, err, ok, dt = [], None, False, 0.0
    try:
        pd = sqobfs.PinnedArray(ctx, nin)
        pins.append(pd)
        po = sqobfs.PinnedArray(ctx, nout)
        pins.append(po)
        pd.array[:] = np.frombuffer(rng.bytes(nin), np.uint8)
        in_off = np.arange(n, dtype=np.uint64) * slot(L)
        out_off = np.arange(n, dtype=np.uint64) * slot(L + S)
        salt = np.frombuffer(rng.bytes(n * S), np.uint8).copy()
        out_len = np.zeros(n, np.uint32)
        hb = sqobfs.HostBatch(pd.array, in_off, np.full(n, L, np.uint32), po.array, out_off,
                              out_len, salt, flags=sqobfs.FLAG_OUT_UNINIT)
        b = hb.as_batch()
        sqobfs.run_host(ctx, kr, sqobfs.OBFUSCATE, b)  # (warm: staging buffers, clocks)
        ok = bool(hb.out_len[0] == L + S and hb.out_len[-1] == L + S)
    except Exception as e:  # (reported below; this rank still joins the collectives)
        err = f"{type(e).__name__}: {e}"
    if dist:
        dist.barrier()
    if err is None:
        try:
            t0 = time.perf_counter()
            for _ in range(reps):
                sqobfs.run_host(ctx, kr, sqobfs.OBFUSCATE, b)
            dt = time.perf_counter() - t0
        except Exception as e:
            err = f"{type(e).__name__}: {e}"
    for p in pins:
        p.free()
    own = n * L * reps / dt / 2**30 if err is None else 0.0
    if dist:
        t = torch.tensor([own, dt, 1.0 if ok else 0.0, 0.0 if err is None else 1.0],
                         dtype=torch.float64, device=tdev)
        g = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(g, t)
        rates = [float(x[0]) for x in g]
        wall = max(float(x[1]) for x in g)
        ok = all(float(x[2]) > 0 for x in g)
        failed = [r for r, x in enumerate(g) if float(x[3]) > 0]
    else:
        rates, wall, failed = [own], dt, ([0] if err else [])
    res = {} if failed else {"aggregate_gib_s": round(n * L * reps * world / wall / 2**30, 3)}
    res.update({"per_rank": [round(r, 3) for r in rates], "wall_s": round(wall, 5),
           "packets_per_rank": n, "payload_bytes": L, "reps": reps, "out_len_ok": ok,
           "rule": "sum over ranks of n x L x reps / max-over-ranks wall; all ranks released "
                   "by one barrier after the timed region (not part of `value`)",
           "path": "sqobfs_run_host, page-locked caller slots, SQOBFS_FLAG_OUT_UNINIT, "
                   "host salts"})
    if failed:
        res["failed_ranks"] = failed
        if err:
            res["error"] = err  # (this rank's; rank 0 prints the line)
    return res


def e2e_rate(torch, sqobfs, ctx, kr, kind, n, L):
    """Host-resident batches through sqobfs_run_host (chunked H2D | kernel |
    D2H pipeline): caller buffers pageable (staged through pinned memory by
    host threads) and page-locked (DMA directly), plus the latter with
    SQOBFS_FLAG_OUT_UNINIT (no copy-in of the output range).  Rates count
    payload bytes (DESIGN.md e2e rate)."""
    import numpy as np
    S = 8 if kind == 0 else 16
    rng = np.random.Generator(np.random.PCG64(9))
    nin, nout = n * slot(L), n * slot(L + S)
    in_off = np.arange(n, dtype=np.uint64) * slot(L)
    out_off = np.arange(n, dtype=np.uint64) * slot(L + S)
    salt = rng.integers(0, 256, n * S, dtype=np.uint8)
    res = {"packets": n, "payload_bytes": L}
    pins = []
    for mode in ("pageable", "pinned", "pinned_out_uninit", "slots2048"):
        if mode == "slots2048":
            # the Go Slots.Run geometry: fixed 2,048-byte slots in page-locked
            # memory, outputs read up to out_len (OUT_UNINIT), whole lines
            # (OUT_LINES): run_host stages the datagrams' bytes only
            pd, po = sqobfs.PinnedArray(ctx, n * 2048), sqobfs.PinnedArray(ctx, n * 2048)
            pins += [pd, po]
            pd.array[:] = rng.integers(0, 256, n * 2048, dtype=np.uint8)
            offs = np.arange(n, dtype=np.uint64) * 2048
            hb = sqobfs.HostBatch(pd.array, offs, np.full(n, L, np.uint32), po.array, offs,
                                  np.zeros(n, np.uint32), salt,
                                  flags=sqobfs.FLAG_OUT_UNINIT | sqobfs.FLAG_OUT_LINES)
            b = hb.as_batch()
            sqobfs.run_host(ctx, kr, sqobfs.OBFUSCATE, b)
            reps = 5
            t0 = time.perf_counter()
            for _ in range(reps):
                sqobfs.run_host(ctx, kr, sqobfs.OBFUSCATE, b)
            dt = (time.perf_counter() - t0) / reps
            res[mode] = {"GiB_s_payload": round(n * L / dt / 2**30, 3),
                         "ms_per_batch": round(dt * 1e3, 3)}
            continue
        if mode == "pageable":
            data = rng.integers(0, 256, nin, dtype=np.uint8)
            out = np.zeros(nout, np.uint8)
        elif mode == "pinned":
            pd, po = sqobfs.PinnedArray(ctx, nin), sqobfs.PinnedArray(ctx, nout)
            pins += [pd, po]
            pd.array[:] = rng.integers(0, 256, nin, dtype=np.uint8)
            po.array[:] = 0
            data, out = pd.array, po.array
        hb = sqobfs.HostBatch(data, in_off, np.full(n, L, np.uint32), out, out_off,
                              np.zeros(n, np.uint32), salt,
                              flags=sqobfs.FLAG_OUT_UNINIT if mode.endswith("uninit") else 0)
        b = hb.as_batch()
        sqobfs.run_host(ctx, kr, sqobfs.OBFUSCATE, b)
        reps = 5
        t0 = time.perf_counter()
        for _ in range(reps):
            sqobfs.run_host(ctx, kr, sqobfs.OBFUSCATE, b)
        dt = (time.perf_counter() - t0) / reps
        res[mode] = {"GiB_s_payload": round(n * L / dt / 2**30, 3),
                     "ms_per_batch": round(dt * 1e3, 3)}
    for p in pins:
        p.free()
    res["path"] = ("sqobfs_run_host: H2D | kernel | D2H pipeline on 3 HIP streams (8 chunks, 16 "
                   "with page-locked buffers, the last cut in three); "
                   "fixed-stride page-locked slots staged as packed rows (2-D copies)")
    return res


def warm_up(torch, dev, call, seconds: float = 0.15, least: int = 2) -> int:
    """Untimed launches for at least `seconds` of wall time (a fresh process's
    first launches run slower); returns the count."""
    k, t0 = 0, time.perf_counter()
    while k < least or time.perf_counter() - t0 < seconds:
        call()
        k += 1
        if k % 4 == 0:
            torch.cuda.synchronize(dev)
    torch.cuda.synchronize(dev)
    return k


def quic_rate(torch, sqobfs, ctx, dev, steps, n=1 << 20, payload=1350, cpu_seconds=2.0,
              suite=0):
    """QUIC 1-RTT packet protection: seal and open
    of n short-header packets (1 + 8-byte DCID + 2-byte packet number +
    `payload` bytes), dense in HBM, one key; suite 0 = ChaCha20-Poly1305,
    1 = AES-128-GCM.  Algorithmic bytes per packet: seal reads len, writes
    len + 16; open reads len + 16, writes len.  Parity: sampled packets
    against the oracle.  CPU legs on bounded samples: the oracle's threaded
    or_quic_seal_batch2 (scalar C port), and OpenSSL libcrypto
    (oracle/ossl_quic.c: AES-NI / vector code, the class of code quic-go
    runs)."""
    import ctypes
    import numpy as np
    import oracle_lib as ol
    hdr = 11
    ln = hdr + payload
    kl = 16 if suite else 32
    rng = np.random.Generator(np.random.PCG64(12))
    key, iv, hp = (rng.integers(0, 256, m, dtype=np.uint8).tobytes() for m in (kl, 12, kl))
    in_off = torch.arange(n, device=dev, dtype=torch.int64) * ln
    out_off = torch.arange(n, device=dev, dtype=torch.int64) * (ln + 16)
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    data = torch.randint(0, 256, (n * ln,), generator=g, device=dev, dtype=torch.uint8)
    data.view(n, ln)[:, 0] = 0x41  # short header, pn_len 2
    pn = torch.arange(n, device=dev, dtype=torch.int64) + 1000
    data.view(n, ln)[:, 9] = ((pn >> 8) & 0xFF).to(torch.uint8)
    data.view(n, ln)[:, 10] = (pn & 0xFF).to(torch.uint8)
    sealed = torch.zeros(n * (ln + 16), device=dev, dtype=torch.uint8)
    opened = torch.zeros(n * ln, device=dev, dtype=torch.uint8)
    lens = torch.full((n,), ln, device=dev, dtype=torch.int32)
    slens = torch.full((n,), ln + 16, device=dev, dtype=torch.int32)
    pno = torch.full((n,), 9, device=dev, dtype=torch.int16)
    largest = pn - 1
    olen = torch.zeros(n, device=dev, dtype=torch.int32)
    olen2 = torch.zeros(n, device=dev, dtype=torch.int32)
    pn_out = torch.zeros(n, device=dev, dtype=torch.int64)
    s = torch.cuda.current_stream(dev).cuda_stream
    res = {"packets": n, "packet_bytes": ln, "payload_bytes": payload,
           "cipher": ("AEAD_AES_128_GCM + AES header protection (RFC 9001)" if suite else
                      "AEAD_CHACHA20_POLY1305 + ChaCha20 header protection (RFC 9001)")}
    with sqobfs.QuicKeyring(ctx, [sqobfs.QuicKey.of(key, iv, hp)], suite) as kr:
        bs = sqobfs.quic_batch(n, data, in_off, lens, sealed, out_off, olen, pno, pn)
        bo = sqobfs.quic_batch(n, sealed, out_off, slens, opened, in_off, olen2, pno, largest,
                               pn_out=pn_out)
        for name, fn, b, alg in (("seal", sqobfs.quic_seal, bs, n * (2 * ln + 16)),
                                 ("open", sqobfs.quic_open, bo, n * (2 * ln + 16))):
            warm_up(torch, dev, lambda: fn(ctx, kr, b, s))
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(steps)]
            for e0, e1 in ev:
                e0.record()
                fn(ctx, kr, b, s)
                e1.record()
            torch.cuda.synchronize(dev)
            ms = sum(e0.elapsed_time(e1) for e0, e1 in ev) / steps
            res[name] = {"kernel_avg_us": round(ms * 1e3, 2),
                         "GiB_s_payload": round(n * payload / (ms * 1e-3) / 2**30, 2),
                         "achieved_GBs": round(alg / (ms * 1e-3) / 1e9, 1),
                         "frac_of_8TBs": round(alg / (ms * 1e-3) / 8e12, 4),
                         "valu_roofline": quic_valu_roofline(
                             "aes_128_gcm" if suite else "chacha20_poly1305", name, ms * 1e3)}
    # several connections in one launch (the multi-key kernels: key_id per
    # packet, keys gathered from the device keyring): 16 keys, key_id = i mod 16
    nk = 16
    mk = [tuple(rng.integers(0, 256, m, dtype=np.uint8).tobytes() for m in (kl, 12, kl))
          for _ in range(nk)]
    kid = (torch.arange(n, device=dev, dtype=torch.int64) % nk).to(torch.int16)
    msealed = torch.zeros_like(sealed)
    mopened = torch.zeros_like(opened)
    molen = torch.zeros_like(olen)
    molen2 = torch.zeros_like(olen2)
    mpn_out = torch.zeros_like(pn_out)
    with sqobfs.QuicKeyring(ctx, [sqobfs.QuicKey.of(*k) for k in mk], suite) as kr:
        bs = sqobfs.quic_batch(n, data, in_off, lens, msealed, out_off, molen, pno, pn, key_id=kid)
        bo = sqobfs.quic_batch(n, msealed, out_off, slens, mopened, in_off, molen2, pno, largest,
                               key_id=kid, pn_out=mpn_out)
        mres = {"keys": nk}
        for name, fn, b in (("seal", sqobfs.quic_seal, bs), ("open", sqobfs.quic_open, bo)):
            warm_up(torch, dev, lambda: fn(ctx, kr, b, s))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(steps):
                fn(ctx, kr, b, s)
            e1.record()
            torch.cuda.synchronize(dev)
            ms = e0.elapsed_time(e1) / steps
            mres[name] = {"kernel_avg_us": round(ms * 1e3, 2),
                          "GiB_s_payload": round(n * payload / (ms * 1e-3) / 2**30, 2)}
        midx = sorted(set([0, n - 1] + list(range(0, n, 8191))))[:150]
        dm = data.view(n, ln)[midx].cpu().numpy()
        slm = msealed.view(n, ln + 16)[midx].cpu().numpy()
        opm = mopened.view(n, ln)[midx].cpu().numpy()
        mok = bool((molen.cpu().numpy() == ln + 16).all() and (molen2.cpu().numpy() == ln).all())
        for k, i in enumerate(midx):
            kk = mk[i % nk]
            want, _ = ol.quic_seal(kk[0], kk[1], kk[2], 1000 + i, dm[k].tobytes(), 9, suite=suite)
            mok = mok and slm[k].tobytes() == want and opm[k].tobytes() == dm[k].tobytes()
        mres["parity_spot_check"] = mok
    res["multi_key"] = mres
    res["fused_salamander"] = quic_fused_rate(torch, sqobfs, ctx, dev, steps, n, ln, data,
                                              in_off, lens, pno, pn, key, iv, hp, suite)
    sn = "aes_128_gcm" if suite else "chacha20_poly1305"
    fs = res["fused_salamander"]
    fs["valu_roofline_fused_seal"] = quic_valu_roofline(sn, "fused_seal", fs["fused_seal_us"])
    fs["valu_roofline_fused_open"] = quic_valu_roofline(sn, "fused_open", fs["fused_open_us"])
    # parity on sampled packets
    idx = sorted(set([0, n - 1] + list(range(0, n, 4099))))[:300]
    d = data.view(n, ln)[idx].cpu().numpy()
    sl = sealed.view(n, ln + 16)[idx].cpu().numpy()
    op = opened.view(n, ln)[idx].cpu().numpy()
    ok = bool((olen.cpu().numpy() == ln + 16).all() and (olen2.cpu().numpy() == ln).all()
              and (pn_out.cpu().numpy() == pn.cpu().numpy()).all())
    for k, i in enumerate(idx):
        want, _ = ol.quic_seal(key, iv, hp, 1000 + i, d[k].tobytes(), 9, suite=suite)
        ok = ok and sl[k].tobytes() == want and op[k].tobytes() == d[k].tobytes()
    res["parity_spot_check"] = ok
    # CPU legs, threaded: the oracle (scalar C restatement) and OpenSSL
    m = 65536 if suite == 0 else 8192
    threads = cpu_share()
    cin = np.tile(d[0], m)
    ci_off = np.arange(m, dtype=np.uint64) * ln
    co_off = np.arange(m, dtype=np.uint64) * (ln + 16)
    cout = np.zeros(m * (ln + 16), np.uint8)
    c_len = np.full(m, ln, np.uint32)
    c_pno = np.full(m, 9, np.uint16)
    c_pn = np.arange(m, dtype=np.uint64)
    args_ = (key, iv, hp, cin.ctypes.data, ci_off.ctypes.data, c_len.ctypes.data,
             c_pno.ctypes.data, c_pn.ctypes.data, m, cout.ctypes.data, co_off.ctypes.data, threads)

    def timed(fn):
        reps, t0 = 0, time.perf_counter()
        while reps < 1 or time.perf_counter() - t0 < cpu_seconds:
            assert fn(suite, *args_) == 0
            reps += 1
        return reps, time.perf_counter() - t0
    reps, dt = timed(ol.lib().or_quic_seal_batch2)
    res["cpu_baseline"] = {"value": round(reps * m * payload / dt / 2**30, 3), "unit": "GiB/s",
                           "cores": threads, "kind": "port",
                           "sample": f"{reps} x {m} packets seal, oracle/oracle.c "
                                     "or_quic_seal_batch2 (scalar C restatement)"}
    so = os.path.join(REPO, "oracle", "libossl_quic.so")
    if os.path.exists(so):
        L2 = ctypes.CDLL(so)
        L2.ossl_quic_seal_batch.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 8 + \
            [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        m_before = m
        reps, dt = timed(L2.ossl_quic_seal_batch)
        chk = ol.quic_seal(key, iv, hp, 0, d[0].tobytes(), 9, suite=suite)[0]
        res["cpu_openssl_threads"] = {
            "value": round(reps * m_before * payload / dt / 2**30, 3),
            "unit": "GiB/s", "cores": threads,
            "matches_oracle": cout[:ln + 16].tobytes() == chk,
            "sample": f"{reps} x {m_before} packets seal, OpenSSL libcrypto EVP "
                      "(oracle/ossl_quic.c), one context per thread; OpenSSL 3.0 "
                      "serialises threads, see cpu_openssl"}
    exe = os.path.join(REPO, "oracle", "ossl_quic_procs")
    if os.path.exists(exe):
        import subprocess

        def procs(p):
            r = subprocess.run([exe, str(suite), str(p), "8192", str(ln), str(cpu_seconds)],
                               capture_output=True, text=True, timeout=120)
            assert r.returncode == 0, r.stderr
            return json.loads(r.stdout)
        one, many = procs(1), procs(threads)
        res["cpu_openssl"] = {
            "value": round(many["gib_s"] * payload / ln, 3), "unit": "GiB/s", "cores": threads,
            "per_core": round(one["gib_s"] * payload / ln, 3),
            "sample": f"OpenSSL libcrypto EVP seal (oracle/ossl_quic.c) in {threads} worker "
                      f"processes x 8192 packets of {ln} B (oracle/ossl_quic_procs); payload "
                      "GiB/s; processes, because OpenSSL 3.0 threads serialise on the EVP "
                      "per-call path (16 threads 6.1 vs 16 processes 24.9 GiB/s on this box)"}
    return res


def quic_fused_rate(torch, sqobfs, ctx, dev, steps, n, ln, data, in_off, lens, pno, pn, key, iv,
                    hp, suite=0):
    """Hysteria2's datagram path: QUIC seal then Salamander obfuscation, as
    two launches (sqobfs_quic_seal into an intermediate buffer, then
    sqobfs_launch) and fused (sqobfs_quic_seal_salamander); and the way in
    (deobfuscate + open vs sqobfs_quic_open_salamander).  Parity of the fused
    wire against the two-launch wire on every byte."""
    import numpy as np
    PSK_ = PSK
    wl = ln + 24
    s = torch.cuda.current_stream(dev).cuda_stream
    g = torch.Generator(device=dev)
    g.manual_seed(9)
    salts = torch.randint(0, 256, (n * 8,), generator=g, device=dev, dtype=torch.uint8)
    sealed = torch.zeros(n * (ln + 16), device=dev, dtype=torch.uint8)
    wire2 = torch.zeros(n * wl, device=dev, dtype=torch.uint8)
    wire1 = torch.zeros(n * wl, device=dev, dtype=torch.uint8)
    opened = torch.zeros(n * ln, device=dev, dtype=torch.uint8)
    s_off = torch.arange(n, device=dev, dtype=torch.int64) * (ln + 16)
    w_off = torch.arange(n, device=dev, dtype=torch.int64) * wl
    slens = torch.full((n,), ln + 16, device=dev, dtype=torch.int32)
    wlens = torch.full((n,), wl, device=dev, dtype=torch.int32)
    z = lambda: torch.zeros(n, device=dev, dtype=torch.int32)  # noqa: E731
    o1, o2, o3, o4, o5 = z(), z(), z(), z(), z()
    largest = pn - 1
    res = {}
    with sqobfs.QuicKeyring(ctx, [sqobfs.QuicKey.of(key, iv, hp)], suite) as kr, \
            sqobfs.Keyring(ctx, sqobfs.SALAMANDER, [PSK_]) as okr:
        b_seal = sqobfs.quic_batch(n, data, in_off, lens, sealed, s_off, o1, pno, pn)
        b_obfs = sqobfs.make_batch(n, sealed, s_off, slens, wire2, w_off, o2, salt=salts)
        b_fused = sqobfs.quic_batch(n, data, in_off, lens, wire1, w_off, o3, pno, pn)
        b_deo = sqobfs.make_batch(n, wire1, w_off, wlens, sealed, s_off, o4)
        b_open = sqobfs.quic_batch(n, sealed, s_off, slens, opened, in_off, o5, pno, largest)
        b_fopen = sqobfs.quic_batch(n, wire1, w_off, wlens, opened, in_off, o5, pno, largest)

        def timed(fn):
            warm_up(torch, dev, fn)
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(steps)]
            for e0, e1 in ev:
                e0.record()
                fn()
                e1.record()
            torch.cuda.synchronize(dev)
            return sum(e0.elapsed_time(e1) for e0, e1 in ev) / steps * 1e3
        two_out = timed(lambda: (sqobfs.quic_seal(ctx, kr, b_seal, s),
                                 sqobfs.launch(ctx, okr, sqobfs.OBFUSCATE, b_obfs, s)))
        fused_out = timed(lambda: sqobfs.quic_seal_salamander(ctx, kr, okr, b_fused, salts, s))
        same = bool(torch.equal(wire1, wire2))
        two_in = timed(lambda: (sqobfs.launch(ctx, okr, sqobfs.DEOBFUSCATE, b_deo, s),
                                sqobfs.quic_open(ctx, kr, b_open, s)))
        fused_in = timed(lambda: sqobfs.quic_open_salamander(ctx, kr, okr, b_fopen, s))
        ok_in = bool((o5 == ln).all()) and bool(torch.equal(opened, data))
    payload = n * (ln - 11)
    for name, us in (("seal_then_obfuscate_us", two_out), ("fused_seal_us", fused_out),
                     ("deobfuscate_then_open_us", two_in), ("fused_open_us", fused_in)):
        res[name] = round(us, 2)
    res["fused_seal_GiB_s_payload"] = round(payload / (fused_out * 1e-6) / 2**30, 2)
    res["fused_open_GiB_s_payload"] = round(payload / (fused_in * 1e-6) / 2**30, 2)
    res["fused_wire_equals_two_launch_wire"] = same
    res["fused_open_round_trip"] = ok_in
    res["traffic_note"] = ("two launches move read L + write L+16 + read L+16 + write L+24 "
                           "per packet; fused: read L + write L+24")
    return res


def udp_quic_rate(sqobfs, ctx, kr, plen, seconds=3.0, batch=256, suite=0):
    """Hysteria2's data path over loopback, one thread: QUIC packets of plen
    bytes (11-byte short header) -> sqobfs_udp_conn_write_quic (seal +
    Salamander in one launch, GSO send) -> sqobfs_udp_conn_read_quic (GRO
    receive, de-obfuscate + open in one launch)."""
    import ctypes
    import socket
    import numpy as np
    rng = np.random.Generator(np.random.PCG64(13))

    def sock():
        s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        s.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 8 << 20)
        s.bind(("127.0.0.1", 0))
        return s
    srv_s, cli_s = sock(), sock()
    kl = 16 if suite else 32
    key, iv, hp = (rng.integers(0, 256, m, dtype=np.uint8).tobytes() for m in (kl, 12, kl))
    qkr = sqobfs.QuicKeyring(ctx, [sqobfs.QuicKey.of(key, iv, hp)], suite)
    srv = sqobfs.UdpConn(ctx, kr, [srv_s.fileno()], slots=batch)
    cli = sqobfs.UdpConn(ctx, kr, [cli_s.fileno()], slots=batch)
    on = cli.set_offload(sqobfs.UDP_TX_GSO) | srv.set_offload(sqobfs.UDP_RX_GRO)
    lib = sqobfs.lib()
    lens = np.full(batch, plen, np.uint32)
    to = (sqobfs.Addr * batch)(*[sqobfs.Addr.of(*srv_s.getsockname())] * batch)
    pn = np.arange(batch, dtype=np.uint64)
    for i in range(batch):
        p = cli.tx_payload(i)
        p[:plen] = rng.integers(0, 256, plen, dtype=np.uint8)
        p[0] = 0x41
    slot0 = lib.sqobfs_udp_conn_tx_payload(cli.handle, 0) - 8  # Salamander: S = 8
    tx = np.ctypeslib.as_array((ctypes.c_uint8 * (batch * 2048)).from_address(slot0))
    tx = tx.reshape(batch, 2048)
    sent = ctypes.c_uint32(0)
    v = sqobfs.UdpView()
    pp = ctypes.c_void_p()
    moved = lost = bad = 0
    base = 0
    t_end = time.perf_counter() + seconds
    t0 = time.perf_counter()
    while time.perf_counter() < t_end:
        # headers (the in-place seal left wire bytes in the slots): first byte
        # and the 2-byte packet number, for the whole batch at once
        seq = np.arange(base, base + batch, dtype=np.int64)
        tx[:, 8] = 0x41
        tx[:, 8 + 9] = (seq >> 8) & 0xFF
        tx[:, 8 + 10] = seq & 0xFF
        pn[:] = np.arange(base, base + batch, dtype=np.uint64)
        assert lib.sqobfs_udp_conn_write_quic(cli.handle, qkr.handle, 0, batch, lens.ctypes.data,
                                              9, pn.ctypes.data, to, ctypes.byref(sent)) == 0
        got = 0
        while got < batch:
            assert lib.sqobfs_udp_conn_read_quic(srv.handle, qkr.handle, 9, max(base, 1) - 1,
                                                 200, ctypes.byref(v), ctypes.byref(pp)) == 0
            if v.count == 0:
                lost += batch - got
                break
            ln = np.ctypeslib.as_array((ctypes.c_uint32 * v.count).from_address(v.len))
            ok = int((ln == plen).sum())
            bad += v.count - ok
            moved += ok  # only datagrams that opened count toward the rate
            got += v.count
        base += batch
    dt = time.perf_counter() - t0
    srv.close()
    cli.close()
    qkr.close()
    srv_s.close()
    cli_s.close()
    return {"suite": ["chacha20_poly1305", "aes_128_gcm"][suite], "quic_packet_bytes": plen,
            "batch": batch, "offload": on, "datagrams_per_s": round(moved / dt),
            "counted": "datagrams that opened (ln == packet length); lost and failed_open "
                       "are excluded",
            "GiB_s_quic_payload": round(moved * (plen - 11) / dt / 2**30, 4),
            "lost": lost, "failed_open": bad,
            "path": "sqobfs_udp_conn_write_quic (QUIC seal + Salamander obfuscate, one launch, "
                    "GSO sendmmsg) -> loopback -> sqobfs_udp_conn_read_quic (GRO recvmmsg, "
                    "deobfuscate + open, one launch), one thread"}


def udp_rate(sqobfs, ctx, kr, kind, L, seconds=3.0, batch=256, nsock=4, offload=0):
    """Loopback UDP end to end through the batched socket layer
    (sqobfs_udp_conn): a client endpoint obfuscates a batch on the GPU
    (device salts) and sends it with sendmmsg to `nsock` server sockets; the
    server endpoint receives the batch with recvmmsg fan-in and deobfuscates
    it on the GPU.  One thread, batch after batch, so the rate is the sum of
    both sides' costs (GPU round trips + syscalls + loopback stack).
    offload: UDP_TX_GSO on the client and / or UDP_RX_GRO on the server
    (runs of batch / nsock datagrams go to each server socket)."""
    import socket
    import numpy as np
    rng = np.random.Generator(np.random.PCG64(11))

    def sock():
        s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        s.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 8 << 20)
        s.bind(("127.0.0.1", 0))
        return s
    srv_s = [sock() for _ in range(nsock)]  # fan-in, as hysteria port hopping
    cli_s = sock()
    to = [sqobfs.Addr.of("127.0.0.1", srv_s[i * nsock // batch].getsockname()[1])
          for i in range(batch)]
    arr = (sqobfs.Addr * batch)(*to)
    lens = np.full(batch, L, np.uint32)
    srv = sqobfs.UdpConn(ctx, kr, [s.fileno() for s in srv_s], slots=batch)
    cli = sqobfs.UdpConn(ctx, kr, [cli_s.fileno()], slots=batch)
    on = cli.set_offload(offload & sqobfs.UDP_TX_GSO) | srv.set_offload(offload & sqobfs.UDP_RX_GRO)
    for i in range(batch):
        cli.tx_payload(i)[:L] = rng.integers(0, 256, L, dtype=np.uint8)
    import ctypes
    sent = ctypes.c_uint32(0)
    lib = sqobfs.lib()
    v = sqobfs.UdpView()
    batches = moved = lost = 0
    t_end = time.perf_counter() + seconds
    t0 = time.perf_counter()
    while time.perf_counter() < t_end:
        st = lib.sqobfs_udp_conn_write(cli.handle, 0, batch, lens.ctypes.data, arr,
                                       ctypes.byref(sent))
        assert st == 0 and sent.value == batch
        got = 0
        while got < batch:
            st = lib.sqobfs_udp_conn_read(srv.handle, 200, ctypes.byref(v))
            assert st == 0
            if v.count == 0:  # dropped by the loopback stack
                lost += batch - got
                break
            got += v.count
        moved += got
        batches += 1
    dt = time.perf_counter() - t0
    srv.close()
    cli.close()
    # the same loop with the GPU step removed: raw sendmmsg / recvmmsg of
    # already-obfuscated wire bytes (the socket layer's own ceiling here)
    S = 8 if kind == 0 else 16
    wire = rng.integers(0, 256, batch * (L + S), dtype=np.uint8)
    off = np.arange(batch, dtype=np.uint64) * (L + S)
    wlen = np.full(batch, L + S, np.uint32)
    slots = np.zeros(batch * 2048, np.uint8)
    fds = np.array([s.fileno() for s in srv_s], np.int32)
    rlen = np.zeros(batch, np.uint32)
    rfi = np.zeros(batch, np.uint16)
    cnt = ctypes.c_uint32(0)
    raw = 0
    t_end = time.perf_counter() + seconds / 2
    t1 = time.perf_counter()
    while time.perf_counter() < t_end:
        assert lib.sqobfs_udp_send(cli_s.fileno(), wire.ctypes.data, off.ctypes.data,
                                   wlen.ctypes.data, arr, batch, ctypes.byref(sent)) == 0
        got = 0
        while got < batch:
            assert lib.sqobfs_udp_recv(fds.ctypes.data, nsock, slots.ctypes.data, 2048, 0,
                                       batch, 200, rlen.ctypes.data, rfi.ctypes.data, None,
                                       ctypes.byref(cnt)) == 0
            if cnt.value == 0:
                break
            got += cnt.value
        raw += got
    dt_raw = time.perf_counter() - t1
    for s in srv_s + [cli_s]:
        s.close()
    return {"payload_bytes": L, "batch": batch, "server_sockets": nsock, "batches": batches,
            "offload": {"asked": offload, "in_effect": on},
            "datagrams_per_s": round(moved / dt), "GiB_s_payload": round(moved * L / dt / 2**30, 4),
            "lost": lost,
            "sockets_only_datagrams_per_s": round(raw / dt_raw),
            "path": "sqobfs_udp_conn_write (GPU obfuscate in the mapped slots, device salts, "
                    "sendmmsg) -> loopback -> sqobfs_udp_conn_read (recvmmsg fan-in over the "
                    "server sockets, GPU deobfuscate in the mapped slots), one thread"}


if __name__ == "__main__":
    sys.exit(main() or 0)
