"""bench.py's multi-rank path on the one-GPU box: two ranks launched by
torch.distributed.run share GPU 0 over gloo (RCCL refuses two ranks on one
device; the driver's 1/2/4/8-GPU runs use nccl, one rank per GPU).  Covers
what N > 1 adds to the single-GPU bench: the barrier-bracketed timing, the
max over ranks, the whole-job sum of payload bytes, the parity AND over
ranks, rank 0 printing one line, and configs[4]'s contiguous shards (strong
scaling) next to the weak-scaling configs[1]."""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("config,packets,scaling,launcher", [
    ("salamander-1m", 65536, "weak", "torchrun"),
    ("salamander-16m-256psk", 131072, "strong", "torchrun"),
    # the bare command: bench.py starts its own ranks (the driver's SCALE form)
    ("salamander-1m", 65536, "weak", "bare"),
    ("salamander-16m-256psk", 131072, "strong", "bare")])
def test_bench_two_ranks(config, packets, scaling, launcher):
    pre = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port())] \
        if launcher == "torchrun" else [sys.executable]
    cmd = pre + [os.path.join(REPO, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
           "--steps", "3", "--warmup", "1", "--warmup-s", "0", "--no-cpu-baseline",
           "--config", config, "--packets", str(packets)]
    env = dict(os.environ, OMP_NUM_THREADS="4")
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["scaling"] == scaling
    assert d["parity_spot_check"] is True
    assert d["value"] > 0 and d["ms_per_step"] > 0
    # whole-job payload over the max-over-ranks wall time
    per_rank = packets if scaling == "weak" else packets // 2
    total = 2 * per_rank * 1350 * d["steps"]
    assert abs(d["value"] - total / (d["ms_per_step"] * d["steps"] * 1e-3) / 2**30) \
        <= 0.01 * d["value"]  # ms_per_step is rounded to 0.1 us
    assert d["config"]["packets_per_gpu"] == per_rank
    # the host-staged batch on both ranks at once, after the timed region
    e = d["e2e"]
    assert len(e["per_rank"]) == 2 and all(r > 0 for r in e["per_rank"]) and e["out_len_ok"]
    payload = 2 * e["packets_per_rank"] * e["payload_bytes"] * e["reps"]
    assert abs(e["aggregate_gib_s"] - payload / e["wall_s"] / 2**30) <= 0.01 * e["aggregate_gib_s"]
    # the max-over-ranks wall: the aggregate is at most the ranks' own rates summed
    assert e["aggregate_gib_s"] <= sum(e["per_rank"]) * 1.01


def test_bench_one_rank_carries_e2e_and_no_e2e_skips_it():
    """The default N = 1 line carries the host-staged e2e key (one rank);
    --no-e2e leaves it out."""
    base = [sys.executable, os.path.join(REPO, "bench.py"), "--steps", "3", "--warmup", "1",
            "--warmup-s", "0", "--no-cpu-baseline", "--packets", "65536"]
    for extra, want in (([], True), (["--no-e2e"], False)):
        r = subprocess.run(base + extra, cwd=REPO, capture_output=True, text=True, timeout=110)
        assert r.returncode == 0, r.stderr[-3000:]
        d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
        assert ("e2e" in d) == want
        if want:
            e = d["e2e"]
            assert len(e["per_rank"]) == 1 and e["out_len_ok"]
            assert abs(e["aggregate_gib_s"] - e["per_rank"][0]) <= 0.01 * e["aggregate_gib_s"]


def test_bare_launch_stops_ranks_on_failure():
    """A rank that fails makes the bare command exit non-zero, promptly, with
    no JSON line (the other rank is stopped, not left in its barrier)."""
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--dist-backend",
           "gloo", "--steps", "1", "--warmup", "1", "--warmup-s", "0", "--no-cpu-baseline",
           "--packets", "1024", "--layout", "inplace", "--direction", "deobfuscate"]
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=110)
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
