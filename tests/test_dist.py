"""Multi-rank logic on the CPU (gloo, world_size 2): the sharding used by
bench.py and the scaling report, checked with the oracle standing in for the
device (packets are independent, so a sharded run must equal a single run
byte for byte; there is no data-path collective)."""
from __future__ import annotations

import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench
import oracle_lib as ol
import sqobfs


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_shards_partition_the_batch(world):
    n_total = bench.CONFIGS["salamander-16m-256psk"][1]
    seen = 0
    for r in range(world):
        n, first = bench.shard("salamander-16m-256psk", n_total, world, r)
        assert first == seen
        seen += n
    assert seen == n_total
    # weak-scaling configs: every rank has the full per-GPU batch
    n, first = bench.shard("salamander-1m", 1 << 20, world, world - 1)
    assert n == 1 << 20 and first == (world - 1) << 20


def _batch(first, n, S, psks):
    """Deterministic packets first..first+n (global ids), psk_id = id % 256."""
    ids = np.arange(first, first + n)
    rng = [np.random.Generator(np.random.PCG64(int(i))) for i in ids]
    pk = [r.integers(0, 256, int(r.integers(0, 300)), dtype=np.uint8).tobytes() for r in rng]
    salts = np.concatenate([np.random.Generator(np.random.PCG64(10**6 + int(i))).integers(
        0, 256, S, dtype=np.uint8) for i in ids])
    data, off, ln = sqobfs.pack(pk, align=1)
    oo = np.cumsum([0] + [len(p) + S for p in pk[:-1]]).astype(np.uint64)
    out = np.zeros(int(oo[-1]) + len(pk[-1]) + S + 8, np.uint8)
    hb = sqobfs.HostBatch(data, off, ln, out, oo, np.zeros(n, np.uint32), salts,
                          (ids % len(psks)).astype(np.uint16))
    ol.batch_run(0, 0, psks, hb, nthreads=1)
    return np.array([ol.fnv64(out[int(o):int(o) + int(l) + S]) for o, l in zip(oo, ln)],
                    dtype=np.uint64)


def _worker(rank, world, n_total, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    psks = [bytes([k]) * (8 + k % 57) for k in range(256)]
    n, first = bench.shard("salamander-16m-256psk", n_total, world, rank)
    h = torch.from_numpy(_batch(first, n, 8, psks).view(np.int64))
    parts = [torch.zeros(bench.shard("salamander-16m-256psk", n_total, world, r)[0],
                         dtype=torch.int64) for r in range(world)]
    dist.all_gather(parts, h)
    t = bench.max_over_ranks(torch, dist, float(rank + 1), torch.device("cpu"))
    if rank == 0:
        q.put((torch.cat(parts).numpy().tobytes(), t))
    dist.destroy_process_group()


def test_sharded_equals_single_gloo_world2():
    n_total = 600
    psks = [bytes([k]) * (8 + k % 57) for k in range(256)]
    single = _batch(0, n_total, 8, psks)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29611
    procs = [ctx.Process(target=_worker, args=(r, 2, n_total, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got, tmax = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert np.frombuffer(got, dtype=np.uint64).tolist() == single.tolist()
    assert tmax == 2.0  # max over ranks, as bench.py reports time


def test_bench_bare_launch_refuses_more_ranks_than_gpus():
    """`bench.py --gpus 2` without torchrun starts its own ranks, one per GPU:
    with fewer GPUs visible (none here) and no gloo opt-in it refuses before
    starting any rank, with a non-zero exit and no JSON line."""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2"],
                       cwd=repo, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 2, r.stderr[-2000:]
    assert "GPU(s) visible" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


class _StubSqobfs:
    """Just enough of the sqobfs binding for bench.e2e_all_ranks on the CPU:
    page-locked arrays are numpy arrays (refused on `fail_rank`), run_host
    writes the out_len the contract gives."""
    OBFUSCATE = 0
    FLAG_OUT_UNINIT = 1

    def __init__(self, rank, fail_rank):
        self.rank, self.fail_rank = rank, fail_rank

    def PinnedArray(self, ctx, nbytes):  # noqa: N802 (the binding's name)
        if self.rank == self.fail_rank:
            raise MemoryError("page-locked allocation refused (stub)")

        class _P:
            array = np.zeros(nbytes, np.uint8)

            def free(self):
                pass
        return _P()

    def HostBatch(self, data, in_off, in_len, out, out_off, out_len, salt, flags=0):  # noqa: N802
        class _H:
            pass
        h = _H()
        h.in_len, h.out_len = in_len, out_len
        h.as_batch = lambda: h
        return h

    def run_host(self, ctx, kr, direction, b):
        import time
        time.sleep(0.005)  # (a wall time the 5-decimal rounding of wall_s keeps)
        b.out_len[:] = b.in_len + 8


def _e2e_worker(rank, world, port, fail_rank, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = bench.e2e_all_ranks(torch, _StubSqobfs(rank, fail_rank), None, None, 0, dist,
                              torch.device("cpu"), world, n=4096, reps=2)
    if rank == 0:
        q.put(res)
    dist.destroy_process_group()


@pytest.mark.parametrize("fail_rank", [-1, 1])
def test_bench_e2e_leg_survives_a_failed_rank(fail_rank):
    """bench.py's host-staged leg on 2 gloo ranks: when one rank's part fails
    (its page-locked buffers refused), every rank still joins the barrier and
    the gather -- nothing hangs -- and rank 0 reports the failed rank instead
    of an aggregate; with no failure, the aggregate is both ranks' payload
    over the max-over-ranks wall."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29621 + (fail_rank + 1)
    procs = [ctx.Process(target=_e2e_worker, args=(r, 2, port, fail_rank, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert len(res["per_rank"]) == 2
    if fail_rank < 0:
        assert "failed_ranks" not in res and res["out_len_ok"]
        payload = 2 * 4096 * 1350 * 2
        assert abs(res["aggregate_gib_s"] - payload / res["wall_s"] / 2**30) <= 0.01 * res["aggregate_gib_s"]
    else:
        assert res["failed_ranks"] == [1] and "aggregate_gib_s" not in res
        assert res["per_rank"][1] == 0.0 and not res["out_len_ok"]
