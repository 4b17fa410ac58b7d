"""BASELINE.json configs at full size on the GPU, checked through properties
that do not need the oracle to process the whole batch:
  * obfuscate -> deobfuscate is the identity on every payload byte (whole
    batch compared on the device),
  * every out_len follows the length rules,
  * sampled packets (first, last, every 4099th) are byte-identical to the
    oracle, and the per-packet FNV checksums of the sample match
    (checksum of checksums),
  * bytes between packets of the wire-dense output are all written.
Plus the bench's multi-rank path (2 gloo ranks sharing the GPU)."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle_lib as ol

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run_config(config: str, n_override=None):
    import torch
    import bench
    import sqobfs
    kind, n_total, L, n_psk = bench.CONFIGS[config]
    n, first = bench.shard(config, n_total, 8 if config == "salamander-16m-256psk" else 1, 0)
    if n_override:
        n = n_override
    dev = torch.device("cuda", 0)
    sh = bench.build_shard(torch, dev, kind, n, L, n_psk, 0, 1, config, "dense", first)
    S = sh["S"]
    with sqobfs.Context(0) as ctx, sqobfs.Keyring(ctx, kind, sh["psks"]) as kr:
        b = sqobfs.make_batch(n, sh["data"], sh["in_off"], sh["lens"], sh["out"], sh["out_off"],
                              sh["out_len"], sh["salt"], sh["psk_id"])
        sqobfs.launch(ctx, kr, sqobfs.OBFUSCATE, b)
        torch.cuda.synchronize()
        lens = sh["lens"].to(torch.int64)
        assert torch.equal(sh["out_len"].to(torch.int64), lens + S)
        # wire-dense output: every byte between the first and last packet written
        lead = int(sh["out_off"][0].item())
        end = int((sh["out_off"][-1] + lens[-1] + S).item())
        assert int((sh["out"][lead:end] == 0).sum().item()) < (end - lead) // 128  # ~1/256 zeros
        # round trip on the whole batch
        back = torch.full_like(sh["data"], 0)
        wl = (lens + S).to(torch.int32)
        olen2 = torch.zeros_like(sh["out_len"])
        b2 = sqobfs.make_batch(n, sh["out"], sh["out_off"], wl, back, sh["in_off"], olen2, None,
                               sh["psk_id"])
        sqobfs.launch(ctx, kr, sqobfs.DEOBFUSCATE, b2)
        torch.cuda.synchronize()
        assert torch.equal(olen2.to(torch.int64), lens)
        # non-payload input bytes are zero (bench.build_shard) and `back`
        # starts zeroed, so the whole buffers must match
        assert torch.equal(back, sh["data"])
    # sampled oracle parity + checksum of checksums
    saved = bench.save_samples(sh, n)
    assert bench.spot_check(torch, sh, kind, n, sh["out"], saved, 1)
    write = ol.salamander_write if kind == 0 else ol.xplus_write
    ids = sh["psk_id"].cpu().numpy() if sh["psk_id"] is not None else None
    out_off = sh["out_off"].cpu().numpy()
    h_gpu = h_ref = 0
    for i, p in saved.items():
        s = sh["salt"][i * S:(i + 1) * S].cpu().numpy().tobytes()
        w, _ = write(sh["psks"][int(ids[i]) if ids is not None else 0], s, p)
        got = sh["out"][int(out_off[i]):int(out_off[i]) + len(w)].cpu().numpy()
        h_gpu = ol.fnv64(got, h_gpu)
        h_ref = ol.fnv64(np.frombuffer(w, np.uint8).copy(), h_ref)
    assert h_gpu == h_ref


def test_config2_salamander_1m_x_1350():
    _run_config("salamander-1m")


def test_config3_xplus_1m_x_1200():
    _run_config("xplus-1m")


def test_config4_salamander_ragged_4m():
    _run_config("salamander-ragged-4m")


def test_config5_salamander_256psk_one_of_8_shards():
    _run_config("salamander-16m-256psk")


def test_bench_two_ranks_share_gpu():
    """bench.py's multi-rank path (barrier, max-over-ranks timing, sharded
    configs[4]) with 2 gloo ranks on one GPU."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29533", os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--dist-backend", "gloo", "--steps", "3", "--warmup", "1",
           "--no-cpu-baseline", "--config", "salamander-16m-256psk"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    d = json.loads(line)
    assert d["n_gpus"] == 2 and d["parity_spot_check"] is True
    assert d["config"]["packets_per_gpu"] == (1 << 24) // 2
    assert d["scaling"] == "strong"
