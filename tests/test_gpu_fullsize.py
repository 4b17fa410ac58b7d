"""BASELINE.json configs at full size on the GPU, checked bit-exactly against
the oracle on EVERY packet of the batch (no sampling):

  * the HIP obfuscate output is compared, byte for byte over the whole output
    buffer, with the threaded C restatement (`or_batch_run`, 16 host threads)
    run over the same host copies of payloads, salts, offsets and PSK ids;
  * the HIP deobfuscate of that wire batch is compared the same way with the
    restatement's deobfuscate, and the decoded payloads with the input;
  * every out_len is compared with the restatement's;
  * dense outputs: the bytes outside the datagrams are untouched.

The restatement writes exactly the datagram bytes; its output buffer starts
as a copy of the GPU's, so the comparison covers every datagram byte and, in
slotted layouts, leaves the padding the batch declared scratch
(SQOBFS_FLAG_OUT_BLOCKS / _OUT_LINES) as the GPU wrote it.

Configs:
  configs[0]  65,536 x 1200 B Salamander round trip (the CPU config, on the HIP path)
  configs[1]  1,048,576 x 1350 B Salamander (dense and the Go Slots' 2048-byte slots)
  configs[2]  1,048,576 x 1200 B XPlus
  configs[3]  4,194,304 ragged U[64,1452] Salamander, dense and 16-byte-aligned slots
  configs[4]  one whole 2,097,152-packet shard (rank 3 of 8) with 256 PSKs

Reference behaviour: hysteria2/salamander.go:42-70, hysteria/xplus.go:46-75.
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
ORACLE_THREADS = 16  # the GPU box's CPU share


def _host(t):
    return None if t is None else t.cpu().numpy()


def _full_parity(config: str, layout: str = "dense", n=None, L="config", rank=0, world=1,
                 slot_flag=None):
    import torch
    import bench
    import sqobfs
    kind, n_total, cL, n_psk = bench.CONFIGS[config]
    if L == "config":
        L = cL
    if n is None:
        n, first = bench.shard(config, n_total, world, rank)
    else:
        first = 0
    dev = torch.device("cuda", 0)
    sh = bench.build_shard(torch, dev, kind, n, L, n_psk, rank, world, config, layout, first)
    S = sh["S"]
    flags = 0
    if sh["slotted"]:
        flags = sqobfs.FLAG_OUT_LINES if slot_flag == "lines" else sqobfs.FLAG_OUT_BLOCKS
    lens = sh["lens"]
    h_data, h_in_off, h_lens = _host(sh["data"]), _host(sh["in_off"]), _host(lens)
    h_out_off, h_salt = _host(sh["out_off"]), _host(sh["salt"])
    h_ids = _host(sh["psk_id"])
    h_ids = None if h_ids is None else h_ids.view(np.uint16)
    with sqobfs.Context(0) as ctx, sqobfs.Keyring(ctx, kind, sh["psks"]) as kr:
        ctx.unit_packets = sqobfs.unit_packets_for(sh["payload_bytes"], n, n_psk > 1, kind)
        # -------- obfuscate: every datagram vs the restatement
        b = sqobfs.make_batch(n, sh["data"], sh["in_off"], lens, sh["out"], sh["out_off"],
                              sh["out_len"], sh["salt"], sh["psk_id"], flags=flags)
        sqobfs.launch(ctx, kr, sqobfs.OBFUSCATE, b)
        torch.cuda.synchronize()
        g_out, g_len = _host(sh["out"]), _host(sh["out_len"])
        ref_out, ref_len = g_out.copy(), np.zeros(n, np.uint32)
        hb = sqobfs.HostBatch(h_data, h_in_off.view(np.uint64), h_lens.view(np.uint32), ref_out,
                              h_out_off.view(np.uint64), ref_len, h_salt, h_ids)
        # the restatement must write every datagram byte: poison its copy first
        # so an unwritten byte cannot pass as the GPU's
        if layout == "dense":
            lead = int(h_out_off[0])
            end = int(h_out_off[-1]) + int(h_lens[-1]) + S
            ref_out[lead:end] ^= 0x5A
            assert not g_out[:lead].any() and not g_out[end:].any(), "write outside the datagrams"
        ol.batch_run(kind, ol.OBFUSCATE, sh["psks"], hb, ORACLE_THREADS)
        assert np.array_equal(ref_len, g_len.view(np.uint32))
        assert np.array_equal(ref_len, h_lens.astype(np.uint32) + S)
        if not np.array_equal(ref_out, g_out):
            bad = np.flatnonzero(ref_out != g_out)
            pytest.fail(f"{config}/{layout} obfuscate: {bad.size} bytes differ, first at {bad[0]}")
        del ref_out
        # -------- deobfuscate the wire batch: every payload vs the restatement
        wl = (lens + S).to(torch.int32)
        if sh["slotted"]:
            back_off = sh["in_off"]
            back = torch.zeros_like(sh["data"])
        else:
            l64 = lens.to(torch.int64)
            back_off = torch.cumsum(l64, 0) - l64 + 64
            back = torch.zeros(int(sh["payload_bytes"]) + 128, device=dev, dtype=torch.uint8)
        olen2 = torch.zeros_like(sh["out_len"])
        b2 = sqobfs.make_batch(n, sh["out"], sh["out_off"], wl, back, back_off, olen2, None,
                               sh["psk_id"], flags=flags)
        sqobfs.launch(ctx, kr, sqobfs.DEOBFUSCATE, b2)
        torch.cuda.synchronize()
        g_back, g_len2 = _host(back), _host(olen2)
        h_back_off = _host(back_off).view(np.uint64)
        ref_back, ref_len2 = g_back.copy(), np.zeros(n, np.uint32)
        if not sh["slotted"]:
            ref_back[64:64 + sh["payload_bytes"]] ^= 0xA5
            assert not g_back[:64].any() and not g_back[64 + sh["payload_bytes"]:].any()
        hb2 = sqobfs.HostBatch(g_out, h_out_off.view(np.uint64), _host(wl).view(np.uint32),
                               ref_back, h_back_off, ref_len2, None, h_ids)
        ol.batch_run(kind, ol.DEOBFUSCATE, sh["psks"], hb2, ORACLE_THREADS)
        assert np.array_equal(ref_len2, g_len2.view(np.uint32))
        assert np.array_equal(ref_len2, h_lens.astype(np.uint32))
        if not np.array_equal(ref_back, g_back):
            bad = np.flatnonzero(ref_back != g_back)
            pytest.fail(f"{config}/{layout} deobfuscate: {bad.size} bytes differ, first at {bad[0]}")
        # the round trip is the identity on every payload: decode once more,
        # byte-exactly, into the input's own layout (its non-payload bytes are
        # zero, bench.build_shard) and compare the whole buffers
        again = torch.zeros_like(sh["data"])
        b3 = sqobfs.make_batch(n, sh["out"], sh["out_off"], wl, again, sh["in_off"], olen2, None,
                               sh["psk_id"])
        sqobfs.launch(ctx, kr, sqobfs.DEOBFUSCATE, b3)
        torch.cuda.synchronize()
        assert torch.equal(again, sh["data"])
    return n


def test_config0_salamander_64k_x_1200_on_hip():
    """configs[0]'s workload (the reference's CPU case) through the HIP path."""
    assert _full_parity("salamander-1m", n=65536, L=1200) == 65536


def test_config1_salamander_1m_x_1350():
    _full_parity("salamander-1m")


def test_config1_salamander_1m_slot2048_lines():
    """The Go Slots geometry: 2048-byte slots, SQOBFS_FLAG_OUT_LINES."""
    _full_parity("salamander-1m", layout="slot2048", slot_flag="lines")


def test_config2_xplus_1m_x_1200():
    _full_parity("xplus-1m")


def test_config3_salamander_ragged_4m_dense():
    _full_parity("salamander-ragged-4m")


def test_config3_salamander_ragged_4m_slot16():
    """SURVEY.md 8(d)'s own layout for configs[3]: 16-byte-aligned slots."""
    _full_parity("salamander-ragged-4m", layout="slot16")


def test_config4_salamander_256psk_one_whole_shard():
    """One of configs[4]'s eight 2,097,152-packet shards (rank 3: global
    packet ids 6,291,456.., psk_id = i mod 256), every packet checked."""
    assert _full_parity("salamander-16m-256psk", rank=3, world=8) == (1 << 24) // 8


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
