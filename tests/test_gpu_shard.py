"""Several contexts in one process (sqobfs_run_host_sharded, sqobfs_shard_run):
the sharded result equals the single-context result byte for byte.  The GPU
box has one GPU, so the shards are two contexts on device 0 -- the same
code path as one context per GPU (each shard has its own streams, staging
and keyring)."""
from __future__ import annotations

import numpy as np
import pytest
import sqobfs
from sqobfs import DEOBFUSCATE, OBFUSCATE, SALAMANDER, XPLUS

import gpu_harness as gh

pytestmark = pytest.mark.gpu

PSKS = [b"sing-quic-mi355x-bench-psk", b"", b"y" * 130]


@pytest.fixture(scope="module")
def ctxs():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    cs = [sqobfs.Context(0), sqobfs.Context(0)]
    yield cs
    for c in cs:
        c.close()


@pytest.mark.parametrize("kind", [SALAMANDER, XPLUS])
@pytest.mark.parametrize("direction", [OBFUSCATE, DEOBFUSCATE])
@pytest.mark.parametrize("layout", ["dense", "shuffled", "inplace"])
def test_run_host_sharded_matches_single(ctxs, kind, direction, layout):
    """'shuffled' permutes the packets so the shards' byte spans interleave and
    'inplace' decodes / encodes in the input buffer: shards whose output span
    meets another shard's span must not run at once (each copies its whole
    span), so the batch runs on one context -- the result is the same."""
    rng = np.random.Generator(np.random.PCG64(500 + 2 * kind + direction))
    n = 30000
    lens = rng.integers(0, 1500, n)
    ids = rng.integers(0, len(PSKS), n)
    hb = gh.make_case(rng, kind, direction, lens, PSKS, psk_ids=ids, in_align=1, out_align=1,
                      inplace=layout == "inplace")
    if layout == "shuffled":
        perm = rng.permutation(n)
        S = sqobfs.SALT_LEN[kind]
        hb.in_off, hb.in_len, hb.out_off = hb.in_off[perm], hb.in_len[perm], hb.out_off[perm]
        if hb.salt is not None:
            hb.salt = hb.salt.reshape(n, S)[perm].reshape(-1).copy()
        hb.psk_id = hb.psk_id[perm]
        if hb.in_cap is not None:
            hb.in_cap = hb.in_cap[perm]
    ref = gh.run_oracle(kind, direction, PSKS, hb)
    one = gh.clone(hb)
    krs = [sqobfs.Keyring(c, kind, PSKS) for c in ctxs]
    try:
        sqobfs.run_host(ctxs[0], krs[0], direction, one.as_batch())
        sqobfs.run_host_sharded(ctxs, krs, direction, hb.as_batch())
    finally:
        for k in krs:
            k.close()
    gh.assert_same(one, ref, "single context")
    gh.assert_same(hb, one, "sharded over two contexts")


@pytest.mark.parametrize("kind", [SALAMANDER, XPLUS])
def test_shard_run_device_resident(ctxs, kind):
    """Device-resident shards cut by bytes (sqobfs_shard_cuts), each launched
    on its own context's stream by sqobfs_shard_run."""
    import torch
    rng = np.random.Generator(np.random.PCG64(520 + kind))
    n = 40000
    lens = rng.integers(64, 1453, n)
    hb = gh.make_case(rng, kind, OBFUSCATE, lens, PSKS[:1])
    ref = gh.run_oracle(kind, OBFUSCATE, PSKS[:1], hb)
    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
    d_in, d_out = t(hb.data), t(hb.out)
    d_off, d_len, d_ooff = t(hb.in_off), t(hb.in_len), t(hb.out_off)
    d_olen, d_salt = t(hb.out_len), t(hb.salt)
    cut = sqobfs.shard_cuts(hb.in_len, 2).astype(np.int64)
    S = sqobfs.SALT_LEN[kind]
    bs = [sqobfs.make_batch(int(b - a), d_in, d_off[a:b], d_len[a:b], d_out, d_ooff[a:b],
                            d_olen[a:b], d_salt[S * a:S * b], None, None, None, 0)
          for a, b in zip(cut[:-1], cut[1:])]
    krs = [sqobfs.Keyring(c, kind, PSKS[:1]) for c in ctxs]
    try:
        torch.cuda.synchronize(dev)
        sqobfs.shard_run(ctxs, krs, OBFUSCATE, bs)
    finally:
        for k in krs:
            k.close()
    hb.out[:] = d_out.cpu().numpy()
    hb.out_len[:] = d_olen.cpu().numpy()
    gh.assert_same(hb, ref, "device shards")


@pytest.mark.parametrize("kind", [SALAMANDER, XPLUS])
def test_shard_launch_steps_in_flight(kind):
    """sqobfs_shard_launch: several steps queued before any is waited for
    (tickets), obfuscate then deobfuscate in flight together, each shard on
    its own context -- on distinct GPUs when the box has more than one, else
    on device 0 (the same path); both steps equal the oracle."""
    import torch
    ndev = torch.cuda.device_count()
    devs = [0, 1] if ndev > 1 else [0, 0]
    rng = np.random.Generator(np.random.PCG64(540 + kind))
    S = sqobfs.SALT_LEN[kind]
    n = 20000
    lens = rng.integers(64, 1453, n)
    hb = gh.make_case(rng, kind, OBFUSCATE, lens, PSKS[:1])
    ref = gh.run_oracle(kind, OBFUSCATE, PSKS[:1], hb)
    cut = sqobfs.shard_cuts(hb.in_len, 2).astype(np.int64)
    ctxs = [sqobfs.Context(d) for d in devs]
    krs = [sqobfs.Keyring(c, kind, PSKS[:1]) for c in ctxs]
    try:
        parts = []
        for k, (a, b) in enumerate(zip(cut[:-1], cut[1:])):
            dev = torch.device("cuda", devs[k])
            t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)  # noqa: E731
            m = int(b - a)
            base = int(hb.in_off[a])
            end = int(hb.in_off[b - 1]) + int(hb.in_len[b - 1])
            clean = np.zeros(end - base, np.uint8)  # payload bytes only
            for i in range(int(a), int(b)):
                o = int(hb.in_off[i]) - base
                clean[o:o + int(hb.in_len[i])] = hb.data[o + base:o + base + int(hb.in_len[i])]
            d_in = t(clean)
            d_ioff = t(hb.in_off[a:b] - base)
            d_len = t(hb.in_len[a:b])
            obase = int(hb.out_off[a])
            oend = int(hb.out_off[b - 1]) + int(hb.in_len[b - 1]) + S
            d_out = torch.zeros(oend - obase, dtype=torch.uint8, device=dev)
            d_ooff = t(hb.out_off[a:b] - obase)
            d_olen = torch.zeros(m, dtype=torch.int32, device=dev)
            d_back = torch.zeros_like(d_in)
            d_blen = torch.zeros(m, dtype=torch.int32, device=dev)
            d_wlen = t((hb.in_len[a:b] + S).astype(np.uint32))
            d_salt = t(hb.salt[S * a:S * b])
            # (each batch holds its tensors: shard 0's must outlive this loop,
            # or shard 1's allocations reuse their memory before the launch)
            obf = sqobfs.make_batch(m, d_in, d_ioff, d_len, d_out, d_ooff, d_olen, d_salt)
            deo = sqobfs.make_batch(m, d_out, d_ooff, d_wlen, d_back, d_ioff, d_blen)
            assert obf._keep[1] is d_ioff and deo._keep[2] is d_wlen
            parts.append((a, b, obase, d_in, d_out, d_olen, d_back, d_blen, obf, deo))
            torch.cuda.synchronize(dev)
        t1 = sqobfs.shard_launch(ctxs, krs, OBFUSCATE, [p[8] for p in parts])
        t2 = sqobfs.shard_launch(ctxs, krs, DEOBFUSCATE, [p[9] for p in parts])
        t2.wait()  # (stream order: the decode ran after the encode)
        assert t1.done()
        t1.wait()
        for a, b, obase, d_in, d_out, d_olen, d_back, d_blen, _, _ in parts:
            got = d_out.cpu().numpy()
            for i in range(int(a), int(b), 97):
                o = int(hb.out_off[i]) - obase
                L = int(hb.in_len[i]) + S
                assert got[o:o + L].tobytes() == \
                    ref.out[int(hb.out_off[i]):int(hb.out_off[i]) + L].tobytes()
            assert np.array_equal(d_olen.cpu().numpy(), ref.out_len[a:b].astype(np.int32))
            assert torch.equal(d_back, d_in)
            assert np.array_equal(d_blen.cpu().numpy(), hb.in_len[a:b].astype(np.int32))
    finally:
        for k in krs:
            k.close()
        for c in ctxs:
            c.close()
