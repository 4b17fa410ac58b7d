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
