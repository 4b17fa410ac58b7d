"""Keyring release (sqobfs_keyring_destroy, sqobfs_quic_keyring_destroy) does
not block and does not wait for other work on the device: its device memory
is freed in stream order after the launches that used it.  Hysteria's port
hopping re-dials (and so re-keys) every 30 s (hysteria/hop.go:114); a
connection closing must not stall the others."""
from __future__ import annotations

import time

import numpy as np
import pytest
import sqobfs
from sqobfs import OBFUSCATE, SALAMANDER

import gpu_harness as gh

pytestmark = pytest.mark.gpu

PSK = b"sing-quic-mi355x-bench-psk"


def _big_batch(torch, dev, n=1 << 20, L=1350):
    data = torch.randint(0, 256, (n * L + 64,), device=dev, dtype=torch.uint8)
    out = torch.zeros(n * (L + 8) + 64, device=dev, dtype=torch.uint8)
    lens = torch.full((n,), L, device=dev, dtype=torch.int32)
    in_off = torch.arange(n, device=dev, dtype=torch.int64) * L
    out_off = torch.arange(n, device=dev, dtype=torch.int64) * (L + 8)
    salt = torch.randint(0, 256, (n * 8,), device=dev, dtype=torch.uint8)
    olen = torch.zeros(n, device=dev, dtype=torch.int32)
    keep = (data, out, lens, in_off, out_off, salt, olen)
    return sqobfs.make_batch(n, data, in_off, lens, out, out_off, olen, salt), keep


def test_destroy_does_not_wait_for_another_contexts_work():
    import torch
    dev = torch.device("cuda", 0)
    a, b = sqobfs.Context(0), sqobfs.Context(0)
    try:
        kra = sqobfs.Keyring(a, SALAMANDER, [PSK])
        batch, keep = _big_batch(torch, dev)
        # context B: a connection opens and runs a small batch ...
        rng = np.random.Generator(np.random.PCG64(9))
        hb = gh.make_case(rng, SALAMANDER, OBFUSCATE, rng.integers(0, 1500, 64), [PSK])
        krb = sqobfs.Keyring(b, SALAMANDER, [PSK])
        gh.run_host(b, krb, OBFUSCATE, hb)
        torch.cuda.synchronize(dev)
        busy = torch.cuda.ExternalStream(a.stream, device=dev)
        for _ in range(100):  # ~50 ms of work queued on context A
            sqobfs.launch(a, kra, OBFUSCATE, batch, a.stream)
        # ... and closes while A is busy
        t0 = time.perf_counter()
        krb.close()
        dt = time.perf_counter() - t0
        still_busy = not busy.query()
        torch.cuda.synchronize(dev)
        kra.close()
        assert still_busy, "context A's queue drained before the check: not a test"
        assert dt < 2e-3, f"keyring destroy took {dt * 1e3:.2f} ms with another context busy"
        ref = gh.run_oracle(SALAMANDER, OBFUSCATE, [PSK], hb)
        gh.assert_same(hb, ref, "batch before the release")
    finally:
        a.close()
        b.close()


def test_destroy_while_its_own_launch_runs():
    """Destroyed right after an asynchronous launch that reads its table: the
    launch still sees the keyring (the free waits for it), the call returns
    at once."""
    import torch
    dev = torch.device("cuda", 0)
    with sqobfs.Context(0) as ctx:
        rng = np.random.Generator(np.random.PCG64(10))
        lens = rng.integers(0, 1500, 200000)
        psks = [PSK, b"", b"z" * 150]
        ids = rng.integers(0, 3, lens.size)
        hb = gh.make_case(rng, SALAMANDER, OBFUSCATE, lens, psks, psk_ids=ids)
        ref = gh.run_oracle(SALAMANDER, OBFUSCATE, psks, hb)
        t = lambda x: None if x is None else torch.from_numpy(x).to(dev)  # noqa: E731
        d = [t(x) for x in (hb.data, hb.in_off, hb.in_len, hb.out, hb.out_off, hb.out_len,
                            hb.salt, hb.psk_id)]
        b = sqobfs.make_batch(hb.n, *d)
        s = torch.cuda.current_stream(dev)
        torch.cuda.synchronize(dev)
        kr = sqobfs.Keyring(ctx, SALAMANDER, psks)
        for _ in range(8):  # in place of one: the last launch's output is checked
            sqobfs.launch(ctx, kr, OBFUSCATE, b, s.cuda_stream)
        t0 = time.perf_counter()
        kr.close()
        dt = time.perf_counter() - t0
        pending = not s.query()
        torch.cuda.synchronize(dev)
        hb.out[:] = d[3].cpu().numpy()
        hb.out_len[:] = d[5].cpu().numpy()
        gh.assert_same(hb, ref, "launches racing the keyring release")
        assert pending and dt < 2e-3, (pending, dt)


def test_sync_spin_is_opt_in():
    with sqobfs.Context(0) as ctx:
        L = sqobfs.lib()
        assert L.sqobfs_set_sync_spin(ctx.handle, 0) == 0
        ctx.sync(ctx.stream)
        assert L.sqobfs_set_sync_spin(ctx.handle, 1000) == 0
        ctx.sync(ctx.stream)
        assert L.sqobfs_set_sync_spin(None, 10) == sqobfs.SQ_EINVAL


def test_caller_stream_released_before_destroy():
    """A caller that destroys its own stream first releases it from the
    keyring (sqobfs_keyring_release_stream): the launch on it completes, and
    the keyring's later release never touches the destroyed handle (ADVICE
    round 3: the fence used to record on every stream it had seen)."""
    import torch
    dev = torch.device("cuda", 0)
    with sqobfs.Context(0) as ctx:
        kr = sqobfs.Keyring(ctx, SALAMANDER, [PSK])
        st = torch.cuda.Stream(dev)
        batch, keep = _big_batch(torch, dev, n=1 << 16)
        torch.cuda.synchronize(dev)
        sqobfs.launch(ctx, kr, OBFUSCATE, batch, st.cuda_stream)
        kr.release_stream(st.cuda_stream)  # waits for the launch
        assert st.query()
        olen = keep[6]
        assert int(olen.min().item()) == 1358 and int(olen.max().item()) == 1358
        del st  # torch destroys (or recycles) the stream
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        kr.close()
        assert time.perf_counter() - t0 < 0.05
        # releasing a stream the keyring never saw, or the null stream, is fine
        kr2 = sqobfs.Keyring(ctx, SALAMANDER, [PSK])
        kr2.release_stream(0)
        kr2.release_stream(torch.cuda.Stream(dev).cuda_stream)
        kr2.close()
