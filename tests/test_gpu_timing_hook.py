"""sqobfs_debug_time_next_launch (bench.py's per-launch timing): the armed
launch records its event pair with its own dispatch and its output is the
oracle's, as without the hook; the hook is spent by that launch (an empty
batch spends it too), and a later launch runs untimed."""
from __future__ import annotations

import numpy as np
import pytest
import sqobfs
from sqobfs import OBFUSCATE, SALAMANDER, XPLUS

import gpu_harness as gh

pytestmark = pytest.mark.gpu

PSK = [b"sing-quic-mi355x-bench-psk"]


@pytest.fixture(scope="module")
def ctx():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    c = sqobfs.Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("kind", [SALAMANDER, XPLUS])
def test_armed_launch_is_timed_and_exact(ctx, kind):
    rng = np.random.Generator(np.random.PCG64(4400 + kind))
    lens = rng.integers(0, 1500, 20000)
    hb = gh.make_case(rng, kind, OBFUSCATE, lens, PSK)
    ref = gh.run_oracle(kind, OBFUSCATE, PSK, hb)
    ev = sqobfs.DispatchEvents(2)
    try:
        with sqobfs.Keyring(ctx, kind, PSK) as kr:
            ev.arm(0)
            gh.run_device(ctx, kr, OBFUSCATE, hb)
            ms = ev.elapsed_ms(0)
            gh.assert_same(hb, ref, f"armed launch kind={kind}")
            assert 0.0 < ms < 1000.0, ms
            # spent: the next launch records nothing into pair 1 or 0
            hb2 = gh.clone(hb)
            gh.run_device(ctx, kr, OBFUSCATE, hb2)
            assert ev.elapsed_ms(0) == ms
            with pytest.raises(sqobfs.SqError):
                ev.elapsed_ms(1)
    finally:
        ev.close()


def test_empty_batch_spends_the_hook(ctx):
    rng = np.random.Generator(np.random.PCG64(4410))
    hb0 = gh.make_case(rng, SALAMANDER, OBFUSCATE, np.zeros(0, dtype=np.int64), PSK)
    hb = gh.make_case(rng, SALAMANDER, OBFUSCATE, rng.integers(0, 1500, 5000), PSK)
    ref = gh.run_oracle(SALAMANDER, OBFUSCATE, PSK, hb)
    ev = sqobfs.DispatchEvents(1)
    try:
        with sqobfs.Keyring(ctx, SALAMANDER, PSK) as kr:
            ev.arm(0)
            gh.run_device(ctx, kr, OBFUSCATE, hb0)  # n == 0: nothing launched
            gh.run_device(ctx, kr, OBFUSCATE, hb)
            gh.assert_same(hb, ref, "after an empty armed batch")
            with pytest.raises(sqobfs.SqError):
                ev.elapsed_ms(0)
    finally:
        ev.close()


def test_stale_hip_error_is_not_the_launch_s(ctx):
    """A failed HIP call of the caller's, left unread on this thread, is not
    taken for the next keyring build's or launch's error."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipEventCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
    hip.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p,
                                        ctypes.c_void_p]
    hip.hipEventDestroy.argtypes = [ctypes.c_void_p]
    a, b = ctypes.c_void_p(), ctypes.c_void_p()
    assert hip.hipEventCreate(ctypes.byref(a)) == 0 and hip.hipEventCreate(ctypes.byref(b)) == 0
    ms = ctypes.c_float()
    try:
        for kind in (SALAMANDER, XPLUS):
            # never recorded: fails, and the error stays unread
            assert hip.hipEventElapsedTime(ctypes.byref(ms), a, b) != 0
            rng = np.random.Generator(np.random.PCG64(4420 + kind))
            hb = gh.make_case(rng, kind, OBFUSCATE, rng.integers(0, 1500, 3000), PSK)
            ref = gh.run_oracle(kind, OBFUSCATE, PSK, hb)
            with sqobfs.Keyring(ctx, kind, PSK) as kr:
                assert hip.hipEventElapsedTime(ctypes.byref(ms), a, b) != 0
                gh.run_device(ctx, kr, OBFUSCATE, hb)
            gh.assert_same(hb, ref, f"after a stale error kind={kind}")
    finally:
        hip.hipGetLastError()
        hip.hipEventDestroy(a)
        hip.hipEventDestroy(b)
