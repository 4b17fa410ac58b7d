"""The CPU path and the GPU path agree (the packet conn engine switches
between them per batch, include/sqobfs.h):
  * every keyring's host hash state equals the state psk_prepare_kernel made
    on the GPU, byte for byte, for PSKs of 0..300 bytes;
  * sqobfs_cpu_run and a launch give identical bytes on the same batch;
  * SQOBFS_FLAG_DEVICE_SALT on the CPU path draws the context's ChaCha20
    stream (one sequence number per call, as a launch), so CPU and GPU salts
    of one context never repeat and follow include/sqobfs.h's construction."""
from __future__ import annotations

import numpy as np
import pytest
import sqobfs
from sqobfs import DEOBFUSCATE, OBFUSCATE, SALAMANDER, XPLUS

import gpu_harness as gh
import oracle_lib as ol

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kind", [SALAMANDER, XPLUS])
def test_host_and_device_keyring_state_identical(kind):
    rng = np.random.Generator(np.random.PCG64(50 + kind))
    psks = [rng.integers(0, 256, L, dtype=np.uint8).tobytes() for L in range(0, 301)]
    with sqobfs.Context(0) as ctx, sqobfs.Keyring(ctx, kind, psks) as kr:
        assert kr.device_check() == 0


@pytest.mark.parametrize("kind", [SALAMANDER, XPLUS])
@pytest.mark.parametrize("direction", [OBFUSCATE, DEOBFUSCATE])
def test_cpu_run_equals_launch(kind, direction):
    rng = np.random.Generator(np.random.PCG64(60 + 2 * kind + direction))
    psks = [rng.integers(0, 256, L, dtype=np.uint8).tobytes() for L in (0, 7, 26, 39, 40, 127,
                                                                         128, 200)]
    n = 3000
    ids = rng.integers(0, len(psks), n)
    lens = rng.integers(0, 1500, n)
    hb = gh.make_case(rng, kind, direction, lens, psks, psk_ids=ids, in_align=1, out_lead=5)
    gpu, cpu = gh.clone(hb), gh.clone(hb)
    with sqobfs.Context(0) as ctx, sqobfs.Keyring(ctx, kind, psks) as kr:
        gh.run_device(ctx, kr, direction, gpu)
        sqobfs.cpu_run(kr, direction, cpu.as_batch())
    gh.assert_same(cpu, gpu, f"cpu vs gpu kind={kind} dir={direction}")
    gh.assert_same(cpu, gh.run_oracle(kind, direction, psks, hb), "cpu vs oracle")


@pytest.mark.parametrize("kind", [SALAMANDER, XPLUS])
def test_cpu_salts_share_the_context_stream(kind):
    S = sqobfs.SALT_LEN[kind]
    key = bytes(range(7, 39))
    rng = np.random.Generator(np.random.PCG64(70 + kind))
    psks = [b"salt-stream"]
    n = 300
    with sqobfs.Context(0) as ctx, sqobfs.Keyring(ctx, kind, psks) as kr:
        ctx.salt_key(key, 41)
        outs = []
        for use_cpu in (True, False, True):
            hb = gh.make_case(rng, kind, OBFUSCATE, rng.integers(0, 1400, n), psks)
            hb.flags, hb.salt = sqobfs.FLAG_DEVICE_SALT, None
            hb.salt_out = np.zeros(n * S, np.uint8)
            if use_cpu:
                sqobfs.cpu_run(kr, OBFUSCATE, hb.as_batch())
            else:
                gh.run_device(ctx, kr, OBFUSCATE, hb)
            outs.append(hb)
        assert ctx.salt_seq == 44
    for k, hb in enumerate(outs):  # sequence numbers 41, 42, 43 in call order
        want = np.frombuffer(ol.device_salts(key, 41 + k, n, S), np.uint8)
        assert np.array_equal(hb.salt_out, want), k
        ref = gh.clone(hb)
        ref.flags, ref.salt = 0, want.copy()
        gh.assert_same(hb, gh.run_oracle(kind, OBFUSCATE, psks, ref), f"salts call {k}")
