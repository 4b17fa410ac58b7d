"""Deterministic placement regression for round 4's illegal-address fault
("What's weak" 7): `__builtin_amdgcn_readfirstlane` returns a
signed int, so a table address whose low 32-bit word had bit 31 set was
sign-extended when it was widened back into a 64-bit key-entry address
(fixed by `rfl32`, sing-quic_amd/csrc/sq_quic_gcm.hip).  The grouped
multi-key GCM test hit that only when the allocator happened to place the
keyring there.  Here every keyring table and the grouping scratch are
carved from a region whose low words are 0x80000100 and up
(sqobfs_debug_device_pool), and the test asserts that they were, so the
placement cannot silently become vacuous.  Checked against the oracle:
the multi-key AES-128-GCM launch (grouped and staged), ChaCha20-Poly1305
multi-key, and the multi-PSK obfuscation kernels of both schemes."""
from __future__ import annotations

import numpy as np
import pytest
import sqobfs
from sqobfs import DEOBFUSCATE, OBFUSCATE, SALAMANDER, XPLUS

import gpu_harness as gh
import oracle_lib as ol
from test_gpu_quic import _random_packets, ctx, run  # noqa: F401  (fixture)
from test_gpu_quic_gcm import _keys

pytestmark = pytest.mark.gpu

REGION = 64 << 20
LOW = 0x80000100  # the region's low 32-bit word: bit 31 set, room below 2^32


@pytest.fixture
def bit31_pool():
    import torch
    dev = torch.device("cuda", 0)
    # 4 GiB + the region: some offset in it has the wanted low word
    pool = torch.empty((1 << 32) + REGION, dtype=torch.uint8, device=dev)
    base = pool.data_ptr()
    region = base + (LOW - (base & 0xFFFFFFFF)) % (1 << 32)
    assert region + REGION <= base + pool.numel()
    assert (region & 0xFFFFFFFF) == LOW and (region + REGION - 1) & 0x80000000
    sqobfs.debug_device_pool(region, REGION)
    state = {"region": region, "used": None}
    try:
        yield state
    finally:
        state["used"] = sqobfs.debug_device_pool(None)
        torch.cuda.synchronize(dev)
        del pool


def _carved(state):
    used = sqobfs.debug_device_pool(state["region"], REGION)  # (re-armed, count read)
    assert used > 0, "nothing was carved from the bit-31 region: the test is vacuous"
    lo, hi = state["region"], state["region"] + used
    assert (lo & 0xFFFFFFFF) >= 0x80000000 and ((hi - 1) & 0xFFFFFFFF) >= 0x80000000
    return used


@pytest.mark.parametrize("suite", [sqobfs.QUIC_AES_128_GCM, sqobfs.QUIC_CHACHA20_POLY1305])
def test_quic_multi_key_at_bit31_addresses(ctx, bit31_pool, suite):  # noqa: F811
    """16 keys over 20,000 packets (the grouped, staged GCM kernel reads
    gmeta and the key table through readfirstlane'd words), seal then open."""
    rng = np.random.Generator(np.random.PCG64(31 + suite))
    if suite == sqobfs.QUIC_AES_128_GCM:
        kb, keys = _keys(rng, 16)
    else:  # ChaCha20-Poly1305: 32-byte key and hp
        kb = [tuple(rng.integers(0, 256, m, dtype=np.uint8).tobytes() for m in (32, 12, 32))
              for _ in range(16)]
        keys = [sqobfs.QuicKey.of(*k) for k in kb]
    n = 20000
    pkts, pnos, pns = _random_packets(rng, n)
    kid = rng.integers(0, 16, n)
    out, oo, ol_, _, _ = run(ctx, keys, True, pkts, pnos, pns, key_ids=kid, suite=suite)
    osuite = ol.AES128GCM if suite == sqobfs.QUIC_AES_128_GCM else ol.CHACHA20
    prot = []
    for i, p in enumerate(pkts):
        want, r = ol.quic_seal(*kb[kid[i]], pns[i], p, pnos[i], suite=osuite)
        assert ol_[i] == r == len(p) + 16, i
        got = out[int(oo[i]):int(oo[i]) + r].tobytes()
        assert got == want, i
        prot.append(got)
    out2, oo2, ol2, pno2, _ = run(ctx, keys, False, prot, pnos, pns, key_ids=kid, suite=suite)
    for i, p in enumerate(pkts):
        assert ol2[i] == len(p) and pno2[i] == pns[i], i
        assert out2[int(oo2[i]):int(oo2[i]) + ol2[i]].tobytes() == p, i
    _carved(bit31_pool)


@pytest.mark.parametrize("kind", [SALAMANDER, XPLUS])
@pytest.mark.parametrize("direction", [OBFUSCATE, DEOBFUSCATE])
def test_obfuscation_multi_psk_at_bit31_addresses(ctx, bit31_pool, kind, direction):  # noqa: F811
    """A 3-PSK keyring (PSKs of 5, 40 and 130 B: one- and two-block keys)
    whose table lies at a bit-31 address; a ragged batch against the oracle."""
    rng = np.random.Generator(np.random.PCG64(310 + 2 * kind + direction))
    psks = [rng.integers(0, 256, k, dtype=np.uint8).tobytes() for k in (5, 40, 130)]
    n = 5000
    lens = rng.integers(0, 1500, n)
    ids = rng.integers(0, 3, n).astype(np.uint16)
    hb = gh.make_case(rng, kind, direction, lens, psks, psk_ids=ids)
    ref = gh.run_oracle(kind, direction, psks, hb)
    kr = sqobfs.Keyring(ctx, kind, psks)
    try:
        gh.run_device(ctx, kr, direction, hb)
    finally:
        kr.close()
    gh.assert_same(hb, ref, f"kind {kind} dir {direction} at a bit-31 table")
    _carved(bit31_pool)
