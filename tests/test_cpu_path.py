"""The product's CPU path (host/sq_cpu.cpp through sqobfs_cpu_run and host
keyrings), against the oracle on the same inputs -- no GPU needed.

This is the byte work the packet conn engine does without a GPU, for small
batches and after a failed launch (include/sqobfs.h); it must give the
reference's bytes exactly as the kernels do (hysteria2/salamander.go:42-70,
hysteria/xplus.go:46-75).  Its hashes are its own (RFC 7693 BLAKE2b, FIPS
180-4 SHA-256, RFC 8439 ChaCha20), not the oracle's."""
from __future__ import annotations

import json
import os

import numpy as np
import pytest
import sqobfs
from sqobfs import DEOBFUSCATE, OBFUSCATE, SALAMANDER, XPLUS

import gpu_harness as gh
import oracle_lib as ol

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")


def _cpu(kind, direction, psks, hb):
    got = gh.clone(hb)
    with sqobfs.Keyring(None, kind, psks) as kr:
        sqobfs.cpu_run(kr, direction, got.as_batch())
    return got


@pytest.mark.parametrize("kind", [SALAMANDER, XPLUS])
@pytest.mark.parametrize("direction", [OBFUSCATE, DEOBFUSCATE])
def test_ragged_batch_matches_oracle(kind, direction):
    rng = np.random.Generator(np.random.PCG64(100 + 2 * kind + direction))
    lens = np.concatenate([np.arange(0, 70), rng.integers(0, 1500, 700), [4000, 9000]])
    psks = [b"sing-quic-mi355x-bench-psk"]
    hb = gh.make_case(rng, kind, direction, lens, psks, in_align=1, out_lead=3, gaps=True)
    gh.assert_same(_cpu(kind, direction, psks, hb), gh.run_oracle(kind, direction, psks, hb),
                   f"cpu kind={kind} dir={direction}")


@pytest.mark.parametrize("kind", [SALAMANDER, XPLUS])
def test_every_psk_length_and_block_boundary(kind):
    """PSKs of 0..300 bytes (BLAKE2b 128-byte and SHA-256 55/64/119-byte block
    edges: one or two compressions per packet from the host midstate)."""
    rng = np.random.Generator(np.random.PCG64(7 + kind))
    psks = [rng.integers(0, 256, L, dtype=np.uint8).tobytes() for L in range(0, 301)]
    n = 1800
    ids = np.arange(n) % len(psks)
    for direction in (OBFUSCATE, DEOBFUSCATE):
        lens = rng.integers(0, 300, n)
        hb = gh.make_case(rng, kind, direction, lens, psks, psk_ids=ids)
        gh.assert_same(_cpu(kind, direction, psks, hb), gh.run_oracle(kind, direction, psks, hb),
                       f"psk lengths kind={kind} dir={direction}")


@pytest.mark.parametrize("kind", [SALAMANDER, XPLUS])
@pytest.mark.parametrize("direction", [OBFUSCATE, DEOBFUSCATE])
def test_in_place_layouts(kind, direction):
    """The vectorised writers' headroom layout (salamander.go:81-93) and the
    decode in place behind the salt (the packet conn engine's slots)."""
    rng = np.random.Generator(np.random.PCG64(31 + kind + 2 * direction))
    lens = rng.integers(0, 1500, 400)
    psks = [b"k" * 45]
    hb = gh.make_case(rng, kind, direction, lens, psks, inplace=True)
    gh.assert_same(_cpu(kind, direction, psks, hb), gh.run_oracle(kind, direction, psks, hb),
                   f"in place kind={kind} dir={direction}")


def test_xplus_read_buffer_quirk():
    """xplus.go:55 XORs to len(p), not n: in_cap > n decodes the extra bytes."""
    rng = np.random.Generator(np.random.PCG64(3))
    lens = rng.integers(0, 1300, 300)
    psks = [b"xplus-key"]
    hb = gh.make_case(rng, XPLUS, DEOBFUSCATE, lens, psks, cap_extra=rng.integers(0, 700, 300))
    gh.assert_same(_cpu(XPLUS, DEOBFUSCATE, psks, hb),
                   gh.run_oracle(XPLUS, DEOBFUSCATE, psks, hb), "xplus in_cap")


def test_golden_vectors():
    """tests/golden (made by oracle/py_oracle.py with hashlib)."""
    for name, kind in (("salamander_write.json", SALAMANDER), ("xplus_write.json", XPLUS)):
        cases = json.load(open(os.path.join(GOLDEN, name)))
        cases = cases["cases"] if isinstance(cases, dict) else cases
        for c in cases:
            psk, salt, pay = (bytes.fromhex(c[k]) for k in ("psk", "salt", "payload"))
            wire = bytes.fromhex(c["wire"])
            S = sqobfs.SALT_LEN[kind]
            hb = sqobfs.HostBatch(np.frombuffer(pay + b"\0", np.uint8).copy(),
                                  np.array([0], np.uint64), np.array([len(pay)], np.uint32),
                                  np.zeros(len(pay) + S + 1, np.uint8), np.array([0], np.uint64),
                                  np.zeros(1, np.uint32),
                                  np.frombuffer(salt, np.uint8).copy())
            with sqobfs.Keyring(None, kind, [psk]) as kr:
                sqobfs.cpu_run(kr, OBFUSCATE, hb.as_batch())
            assert hb.out[:len(wire)].tobytes() == wire, (name, c["psk"], c["payload"][:32])
            assert int(hb.out_len[0]) == len(pay) + S


def test_bad_psk_id_and_empty_batch():
    psks = [b"a", b"bb"]
    hb = sqobfs.HostBatch(np.zeros(64, np.uint8), np.array([0, 16], np.uint64),
                          np.array([10, 10], np.uint32), np.zeros(64, np.uint8),
                          np.array([0, 32], np.uint64), np.zeros(2, np.uint32),
                          np.zeros(16, np.uint8), np.array([1, 7], np.uint16))
    with sqobfs.Keyring(None, SALAMANDER, psks) as kr:
        sqobfs.cpu_run(kr, OBFUSCATE, hb.as_batch())
        assert int(hb.out_len[0]) == 18 and int(hb.out_len[1]) == sqobfs.BAD_PSK
        assert not hb.out[32:].any()  # nothing written for the bad id
        empty = sqobfs.HostBatch(np.zeros(1, np.uint8), np.zeros(0, np.uint64),
                                 np.zeros(0, np.uint32), np.zeros(1, np.uint8),
                                 np.zeros(0, np.uint64), np.zeros(0, np.uint32))
        sqobfs.cpu_run(kr, OBFUSCATE, empty.as_batch())
        with pytest.raises(sqobfs.SqError):  # obfuscate needs salts
            sqobfs.cpu_run(kr, OBFUSCATE, sqobfs.make_batch(1, hb.data, hb.in_off, hb.in_len,
                                                             hb.out, hb.out_off, hb.out_len))


@pytest.mark.parametrize("kind", [SALAMANDER, XPLUS])
def test_generated_salts_are_the_wire_salts(kind):
    """SQOBFS_FLAG_DEVICE_SALT on a host keyring: salts from the process's
    ChaCha20 generator, returned in salt_out, fresh per call, and the wire is
    the reference's WriteTo for them."""
    rng = np.random.Generator(np.random.PCG64(11))
    S = sqobfs.SALT_LEN[kind]
    lens = rng.integers(0, 1400, 64)
    psks = [b"generated-salts"]
    hb = gh.make_case(rng, kind, OBFUSCATE, lens, psks)
    hb.flags = sqobfs.FLAG_DEVICE_SALT
    hb.salt = None
    hb.salt_out = np.zeros(64 * S, np.uint8)
    with sqobfs.Keyring(None, kind, psks) as kr:
        sqobfs.cpu_run(kr, OBFUSCATE, hb.as_batch())
        first = hb.salt_out.copy()
        sqobfs.cpu_run(kr, OBFUSCATE, hb.as_batch())
    assert not np.array_equal(first, hb.salt_out)  # a new sequence number per call
    assert len({first[i * S:(i + 1) * S].tobytes() for i in range(64)}) == 64
    write = ol.salamander_write if kind == SALAMANDER else ol.xplus_write
    for i in range(64):
        o, L = int(hb.out_off[i]), int(lens[i])
        p = hb.data[int(hb.in_off[i]):int(hb.in_off[i]) + L].tobytes()
        w, _ = write(psks[0], hb.salt_out[i * S:(i + 1) * S].tobytes(), p)
        assert hb.out[o:o + L + S].tobytes() == w


@pytest.mark.parametrize("force", ["portable", "avx2"])
def test_portable_compressions_too(force):
    """The CPU path picks AVX2 BLAKE2b / SHA-NI SHA-256 and the AVX-512
    multi-buffer key groups where the host has them; the portable
    compressions (hosts without: SQOBFS_CPU_PORTABLE=1 forces them) and the
    AVX2 multi-buffer width (SQOBFS_CPU_MB=avx2) pass the same tests."""
    import subprocess
    import sys
    env = dict(os.environ, **({"SQOBFS_CPU_PORTABLE": "1"} if force == "portable"
                              else {"SQOBFS_CPU_MB": "avx2"}))
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                        os.path.abspath(__file__), "-k", "not portable"],
                       capture_output=True, text=True, env=env, timeout=600,
                       cwd=os.path.dirname(os.path.abspath(__file__)))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
