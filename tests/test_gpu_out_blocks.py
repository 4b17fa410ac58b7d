"""SQOBFS_FLAG_OUT_BLOCKS (outputs own their 16-byte blocks; slotted layouts):
every output byte equals the oracle's (the reference's WriteTo / ReadFrom,
salamander.go:42-93, xplus.go:46-98), out_len too, and the only other bytes
that change are inside the 16-byte blocks a packet's own output touches --
the padding the flag declares scratch."""
from __future__ import annotations

import numpy as np
import pytest
import sqobfs
from sqobfs import DEOBFUSCATE, OBFUSCATE, SALAMANDER, XPLUS

import gpu_harness as gh

pytestmark = pytest.mark.gpu

KINDS = [SALAMANDER, XPLUS]
DIRS = [OBFUSCATE, DEOBFUSCATE]
PSK = b"sing-quic-mi355x-bench-psk"
PSKS = [PSK, b"", b"q" * 140]


@pytest.fixture(scope="module")
def ctx():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    c = sqobfs.Context(0)
    yield c
    c.close()


def scratch_mask(hb, ref):
    """Bytes allowed to differ: a packet's own blocks outside its output."""
    m = np.zeros(hb.out.size, dtype=bool)
    for o, n in zip(hb.out_off.astype(np.int64), ref.out_len.astype(np.int64)):
        if n <= 0 or n >= 0xFFFFFFF0:
            continue
        lo, hi = o & ~15, (o + n + 15) & ~15
        m[lo:o] = True
        m[o + n:hi] = True
    return m


def make(rng, kind, direction, layout, multi, n=3000):
    S = sqobfs.SALT_LEN[kind]
    lens = np.concatenate([np.arange(0, 48), rng.integers(0, 1500, n - 48)])
    if layout == "slot2048":
        lens = np.minimum(lens, 2048 - S - 16)
    ids = rng.integers(0, len(PSKS), lens.size) if multi else None
    psks = PSKS if multi else [PSK]
    kw = dict(psk_ids=ids, in_align=16, out_align=16)
    if layout == "inplace16":
        kw["inplace"] = True
    elif layout == "lead5":          # slots at 16k + 5: unaligned heads, aligned blocks
        kw.update(out_lead=5, in_lead=3)
    elif layout == "lead13":         # rs % 16 + S > 16 for obfuscate: byte-exact head kept
        kw.update(out_lead=13, in_lead=1)
    hb = gh.make_case(rng, kind, direction, lens, psks, **kw)
    if layout == "slot2048":         # fixed 2048-byte slots, as the Go Slots / the endpoint
        hb = gh.make_case(rng, kind, direction, lens, psks, psk_ids=ids, in_align=2048,
                          out_align=2048)
    return hb, psks


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("direction", DIRS)
@pytest.mark.parametrize("layout", ["slot16", "slot2048", "inplace16", "lead5", "lead13"])
@pytest.mark.parametrize("multi", [False, True])
def test_out_blocks_device(ctx, kind, direction, layout, multi):
    rng = np.random.Generator(np.random.PCG64(7000 + 100 * kind + 10 * direction + multi +
                                              1000 * ["slot16", "slot2048", "inplace16", "lead5",
                                                      "lead13"].index(layout)))
    hb, psks = make(rng, kind, direction, layout, multi)
    ref = gh.run_oracle(kind, direction, psks, hb)
    hb.flags = sqobfs.FLAG_OUT_BLOCKS
    with sqobfs.Keyring(ctx, kind, psks) as kr:
        gh.run_device(ctx, kr, direction, hb)
    assert np.array_equal(hb.out_len, ref.out_len)
    free = scratch_mask(hb, ref)
    bad = np.nonzero((hb.out != ref.out) & ~free)[0]
    assert bad.size == 0, f"{bad.size} bytes outside the scratch padding differ, first at {bad[0]}"
    # and the padding really is written whole somewhere (the fast path ran)
    if layout in ("slot16", "lead5"):
        assert ((hb.out != ref.out) & free).any()


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("direction", DIRS)
@pytest.mark.parametrize("pinned", [False, True])
def test_out_blocks_run_host(ctx, kind, direction, pinned):
    """Through sqobfs_run_host: the staging copy keeps every byte's address
    modulo 16, so the blocks the kernel writes whole are the caller's."""
    rng = np.random.Generator(np.random.PCG64(7500 + 10 * kind + direction + 4 * pinned))
    hb, psks = make(rng, kind, direction, "lead5", True, n=20000)
    ref = gh.run_oracle(kind, direction, psks, hb)
    hb.flags = sqobfs.FLAG_OUT_BLOCKS | sqobfs.FLAG_OUT_UNINIT
    keep = []
    try:
        if pinned:
            for name in ("data", "out"):
                a = getattr(hb, name)
                p = sqobfs.PinnedArray(ctx, a.size + 16)
                # the same address modulo 16 as the pageable copy
                sh = (a.ctypes.data - p.array.ctypes.data) % 16
                v = p.array[sh:sh + a.size]
                v[:] = a
                keep.append(p)
                setattr(hb, name, v)
        with sqobfs.Keyring(ctx, kind, psks) as kr:
            gh.run_host(ctx, kr, direction, hb)
        assert np.array_equal(hb.out_len, ref.out_len)
        free = scratch_mask(hb, ref)
        # OUT_UNINIT: bytes outside every output block are unspecified too
        inside = np.zeros(hb.out.size, dtype=bool)
        for o, n in zip(hb.out_off.astype(np.int64), ref.out_len.astype(np.int64)):
            if 0 < n < 0xFFFFFFF0:
                inside[o:o + n] = True
        bad = np.nonzero((hb.out != ref.out) & inside)[0]
        assert bad.size == 0, f"{bad.size} output bytes differ, first at {bad[0]}"
        assert not ((hb.out != ref.out) & free & inside).any()
    finally:
        for p in keep:
            p.free()


def make_lines(rng, kind, direction, multi, lead, n=3000, inplace=False):
    """Fixed 2048-byte slots (the Go Slots / the packet conn engine), outputs
    short enough that the padding to the next 128-byte line stays in the
    slot wherever the buffer lies; `inplace`: each packet transformed in its
    own slot (the vectorised WriteTo's headroom layout, or decoded behind
    its salt)."""
    S = sqobfs.SALT_LEN[kind]
    lens = np.concatenate([np.arange(0, 48), rng.integers(0, 2048 - S - 128, n - 48)])
    lens[48:80] = 2048 - S - 128 - np.arange(32)  # the longest ones
    ids = rng.integers(0, len(PSKS), lens.size) if multi else None
    psks = PSKS if multi else [PSK]
    if inplace:
        hb = gh.make_case(rng, kind, direction, lens, psks, psk_ids=ids, in_align=2048,
                          in_lead=lead, inplace=True)
    else:
        hb = gh.make_case(rng, kind, direction, lens, psks, psk_ids=ids, in_align=2048,
                          out_align=2048, in_lead=lead, out_lead=lead)
    return hb, psks


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("direction", DIRS)
@pytest.mark.parametrize("lead,inplace", [(0, False), (64, False), (8, False), (0, True),
                                          (8, True)])
@pytest.mark.parametrize("multi", [False, True])
def test_out_lines_device(ctx, kind, direction, lead, inplace, multi):
    """Every output byte and out_len equal the oracle's; only the packet's own
    head block and its last line's padding may change; the padding is
    written (the lines are whole)."""
    rng = np.random.Generator(np.random.PCG64(7700 + 100 * kind + 10 * direction + multi + lead +
                                              5 * inplace))
    hb, psks = make_lines(rng, kind, direction, multi, lead, inplace=inplace)
    ref = gh.run_oracle(kind, direction, psks, hb)
    hb.flags = sqobfs.FLAG_OUT_LINES
    with sqobfs.Keyring(ctx, kind, psks) as kr:
        gh.run_device(ctx, kr, direction, hb)
    assert np.array_equal(hb.out_len, ref.out_len)
    # the device copy lies 128-byte aligned (torch): line ends by buffer offset
    m = np.zeros(hb.out.size, dtype=bool)
    for o, n in zip(hb.out_off.astype(np.int64), ref.out_len.astype(np.int64)):
        if 0 < n < 0xFFFFFFF0:
            m[o & ~15:o] = True
            m[o + n:(o + n + 127) & ~127] = True
    bad = np.nonzero((hb.out != ref.out) & ~m)[0]
    assert bad.size == 0, f"{bad.size} bytes outside the scratch padding differ, first at {bad[0]}"
    # the padding past the 16-byte block is written somewhere (pad blocks ran)
    past = np.zeros(hb.out.size, dtype=bool)
    for o, n in zip(hb.out_off.astype(np.int64), ref.out_len.astype(np.int64)):
        if 0 < n < 0xFFFFFFF0:
            past[(o + n + 15) & ~15:(o + n + 127) & ~127] = True
    assert ((hb.out != ref.out) & past).any()


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("direction", DIRS)
@pytest.mark.parametrize("pinned", [False, True])
def test_out_lines_run_host(ctx, kind, direction, pinned):
    """Through sqobfs_run_host: the staging keeps output addresses modulo 128
    and stages the last line's padding."""
    rng = np.random.Generator(np.random.PCG64(7900 + 10 * kind + direction + 4 * pinned))
    hb, psks = make_lines(rng, kind, direction, True, 64, n=20000)
    ref = gh.run_oracle(kind, direction, psks, hb)
    hb.flags = sqobfs.FLAG_OUT_LINES | sqobfs.FLAG_OUT_UNINIT
    keep = []
    try:
        if pinned:
            for name in ("data", "out"):
                a = getattr(hb, name)
                p = sqobfs.PinnedArray(ctx, a.size + 128)
                sh = (a.ctypes.data - p.array.ctypes.data) % 128
                v = p.array[sh:sh + a.size]
                v[:] = a
                keep.append(p)
                setattr(hb, name, v)
        with sqobfs.Keyring(ctx, kind, psks) as kr:
            gh.run_host(ctx, kr, direction, hb)
        assert np.array_equal(hb.out_len, ref.out_len)
        inside = np.zeros(hb.out.size, dtype=bool)
        for o, n in zip(hb.out_off.astype(np.int64), ref.out_len.astype(np.int64)):
            if 0 < n < 0xFFFFFFF0:
                inside[o:o + n] = True
        bad = np.nonzero((hb.out != ref.out) & inside)[0]
        assert bad.size == 0, f"{bad.size} output bytes differ, first at {bad[0]}"
    finally:
        for p in keep:
            p.free()
