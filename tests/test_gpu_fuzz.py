"""Seeded random combinations of what the other parity files test one axis
at a time: scheme, direction, batch size, length distribution, PSK set
(empty, short, multi-block, several per batch), buffer layout (dense with
gaps, unaligned, 16-byte slots, in place, 128-byte-line slots), batch flags
(SQOBFS_FLAG_OUT_BLOCKS / OUT_LINES) and unit size -- each case against the
oracle's restatement of the reference (salamander.go:42-93,
xplus.go:46-98): every out_len and every output byte, and no byte outside
the outputs changed except the slot padding a flag declares scratch."""
from __future__ import annotations

import numpy as np
import pytest
import sqobfs
from sqobfs import DEOBFUSCATE, OBFUSCATE, SALAMANDER, XPLUS

import gpu_harness as gh

pytestmark = pytest.mark.gpu

LAYOUTS = ["dense", "gaps", "unaligned", "slot16", "inplace", "lines128"]
UNITS = [0, 1, 3, 16, 28, 62]


@pytest.fixture(scope="module")
def ctx():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    c = sqobfs.Context(0)
    yield c
    c.close()


def _case(seed):
    rng = np.random.Generator(np.random.PCG64(31337 + seed))
    kind = int(rng.integers(0, 2))
    direction = int(rng.integers(0, 2))
    n = (int(rng.choice([1, 2, 7, 63, 64, 65])) if rng.random() < 0.4
         else int(rng.integers(100, 6000)))
    dist = rng.choice(["uniform", "tiny", "mtu", "jumbo"], p=[0.5, 0.2, 0.2, 0.1])
    hi = {"uniform": 1500, "tiny": 41, "mtu": 1453, "jumbo": 9000}[dist]
    lo = 1200 if dist == "mtu" else 0
    lens = rng.integers(lo, hi, n)
    npsk = int(rng.choice([1, 1, 2, 5, 8]))
    psks = [rng.integers(0, 256, int(rng.choice([0, 1, 26, 39, 40, 64, 120, 129, 200])),
                         dtype=np.uint8).tobytes() for _ in range(npsk)]
    ids = rng.integers(0, npsk, n) if npsk > 1 else None
    layout = LAYOUTS[int(rng.integers(0, len(LAYOUTS)))]
    unit = int(rng.choice(UNITS))
    return rng, kind, direction, lens, psks, ids, layout, unit


def _build(rng, kind, direction, lens, psks, ids, layout):
    kw = dict(psk_ids=ids)
    flags = 0
    if layout == "dense":
        kw.update(in_align=1, out_align=1)
    elif layout == "gaps":
        kw.update(in_align=1, out_align=1, gaps=True)
    elif layout == "unaligned":
        kw.update(in_align=int(rng.choice([1, 4, 16])), in_lead=int(rng.integers(0, 16)),
                  out_align=int(rng.choice([1, 4, 16])), out_lead=int(rng.integers(0, 16)))
    elif layout == "slot16":
        kw.update(in_align=16, out_align=16, in_lead=int(rng.integers(0, 16)),
                  out_lead=int(rng.integers(0, 16)))
        flags = sqobfs.FLAG_OUT_BLOCKS
    elif layout == "inplace":
        kw.update(inplace=True, in_align=16)
        flags = int(rng.choice([0, sqobfs.FLAG_OUT_BLOCKS]))
    elif layout == "lines128":
        kw.update(in_align=128, out_align=128)
        flags = sqobfs.FLAG_OUT_LINES
    hb = gh.make_case(rng, kind, direction, lens, psks, **kw)
    return hb, flags


def _scratch(hb, ref, flags):
    """Bytes a flag lets the launch leave unspecified: a packet's own blocks
    (OUT_BLOCKS) or lines (OUT_LINES) outside its output."""
    m = np.zeros(hb.out.size, dtype=bool)
    if not flags:
        return m
    g = 128 if flags & sqobfs.FLAG_OUT_LINES else 16
    for o, n in zip(hb.out_off.astype(np.int64), ref.out_len.astype(np.int64)):
        if n <= 0 or n >= 0xFFFFFFF0:
            continue
        lo, hi = o & ~15, min(hb.out.size, (o + n + g - 1) & ~(g - 1))
        m[lo:o] = True
        m[o + n:hi] = True
    return m


@pytest.mark.parametrize("seed", range(40))
def test_random_combination(ctx, seed):
    rng, kind, direction, lens, psks, ids, layout, unit = _case(seed)
    hb, flags = _build(rng, kind, direction, lens, psks, ids, layout)
    ref = gh.run_oracle(kind, direction, psks, hb)
    hb.flags = flags
    ctx.unit_packets = unit
    try:
        with sqobfs.Keyring(ctx, kind, psks) as kr:
            gh.run_device(ctx, kr, direction, hb)
    finally:
        ctx.unit_packets = 0
    what = (f"seed {seed}: kind {kind} dir {direction} n {lens.size} psks "
            f"{[len(p) for p in psks]} layout {layout} flags {flags} unit {unit}")
    assert np.array_equal(hb.out_len, ref.out_len), what + ": out_len"
    bad = np.nonzero((hb.out != ref.out) & ~_scratch(hb, ref, flags))[0]
    assert bad.size == 0, f"{what}: {bad.size} bytes differ, first at {bad[0]}"
