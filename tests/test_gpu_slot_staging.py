"""sqobfs_run_host with fixed-stride slots in page-locked memory (the Go
Slots, socket batches): only the first bytes of each slot cross PCIe, rows
packed at the datagrams' width with 2-D copies (sq_api.hip slot_pack).
Every output byte and out_len equal the oracle's (the reference's WriteTo /
ReadFrom, salamander.go:42-70, xplus.go:46-75); bytes outside the outputs
keep their values unless the batch's flags declare them scratch; the
staging really is the packed size."""
from __future__ import annotations

import numpy as np
import pytest
import sqobfs
from sqobfs import DEOBFUSCATE, OBFUSCATE, SALAMANDER, XPLUS

import gpu_harness as gh

pytestmark = pytest.mark.gpu

PSKS = [b"sing-quic-mi355x-bench-psk", b"", b"q" * 140]


@pytest.fixture(scope="module", autouse=True)
def torch_first():
    """torch's HIP runtime comes up before the library's contexts (as in the
    other GPU test modules), whatever order the modules run in."""
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"


def slotted(rng, kind, direction, n, slot, lead, cap_extra=False, max_len=1452):
    """n datagrams in fixed slots of `slot` bytes (packet i at lead + i slot,
    input and output buffers alike), quic-go-sized (up to 1,452 B of
    payload); XPlus deobfuscate optionally reads past the datagram (in_cap,
    xplus.go:55)."""
    S = sqobfs.SALT_LEN[kind]
    lens = np.concatenate([np.arange(0, 40), rng.integers(0, max_len, n - 40)])
    lens[40:60] = max_len - np.arange(20)
    ids = rng.integers(0, len(PSKS), n)
    extra = rng.integers(0, 128, n) if cap_extra else None
    d = gh.make_case(rng, kind, direction, lens, PSKS, psk_ids=ids, cap_extra=extra)
    caps = d.in_cap.astype(np.int64) if d.in_cap is not None else d.in_len.astype(np.int64)
    in_off = (lead + slot * np.arange(n)).astype(np.uint64)
    out_off = in_off.copy()
    data = rng.integers(0, 256, lead + slot * n + 256, dtype=np.uint8)  # junk between packets
    for i in range(n):
        o, c = int(d.in_off[i]), int(caps[i])
        assert c + (S if direction == OBFUSCATE else 0) <= slot
        data[int(in_off[i]):int(in_off[i]) + c] = d.data[o:o + c]
    out = np.full(lead + slot * n + 256, gh.SENTINEL, dtype=np.uint8)
    return sqobfs.HostBatch(data, in_off, d.in_len.copy(), out, out_off,
                            np.zeros(n, dtype=np.uint32), d.salt, d.psk_id, d.in_cap)


def pin(ctx, hb, keep, phase=0):
    for name in ("data", "out"):
        a = getattr(hb, name)
        p = sqobfs.PinnedArray(ctx, a.size + 256)
        v = p.array[phase:phase + a.size]
        v[:] = a
        keep.append(p)
        setattr(hb, name, v)


@pytest.mark.parametrize("kind", [SALAMANDER, XPLUS])
@pytest.mark.parametrize("direction", [OBFUSCATE, DEOBFUSCATE])
@pytest.mark.parametrize("flags", ["none", "blocks", "lines", "lines+uninit"])
def test_slot_staging(kind, direction, flags):
    _slot_staging(kind, direction, flags, 2048)


@pytest.mark.parametrize("kind", [SALAMANDER, XPLUS])
@pytest.mark.parametrize("direction", [OBFUSCATE, DEOBFUSCATE])
def test_slot_staging_1536_lines(kind, direction):
    """1,536-byte slots (12 whole 128-byte lines: wire <= 1,468 B for both
    schemes), the stride DESIGN.md section 5 compared with 2,048."""
    _slot_staging(kind, direction, "lines+uninit", 1536)


def _slot_staging(kind, direction, flags, slot):
    rng = np.random.Generator(np.random.PCG64(8100 + 10 * kind + direction + slot +
                                              100 * ["none", "blocks", "lines",
                                                     "lines+uninit"].index(flags)))
    n = 9000  # several pipeline chunks
    hb = slotted(rng, kind, direction, n, slot, lead=0 if flags != "none" else 5,
                 cap_extra=kind == XPLUS and direction == DEOBFUSCATE and slot >= 2048)
    ref = gh.run_oracle(kind, direction, PSKS, hb)
    hb.flags = {"none": 0, "blocks": sqobfs.FLAG_OUT_BLOCKS, "lines": sqobfs.FLAG_OUT_LINES,
                "lines+uninit": sqobfs.FLAG_OUT_LINES | sqobfs.FLAG_OUT_UNINIT}[flags]
    keep = []
    with sqobfs.Context(0) as ctx:
        try:
            pin(ctx, hb, keep)
            with sqobfs.Keyring(ctx, kind, PSKS) as kr:
                gh.run_host(ctx, kr, direction, hb)
                # packed: well under the two 2,048-byte-slot spans (1,536-byte
                # slots of whole lines hold rows of 1,536: nothing to pack)
                if slot == 2048:
                    assert ctx.staging_bytes < 2 * n * slot * 7 // 8, ctx.staging_bytes
            assert np.array_equal(hb.out_len, ref.out_len)
            out = hb.out.copy()
        finally:
            for p in keep:
                p.free()
    inside = np.zeros(out.size, dtype=bool)
    scratch = np.zeros(out.size, dtype=bool)
    S = sqobfs.SALT_LEN[kind]
    ext = ref.out_len.astype(np.int64)
    if hb.in_cap is not None:  # XPlus ReadFrom writes up to len(p) - 16 (xplus.go:55)
        caps = hb.in_cap.astype(np.int64)
        ext = np.where(hb.in_len.astype(np.int64) >= S, caps - S, ext)
    for o, m in zip(hb.out_off.astype(np.int64), ext):
        if 0 < m < 0xFFFFFFF0:
            inside[o:o + m] = True
            scratch[o & ~15:o] = True
            scratch[o + m:(o + m + 127) & ~127 if "lines" in flags else (o + m + 15) & ~15] = True
    bad = np.nonzero((out != ref.out) & inside)[0]
    assert bad.size == 0, f"{bad.size} output bytes differ, first at {bad[0]}"
    if flags == "none":
        assert np.array_equal(out, ref.out), "bytes outside the outputs changed"
    elif flags in ("blocks", "lines"):
        bad = np.nonzero((out != ref.out) & ~scratch & ~inside)[0]
        assert bad.size == 0, f"{bad.size} preserved bytes changed, first at {bad[0]}"


@pytest.mark.parametrize("kind", [SALAMANDER, XPLUS])
def test_slot_staging_round_trip_odd_stride(kind):
    """A stride that is not a multiple of 16 (no block flags) and a buffer
    phase of 3: obfuscate then deobfuscate through packed staging gives the
    payloads back; the wire equals the oracle's."""
    rng = np.random.Generator(np.random.PCG64(8300 + kind))
    S = sqobfs.SALT_LEN[kind]
    n, slot = 5000, 1900 + 7
    hb = slotted(rng, kind, OBFUSCATE, n, slot, lead=3)
    hb.psk_id = None
    lens = hb.in_len.astype(np.int64)
    hb.in_len[lens == 0] = 1  # (a 0-byte payload's 8-byte wire reads back as 8 bytes)
    ref = gh.run_oracle(kind, OBFUSCATE, [PSKS[0]], hb)
    keep = []
    with sqobfs.Context(0) as ctx:
        try:
            pin(ctx, hb, keep, phase=3)
            with sqobfs.Keyring(ctx, kind, [PSKS[0]]) as kr:
                gh.run_host(ctx, kr, OBFUSCATE, hb)
                assert np.array_equal(hb.out, ref.out)
                assert np.array_equal(hb.out_len, ref.out_len)
                # decode the wire (now the input) into fresh slots
                back = sqobfs.PinnedArray(ctx, hb.data.size + 256)
                keep.append(back)
                b = back.array[:hb.data.size]
                b[:] = 0
                hb2 = sqobfs.HostBatch(hb.out, hb.out_off, (hb.in_len + S).astype(np.uint32), b,
                                       hb.in_off, np.zeros(n, np.uint32), None, None, None)
                gh.run_host(ctx, kr, DEOBFUSCATE, hb2)
                for i in range(0, n, 97):
                    o, m = int(hb.in_off[i]), int(hb.in_len[i])
                    assert bytes(b[o:o + m]) == bytes(hb.data[o:o + m]), f"packet {i}"
                assert np.array_equal(hb2.out_len, hb.in_len)
        finally:
            for p in keep:
                p.free()
