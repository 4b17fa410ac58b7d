"""Parity of the gfx950 path (through the C ABI) with the CPU oracle.

Bit-exact comparison of every output byte (including the bytes around each
packet's output region, which must stay untouched) and every out_len, on
seeded inputs: golden vectors, ragged batches, unaligned offsets, in-place
layouts, multi-PSK keyrings, the reference's short-datagram and XPlus
read-buffer quirks.  Full BASELINE sizes are covered in test_gpu_fullsize.py.
"""
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


@pytest.fixture(scope="module")
def ctx():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    c = sqobfs.Context(0)
    yield c
    c.close()


def check(ctx, kind, direction, psks, hb, what, path="device"):
    ref = gh.run_oracle(kind, direction, psks, hb)
    with sqobfs.Keyring(ctx, kind, psks) as kr:
        if path == "device":
            gh.run_device(ctx, kr, direction, hb)
        else:
            gh.run_host(ctx, kr, direction, hb)
    gh.assert_same(hb, ref, what)


# ---------------------------------------------------------------- golden

@pytest.mark.parametrize("kind", KINDS)
def test_golden_write_vectors(ctx, golden, kind):
    """All golden write vectors in ONE batch: one keyring entry per vector
    (PSK lengths 0..300), psk_id per packet."""
    vs = golden("salamander_write.json" if kind == SALAMANDER else "xplus_write.json")
    psks = [bytes.fromhex(v["psk"]) for v in vs]
    pays = [bytes.fromhex(v["payload"]) for v in vs]
    S = sqobfs.SALT_LEN[kind]
    data, off, ln = sqobfs.pack(pays)
    oo, end = gh._place([S + len(p) for p in pays], 16, 0)
    out = np.full(end + 64, gh.SENTINEL, np.uint8)
    salt = np.frombuffer(b"".join(bytes.fromhex(v["salt"]) for v in vs), np.uint8).copy()
    hb = sqobfs.HostBatch(data, off, ln, out, oo, np.zeros(len(vs), np.uint32), salt,
                          np.arange(len(vs), dtype=np.uint16))
    with sqobfs.Keyring(ctx, kind, psks) as kr:
        gh.run_device(ctx, kr, OBFUSCATE, hb)
    for i, v in enumerate(vs):
        w = bytes.fromhex(v["wire"])
        assert hb.out[int(oo[i]):int(oo[i]) + len(w)].tobytes() == w, f"vector {i}"
        assert hb.out_len[i] == len(w)


@pytest.mark.parametrize("kind", KINDS)
def test_golden_read_vectors(ctx, golden, kind):
    vs = golden("salamander_read.json" if kind == SALAMANDER else "xplus_read.json")
    S = sqobfs.SALT_LEN[kind]
    full = [bytes.fromhex(v.get("buffer_full", v["datagram"])) for v in vs]
    dl = [len(bytes.fromhex(v["datagram"])) for v in vs]
    data, off, _ = sqobfs.pack(full)
    caps = np.array([len(f) for f in full], np.uint32)
    osz = [gh.out_size(kind, DEOBFUSCATE, n, c) for n, c in zip(dl, caps)]
    oo, end = gh._place(osz, 16, 0)
    out = np.full(end + 64, gh.SENTINEL, np.uint8)
    hb = sqobfs.HostBatch(data, off, np.array(dl, np.uint32), out, oo,
                          np.zeros(len(vs), np.uint32), None, None,
                          caps if kind == XPLUS else None)
    with sqobfs.Keyring(ctx, kind, [bytes.fromhex(vs[0]["psk"])]) as kr:
        gh.run_device(ctx, kr, DEOBFUSCATE, hb)
    for i, v in enumerate(vs):
        after = bytes.fromhex(v["buffer_after"])
        ret = v["read_ret"]
        assert hb.out_len[i] == ret, f"vector {i}"
        # product output = what ReadFrom leaves in p[0 : out region)
        got = hb.out[int(oo[i]):int(oo[i]) + osz[i]].tobytes()
        assert got == after[:osz[i]], f"vector {i}"


def test_survey_examples(ctx, golden):
    for ex in golden("survey_examples.json"):
        kind = SALAMANDER if ex["kind"] == "salamander" else XPLUS
        pay = bytes.fromhex(ex["payload"])
        data, off, ln = sqobfs.pack([pay])
        S = sqobfs.SALT_LEN[kind]
        out = np.zeros(S + len(pay) + 64, np.uint8)
        hb = sqobfs.HostBatch(data, off, ln, out, np.zeros(1, np.uint64), np.zeros(1, np.uint32),
                              np.frombuffer(bytes.fromhex(ex["salt"]), np.uint8).copy())
        with sqobfs.Keyring(ctx, kind, [bytes.fromhex(ex["psk"])]) as kr:
            gh.run_host(ctx, kr, OBFUSCATE, hb)
        assert out[:S + len(pay)].tobytes().hex() == ex["wire"]


# ---------------------------------------------------------------- ragged

@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("direction", DIRS)
@pytest.mark.parametrize("dist", ["tiny", "mixed", "mtu"])
def test_ragged_single_psk(ctx, kind, direction, dist):
    rng = np.random.Generator(np.random.PCG64(100 + 10 * kind + direction))
    n = {"tiny": 3000, "mixed": 2500, "mtu": 700}[dist]
    lo, hi = {"tiny": (0, 70), "mixed": (0, 1500), "mtu": (1200, 1500)}[dist]
    lens = rng.integers(lo, hi + 1, n)
    hb = gh.make_case(rng, kind, direction, lens, [PSK])
    check(ctx, kind, direction, [PSK], hb, f"{kind}/{direction}/{dist}")


def wire_dense_case(rng, kind, direction, lens, lead=0):
    """The bench's dense layout: obfuscate outputs (wire datagrams) back to
    back, each payload at the same position of an input buffer of the same
    shape (S bytes of headroom in front); deobfuscate reads such a wire
    buffer and writes the payloads back to back.  One uniform, 16-byte
    aligned input/output shift for every packet: the stream also loads the
    special blocks' inputs here."""
    S = sqobfs.SALT_LEN[kind]
    lens = np.asarray(lens, np.int64)
    wire = lens + S
    w_off = (np.cumsum(wire) - wire + lead).astype(np.uint64)
    end = int(wire.sum()) + lead
    if direction == OBFUSCATE:
        data = rng.integers(0, 256, end + 64, dtype=np.uint8)  # headroom holds junk
        out = np.full(end + 64, gh.SENTINEL, np.uint8)
        salt = rng.integers(0, 256, len(lens) * S, dtype=np.uint8)
        return sqobfs.HostBatch(data, w_off + S, lens.astype(np.uint32), out, w_off,
                                np.zeros(len(lens), np.uint32), salt)
    data = rng.integers(0, 256, end + 64, dtype=np.uint8)
    # output slots by the reference's return lengths (a datagram of <= 8
    # bytes comes back whole, salamander.go:47-49)
    osz = np.array([gh.out_size(kind, direction, int(w), int(w)) for w in wire], np.int64)
    p_off = (np.cumsum(osz) - osz + lead).astype(np.uint64)
    out = np.full(int(osz.sum()) + lead + 64, gh.SENTINEL, np.uint8)
    return sqobfs.HostBatch(data, w_off, wire.astype(np.uint32), out, p_off,
                            np.zeros(len(lens), np.uint32))


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("direction", DIRS)
@pytest.mark.parametrize("lead", [0, 8, 16])
def test_wire_dense_layout(ctx, kind, direction, lead):
    rng = np.random.Generator(np.random.PCG64(700 + 10 * kind + direction + lead))
    lens = np.concatenate([np.arange(0, 40), rng.integers(0, 1500, 1500),
                           np.full(300, 1350)])
    hb = wire_dense_case(rng, kind, direction, lens, lead)
    check(ctx, kind, direction, [PSK], hb, f"{kind}/{direction}/dense{lead}")


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("direction", DIRS)
def test_jumbo_units(ctx, kind, direction):
    """Units whose flat block space exceeds the block map (4,096 blocks per
    32 packets): jumbo datagrams and a few 70 KB buffers (GSO-sized), next to
    MTU-sized units, so both stream lookups run in one launch."""
    rng = np.random.Generator(np.random.PCG64(800 + 10 * kind + direction))
    lens = np.concatenate([rng.integers(1500, 9001, 200), rng.integers(0, 1500, 100),
                           rng.integers(60000, 70001, 6), rng.integers(0, 200, 40)])
    rng.shuffle(lens[:200])
    hb = gh.make_case(rng, kind, direction, lens, [PSK], in_align=1, out_align=16, out_lead=3)
    check(ctx, kind, direction, [PSK], hb, f"{kind}/{direction}/jumbo")
    hb = wire_dense_case(rng, kind, direction, lens)
    check(ctx, kind, direction, [PSK], hb, f"{kind}/{direction}/jumbo-dense")


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("direction", DIRS)
def test_single_psk_lengths(ctx, kind, direction):
    """One-entry keyrings (no psk_id: the single-PSK kernels, which read the
    keyring's entry 0 from the kernel arguments) for PSK lengths that put the
    salt at every byte position of a one-block final message, across the
    one/two-block boundary (PSK tail 120 / 121 / 127 B) and past whole
    blocks."""
    rng = np.random.Generator(np.random.PCG64(950 + 10 * kind + direction))
    lens = np.concatenate([np.arange(0, 24), rng.integers(0, 1500, 120)])
    for k in list(range(0, 136, 3)) + [119, 120, 121, 122, 126, 127, 128, 129,
                                       247, 248, 249, 255, 256, 300]:
        psk = rng.integers(0, 256, k, dtype=np.uint8).tobytes()
        hb = gh.make_case(rng, kind, direction, lens, [psk], in_align=4, out_lead=8)
        check(ctx, kind, direction, [psk], hb, f"{kind}/{direction}/psk{k}")


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("direction", DIRS)
def test_xcd_remapped_launch(ctx, kind, direction):
    """Launches of at least 2^18 units take the XCD-contiguous unit order
    (sq_kernels.hip kXcdMinUnits): one-packet units over 600,001 short
    datagrams (an odd grid, not a multiple of 8 workgroups) give the
    oracle's bytes, neighbours and out_len for every packet."""
    S = sqobfs.SALT_LEN[kind]
    rng = np.random.Generator(np.random.PCG64(4400 + 10 * kind + direction))
    n = 600_001
    lens = rng.integers(0, 96, n).astype(np.int64)
    if direction == DEOBFUSCATE:
        lens += S // 2  # some below S (passthrough / dropped), most above
    in_off = np.cumsum(lens) - lens + 5
    data = rng.integers(0, 256, int(lens.sum()) + 64, dtype=np.uint8)
    osz = np.array([gh.out_size(kind, direction, int(L), int(L)) for L in lens], dtype=np.int64)
    out_off = np.cumsum(osz) - osz + 3
    out = np.full(int(osz.sum()) + 64, gh.SENTINEL, dtype=np.uint8)
    salt = rng.integers(0, 256, n * S, dtype=np.uint8) if direction == OBFUSCATE else None
    hb = sqobfs.HostBatch(data, in_off.astype(np.uint64), lens.astype(np.uint32), out,
                          out_off.astype(np.uint64), np.zeros(n, dtype=np.uint32), salt, None,
                          None)
    ctx.unit_packets = 1
    try:
        check(ctx, kind, direction, [PSK], hb, "xcd-remapped launch")
    finally:
        ctx.unit_packets = 0


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("direction", DIRS)
def test_unit_sizes(ctx, kind, direction):
    """Every unit size gives the same bytes (sqobfs_set_unit_packets): unit
    boundaries, donation and the neighbour lanes move with it.  Ragged and
    dense layouts, a 256-entry keyring, 1..62 packets per wavefront."""
    rng = np.random.Generator(np.random.PCG64(900 + 10 * kind + direction))
    lens = np.concatenate([np.arange(0, 40), rng.integers(0, 1500, 900), np.full(200, 1350)])
    psks = [rng.integers(0, 256, int(k), dtype=np.uint8).tobytes()
            for k in rng.integers(0, 140, 256)]
    ids = rng.integers(0, 256, len(lens)).astype(np.uint16)
    default = ctx.unit_packets
    try:
        for ppw in (1, 2, 7, 16, 26, 31, 33, 40, 62):
            ctx.unit_packets = ppw
            assert ctx.unit_packets == ppw
            hb = gh.make_case(rng, kind, direction, lens, [PSK], in_align=4, out_lead=8)
            check(ctx, kind, direction, [PSK], hb, f"{kind}/{direction}/ppw{ppw}")
            hb = wire_dense_case(rng, kind, direction, lens, lead=8)
            check(ctx, kind, direction, [PSK], hb, f"{kind}/{direction}/ppw{ppw}/dense")
            hb = gh.make_case(rng, kind, direction, lens, psks, psk_ids=ids)
            check(ctx, kind, direction, psks, hb, f"{kind}/{direction}/ppw{ppw}/multi")
    finally:
        ctx.unit_packets = 0
    assert ctx.unit_packets == default
    with pytest.raises(sqobfs.SqError):
        ctx.unit_packets = 63


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("direction", DIRS)
@pytest.mark.parametrize("in_align,in_lead,out_align,out_lead",
                         [(1, 0, 1, 0), (1, 3, 16, 0), (16, 0, 1, 5), (16, 8, 16, 8),
                          (16, 4, 16, 12), (4, 0, 8, 0)])
def test_unaligned_layouts(ctx, kind, direction, in_align, in_lead, out_align, out_lead):
    rng = np.random.Generator(np.random.PCG64(7 + in_align + in_lead * 3 + out_lead))
    lens = np.concatenate([np.arange(0, 80), rng.integers(0, 1500, 400)])
    hb = gh.make_case(rng, kind, direction, lens, [PSK], in_align=in_align, in_lead=in_lead,
                      out_align=out_align, out_lead=out_lead, gaps=True)
    check(ctx, kind, direction, [PSK], hb, "unaligned")


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("direction", DIRS)
def test_in_place(ctx, kind, direction):
    """Headroom layout (obfs) / decode at +S (deobfs): output over input."""
    rng = np.random.Generator(np.random.PCG64(55 + kind + direction))
    lens = np.concatenate([np.arange(0, 70), rng.integers(0, 1500, 600)])
    hb = gh.make_case(rng, kind, direction, lens, [PSK], inplace=True)
    check(ctx, kind, direction, [PSK], hb, "in place")


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("direction", DIRS)
def test_multi_psk_256(ctx, kind, direction):
    """Config-5 shape: 256 PSKs of length U[8,64] (some cross SHA-256's
    39-byte two-block boundary), psk_id = i mod 256."""
    rng = np.random.Generator(np.random.PCG64(3))
    psks = [rng.integers(0, 256, int(k), dtype=np.uint8).tobytes()
            for k in rng.integers(8, 65, 256)]
    n = 3000
    ids = (np.arange(n) % 256).astype(np.uint16)
    lens = rng.integers(0, 1460, n)
    hb = gh.make_case(rng, kind, direction, lens, psks, psk_ids=ids)
    check(ctx, kind, direction, psks, hb, "multi psk")


@pytest.mark.parametrize("kind", KINDS)
def test_long_and_empty_psks(ctx, kind):
    psks = [b"", b"x", b"y" * 39, b"z" * 40, b"w" * 120, b"v" * 121, b"u" * 128,
            b"t" * 255, b"s" * 1000]
    rng = np.random.Generator(np.random.PCG64(11))
    n = 900
    ids = rng.integers(0, len(psks), n).astype(np.uint16)
    for direction in DIRS:
        hb = gh.make_case(rng, kind, direction, rng.integers(0, 400, n), psks, psk_ids=ids)
        check(ctx, kind, direction, psks, hb, "long psk")


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("longest", [0, 1, 8, 24, 39, 40, 55, 56, 63, 64, 72, 73, 119, 120, 121,
                                     127, 128])
def test_keyring_hot_bounds(ctx, kind, longest):
    """The multi-PSK kernels load only the entry words the keyring's longest
    PSK needs, and no chaining value when no PSK has a PSK-only block
    (sq_api.hip keyring_hot_words): keyrings whose longest PSK sits at each
    boundary of those bounds (one more message word; BLAKE2b's one/two-block
    final at tail 120/121; a PSK-only block at 64 / 128 bytes; SHA-256's
    one/two-block final at 39/40 and BLAKE2b's ten/eleven message words at
    72/73)."""
    rng = np.random.Generator(np.random.PCG64(1300 + longest + 7 * kind))
    ks = list(rng.integers(0, longest + 1, 40)) + [longest]
    psks = [rng.integers(0, 256, int(k), dtype=np.uint8).tobytes() for k in ks]
    n = 700
    ids = rng.integers(0, len(psks), n).astype(np.uint16)
    for direction in DIRS:
        hb = gh.make_case(rng, kind, direction, rng.integers(0, 600, n), psks, psk_ids=ids)
        check(ctx, kind, direction, psks, hb, f"hot bounds {longest}")


def test_xplus_read_buffer_quirk(ctx):
    """xplus.go:55 XORs up to len(p) - 16, not n - 16."""
    rng = np.random.Generator(np.random.PCG64(12))
    n = 800
    lens = rng.integers(0, 1300, n)
    extra = rng.integers(0, 700, n)
    hb = gh.make_case(rng, XPLUS, DEOBFUSCATE, lens, [PSK], cap_extra=extra)
    check(ctx, XPLUS, DEOBFUSCATE, [PSK], hb, "xplus cap")


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("direction", DIRS)
def test_host_staged_path(ctx, kind, direction):
    rng = np.random.Generator(np.random.PCG64(21 + kind + 2 * direction))
    lens = rng.integers(0, 1500, 1500)
    hb = gh.make_case(rng, kind, direction, lens, [PSK], in_align=1, out_align=1)
    check(ctx, kind, direction, [PSK], hb, "host path", path="host")


def _pin(ctx, hb, keep):
    """Move hb's data/out into page-locked memory (run_host's DMA path)."""
    inplace = hb.out is hb.data
    pd = sqobfs.PinnedArray(ctx, hb.data.size)
    pd.array[:] = hb.data
    keep.append(pd)
    hb.data = pd.array
    if inplace:
        hb.out = hb.data
    else:
        po = sqobfs.PinnedArray(ctx, hb.out.size)
        po.array[:] = hb.out
        keep.append(po)
        hb.out = po.array


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("direction", DIRS)
@pytest.mark.parametrize("layout", ["dense", "gaps", "inplace", "shuffled"])
@pytest.mark.parametrize("pinned", [False, True])
def test_host_pipeline(ctx, kind, direction, layout, pinned):
    """Batches big enough for run_host's chunked H2D/kernel/D2H pipeline
    (several chunks), with pageable and pinned caller buffers, 3 PSKs.
    'shuffled' permutes the packet order so chunks' byte ranges interleave
    (the single-chunk fallback)."""
    rng = np.random.Generator(np.random.PCG64(300 + kind + 2 * direction + 4 * pinned))
    n = 20000
    lens = rng.integers(0, 1500, n)
    psks = [PSK, b"", b"x" * 200]
    ids = rng.integers(0, 3, n)
    hb = gh.make_case(rng, kind, direction, lens, psks, psk_ids=ids,
                      in_align=1 if layout == "gaps" else 16,
                      out_align=1 if layout == "gaps" else 16,
                      gaps=layout == "gaps", inplace=layout == "inplace")
    if layout == "shuffled":
        perm = rng.permutation(n)
        S = sqobfs.SALT_LEN[kind]
        hb.in_off, hb.in_len, hb.out_off = hb.in_off[perm], hb.in_len[perm], hb.out_off[perm]
        if hb.salt is not None:
            hb.salt = hb.salt.reshape(n, S)[perm].reshape(-1).copy()
        if hb.psk_id is not None:
            hb.psk_id = hb.psk_id[perm]
        if hb.in_cap is not None:
            hb.in_cap = hb.in_cap[perm]
    keep = []
    try:
        if pinned:
            _pin(ctx, hb, keep)
        check(ctx, kind, direction, psks, hb, f"host pipeline {layout}", path="host")
    finally:
        for k in keep:
            k.free()


@pytest.mark.parametrize("kind", KINDS)
def test_host_out_uninit_flag(ctx, kind):
    """SQOBFS_FLAG_OUT_UNINIT: every packet's output region and out_len are
    exact; bytes between regions are not checked."""
    rng = np.random.Generator(np.random.PCG64(77 + kind))
    n = 12000
    lens = rng.integers(0, 1500, n)
    hb = gh.make_case(rng, kind, OBFUSCATE, lens, [PSK], gaps=True)
    ref = gh.run_oracle(kind, OBFUSCATE, [PSK], hb)
    hb.flags = sqobfs.FLAG_OUT_UNINIT
    with sqobfs.Keyring(ctx, kind, [PSK]) as kr:
        gh.run_host(ctx, kr, OBFUSCATE, hb)
    assert np.array_equal(hb.out_len, ref.out_len)
    mask = np.zeros(hb.out.size, bool)
    for o, L in zip(hb.out_off.astype(np.int64), ref.out_len.astype(np.int64)):
        mask[o:o + L] = True
    assert np.array_equal(hb.out[mask], ref.out[mask])


def test_empty_batch_and_zero_length(ctx):
    with sqobfs.Keyring(ctx, SALAMANDER, [PSK]) as kr:
        b = sqobfs.Batch()
        sqobfs.launch(ctx, kr, OBFUSCATE, b)
        ctx.sync()
    rng = np.random.Generator(np.random.PCG64(1))
    for kind in KINDS:
        for direction in DIRS:
            hb = gh.make_case(rng, kind, direction, [0] * 130, [PSK])
            check(ctx, kind, direction, [PSK], hb, "zero length")


def test_bad_psk_id_marked_and_untouched(ctx):
    rng = np.random.Generator(np.random.PCG64(2))
    hb = gh.make_case(rng, SALAMANDER, OBFUSCATE, [100] * 70, [PSK], psk_ids=[0] * 70)
    hb.psk_id[5] = 9
    before = hb.out.copy()
    with sqobfs.Keyring(ctx, SALAMANDER, [PSK, b"second"]) as kr:
        gh.run_device(ctx, kr, OBFUSCATE, hb)
        assert hb.out_len[5] == sqobfs.BAD_PSK
        o = int(hb.out_off[5])
        assert np.array_equal(hb.out[o:o + 108], before[o:o + 108])
        with pytest.raises(sqobfs.SqError) as e:
            gh.run_host(ctx, kr, OBFUSCATE, hb)
        assert e.value.status == sqobfs.SQ_EPSK


def test_kind_mismatch_rejected(ctx):
    import ctypes
    with sqobfs.Keyring(ctx, XPLUS, [PSK]) as kr:
        b = sqobfs.Batch()
        b.n = 1
        st = sqobfs.lib().sqobfs_salamander_obfuscate(ctx.handle, kr.handle, ctypes.byref(b),
                                                      None)
        assert st == sqobfs.SQ_EINVAL


def test_round_trip_random(ctx):
    """obfuscate -> deobfuscate is the identity on the payload (both kinds)."""
    rng = np.random.Generator(np.random.PCG64(77))
    for kind in KINDS:
        S = sqobfs.SALT_LEN[kind]
        lens = rng.integers(0, 1500, 2000)
        hb = gh.make_case(rng, kind, OBFUSCATE, lens, [PSK], out_align=1)
        with sqobfs.Keyring(ctx, kind, [PSK]) as kr:
            gh.run_device(ctx, kr, OBFUSCATE, hb)
            osz = [gh.out_size(kind, DEOBFUSCATE, S + int(L), S + int(L)) for L in lens]
            oo, end = gh._place(osz, 1, 3)
            back = sqobfs.HostBatch(hb.out, hb.out_off, hb.out_len.copy(),
                                    np.zeros(end + 64, np.uint8), oo,
                                    np.zeros(len(lens), np.uint32))
            gh.run_device(ctx, kr, DEOBFUSCATE, back)
        for i, L in enumerate(lens):
            a, b = int(hb.in_off[i]), int(oo[i])
            assert back.out[b:b + int(L)].tobytes() == hb.data[a:a + int(L)].tobytes()


# ---------------------------------------------------------------- device salts

@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("path", ["device", "host"])
@pytest.mark.parametrize("with_out", [True, False])
def test_device_salt(ctx, kind, path, with_out):
    """SQOBFS_FLAG_DEVICE_SALT: salts are the ChaCha20 keystream of
    (context key, 'sqob' || le64(seq)); the wire is the oracle's obfuscation
    with exactly those salts; `salt` is ignored; seq advances per launch."""
    import oracle_lib as ol
    S = sqobfs.SALT_LEN[kind]
    rng = np.random.Generator(np.random.PCG64(900 + kind + 2 * (path == "host") + 4 * with_out))
    n = 3000  # one run_host chunk
    lens = rng.integers(0, 1500, n)
    psks = [PSK, b"q" * 77]
    ids = rng.integers(0, 2, n)
    key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    seq0 = int(rng.integers(0, 2**40))
    for launch in range(2):
        hb = gh.make_case(rng, kind, OBFUSCATE, lens, psks, psk_ids=ids, in_align=1, out_align=1)
        expect = np.frombuffer(ol.device_salts(key, seq0 + launch, n, S), np.uint8)
        ref_in = gh.clone(hb)
        ref_in.salt = expect.copy()
        ref = gh.run_oracle(kind, OBFUSCATE, psks, ref_in)
        hb.salt = rng.integers(0, 256, n * S, dtype=np.uint8)  # must be ignored
        hb.flags = sqobfs.FLAG_DEVICE_SALT
        hb.salt_out = np.zeros(n * S, np.uint8) if with_out else None
        if launch == 0:
            ctx.salt_key(key, seq0)
        with sqobfs.Keyring(ctx, kind, psks) as kr:
            if path == "device":
                gh.run_device(ctx, kr, OBFUSCATE, hb)
            else:
                gh.run_host(ctx, kr, OBFUSCATE, hb)
        assert ctx.salt_seq == seq0 + launch + 1
        if with_out:
            assert np.array_equal(hb.salt_out, expect), "salt_out differs from ChaCha20"
        gh.assert_same(hb, ref, f"device salt {path} launch {launch}")


def test_device_salt_rejected_for_deobfuscate(ctx):
    rng = np.random.Generator(np.random.PCG64(5))
    hb = gh.make_case(rng, SALAMANDER, DEOBFUSCATE, [40, 50], [PSK])
    hb.flags = sqobfs.FLAG_DEVICE_SALT
    with sqobfs.Keyring(ctx, SALAMANDER, [PSK]) as kr:
        with pytest.raises(sqobfs.SqError):
            gh.run_host(ctx, kr, DEOBFUSCATE, hb)


@pytest.mark.parametrize("kind", KINDS)
def test_host_staging_is_span_sized(kind):
    """run_host stages only the byte spans the batch touches: a batch sitting
    1 GiB into its (pageable) buffers needs kilobytes of staging, not 1 GiB,
    and still matches the oracle."""
    rng = np.random.Generator(np.random.PCG64(91 + kind))
    lens = rng.integers(0, 1500, 3000)
    hb = gh.make_case(rng, kind, OBFUSCATE, lens, [PSK], in_align=1, out_align=1)
    ref = gh.run_oracle(kind, OBFUSCATE, [PSK], hb)
    base = 1 << 30
    big_in = np.zeros(base + hb.data.size, np.uint8)   # untouched pages stay unbacked
    big_out = np.zeros(base + hb.out.size, np.uint8)
    big_in[base:] = hb.data
    big_out[base:] = hb.out
    hb.data, hb.out = big_in, big_out
    hb.in_off = hb.in_off + base
    hb.out_off = hb.out_off + base
    with sqobfs.Context(0) as c2, sqobfs.Keyring(c2, kind, [PSK]) as kr:
        gh.run_host(c2, kr, OBFUSCATE, hb)
        assert c2.staging_bytes < 32 << 20, c2.staging_bytes
    assert np.array_equal(hb.out_len, ref.out_len)
    assert np.array_equal(big_out[base:], ref.out)
    assert not big_out[:base].any()


@pytest.mark.parametrize("kind", KINDS)
def test_host_failure_drains_pipeline(ctx, kind):
    """A failure in the middle of run_host's pipeline (injected at chunk 2)
    returns an error only after every copy has finished: the caller's pinned
    output does not change afterwards.  The context stays usable."""
    import time
    rng = np.random.Generator(np.random.PCG64(95 + kind))
    n = 20000
    lens = rng.integers(0, 1500, n)
    hb = gh.make_case(rng, kind, OBFUSCATE, lens, [PSK])
    ref = gh.run_oracle(kind, OBFUSCATE, [PSK], hb)
    keep = []
    try:
        _pin(ctx, hb, keep)
        with sqobfs.Keyring(ctx, kind, [PSK]) as kr:
            sqobfs.debug_fail_chunk(2)
            with pytest.raises(sqobfs.SqError) as ei:
                gh.run_host(ctx, kr, OBFUSCATE, hb)
            assert ei.value.status == sqobfs.SQ_EDEVICE
            snap = hb.out.copy()
            time.sleep(0.05)
            assert np.array_equal(hb.out, snap), "a copy was still writing after the error"
            gh.run_host(ctx, kr, OBFUSCATE, hb)  # the hook fired once
        gh.assert_same(hb, ref, "after an injected failure")
    finally:
        sqobfs.debug_fail_chunk(-1)
        for k in keep:
            k.free()


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("pinned", [False, True])
def test_host_pipeline_device_salts(ctx, kind, pinned):
    """SQOBFS_FLAG_DEVICE_SALT through run_host's multi-piece pipeline (20,000
    packets: 5 chunks, the last cut in three): every piece is a launch with
    its own sequence number, salt_out comes back piece by piece (per landed
    piece with pageable output, in one copy with page-locked output), and the
    wire is the oracle's obfuscation with exactly those salts."""
    S = sqobfs.SALT_LEN[kind]
    rng = np.random.Generator(np.random.PCG64(610 + kind + 2 * pinned))
    n = 20000
    lens = rng.integers(0, 1500, n)
    psks = [PSK, b"r" * 33]
    ids = rng.integers(0, 2, n)
    hb = gh.make_case(rng, kind, OBFUSCATE, lens, psks, psk_ids=ids, in_align=1, out_align=1)
    hb.flags = sqobfs.FLAG_DEVICE_SALT
    hb.salt_out = np.zeros(n * S, np.uint8)
    keep = []
    try:
        if pinned:
            _pin(ctx, hb, keep)
        seq0 = ctx.salt_seq
        with sqobfs.Keyring(ctx, kind, psks) as kr:
            gh.run_host(ctx, kr, OBFUSCATE, hb)
        assert ctx.salt_seq - seq0 == 7, "one sequence number per piece (5 chunks, last cut in 3)"
        salts = hb.salt_out.reshape(n, S)
        assert len({bytes(r) for r in salts}) == n, "salts repeat across pieces"
        ref_in = gh.clone(hb)
        ref_in.flags = 0
        ref_in.salt = hb.salt_out.copy()
        ref = gh.run_oracle(kind, OBFUSCATE, psks, ref_in)
        gh.assert_same(hb, ref, f"run_host device salts pinned={pinned}")
    finally:
        for k in keep:
            k.free()


@pytest.mark.parametrize("kind", KINDS)
def test_host_failure_pageable_pieces(ctx, kind):
    """A failure injected at piece 4 of a pageable batch (its landed pieces
    are copied out while later ones move): the error comes back, out_len of
    the failed batch is not trusted, and the context reruns the batch
    correctly."""
    rng = np.random.Generator(np.random.PCG64(620 + kind))
    n = 20000
    lens = rng.integers(0, 1500, n)
    hb = gh.make_case(rng, kind, OBFUSCATE, lens, [PSK])
    ref = gh.run_oracle(kind, OBFUSCATE, [PSK], hb)
    try:
        with sqobfs.Keyring(ctx, kind, [PSK]) as kr:
            sqobfs.debug_fail_chunk(4)
            with pytest.raises(sqobfs.SqError) as ei:
                gh.run_host(ctx, kr, OBFUSCATE, hb)
            assert ei.value.status == sqobfs.SQ_EDEVICE
            gh.run_host(ctx, kr, OBFUSCATE, hb)
        gh.assert_same(hb, ref, "after an injected failure (pageable pieces)")
    finally:
        sqobfs.debug_fail_chunk(-1)
