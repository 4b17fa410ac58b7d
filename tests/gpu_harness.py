"""Builds ragged batches, runs them through the product (C ABI -> gfx950) and
through the CPU oracle, and compares.  Used by the -m gpu tests, smoke() and
bench.py's parity spot-check."""
from __future__ import annotations

import numpy as np
import sqobfs
from sqobfs import DEOBFUSCATE, OBFUSCATE, SALT_LEN, SALAMANDER, HostBatch

import oracle_lib as ol

SENTINEL = 0xA5


def out_size(kind: int, direction: int, n: int, cap: int) -> int:
    S = SALT_LEN[kind]
    if direction == OBFUSCATE:
        return S + n
    if kind == SALAMANDER:
        return n if n <= S else n - S
    return 0 if n < S else cap - S


def _place(sizes, align, lead, gap_rng=None):
    offs, pos = [], lead
    for sz in sizes:
        offs.append(pos)
        pos += sz
        if gap_rng is not None:
            pos += int(gap_rng.integers(0, 5))
        if align > 1:
            pos = (pos + align - 1) // align * align + lead
    return np.array(offs, dtype=np.uint64), pos


def make_case(rng: np.random.Generator, kind: int, direction: int, lens, psks,
              psk_ids=None, in_align=16, in_lead=0, out_align=16, out_lead=0,
              cap_extra=None, real_wire=True, inplace=False, gaps=False) -> HostBatch:
    """A HostBatch with random contents.  For deobfuscate, `lens` are datagram
    lengths; with real_wire half the datagrams are genuine obfuscated packets."""
    S = SALT_LEN[kind]
    lens = [int(x) for x in lens]
    n = len(lens)
    caps = list(lens)
    if direction == DEOBFUSCATE and kind != SALAMANDER and cap_extra is not None:
        caps = [L + int(e) for L, e in zip(lens, cap_extra)]
    pk = []
    for i, (L, C) in enumerate(zip(lens, caps)):
        b = rng.integers(0, 256, C, dtype=np.uint8).tobytes()
        if direction == DEOBFUSCATE and real_wire and L > S and i % 2 == 0:
            psk = psks[int(psk_ids[i]) if psk_ids is not None else 0]
            salt = b[:S]
            w = (ol.salamander_write if kind == SALAMANDER else ol.xplus_write)(
                psk, salt, b[S:L])[0]
            b = w + b[L:]
        pk.append(b)
    osz = [out_size(kind, direction, L, C) for L, C in zip(lens, caps)]
    grng = rng if gaps else None
    if inplace:
        # one buffer: payload output exactly over the payload input
        if direction == OBFUSCATE:   # headroom layout: [salt | payload]
            in_off, end = _place([S + L for L in lens], in_align, in_lead, grng)
            out_off = in_off.copy()
            in_off = in_off + S
        else:                        # decode in place: payload stays at +S
            in_off, end = _place([c + S for c in caps], in_align, in_lead, grng)
            out_off = in_off + S
        buf = np.full(end + 64, SENTINEL, dtype=np.uint8)
        for o, b in zip(in_off, pk):
            buf[int(o):int(o) + len(b)] = np.frombuffer(b, np.uint8)
        data = out = buf
    else:
        in_off, end = _place(caps, in_align, in_lead, grng)
        data = rng.integers(0, 256, end + 64, dtype=np.uint8)  # junk between packets
        for o, b in zip(in_off, pk):
            data[int(o):int(o) + len(b)] = np.frombuffer(b, np.uint8)
        out_off, oend = _place(osz, out_align, out_lead, grng)
        out = np.full(oend + 64, SENTINEL, dtype=np.uint8)
    salt = rng.integers(0, 256, n * S, dtype=np.uint8) if direction == OBFUSCATE else None
    in_cap = np.array(caps, dtype=np.uint32) if caps != lens else None
    ids = None if psk_ids is None else np.asarray(psk_ids, dtype=np.uint16)
    return HostBatch(data, in_off, np.array(lens, dtype=np.uint32), out, out_off,
                     np.zeros(n, dtype=np.uint32), salt, ids, in_cap)


def clone(hb: HostBatch) -> HostBatch:
    inplace = hb.out is hb.data
    data = hb.data.copy()
    out = data if inplace else hb.out.copy()
    c = lambda a: None if a is None else a.copy()  # noqa: E731
    return HostBatch(data, hb.in_off.copy(), hb.in_len.copy(), out, hb.out_off.copy(),
                     hb.out_len.copy(), c(hb.salt), c(hb.psk_id), c(hb.in_cap), hb.flags,
                     c(hb.salt_out))


def run_oracle(kind, direction, psks, hb: HostBatch, nthreads=4) -> HostBatch:
    ref = clone(hb)
    ol.batch_run(kind, direction, psks, ref, nthreads=nthreads)
    return ref


def run_device(ctx: sqobfs.Context, kr: sqobfs.Keyring, direction: int, hb: HostBatch,
               stream=None) -> None:
    """Copy the batch to HBM (torch tensors), launch through the C ABI on the
    current torch stream, copy the results back into hb."""
    import torch
    dev = torch.device("cuda", ctx.device)

    def t(a):
        return None if a is None else torch.from_numpy(a).to(dev)
    inplace = hb.out is hb.data
    d_data = t(hb.data)
    d_out = d_data if inplace else t(hb.out)
    d = dict(in_off=t(hb.in_off), in_len=t(hb.in_len), out_off=t(hb.out_off),
             out_len=t(hb.out_len), salt=t(hb.salt), psk_id=t(hb.psk_id), in_cap=t(hb.in_cap),
             salt_out=t(hb.salt_out))
    b = sqobfs.make_batch(hb.n, d_data, d["in_off"], d["in_len"], d_out, d["out_off"],
                          d["out_len"], d["salt"], d["psk_id"], d["in_cap"], d["salt_out"],
                          hb.flags)
    s = torch.cuda.current_stream(dev).cuda_stream if stream is None else stream
    sqobfs.launch(ctx, kr, direction, b, s)
    torch.cuda.synchronize(dev)
    hb.out[:] = d_out.cpu().numpy()
    hb.out_len[:] = d["out_len"].cpu().numpy()
    if hb.salt_out is not None:
        hb.salt_out[:] = d["salt_out"].cpu().numpy()


def run_host(ctx, kr, direction, hb: HostBatch) -> None:
    sqobfs.run_host(ctx, kr, direction, hb.as_batch())


def assert_same(got: HostBatch, ref: HostBatch, what=""):
    assert np.array_equal(got.out_len, ref.out_len), f"{what}: out_len differs at " \
        f"{np.nonzero(got.out_len != ref.out_len)[0][:10]}"
    if not np.array_equal(got.out, ref.out):
        bad = np.nonzero(got.out != ref.out)[0]
        pk = np.searchsorted(got.out_off.astype(np.int64), bad[:1], side="right") - 1
        raise AssertionError(f"{what}: {bad.size} output bytes differ, first at {bad[0]} "
                             f"(packet ~{pk[0]}, got {got.out[bad[0]]:#x} "
                             f"want {ref.out[bad[0]]:#x})")
