"""CPU-side checks of the C-ABI boundary (no compute calls, no GPU needed)."""
from __future__ import annotations

import ctypes
import os
import re
import subprocess

import pytest
import sqobfs

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_header_symbol():
    L = sqobfs.lib()
    syms = sqobfs.header_symbols()
    assert len(syms) >= 18
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    # exported with C linkage (unmangled) in the dynamic symbol table
    nm = subprocess.run(["nm", "-D", "--defined-only", sqobfs.LIB_PATH], capture_output=True,
                        text=True, check=True).stdout
    exported = set(re.findall(r"\bT (sqobfs_\w+)", nm))
    assert set(syms) <= exported, set(syms) - exported


def test_header_is_plain_c():
    """The boundary header compiles as C99 with no HIP/torch types."""
    src = open(sqobfs.HEADER_PATH).read()
    assert "hip" not in re.sub(r"/\*.*?\*/", "", src, flags=re.S).lower()
    out = subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-fsyntax-only", "-x", "c",
                          sqobfs.HEADER_PATH], capture_output=True, text=True)
    assert out.returncode == 0, out.stderr


def test_batch_struct_layout_matches_header():
    """ctypes mirror of sqobfs_batch has the C layout (offsetof via gcc)."""
    prog = r'''
#include <stdio.h>
#include <stddef.h>
#include "sqobfs.h"
int main(void){printf("%zu %zu %zu %zu %zu\n", sizeof(sqobfs_batch),
 offsetof(sqobfs_batch,in), offsetof(sqobfs_batch,out_len), offsetof(sqobfs_batch,psk_id),
 offsetof(sqobfs_batch,in_cap));return 0;}'''
    exe = "/tmp/sq_layout_probe"
    subprocess.run(["gcc", "-x", "c", "-", "-I", os.path.join(REPO, "include"), "-o", exe],
                   input=prog, text=True, check=True)
    got = [int(x) for x in subprocess.run([exe], capture_output=True, text=True).stdout.split()]
    B = sqobfs.Batch
    assert got == [ctypes.sizeof(B), B.in_.offset, B.out_len.offset, B.psk_id.offset,
                   B.in_cap.offset]


def test_engine_info_layout_matches_header():
    """ctypes mirror of sqobfs_engine_info has the C layout (round 5 grew it:
    load routing, affinity and the coalesced-launch counters; round 6, ABI 6:
    the completer's counters)."""
    fields = ["pool_bytes", "route_bytes", "cpus", "group_max", "launches", "group_launches",
              "group_batches", "async_launches", "streams"]
    prog = ('#include <stdio.h>\n#include <stddef.h>\n#include "sqobfs.h"\n'
            'int main(void){printf("%zu' + ' %zu' * len(fields) + '\\n", sizeof(sqobfs_engine_info)'
            + "".join(f", offsetof(sqobfs_engine_info,{f})" for f in fields) + ");return 0;}")
    exe = "/tmp/sq_engine_info_probe"
    subprocess.run(["gcc", "-x", "c", "-", "-I", os.path.join(REPO, "include"), "-o", exe],
                   input=prog, text=True, check=True)
    got = [int(x) for x in subprocess.run([exe], capture_output=True, text=True).stdout.split()]
    E = sqobfs.EngineInfo
    assert got == [ctypes.sizeof(E)] + [getattr(E, f).offset for f in fields]


def test_engine_set_group_bounds():
    """sqobfs_engine_set_group (host logic): 0..64 batches per launch."""
    L = sqobfs.lib()
    assert L.sqobfs_engine_set_group(None, 65) == sqobfs.SQ_EINVAL
    sqobfs.engine_set_group(None, 0)  # (the host engine: no launches to coalesce)


def test_abi_version_and_strerror():
    L = sqobfs.lib()
    assert L.sqobfs_abi_version() == 6
    for st in (0, -1, -2, -3, -4, -5, -6, -7, -8):
        assert sqobfs.strerror(st) != "unknown status"


def test_null_arguments_rejected_without_gpu():
    L = sqobfs.lib()
    assert L.sqobfs_open(0, None) == sqobfs.SQ_EINVAL
    assert L.sqobfs_sync(None, None) == sqobfs.SQ_EINVAL
    b = sqobfs.Batch()
    assert L.sqobfs_launch(None, None, 0, ctypes.byref(b), None) == sqobfs.SQ_EINVAL
    assert L.sqobfs_run_host(None, None, 0, ctypes.byref(b)) == sqobfs.SQ_EINVAL
    assert L.sqobfs_keyring_create(None, 0, 1, None, None, None, None) == sqobfs.SQ_EINVAL


@pytest.mark.skipif(os.environ.get("SQ_ASSUME_GPU") == "1", reason="GPU box")
def test_no_gpu_reports_enodev_not_fallback():
    """Without a GPU the device entry points fail loudly (never a silent CPU
    fallback); the CPU path is explicit (host keyrings, tests/test_cpu_path.py)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(sqobfs.SqError) as e:
        sqobfs.Context(0)
    assert e.value.status == sqobfs.SQ_ENODEV


def test_shard_cuts_balance_bytes():
    """sqobfs_shard_cuts (host logic, no GPU): contiguous, covering, and
    balanced by cumulative bytes for ragged batches."""
    import numpy as np
    rng = np.random.Generator(np.random.PCG64(5))
    for n, parts in [(0, 3), (1, 4), (7, 8), (100_000, 8), (100_000, 3)]:
        lens = rng.integers(64, 1453, n).astype(np.uint32)
        cut = sqobfs.shard_cuts(lens, parts)
        assert cut[0] == 0 and cut[-1] == n and np.all(np.diff(cut.astype(np.int64)) >= 0)
        if n >= 1000:
            w = lens.astype(np.int64) + 64
            share = np.add.reduceat(w, cut[:-1].astype(np.int64)) if n else w
            assert share.max() - share.min() <= 2 * (1452 + 64), share
    # a skewed batch: one half tiny, one half large -> cut far from n/2
    lens = np.concatenate([np.full(5000, 0, np.uint32), np.full(5000, 1400, np.uint32)])
    cut = sqobfs.shard_cuts(lens, 2)
    assert abs(int(cut[1]) - 7391) <= 1  # (5000*64 + 5000*1464) / 2 bytes each side


def test_unit_packets_for_sizes_units_by_bytes():
    """sqobfs_unit_packets_for (host logic, no GPU): ~21.7 KB of payload per
    wavefront, 31.5 KB with a multi-PSK keyring, clamped to 1..62; the BASELINE
    configs get the unit sizes the in-process sweeps measured best
    (DESIGN.md section 5)."""
    f = sqobfs.unit_packets_for
    assert f(1350 << 20, 1 << 20) == 16          # configs[1]
    assert f(1200 << 20, 1 << 20) == 18          # (Salamander rule at 1,200 B)
    assert f(1200 << 20, 1 << 20, kind=sqobfs.XPLUS) == 16  # configs[2]
    assert f(1200 << 20, 1 << 20, True, sqobfs.XPLUS) == 26  # multi-PSK XPlus: 31.5 KB
    assert f(758 * (4 << 20), 4 << 20) == 28     # configs[3] (mean of U[64, 1452])
    assert f(1350 * (16 << 20), 16 << 20, True) == 23  # configs[4]
    assert f(64 * 100_000, 100_000) == 49 and f(0, 1 << 20) == 62
    assert f(70_000 * 8, 8) == 1
    for mean in range(1, 100_000, 997):
        u = f(mean * 1000, 1000)
        assert 1 <= u <= 62


def test_unit_packets_spread_small_batches():
    """Small batches run as at least 2,048 wavefronts (latency: a 256-datagram
    socket batch is 256 one-packet waves, not 10 waves of 26 packets)."""
    f = sqobfs.unit_packets_for
    for n in (1, 16, 64, 256, 1024, 2048):
        assert f(1350 * n, n) == 1
    assert f(1350 * 4096, 4096) == 2
    assert f(1350 * 16384, 16384) == 8
    assert f(64 * 8192, 8192) == 4  # short packets: the spread rule binds


def test_batch_flags_match_header():
    """The ctypes binding's batch flags are the header's (the Go binding
    takes them from the header through cgo)."""
    import re
    text = open(os.path.join(REPO, "include", "sqobfs.h")).read()
    defs = {m.group(1): int(m.group(2)) for m in
            re.finditer(r"#define SQOBFS_FLAG_(\w+) (\d+)u", text)}
    assert defs == {"OUT_UNINIT": 1, "DEVICE_SALT": 2, "OUT_BLOCKS": 4, "OUT_LINES": 8}
    for name, v in defs.items():
        assert getattr(sqobfs, "FLAG_" + name) == v, name
