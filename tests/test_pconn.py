"""The obfuscating packet conn engine (sqobfs_pconn_*, the core of the Go
drop-in go/sqobfs.Conn): tests/cpp/test_pconn.c, threaded, over loopback UDP,
checked against the oracle's ReadFrom / WriteTo restatement."""
from __future__ import annotations

import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "tests", "cpp", "test_pconn.c")
OUT = os.path.join(REPO, "build", "test_pconn")


def _compile() -> str:
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle")], check=True)
    lib = os.path.join(REPO, "sing-quic_amd")
    cmd = ["gcc", "-std=c11", "-O1", "-Wall", "-Wextra", "-I", os.path.join(REPO, "include"),
           "-I", os.path.join(REPO, "oracle"), SRC, "-L", lib, "-lsqobfs",
           "-L", os.path.join(REPO, "oracle"), "-loracle", "-lpthread", f"-Wl,-rpath,{lib}",
           f"-Wl,-rpath,{os.path.join(REPO, 'oracle')}", "-o", OUT]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return OUT


def test_pconn_test_compiles_as_c():
    """What cgo sees: plain C against include/sqobfs.h."""
    _compile()


@pytest.mark.gpu
def test_pconn_engine():
    exe = _compile()
    r = subprocess.run([exe], capture_output=True, text=True, timeout=240)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok: pconn engine" in r.stdout
