"""The obfuscating packet conn engine (sqobfs_pconn_*, the core of the Go
drop-in go/sqobfs.Conn): tests/cpp/test_pconn.c, threaded, over loopback UDP,
checked against the oracle's ReadFrom / WriteTo restatement.

Three ways, so the engine's behaviour is covered with and without a GPU:
  * on the MI355X (-m gpu): a context on GPU 0;
  * with no device (CPU): the real libsqobfs.so, host keyrings, every batch
    on the product's CPU path -- the drop-in where no GPU exists;
  * over the CPU device of tests/cpp/sq_devstub.cpp (CPU): the engine built
    without HIP, its GPU-mode paths (launches on streams, waits, injected
    launch failures) exercised, plain and under ASan/UBSan and TSan
    (scripts/dev/cpu_sanitize.sh)."""
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


def test_pconn_engine_without_a_device():
    """The drop-in with no GPU at all: every datagram through the CPU path,
    the same wire / read checks, deadlines, shutdown, sync errors, and the
    shared engine."""
    exe = _compile()
    r = subprocess.run([exe, "nodev"], capture_output=True, text=True, timeout=240)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok: pconn engine [no device]" in r.stdout


@pytest.mark.parametrize("variant", ["plain", "asan", "tsan"])
def test_pconn_engine_on_cpu_device_sanitized(variant):
    """The engine without HIP over a CPU "device" whose streams are threads:
    GPU-mode scheduling, launch / wait hand-offs, injected launch failures;
    ASan+UBSan and TSan halt on the first report."""
    script = os.path.join(REPO, "scripts", "dev", "cpu_sanitize.sh")
    r = subprocess.run([script, variant], capture_output=True, text=True, timeout=1500)
    log = open(os.path.join(REPO, "build", "san", f"{variant}.log")).read()
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:] + log[-3000:]
    assert "ok: pconn engine [device]" in log and "ok: pconn engine [no device]" in log
    assert "Sanitizer" not in log and "runtime error" not in log


@pytest.mark.gpu
def test_pconn_engine():
    exe = _compile()
    r = subprocess.run([exe], capture_output=True, text=True, timeout=240)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok: pconn engine [device]" in r.stdout
