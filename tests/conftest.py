import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "sing-quic_amd"), os.path.join(REPO, "tests"),
          os.path.join(REPO, "oracle"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

# torch before libsqobfs, whatever test runs first: torch's wheel carries its
# own HIP runtime (torch/lib/libamdhip64.so, soname libamdhip64.so.7), which
# libsqobfs then shares.  Loaded the other way round, the library brings
# /opt/rocm's runtime and torch, asking for the file name libamdhip64.so,
# loads a second one that finds no GPU ("No HIP GPUs are available").
try:
    import torch  # noqa: F401,E402
except ImportError:
    pass


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")


@pytest.fixture(scope="session")
def golden():
    import json

    def load(name):
        with open(os.path.join(REPO, "tests", "golden", name)) as f:
            return json.load(f)
    return load
