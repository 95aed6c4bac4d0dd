import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_PARENT = os.path.join(ROOT, "distributed-sieve-e_amd")
for p in (ROOT, PKG_PARENT):
    if p not in sys.path:
        sys.path.insert(0, p)

# Test harness only: DSE_TEST_LIB runs the suite against a variant build of
# libdse.so (tools/build_variant.sh) before it replaces the production one.
if os.environ.get("DSE_TEST_LIB"):
    from mail_sieve_e import _dse as _d
    _d.LIB_PATH = os.environ["DSE_TEST_LIB"]


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")
    config.addinivalue_line("markers", "slow: long CPU-side checks")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as o
    o.lib()
    return o


@pytest.fixture(scope="session")
def ctx():
    # no skip: on the GPU box a missing device or libdse.so must fail loudly
    from mail_sieve_e.sieve import Context
    c = Context(num_gpus=1)
    yield c
    c.close()
