import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "oracle"), os.path.join(REPO, "zfp-par_amd"), os.path.join(REPO, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP product path)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def _ensure_oracle():
    so = os.path.join(REPO, "oracle", "build", "liboracle.so")
    if not os.path.exists(so):
        subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "oracle")])
    return so


@pytest.fixture(scope="session")
def oracle():
    _ensure_oracle()
    from pyoracle import Oracle
    return Oracle()


@pytest.fixture(scope="session")
def ref_capi():
    """The reference library compiled from /root/reference (oracle/_ref)."""
    from pyoracle import REF_SO
    if not os.path.exists(REF_SO):
        pytest.skip("oracle/_ref not built (needs /root/reference; make -C oracle ref)")
    from capi import ZfpCAPI
    return ZfpCAPI(REF_SO)


PRODUCT_SO = os.path.join(REPO, "zfp-par_amd", "lib", "libzfp.so")


@pytest.fixture(scope="session")
def prod():
    """The product library for host-only (no GPU) checks."""
    if not os.path.exists(PRODUCT_SO):
        pytest.fail("product library not built")
    from capi import ZfpCAPI
    return ZfpCAPI(PRODUCT_SO)


@pytest.fixture(scope="session")
def product():
    """The product library; GPU tests fail loudly if it or the GPU is missing."""
    if not os.path.exists(PRODUCT_SO):
        raise RuntimeError("zfp-par_amd/lib/libzfp.so is not built (python -c 'import __graft_entry__ as g; g.build()')")
    try:  # one HIP runtime per process: let torch's (same SONAME) load first
        import torch  # noqa: F401
    except ImportError:
        pass
    from capi import ZfpCAPI
    api = ZfpCAPI(PRODUCT_SO)
    api.enable_index()
    if api.lib.zfp_hip_device_count() <= 0:
        raise RuntimeError("no HIP device visible: the MI355X path cannot run")
    return api


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(REPO, "tests", "golden", "checksums.json")) as f:
        return json.load(f)["entries"]
