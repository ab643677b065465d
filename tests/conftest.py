import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

SEED = 0x6D656D6F


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


@pytest.fixture(scope="session")
def golden():
    z = np.load(os.path.join(ROOT, "tests", "golden", "rs_golden.npz"))  # allow_pickle=False
    return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def O():
    from oracle import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def codec():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from memo_amd import ec
    ec.check_build()  # the loaded kernels were built from this tree's sources
    c = ec.Codec(0)
    yield c
    c.close()


@pytest.fixture(params=["fused", "rows"])
def rebuild_path(request, monkeypatch):
    """Run a rebuild test on both device rebuild paths: the fused
    gf_rebuild_kernel (default) and the two-kernel decode_coef_kernel +
    gf_mac_kernel path: the session codec's MEMO_EC_OPT_REBUILD_PATH, and
    MEMO_EC_REBUILD_FUSED for contexts the test creates itself."""
    v = 1 if request.param == "fused" else 0
    monkeypatch.setenv("MEMO_EC_REBUILD_FUSED", str(v))
    if "codec" in request.fixturenames:
        c = request.getfixturevalue("codec")
        with c.options(rebuild_path=v):
            yield request.param
    else:
        yield request.param
