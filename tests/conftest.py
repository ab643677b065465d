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
    c = ec.Codec(0)
    yield c
    c.close()


@pytest.fixture(params=["fused", "rows"])
def rebuild_path(request, monkeypatch):
    """Run a rebuild test on both device rebuild paths: the fused
    gf_rebuild_kernel (default) and the two-kernel decode_coef_kernel +
    gf_mac_kernel path (MEMO_EC_REBUILD_FUSED=0, read per call)."""
    monkeypatch.setenv("MEMO_EC_REBUILD_FUSED", "1" if request.param == "fused" else "0")
    return request.param
