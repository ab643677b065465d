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


# rebuild_path param -> (rebuild_path, image_min_tiles, image_min_coefs)
REBUILD_PATHS = {"fused": (1, 1, 40), "rows": (0, 1, 40), "lds": (0, 0, 40), "images": (0, 1, 0)}


@pytest.fixture(params=list(REBUILD_PATHS))
def rebuild_path(request, monkeypatch):
    """Run a rebuild test on every device rebuild path: the fused
    gf_rebuild_kernel (default up to 256 MiB); the two-kernel decode rows +
    gf_mac_kernel path as the defaults choose its tables ("rows": per-block
    table images through HBM for multi-tile blocks with costly tables,
    tables built in LDS for the rest, both in one launch of a mixed call);
    the same with tables always built in LDS ("lds") and with images for
    every block size ("images"): the session codec's options, and
    MEMO_EC_REBUILD_FUSED / MEMO_EC_IMAGE_MIN_TILES / MEMO_EC_IMAGE_MIN_COEFS
    for contexts the test creates itself."""
    v, t, cf = REBUILD_PATHS[request.param]
    monkeypatch.setenv("MEMO_EC_REBUILD_FUSED", str(v))
    monkeypatch.setenv("MEMO_EC_IMAGE_MIN_TILES", str(t))
    monkeypatch.setenv("MEMO_EC_IMAGE_MIN_COEFS", str(cf))
    if "codec" in request.fixturenames:
        c = request.getfixturevalue("codec")
        with c.options(rebuild_path=v, image_min_tiles=t, image_min_coefs=cf):
            yield request.param
    else:
        yield request.param
