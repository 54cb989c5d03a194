import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def golden():
    return np.load(os.path.join(GOLDEN, "verify_vectors.npz"))


def golden_batches(g):
    """Yield (msg_len, dict of arrays) per golden batch."""
    for ml in g["msg_lens"]:
        pre = f"m{int(ml)}_"
        yield int(ml), {k[len(pre):]: g[k] for k in g.files if k.startswith(pre)}
