import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")
CASES = ["c1_nobrand", "c1_brand", "micro_d12", "hub_d32"]


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run with -m gpu")


def load_case(name):
    return np.load(os.path.join(GOLDEN, f"{name}.npz"))


def case_dims(z):
    return tuple(int(z[k]) for k in ("U", "I", "B", "d", "K"))


def case_e0(z):
    return np.concatenate([z["param/user_embedding.weight"], z["param/item_embedding.weight"],
                           z["param/brand_embedding.weight"]])


def upstream_grad(n, d):
    """Same seeded G as tests/golden/gen_golden.py::upstream_grad."""
    return np.random.default_rng(7).standard_normal((n, d)).astype(np.float32)


class Cfg:
    def __init__(self, d, k, debug=False):
        self.embedding_dim = d
        self.n_layers = k
        self.debug = debug


@pytest.fixture(scope="session")
def gpu_device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from gcn_recommendation_amd import engine
    engine.load_library()  # fails loudly if the extension is missing
    return torch.device("cuda:0")
