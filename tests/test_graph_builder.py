"""Product-side host graph builder (gcn_recommendation_amd.graph) vs the reference-built Â."""
import numpy as np
import pytest
import torch

from conftest import CASES, case_dims, load_case
from gcn_recommendation_amd import graph


@pytest.mark.parametrize("name", CASES + ["c1_fusion"])
def test_build_norm_adj_matches_reference(name):
    z = load_case(name)
    U, I, B, d, K = case_dims(z)
    adj = graph.build_norm_adj(z["train_user"], z["train_item"], U, I, B, z["ib_item"],
                               z["ib_brand"], bool(z["use_brand"]))
    assert adj.shape == (U + I + B, U + I + B)
    assert adj.dtype == torch.float32 and not adj.is_coalesced()
    idx = adj._indices().numpy()
    np.testing.assert_array_equal(idx[0], z["adj_row"])
    np.testing.assert_array_equal(idx[1], z["adj_col"])
    assert np.array_equal(adj._values().numpy().view(np.uint32), z["adj_val"].view(np.uint32))


def test_generators_shapes_and_determinism():
    u, i = graph.uniform_interactions(100, 50, 1000, 1)
    u2, i2 = graph.uniform_interactions(100, 50, 1000, 1)
    assert np.array_equal(u, u2) and np.array_equal(i, i2)
    assert u.max() < 100 and i.max() < 50
    u, i = graph.powerlaw_interactions(1000, 500, 5000, 2)
    assert len(u) == len(i) == 5000
    assert np.unique(u).size == 1000  # every user has >= 1 interaction
    deg = np.bincount(i, minlength=500)
    assert deg.max() > 10 * max(1, np.median(deg))  # skewed


def test_empty_graph_builds():
    adj = graph.build_norm_adj(np.zeros(0, np.int64), np.zeros(0, np.int64), 3, 4, 0,
                               use_brand=False)
    assert adj._nnz() == 0 and adj.shape == (7, 7)
