"""gcn_recommendation_amd.data: the reference's processed-data format -> the 8-tuple of
main.py:172-347. The raw parquet files of the golden C1 case are re-created exactly as
tests/golden/gen_golden.py wrote them; the split and Â must match the fixture bitwise."""
import json

import numpy as np
import pandas as pd
import pytest
import torch

from conftest import ROOT, load_case
from gcn_recommendation_amd import data


def _write_c1(d, brand):
    rng = np.random.default_rng(0)
    U, I, E = 1000, 1000, 10000
    u = rng.integers(0, U, E)
    it = rng.integers(0, I, E)
    test_items = np.random.default_rng(123).integers(0, I, U)
    pd.DataFrame({"user_idx": u, "item_idx": it}).to_parquet(d / "train.parquet")
    pd.DataFrame({"user_idx": np.arange(U), "item_idx": test_items}).to_parquet(d / "test.parquet")
    if brand:
        ib = (np.arange(I), np.random.default_rng(1).integers(0, 50, I))
        B = 50
    else:
        ib = (np.zeros(0, np.int64), np.zeros(0, np.int64))
        B = 0
    pd.DataFrame({"item_idx": ib[0], "brand_idx": ib[1]}).to_parquet(d / "item_brand.parquet")
    json.dump({"num_users": U, "num_items": I, "num_brands": B}, open(d / "stats.json", "w"))
    np.save(d / "item_embeddings.npy", np.ones((I, 8), np.float32))


def _check(out, z):
    tr, va, te, U, I, B, adj, ib = out
    np.testing.assert_array_equal(tr["user_idx"].to_numpy(), z["train_user"])
    np.testing.assert_array_equal(tr["item_idx"].to_numpy(), z["train_item"])
    np.testing.assert_array_equal(va["user_idx"].to_numpy(), z["val_user"])
    np.testing.assert_array_equal(va["item_idx"].to_numpy(), z["val_item"])
    idx = adj._indices().cpu().numpy()
    np.testing.assert_array_equal(idx[0], z["adj_row"])
    np.testing.assert_array_equal(idx[1], z["adj_col"])
    assert np.array_equal(adj._values().cpu().numpy().view(np.uint32), z["adj_val"].view(np.uint32))


@pytest.mark.parametrize("brand", [False, True])
def test_loader_cpu_matches_reference(tmp_path, brand):
    _write_c1(tmp_path, brand)
    z = load_case("c1_brand" if brand else "c1_nobrand")
    _check(data.load_preprocessed_data(str(tmp_path), "cpu", use_brand=brand, verbose=False), z)
    assert data.load_item_embeddings(str(tmp_path)).shape == (1000, 8)


@pytest.mark.gpu
@pytest.mark.parametrize("brand", [False, True])
def test_loader_device_matches_reference(tmp_path, brand, gpu_device):
    _write_c1(tmp_path, brand)
    z = load_case("c1_brand" if brand else "c1_nobrand")
    out = data.load_preprocessed_data(str(tmp_path), gpu_device, use_brand=brand, verbose=False)
    _check(out, z)
    assert hasattr(out[6], "_lgcn_graph")


def test_loader_missing_stats(tmp_path):
    with pytest.raises(FileNotFoundError):
        data.load_preprocessed_data(str(tmp_path), "cpu")


def test_bench_val_split_is_main_py_split():
    """bench.val_split (the trained-Recall@20 block) is main.py:201-203's split: the row ranked
    1 by groupby(user).rank(method="first", ascending=False) — each user's FIRST row."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    u = np.array([0, 1, 0, 2, 1, 0, 3])
    i = np.array([5, 6, 7, 8, 9, 10, 11])
    tu, ti, vu, vi = bench.val_split(u, i)
    assert list(zip(vu, vi)) == [(0, 5), (1, 6), (2, 8), (3, 11)]
    assert list(zip(tu, ti)) == [(0, 7), (1, 9), (0, 10)]
