"""Pin the CPU oracle (oracle/) against the golden vectors generated from the reference itself
(tests/golden/gen_golden.py imports /root/reference main.py + models/*). Everything is bitwise."""
import numpy as np
import pytest
import torch

from conftest import CASES, case_dims, case_e0, load_case, upstream_grad
from oracle import oracle
from util import sha1


@pytest.mark.parametrize("name", CASES + ["c1_fusion"])
def test_adjacency_builder_bitwise(name):
    """oracle.build_norm_adj == reference load_preprocessed_data's Â (main.py:282-336)."""
    z = load_case(name)
    U, I, B, d, K = case_dims(z)
    r, c, v, n = oracle.build_norm_adj(z["train_user"], z["train_item"], U, I, B, z["ib_item"],
                                       z["ib_brand"], bool(z["use_brand"]))
    assert n == U + I + B
    np.testing.assert_array_equal(r, z["adj_row"])
    np.testing.assert_array_equal(c, z["adj_col"])
    assert np.array_equal(v.view(np.uint32), z["adj_val"].view(np.uint32))


@pytest.mark.parametrize("name", CASES)
def test_forward_layers_and_mean_bitwise(name):
    z = load_case(name)
    U, I, B, d, K = case_dims(z)
    final, layers = oracle.forward(z["adj_row"], z["adj_col"], z["adj_val"], case_e0(z), K,
                                   return_layers=True)
    assert sha1(case_e0(z)) == str(z["sha1/E0"])
    for k in range(K):
        assert sha1(layers[k]) == str(z[f"sha1/E{k + 1}"]), f"layer {k + 1}"
    assert sha1(final) == str(z["sha1/final"])
    np.testing.assert_array_equal(final[:4], z["head/final"])


@pytest.mark.parametrize("name", CASES)
def test_backward_bitwise(name):
    z = load_case(name)
    U, I, B, d, K = case_dims(z)
    G = upstream_grad(U + I + B, d)
    assert sha1(G) == str(z["sha1/G"])
    g0 = oracle.backward(z["adj_row"], z["adj_col"], z["adj_val"], G, K)
    assert sha1(g0[:U]) == str(z["sha1/grad/user_embedding.weight"])
    assert sha1(g0[U:U + I]) == str(z["sha1/grad/item_embedding.weight"])
    assert sha1(g0[U + I:]) == str(z["sha1/grad/brand_embedding.weight"])


def test_fusion_path_bitwise():
    """Fusion: same loop over E0 = [user | leaky_relu(Linear) | brand] (lightgcn_fusion.py)."""
    z = load_case("c1_fusion")
    U, I, B, d, K = case_dims(z)
    e0 = z["full/E0"]
    final = oracle.forward(z["adj_row"], z["adj_col"], z["adj_val"], e0, K)
    assert sha1(final) == str(z["sha1/final"])
    np.testing.assert_array_equal(final, z["full/final"])


@pytest.mark.parametrize("name", CASES + ["c1_fusion"])
def test_evaluate_recall_ndcg_exact(name):
    """oracle.evaluate == main.evaluate (main.py:404-439) on the reference model's embeddings."""
    z = load_case(name)
    U, I, B, d, K = case_dims(z)
    e0 = z["full/E0"] if name == "c1_fusion" else case_e0(z)
    final = oracle.forward(z["adj_row"], z["adj_col"], z["adj_val"], e0, K)
    rec, ndcg = oracle.evaluate(final[:U], final[U:U + I], z["val_user"], z["val_item"],
                                z["train_user"], z["train_item"], int(z["eval_k"]))
    assert rec == float(z["recall"]) and ndcg == float(z["ndcg"])


@pytest.mark.parametrize("K", [1, 2, 3, 4, 8, 16])
def test_mean_is_sequential_sum_then_divide(K):
    """The fused mean epilogue's order: torch.mean(stack) == ((E0+E1)+...+EK)/(K+1) bitwise
    for K+1 <= 17 (lightgcn.py:54); LGCN_MAX_LAYERS is sized from this."""
    g = torch.Generator().manual_seed(K)
    es = [torch.randn(257, 64, generator=g) for _ in range(K + 1)]
    s = es[0].clone()
    for e in es[1:]:
        s = s + e
    assert torch.equal(s / (K + 1), torch.mean(torch.stack(es, 0), 0))


def test_oracle_matches_torch_sparse_mm_unsorted_duplicates():
    """The C restatement equals torch.sparse.mm on an uncoalesced COO in arbitrary stored order
    with duplicate coordinates (what the engine's stable sort must preserve)."""
    rng = np.random.default_rng(0)
    n, nnz, d = 300, 4000, 24
    r = rng.integers(0, n, nnz)
    c = rng.integers(0, n, nnz)
    v = rng.standard_normal(nnz).astype(np.float32)
    x = rng.standard_normal((n, d)).astype(np.float32)
    adj = torch.sparse_coo_tensor(torch.from_numpy(np.vstack([r, c])), torch.from_numpy(v), (n, n))
    want = torch.sparse.mm(adj, torch.from_numpy(x)).numpy()
    got = oracle.spmm(r, c, v, n, x)
    assert np.array_equal(got, want)
