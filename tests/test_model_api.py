"""Drop-in boundary: models.lightgcn.LightGCN / models.lightgcn_fusion.LightGCN_Fusion resolve
through the reference's plugin loader logic (main.py:42-50), keep its constructor semantics,
RNG draw order, parameter/state_dict layout and the 5-tuple; the BPR-loss API matches
main.py:366-402 on the golden batch."""
import importlib

import numpy as np
import pytest
import torch

from conftest import CASES, Cfg, case_dims, load_case
from gcn_recommendation_amd import graph
from gcn_recommendation_amd.loss import bpr_loss_reg
from util import sha1


def get_model(model_name):
    """main.py:42-50, verbatim logic."""
    module_path = f"models.{model_name.lower()}"
    model_module = importlib.import_module(module_path)
    return getattr(model_module, model_name)


def _make(name, z):
    U, I, B, d, K = case_dims(z)
    torch.manual_seed(42)
    if name == "c1_fusion":
        return get_model("LightGCN_Fusion")(U, I, B, Cfg(d, K), pretrained_item_emb=z["content"])
    return get_model("LightGCN")(U, I, B, Cfg(d, K))


@pytest.mark.parametrize("name", CASES + ["c1_fusion"])
def test_ctor_rng_order_and_state_dict(name):
    z = load_case(name)
    m = _make(name, z)
    sd = m.state_dict()
    want = [k[len("param/"):] for k in z.files if k.startswith("param/")]
    assert sorted(sd.keys()) == sorted(want)
    for k in want:
        assert np.array_equal(sd[k].numpy(), z["param/" + k]), k
    # parameter registration order (Adam state order, main.py:469)
    names = [n for n, _ in m.named_parameters()]
    if name == "c1_fusion":
        assert names == ["user_embedding.weight", "item_id_embedding.weight",
                         "brand_embedding.weight", "item_fusion_layer.weight",
                         "item_fusion_layer.bias"]
    else:
        assert names == ["user_embedding.weight", "brand_embedding.weight",
                         "item_embedding.weight"]


def test_ctor_errors():
    with pytest.raises(ValueError):
        get_model("LightGCN")(3, 4, 0, Cfg(8, 2), pretrained_item_emb=np.zeros((4, 5), np.float32))
    with pytest.raises(ValueError):
        get_model("LightGCN_Fusion")(3, 4, 0, Cfg(8, 2), pretrained_item_emb=None)
    m = get_model("LightGCN")(3, 4, 0, Cfg(8, 2), pretrained_item_emb=np.ones((4, 8), np.float32))
    assert torch.equal(m.item_embedding.weight, torch.ones(4, 8))
    assert m.item_embedding.weight.requires_grad


@pytest.mark.parametrize("name", CASES + ["c1_fusion"])
def test_cpu_forward_backward_match_reference(name):
    """CPU adjacency (BASELINE configs[0], plumbing): bitwise = the reference's outputs.
    (Fixtures were generated single-threaded; MKL's GEMM in the fusion Linear is thread-count
    dependent, so run single-threaded here too.)"""
    torch.set_num_threads(1)
    z = load_case(name)
    U, I, B, d, K = case_dims(z)
    m = _make(name, z)
    adj = graph.build_norm_adj(z["train_user"], z["train_item"], U, I, B, z["ib_item"],
                               z["ib_brand"], bool(z["use_brand"]))
    out = m(adj, use_brand=bool(z["use_brand"]))
    assert len(out) == 5
    fu, fi, fb, u0, i0 = out
    assert fu.shape == (U, d) and fi.shape == (I, d) and fb.shape == (B, d)
    assert u0 is m.user_embedding.weight
    assert sha1(torch.cat([fu, fi, fb]).detach().numpy()) == str(z["sha1/final"])
    G = torch.from_numpy(np.random.default_rng(7).standard_normal((U + I + B, d)).astype(np.float32))
    (torch.cat([fu, fi, fb]) * G).sum().backward()
    for n, p in m.named_parameters():
        assert sha1(p.grad.numpy()) == str(z["sha1/grad/" + n]), n


@pytest.mark.parametrize("name", CASES)
def test_bpr_loss_api_matches_reference(name):
    z = load_case(name)
    U, I, B, d, K = case_dims(z)
    m = _make(name, z)
    adj = graph.build_norm_adj(z["train_user"], z["train_item"], U, I, B, z["ib_item"],
                               z["ib_brand"], bool(z["use_brand"]))
    bu, bp, bn = (torch.from_numpy(z[k]) for k in ("bpr_users", "bpr_pos", "bpr_neg"))
    fu, fi, fb, u0, i0 = m(adj, use_brand=bool(z["use_brand"]))
    loss = bpr_loss_reg(fu[bu], fi[bp], fi[bn], u0[bu], i0[bp], i0[bn], 1e-4, brand_loss=False,
                        final_brand_emb=fb if bool(z["use_brand"]) else None)
    assert np.float32(loss.item()) == z["bpr_loss"]
    loss.backward()
    for n, p in m.named_parameters():
        assert sha1(p.grad.numpy()) == str(z["sha1/bpr_grad/" + n]), n


def test_computer_alias():
    z = load_case("micro_d12")
    U, I, B, d, K = case_dims(z)
    m = _make("micro_d12", z)
    adj = graph.build_norm_adj(z["train_user"], z["train_item"], U, I, B, z["ib_item"],
                               z["ib_brand"], True)
    fu, fi = m.set_graph(adj).computer()
    fu2, fi2, _, _, _ = m(adj)
    assert torch.equal(fu, fu2) and torch.equal(fi, fi2)
    with pytest.raises(ValueError):
        _make("micro_d12", z).computer()


def test_use_brand_flag_is_ignored_like_reference():
    z = load_case("micro_d12")
    U, I, B, d, K = case_dims(z)
    m = _make("micro_d12", z)
    adj = graph.build_norm_adj(z["train_user"], z["train_item"], U, I, B, z["ib_item"],
                               z["ib_brand"], True)
    a = m(adj, use_brand=True)[0]
    b = m(adj, use_brand=False)[0]
    assert torch.equal(a, b)


def test_cpu_forward_returns_the_weights_themselves():
    """On a CPU adjacency the ego tables are the weights (the reference's objects); the engine's
    aliases (e0_outputs) exist on the HIP path only. A bad e0_outputs is refused before any
    device work."""
    from gcn_recommendation_amd import engine
    from models.lightgcn import LightGCN
    z = load_case("c1_brand")
    U, I, B, d, K = case_dims(z)
    m = LightGCN(U, I, B, Cfg(d, K))
    adj = graph.build_norm_adj(z["train_user"], z["train_item"], U, I, B, z["ib_item"],
                               z["ib_brand"], bool(z["use_brand"]))
    out = m(adj)
    assert out[3] is m.user_embedding.weight and out[4] is m.item_embedding.weight
    segs = [torch.zeros(2, 4)] * 3
    for bad in (-1, 4):
        with pytest.raises(engine.LgcnError):
            engine.propagate_blocks(adj, segs, 1, e0_outputs=bad)
