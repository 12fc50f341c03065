"""A main.py-style training loop (Adam lr 1e-3 over all parameters, BPR loss with lambda 1e-4,
full-graph forward + backward per batch, main.py:469-531) on the HIP engine vs the same loop on
the CPU reference path, same initial weights and batches: loss trajectories and parameters
stay within fp32 noise."""
import numpy as np
import pytest
import torch

from conftest import Cfg, case_dims, load_case
from gcn_recommendation_amd import graph
from gcn_recommendation_amd.loss import bpr_loss_reg
from models.lightgcn import LightGCN

pytestmark = pytest.mark.gpu


def _train(dev, z, steps=12):
    U, I, B, d, K = case_dims(z)
    torch.manual_seed(42)
    m = LightGCN(U, I, B, Cfg(d, K)).to(dev)
    adj = graph.build_norm_adj(z["train_user"], z["train_item"], U, I, B, z["ib_item"],
                               z["ib_brand"], bool(z["use_brand"]), device=dev)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    rng = np.random.default_rng(5)
    losses = []
    for _ in range(steps):
        bu = torch.from_numpy(rng.integers(0, U, 256)).to(dev)
        bp = torch.from_numpy(rng.integers(0, I, 256)).to(dev)
        bn = torch.from_numpy(rng.integers(0, I, 256)).to(dev)
        opt.zero_grad()
        fu, fi, fb, u0, i0 = m(adj, use_brand=True)
        loss = bpr_loss_reg(fu[bu], fi[bp], fi[bn], u0[bu], i0[bp], i0[bn], 1e-4,
                            final_brand_emb=fb)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    return np.array(losses), {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}


def test_training_loop_gpu_matches_cpu(gpu_device):
    z = load_case("c1_brand")
    lg, pg = _train(gpu_device, z)
    lc, pc = _train(torch.device("cpu"), z)
    np.testing.assert_allclose(lg, lc, rtol=1e-5)
    z0 = {k[len("param/"):]: z[k] for k in z.files if k.startswith("param/")}
    for k in pc:
        np.testing.assert_allclose(pg[k], pc[k], rtol=0, atol=2e-6 * np.abs(pc[k]).max() + 1e-9)
        assert not np.array_equal(pc[k], z0[k]) or pc[k].size == 0, f"{k} never updated"
