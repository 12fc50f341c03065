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


def _ego_grads(dev, z, e0_outputs, dense=False):
    """Weight gradients of one BPR step (main.py:496-499) whose regulariser gathers either the
    engine's ego aliases (e0_outputs=2) or the weights themselves (0)."""
    from gcn_recommendation_amd import engine
    U, I, B, d, K = case_dims(z)
    torch.manual_seed(7)
    w = [torch.randn(n, d, device=dev).requires_grad_() for n in (U, I, B)]
    adj = graph.build_norm_adj(z["train_user"], z["train_item"], U, I, B, z["ib_item"],
                               z["ib_brand"], bool(z["use_brand"]), device=dev)
    out = engine.propagate_blocks(adj, w, K, e0_outputs=e0_outputs)
    fu, fi, fb = out[:3]
    u0, i0 = out[3:] if e0_outputs else (w[0], w[1])
    g = torch.Generator().manual_seed(11)
    bu, bp, bn = (torch.randint(0, n, (512,), generator=g).to(dev) for n in (U, I, I))
    loss = bpr_loss_reg(fu[bu], fi[bp], fi[bn], u0[bu], i0[bp], i0[bn], 1e-4, final_brand_emb=fb)
    if dense:  # every row of every table live: the dense add
        loss = loss + (fu * 1e-3).sum() + (u0 * 2e-3).sum() + (i0 ** 2).sum()
    loss.backward()
    return [t.grad.clone() for t in w]


@pytest.mark.parametrize("dense", [False, True])
def test_ego_alias_gradients_bitwise(gpu_device, dense):
    """PropagateFunction's ego aliases: adding their gradients' nonzero entries into dE0 inside
    the backward gives autograd's dense sum to the bit (row-sparse and dense cases)."""
    z = load_case("c1_brand")
    a = _ego_grads(gpu_device, z, 2, dense)
    b = _ego_grads(gpu_device, z, 0, dense)
    for x, y in zip(a, b):
        assert torch.equal(x.view(torch.int32), y.view(torch.int32))


def test_ego_alias_k0_negative_zero(gpu_device):
    """n_layers = 0: dE0 is G itself and may hold -0; where the ego alias's gradient
    is +0, autograd's sum gives +0 — the aliases' backward must too."""
    from gcn_recommendation_amd import engine
    z = load_case("c1_brand")
    U, I, B, d, _ = case_dims(z)
    adj = graph.build_norm_adj(z["train_user"], z["train_item"], U, I, B, z["ib_item"],
                               z["ib_brand"], bool(z["use_brand"]), device=gpu_device)
    g = torch.Generator().manual_seed(4)
    G = [torch.randn(n, d, generator=g) for n in (U, I, B)]
    E = [torch.randn(n, d, generator=g) for n in (U, I)]
    for t in G:
        t[torch.rand(t.shape, generator=g) < 0.3] = -0.0
    for t in E:
        t[torch.rand(t.shape, generator=g) < 0.5] = 0.0
    G = [t.to(gpu_device) for t in G]
    E = [t.to(gpu_device) for t in E]
    res = []
    for e0_outputs in (2, 0):
        torch.manual_seed(7)
        w = [torch.randn(n, d, device=gpu_device).requires_grad_() for n in (U, I, B)]
        out = engine.propagate_blocks(adj, w, 0, e0_outputs=e0_outputs)
        ego = list(out[3:]) if e0_outputs else [w[0], w[1]]
        torch.autograd.backward(list(out[:3]) + ego, G + E)
        res.append([t.grad.clone() for t in w])
    for x, y in zip(*res):
        assert torch.equal(x.view(torch.int32), y.view(torch.int32))


def test_add_nonzero_matches_dense_add(gpu_device):
    """lgcn_add_nonzero == dst + src bitwise for dst != -0 (zeros of both signs, NaN, inf, odd
    lengths and a misaligned start take the scalar path)."""
    from gcn_recommendation_amd import engine
    lib = engine.load_library()
    g = torch.Generator().manual_seed(3)
    for n, off in ((0, 0), (1, 0), (7, 0), (4096, 0), (4096 + 3, 1), (1 << 20, 0)):
        src = torch.randn(n + off, generator=g)
        src[torch.rand(n + off, generator=g) < 0.6] = 0.0
        src[torch.rand(n + off, generator=g) < 0.1] = -0.0
        if n > 8:
            src[off + 3], src[off + 5] = float("nan"), float("inf")
        dst = torch.randn(n + off, generator=g)
        dst[torch.rand(n + off, generator=g) < 0.2] = 0.0
        s, t = src.to(gpu_device)[off:], dst.to(gpu_device)[off:]
        want = t + s
        with torch.cuda.device(gpu_device):
            assert lib.lgcn_add_nonzero(engine._ptr(s), engine._ptr(t), n,
                                        engine._stream(gpu_device)) == 0
        assert torch.equal(t.view(torch.int32), want.view(torch.int32)), n


def test_fusion_model_user_alias_gradients_bitwise(gpu_device):
    """LightGCN_Fusion returns the engine's user alias (e0_outputs=1): one BPR step's parameter
    gradients equal those of the same step with the user weight itself, to the bit."""
    from models.lightgcn_fusion import LightGCN_Fusion
    from gcn_recommendation_amd import engine
    z = load_case("c1_fusion")
    U, I, B, d, K = case_dims(z)
    content = z["content"] if "content" in z.files else \
        np.random.default_rng(1).standard_normal((I, 32)).astype(np.float32)
    adj = graph.build_norm_adj(z["train_user"], z["train_item"], U, I, B, z["ib_item"],
                               z["ib_brand"], bool(z["use_brand"]), device=gpu_device)
    g = torch.Generator().manual_seed(5)
    bu, bp, bn = (torch.randint(0, n, (256,), generator=g).to(gpu_device) for n in (U, I, I))

    def grads(alias):
        torch.manual_seed(3)
        m = LightGCN_Fusion(U, I, B, Cfg(d, K), pretrained_item_emb=content).to(gpu_device)
        fu, fi, fb, u0, i0 = m(adj)
        if not alias:
            u0 = m.user_embedding.weight
        else:
            assert u0 is not m.user_embedding.weight
            assert u0.data_ptr() == m.user_embedding.weight.data_ptr()
        loss = bpr_loss_reg(fu[bu], fi[bp], fi[bn], u0[bu], i0[bp], i0[bn], 1e-4,
                            final_brand_emb=fb)
        loss.backward()
        return {k: p.grad.clone() for k, p in m.named_parameters()}

    a, b = grads(True), grads(False)
    for k in a:
        assert torch.equal(a[k].view(torch.int32), b[k].view(torch.int32)), k
