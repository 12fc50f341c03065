"""Generate the golden parity fixtures by IMPORTING the reference in this container.

This script is the only place that touches `/root/reference`. It imports the reference's own
`main.load_preprocessed_data` (main.py:172-347), `models.lightgcn.LightGCN` (lightgcn.py:4-81),
`models.lightgcn_fusion.LightGCN_Fusion` (lightgcn_fusion.py:5-64), `main.bpr_loss_reg`
(main.py:366-402) and `main.evaluate` (main.py:404-439), runs them on CPU on small seeded synthetic
graphs, and dumps inputs + outputs as `.npz` data fixtures next to this file. Only data leaves the
reference: edge lists, the normalised adjacency it built, embeddings, gradients, losses, metrics.

Run (in the build container only; the GPU box has no /root/reference):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py [debug]
"""
import contextlib
import io
import json
import os
import sys
import tempfile

import hashlib

import numpy as np
import pandas as pd
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def _import_reference():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    import main as ref_main  # noqa: E402
    from models.lightgcn import LightGCN  # noqa: E402
    from models.lightgcn_fusion import LightGCN_Fusion  # noqa: E402
    return ref_main, LightGCN, LightGCN_Fusion


def sha1(a):
    return hashlib.sha1(np.ascontiguousarray(a).tobytes()).hexdigest()


def _keep(out, name, a, full=False):
    """Outputs are pinned by sha1 of their bytes (bitwise) + a few rows for diagnostics."""
    a = np.ascontiguousarray(a)
    out["sha1/" + name] = np.array(sha1(a))
    out["head/" + name] = a[:4].copy()
    out["absmax/" + name] = np.float64(np.abs(a).max() if a.size else 0.0)
    if full:
        out["full/" + name] = a


def upstream_grad(n, d):
    """Seeded upstream gradient of the final embeddings (numpy PCG64, reproducible in tests)."""
    return np.random.default_rng(7).standard_normal((n, d)).astype(np.float32)


class _Cfg:
    def __init__(self, d, k):
        self.embedding_dim = d
        self.n_layers = k
        self.debug = False


def _write_dataset(d, users, items, test_items, item_brand, U, I, B):
    pd.DataFrame({"user_idx": users, "item_idx": items}).to_parquet(f"{d}/train.parquet")
    pd.DataFrame({"user_idx": np.arange(len(test_items)), "item_idx": test_items}).to_parquet(
        f"{d}/test.parquet")
    ib_items, ib_brands = item_brand
    pd.DataFrame({"item_idx": ib_items, "brand_idx": ib_brands}).to_parquet(f"{d}/item_brand.parquet")
    with open(f"{d}/stats.json", "w") as f:
        json.dump({"num_users": U, "num_items": I, "num_brands": B}, f)


def make_case(name, users, items, U, I, B, item_brand, d, K, use_brand, fusion_c=0, eval_k=20):
    ref_main, LightGCN, LightGCN_Fusion = _import_reference()
    rng = np.random.default_rng(123)
    test_items = rng.integers(0, I, U)
    with tempfile.TemporaryDirectory() as tmp:
        _write_dataset(tmp, users, items, test_items, item_brand, U, I, B)
        with contextlib.redirect_stdout(io.StringIO()):
            tr, va, te, nu, ni, nb, adj, ibdf = ref_main.load_preprocessed_data(
                tmp, "cpu", use_brand=use_brand, debug=False)
    idx = adj._indices().numpy()
    vals = adj._values().numpy()
    out = {
        "U": np.int64(U), "I": np.int64(I), "B": np.int64(B), "d": np.int64(d), "K": np.int64(K),
        "use_brand": np.int64(int(use_brand)),
        # builder inputs AFTER the reference's val split (main.py:201-203)
        "train_user": tr["user_idx"].to_numpy().astype(np.int64),
        "train_item": tr["item_idx"].to_numpy().astype(np.int64),
        "val_user": va["user_idx"].to_numpy().astype(np.int64),
        "val_item": va["item_idx"].to_numpy().astype(np.int64),
        "ib_item": np.asarray(item_brand[0], dtype=np.int64),
        "ib_brand": np.asarray(item_brand[1], dtype=np.int64),
        # the reference's normalised adjacency, in its stored order (main.py:331-336)
        "adj_row": idx[0].astype(np.int32), "adj_col": idx[1].astype(np.int32), "adj_val": vals,
    }
    cfg = _Cfg(d, K)
    content = None
    torch.manual_seed(42)
    if fusion_c:
        content = np.random.default_rng(5).standard_normal((I, fusion_c)).astype(np.float32)
        with contextlib.redirect_stdout(io.StringIO()):
            model = LightGCN_Fusion(nu, ni, nb, cfg, pretrained_item_emb=content)
        out["content"] = content
    else:
        with contextlib.redirect_stdout(io.StringIO()):
            model = LightGCN(nu, ni, nb, cfg)
    state = {k: v.detach().clone().numpy() for k, v in model.state_dict().items()}
    for k, v in state.items():
        out["param/" + k] = v

    # forward, then the hot path's gradient for a seeded upstream gradient G
    fu, fi, fb, u0, i0 = model(adj, use_brand=use_brand)
    G = torch.from_numpy(upstream_grad(U + I + B, d))
    Gu, Gi, Gb = torch.split(G, [U, I, B])
    ((fu * Gu).sum() + (fi * Gi).sum() + (fb * Gb).sum()).backward()
    _keep(out, "final", torch.cat([fu, fi, fb]).detach().numpy(), full=bool(fusion_c))
    out["sha1/G"] = np.array(sha1(G.numpy()))
    for n, p in model.named_parameters():
        _keep(out, "grad/" + n, p.grad.detach().numpy(), full=bool(fusion_c) and "fusion" in n)

    # per-layer outputs E_1..E_K with the reference's own op (torch.sparse.mm, lightgcn.py:45)
    with torch.no_grad():
        if fusion_c:
            ego = torch.cat([model.user_embedding.weight,
                             torch.nn.functional.leaky_relu(model.item_fusion_layer(
                                 torch.cat([model.item_id_embedding.weight,
                                            model.item_content_embedding], 1))),
                             model.brand_embedding.weight])
        else:
            ego = torch.cat([model.user_embedding.weight, model.item_embedding.weight,
                             model.brand_embedding.weight])
        _keep(out, "E0", ego.numpy(), full=bool(fusion_c))
        x = ego
        for k in range(K):
            x = torch.sparse.mm(adj, x)
            _keep(out, f"E{k + 1}", x.numpy())

    # BPR loss API (main.py:366-402, called as in main.py:515-522) on a fixed batch
    model.zero_grad()
    brng = np.random.default_rng(11)
    bu = torch.from_numpy(brng.integers(0, U, 64))
    bp = torch.from_numpy(brng.integers(0, I, 64))
    bn = torch.from_numpy(brng.integers(0, I, 64))
    fu, fi, fb, u0, i0 = model(adj, use_brand=use_brand)
    loss = ref_main.bpr_loss_reg(fu[bu], fi[bp], fi[bn], u0[bu], i0[bp], i0[bn], 1e-4,
                                 brand_loss=False, final_brand_emb=fb if use_brand else None)
    loss.backward()
    out["bpr_users"], out["bpr_pos"], out["bpr_neg"] = bu.numpy(), bp.numpy(), bn.numpy()
    out["bpr_loss"] = np.float32(loss.item())
    for n, p in model.named_parameters():
        _keep(out, "bpr_grad/" + n, p.grad.detach().numpy())

    # Recall@20 / NDCG@20 via the reference's evaluate (main.py:404-439)
    with contextlib.redirect_stdout(io.StringIO()), contextlib.redirect_stderr(io.StringIO()):
        rec, ndcg = ref_main.evaluate(model, va, tr, adj, eval_k, "cpu")
    out["recall"] = np.float64(rec)
    out["ndcg"] = np.float64(ndcg)
    out["eval_k"] = np.int64(eval_k)
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **out)
    print(f"{name}: N={U + I + B} nnz={len(vals)} d={d} K={K} recall={rec:.4f} ndcg={ndcg:.4f}")


def make_debug_case(name, users, items, U, I, B, item_brand, d, K, use_brand):
    """config.debug=True forward (lightgcn.py:49-51 per-layer brand norms, :62-78 cosine check
    and its torch.manual_seed(42) side effect): the printed lines and the CPU generator's next
    draws after the forward."""
    ref_main, LightGCN, _ = _import_reference()
    rng = np.random.default_rng(123)
    test_items = rng.integers(0, I, U)
    with tempfile.TemporaryDirectory() as tmp:
        _write_dataset(tmp, users, items, test_items, item_brand, U, I, B)
        with contextlib.redirect_stdout(io.StringIO()):
            tr, va, te, nu, ni, nb, adj, ibdf = ref_main.load_preprocessed_data(
                tmp, "cpu", use_brand=use_brand, debug=False)
    idx = adj._indices().numpy()
    cfg = _Cfg(d, K)
    cfg.debug = True
    torch.manual_seed(42)
    with contextlib.redirect_stdout(io.StringIO()):
        model = LightGCN(nu, ni, nb, cfg)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        fu, fi, fb, _, _ = model(adj, use_brand=use_brand)
    out = {
        "U": np.int64(U), "I": np.int64(I), "B": np.int64(B), "d": np.int64(d), "K": np.int64(K),
        "use_brand": np.int64(int(use_brand)),
        "train_user": tr["user_idx"].to_numpy().astype(np.int64),
        "train_item": tr["item_idx"].to_numpy().astype(np.int64),
        "ib_item": np.asarray(item_brand[0], dtype=np.int64),
        "ib_brand": np.asarray(item_brand[1], dtype=np.int64),
        "adj_row": idx[0].astype(np.int32), "adj_col": idx[1].astype(np.int32),
        "adj_val": adj._values().numpy(),
        "stdout": np.array(buf.getvalue()),
        "rng_after": torch.rand(8).numpy(),
    }
    _keep(out, "final", torch.cat([fu, fi, fb]).detach().numpy())
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **out)
    print(f"{name}: debug stdout {len(buf.getvalue().splitlines())} lines")


def main_debug():
    rng = np.random.default_rng(0)
    U, I, E = 1000, 1000, 10000
    u = rng.integers(0, U, E)
    it = rng.integers(0, I, E)
    brands = np.random.default_rng(1).integers(0, 50, I)
    make_debug_case("debug_c1_brand", u, it, U, I, 50, (np.arange(I), brands), 64, 2,
                    use_brand=True)
    make_debug_case("debug_c1_brand_k0", u, it, U, I, 50, (np.arange(I), brands), 64, 0,
                    use_brand=True)


def main():
    torch.set_num_threads(1)
    # C1 (BASELINE.json configs[0]): 1k x 1k x 10k uniform, default_rng(0), d=64, K=2
    rng = np.random.default_rng(0)
    U, I, E = 1000, 1000, 10000
    u = rng.integers(0, U, E)
    it = rng.integers(0, I, E)
    make_case("c1_nobrand", u, it, U, I, 0, (np.zeros(0, np.int64), np.zeros(0, np.int64)),
              64, 2, use_brand=False)
    brands = np.random.default_rng(1).integers(0, 50, I)
    make_case("c1_brand", u, it, U, I, 50, (np.arange(I), brands), 64, 2, use_brand=True)
    # Fusion path (lightgcn_fusion.py) on the C1 graph: content dim C=32
    make_case("c1_fusion", u, it, U, I, 50, (np.arange(I), brands), 64, 2, use_brand=True,
              fusion_c=32)

    # micro graph: duplicate edges, users with no train edge, isolated brand, odd d
    rng = np.random.default_rng(3)
    U, I, B = 30, 40, 5
    u = rng.integers(0, 25, 120)           # users 25..29 have no interactions
    it = rng.integers(0, I, 120)
    u = np.concatenate([u, [0, 0, 0, 1, 1]])  # forced duplicates
    it = np.concatenate([it, [3, 3, 3, 7, 7]])
    ib_items = np.arange(I)
    ib_brands = rng.integers(0, B - 1, I)  # brand B-1 stays isolated
    make_case("micro_d12", u, it, U, I, B, (ib_items, ib_brands), 12, 3, use_brand=True, eval_k=5)

    # hub graph: one item with ~2500 neighbours (exercises the chunked long-row path)
    rng = np.random.default_rng(4)
    U, I = 3000, 64
    u = np.concatenate([rng.permutation(U)[:2500], rng.integers(0, U, 3500)])
    it = np.concatenate([np.zeros(2500, np.int64), rng.integers(1, I, 3500)])
    make_case("hub_d32", u, it, U, I, 0, (np.zeros(0, np.int64), np.zeros(0, np.int64)), 32, 3,
              use_brand=False, eval_k=10)


if __name__ == "__main__":
    # `gen_golden.py debug` writes only the debug-diagnostics fixtures
    main_debug() if sys.argv[1:] == ["debug"] else main()
