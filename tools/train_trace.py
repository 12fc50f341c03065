"""One C3 training step (bench.py's bench_train_step: forward + BPR loss + backward + Adam),
run after warm-up between 50-ms idle gaps, for a rocprofv3 kernel trace (tools/timeline.py
splits it at the gaps), and the step's own event timing.

    rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python3 tools/train_trace.py
    python tools/timeline.py OUT
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from gcn_recommendation_amd import engine  # noqa: E402
from gcn_recommendation_amd.loss import bpr_loss_reg  # noqa: E402


def main():
    cfg = bench.CONFIGS[os.environ.get("CFG", "c3")]
    dev = torch.device("cuda:0")
    engine.load_library()
    r, c, v, _, _, _ = bench.make_graph(cfg, "powerlaw", 16)
    U, I = cfg["users"], cfg["items"]
    n, d, K = U + I, cfg["d"], cfg["K"]
    adj = torch.sparse_coo_tensor(torch.from_numpy(np.vstack((r, c))), torch.from_numpy(v),
                                  (n, n)).to(dev)
    gen = torch.Generator().manual_seed(42)
    emb = [bench.xavier(U, d, gen), bench.xavier(I, d, gen)]
    from models.lightgcn import LightGCN
    model = LightGCN.__new__(LightGCN)
    torch.nn.Module.__init__(model)
    model.num_users, model.num_items, model.num_brands = U, I, 0
    model.embedding_dim, model.n_layers, model.debug = d, K, False
    model.user_embedding = torch.nn.Embedding.from_pretrained(emb[0].clone(), freeze=False)
    model.brand_embedding = torch.nn.Embedding(0, d)
    model.item_embedding = torch.nn.Embedding.from_pretrained(emb[1].clone(), freeze=False)
    model.final_brand_emb, model._graph_adj = None, None
    model = model.to(dev)
    fused = os.environ.get("ADAM_FUSED", "")
    opt = torch.optim.Adam(model.parameters(), lr=1e-3,
                           **({"fused": True} if fused == "1" else {}))
    rng = np.random.default_rng(0)

    def step():
        users, pos, neg = (torch.from_numpy(x).to(dev) for x in (
            rng.integers(0, U, 2048), rng.integers(0, I, 2048), rng.integers(0, I, 2048)))
        opt.zero_grad()
        fu, fi, _, u0, i0 = model(adj, use_brand=False)
        loss = bpr_loss_reg(fu[users], fi[pos], fi[neg], u0[users], i0[pos], i0[neg], 1e-4)
        loss.backward()
        opt.step()
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    ts = []
    for _ in range(int(os.environ.get("REPS", "3"))):
        time.sleep(0.05)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        step()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    print("train step ms:", " ".join(f"{t:.2f}" for t in ts), flush=True)


if __name__ == "__main__":
    main()
