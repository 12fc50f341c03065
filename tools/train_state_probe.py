"""Does the C3 training step (bench_train_step's loop) slow down after the GPU has been busy?
Back-to-back steps timed fresh, then after ~SECONDS of propagate_forward calls, then again after
an idle pause (a diagnostic for the gap between tools/train_trace_c3.py and bench.py).

    python tools/train_state_probe.py
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
from models.lightgcn import LightGCN  # noqa: E402


def main():
    cfg = bench.CONFIGS["c3"]
    dev = torch.device("cuda:0")
    r, c, v, _, _, _ = bench.make_graph(cfg, "powerlaw", 16)
    U, I, d, K = cfg["users"], cfg["items"], cfg["d"], cfg["K"]
    n = U + I
    adj = torch.sparse_coo_tensor(torch.from_numpy(np.vstack((r, c))), torch.from_numpy(v),
                                  (n, n)).to(dev)
    gen = torch.Generator().manual_seed(42)
    emb = [bench.xavier(U, d, gen), bench.xavier(I, d, gen)]
    model = LightGCN.__new__(LightGCN)
    torch.nn.Module.__init__(model)
    model.num_users, model.num_items, model.num_brands = U, I, 0
    model.embedding_dim, model.n_layers, model.debug = d, K, False
    model.user_embedding = torch.nn.Embedding.from_pretrained(emb[0].clone(), freeze=False)
    model.brand_embedding = torch.nn.Embedding(0, d)
    model.item_embedding = torch.nn.Embedding.from_pretrained(emb[1].clone(), freeze=False)
    model.final_brand_emb, model._graph_adj = None, None
    model = model.to(dev)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    rng = np.random.default_rng(0)
    batches = [tuple(torch.from_numpy(x).to(dev) for x in (rng.integers(0, U, 2048),
                                                            rng.integers(0, I, 2048),
                                                            rng.integers(0, I, 2048)))
               for _ in range(10)]

    def step(b):
        users, pos, neg = b
        opt.zero_grad()
        fu, fi, fb, u0, i0 = model(adj, use_brand=False)
        loss = bpr_loss_reg(fu[users], fi[pos], fi[neg], u0[users], i0[pos], i0[neg], 1e-4)
        loss.backward()
        opt.step()
        return loss

    def timed_steps(tag):
        torch.cuda.synchronize()
        a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        a.record()
        for b in batches:
            step(b)
        e.record()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        print(f"{tag}: {a.elapsed_time(e) / len(batches):.2f} ms/step GPU, host enqueue "
              f"{(t1 - t0) * 1e3 / len(batches):.2f} ms/step", flush=True)

    for b in batches[:4]:
        step(b)
    timed_steps("fresh")
    timed_steps("fresh again")
    g = engine.graph_from_coo(adj, (U, U + I))
    segs = [model.user_embedding.weight.detach(), model.item_embedding.weight.detach(),
            model.brand_embedding.weight.detach()]
    t_end = time.time() + float(os.environ.get("SECONDS_BUSY", "60"))
    nf = 0
    while time.time() < t_end:
        for _ in range(20):
            engine.propagate_forward(g, segs, K)
        torch.cuda.synchronize()
        nf += 20
    print(f"busy: {nf} forwards", flush=True)
    timed_steps("after busy")
    time.sleep(20)
    timed_steps("after 20 s idle")


if __name__ == "__main__":
    main()
