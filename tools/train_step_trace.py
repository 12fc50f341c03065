"""Host read-backs of main.py's training step on the engine: N steps of
forward (drop-in LightGCN, exact plan) + batch gathers + bpr_loss_reg + backward + Adam on the
C2 power-law graph, nothing read back by the script itself. Run under
`rocprofv3 --kernel-trace --memory-copy-trace --stats` with two step counts: the device-to-host
copy count must not grow with N (tools/train_step_trace.sh).

    python tools/train_step_trace.py --steps N
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from gcn_recommendation_amd.loss import bpr_loss_reg  # noqa: E402
from models.lightgcn import LightGCN  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    cfg = bench.CONFIGS["c2"]
    dev = torch.device("cuda", 0)
    r, c, v, _, _, _ = bench.make_graph(cfg, "powerlaw", 16)
    U, I, d, K = cfg["users"], cfg["items"], cfg["d"], cfg["K"]
    n = U + I
    adj = torch.sparse_coo_tensor(torch.from_numpy(np.vstack((r, c))), torch.from_numpy(v),
                                  (n, n)).to(dev)

    class Cfg:
        embedding_dim, n_layers, debug = d, K, False
    torch.manual_seed(42)
    model = LightGCN(U, I, 0, Cfg()).to(dev)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    rng = np.random.default_rng(0)
    batches = [tuple(torch.from_numpy(x).to(dev) for x in (
        rng.integers(0, U, 2048), rng.integers(0, I, 2048), rng.integers(0, I, 2048)))
        for _ in range(a.steps + 3)]
    torch.cuda.synchronize()

    def step(b):
        users, pos, neg = b
        opt.zero_grad()
        fu, fi, _, u0, i0 = model(adj, use_brand=False)
        loss = bpr_loss_reg(fu[users], fi[pos], fi[neg], u0[users], i0[pos], i0[neg], 1e-4)
        loss.backward()
        opt.step()
        return loss
    for b in batches[:3]:  # plan build, scratch, allocator pools
        step(b)
    torch.cuda.synchronize()
    losses = [step(b) for b in batches[3:]]
    torch.cuda.synchronize()
    print(f"steps {a.steps} last loss {float(losses[-1]):.6f}", flush=True)


if __name__ == "__main__":
    main()
