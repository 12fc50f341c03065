"""Timing probe of the fused evaluation kernel (lgcn_score_topk) at Books scale without building
the graph: random user / item tables (10.3M x d, 4.4M x d), 8192 users with 3 random train
items each, top-20. Prints one JSON line.

    python tools/eval_probe.py [--d 64] [--users 8192] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from gcn_recommendation_amd import evaluate as E  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--d", type=int, default=64)
    ap.add_argument("--users", type=int, default=8192)
    ap.add_argument("--items", type=int, default=4_400_000)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    U = 10_300_000
    ue = torch.randn(U, args.d, device=dev, generator=g) * 0.05
    ie = torch.randn(args.items, args.d, device=dev, generator=g) * 0.05
    rng = np.random.default_rng(0)
    users = np.sort(rng.choice(U, args.users, replace=False))
    mu = np.repeat(users, 3)
    mi = rng.integers(0, args.items, mu.size)
    mrow, mit = E.mask_csr(mu, mi, U)
    res = E.topk_fused(ue, ie, users, mrow, mit, 20)
    torch.cuda.synchronize()
    import hashlib
    h = hashlib.sha1()
    for t in (res if isinstance(res, (tuple, list)) else [res]):
        h.update(t.cpu().numpy().tobytes() if hasattr(t, "cpu") else np.asarray(t).tobytes())
    t0 = time.time()
    for _ in range(args.reps):
        E.topk_fused(ue, ie, users, mrow, mit, 20)
    torch.cuda.synchronize()
    ms = (time.time() - t0) / args.reps * 1e3
    flops = 2.0 * args.users * args.items * args.d
    print(json.dumps({"d": args.d, "users": args.users, "items": args.items, "ms": round(ms, 2),
                      "tflops": round(flops / (ms / 1e3) / 1e12, 1), "sha": h.hexdigest()[:16],
                      "lib": os.environ.get("LGCN_LIB", "product")}), flush=True)


if __name__ == "__main__":
    main()
