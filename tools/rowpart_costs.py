"""rowpart per-rank cost table: the C3 graph's row blocks under the old balance
(nnz + 4 rows) and the walk-cost balance (dist.balanced_row_bounds with the engine's chain cut:
walked rows at WALK_FACTOR x nnz), P = 2, 4, 8. Host only (no GPU).
    python tools/rowpart_costs.py [c3]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from gcn_recommendation_amd import dist  # noqa: E402


def chain_cut(nnz):  # lgcn_chain_max_default: nnz/256 clamped to [8192, 262144]
    return int(min(max(nnz // 256, 8192), 262144))


def main():
    cfg = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c3"]
    r, c, v, _, _, _ = bench.make_graph(cfg, "powerlaw", 16)
    n = cfg["users"] + cfg["items"] + cfg.get("brands", 0)
    deg = np.bincount(r, minlength=n)
    cut = chain_cut(len(v))
    print(f"N={n:,} nnz={len(v):,} chain cut {cut:,}: {int((deg > cut).sum())} walked rows, "
          f"largest {int(deg.max()):,} edges; walk factor {dist.WALK_FACTOR}")
    for P in (2, 4, 8):
        for name, b in (("nnz+4rows", dist.balanced_row_bounds(deg, P)),
                        ("walk-cost", dist.balanced_row_bounds(deg, P, walk_deg=cut))):
            print(f"P={P} {name}: n_max {int(np.diff(b).max()):,} rows")
            cost = dist.row_costs(deg, walk_deg=cut)
            for p in range(P):
                d = deg[b[p]:b[p + 1]]
                w = d > cut
                print(f"  rank {p}: rows {d.size:>10,} nnz {int(d.sum()):>11,} walked "
                      f"{int(w.sum()):>3} (max {int(d[w].max()) if w.any() else 0:>9,}) "
                      f"cost {cost[b[p]:b[p + 1]].sum() / 1e6:8.1f} M")


if __name__ == "__main__":
    main()
