"""Dispatch timeline of a rocprofv3 kernel trace (csv): the dispatches split into bursts at idle
gaps (tools/fwd_trace.py leaves 50 ms between its runs), and per burst every kernel's start/end
(ms from the burst start), queue and duration — grouped by kernel name and queue, longest last.

    python tools/timeline.py <rocprofv3 -d dir> [--bursts -3] [--all]
"""
import argparse
import csv
import glob
import os
import re
from collections import defaultdict


def load(d):
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no *kernel_trace.csv under {d}")
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                             r.get("Queue_Id", "?"), r.get("Stream_Id", r.get("Queue_Id", "?"))))
    rows.sort()
    return rows


def bursts(rows, gap_ns=20_000_000):
    out, cur, last_end = [], [], 0
    for r in rows:
        if cur and r[0] - last_end > gap_ns:
            out.append(cur)
            cur = []
        cur.append(r)
        last_end = max(last_end, r[1]) if len(cur) > 1 else r[1]
    if cur:
        out.append(cur)
    return out


def short(name):
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"\(.*$", "", name.replace("(anonymous namespace)::", ""))
    return name if len(name) < 70 else name[:67] + "..."


def show(b, full):
    t0 = b[0][0]
    t1 = max(r[1] for r in b)
    print(f"burst: {len(b)} dispatches, {(t1 - t0) / 1e6:.3f} ms")
    if full:
        for s, e, nm, q, st in b:
            print(f"  q{q:>3} s{st:>3} {(s - t0) / 1e6:8.3f} -> {(e - t0) / 1e6:8.3f}  "
                  f"({(e - s) / 1e6:7.3f})  {short(nm)}")
        return
    grp = defaultdict(list)
    for s, e, nm, q, st in b:
        grp[(short(nm), st)].append((s, e))
    for (nm, st), v in sorted(grp.items(), key=lambda kv: max(e for _, e in kv[1])):
        first = min(s for s, _ in v)
        last = max(e for _, e in v)
        tot = sum(e - s for s, e in v)
        print(f"  s{st:>3} n={len(v):3d} first {(first - t0) / 1e6:8.3f} last end "
              f"{(last - t0) / 1e6:8.3f} busy {tot / 1e6:8.3f}  {nm}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--bursts", type=int, default=-3, help="show the last N bursts (negative)")
    ap.add_argument("--all", action="store_true", help="every dispatch, not grouped")
    ap.add_argument("--sum", action="store_true",
                    help="per kernel name: dispatches, summed duration, first start / last end")
    a = ap.parse_args()
    bs = bursts(load(a.dir))
    for b in bs[a.bursts:]:
        if a.sum:
            t0 = b[0][0]
            agg = defaultdict(lambda: [0, 0, None, 0])
            for st, en, name, _, _ in b:
                g = agg[name]
                g[0] += 1
                g[1] += en - st
                g[2] = st if g[2] is None else min(g[2], st)
                g[3] = max(g[3], en)
            span = (max(r[1] for r in b) - t0) / 1e6
            print(f"burst: {len(b)} dispatches, {span:.3f} ms, kernel time "
                  f"{sum(g[1] for g in agg.values()) / 1e6:.3f} ms")
            for name, (cnt, tot, f, l) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
                print(f"  n={cnt:4d} sum {tot / 1e6:8.3f}  [{(f - t0) / 1e6:7.3f} -> "
                      f"{(l - t0) / 1e6:7.3f}]  {name[:110]}")
        else:
            show(b, a.all)


if __name__ == "__main__":
    main()
