"""Summarise a tools/profile.sh output directory into profiles/:
  profiles/<round>_<tag>_kernel_stats.csv   rocprofv3 --stats summary (kernel-trace pass)
  profiles/traffic_<tag>.json              HBM bytes per launch of every engine kernel from the
                                           separate FETCH_SIZE / WRITE_SIZE PMC passes

gfx950 correction (MI355X_MICROARCH.md, HBM): FETCH_SIZE counts half the bytes of 16-B/lane
coalesced reads, so hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.

    python tools/summarize_profile.py gpurun_out/prof_c3 c3_powerlaw r01 18686716948
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    return name.split("(int")[0].split("(lgcn")[0].split("(long")[0].strip()


def main(prof, tag, rnd, algo_bytes):
    stats = list(csv.DictReader(open(os.path.join(prof, "trace", "run_kernel_stats.csv"))))
    dst = os.path.join(ROOT, "profiles", f"{rnd}_{tag}_kernel_stats.csv")
    shutil.copy(os.path.join(prof, "trace", "run_kernel_stats.csv"), dst)
    dur = {short(r["Name"]): float(r["AverageNs"]) / 1e6 for r in stats}
    calls = {short(r["Name"]): int(r["Calls"]) for r in stats}
    raw = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        path = os.path.join(prof, f"pmc_{c}", "run_counter_collection.csv")
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(path)):
            agg[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
        for k, v in agg.items():
            raw.setdefault(k, {})[c + "_KB_avg"] = sum(v) / len(v)
    kernels = {}
    for k, v in raw.items():
        if "FETCH_SIZE_KB_avg" in v and "WRITE_SIZE_KB_avg" in v and "anonymous" in k:
            kernels[k] = {"avg_ms": dur.get(k), "calls": calls.get(k),
                          "hbm_bytes_per_launch": int((2 * v["FETCH_SIZE_KB_avg"]
                                                       + v["WRITE_SIZE_KB_avg"]) * 1024),
                          **v}
    def layer_mode(k):  # k_layer<V, G, NV, MODE, RPG, U, NP, XD>
        args = k.split("k_layer<", 1)[1].split(">, ", 1)[1].rstrip(">").split(", ")
        return int(args[2])
    store = [k for k in kernels if "k_layer" in k and layer_mode(k) == 0]
    store = store or [k for k in kernels if "k_layer" in k]
    dom = max(store, key=lambda k: (kernels[k]["avg_ms"] or 0) * (kernels[k]["calls"] or 0))
    sys.path.insert(0, ROOT)
    from bench import kernel_source_hash  # bench.py refuses a traffic file with another stamp
    out = {"command": f"tools/profile.sh {tag} ... (see profiles/README.md)",
           "source_hash": kernel_source_hash(),
           "correction": "hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE "
                         "halves 16-B/lane coalesced reads)",
           "kernel": dom, "avg_duration_ms_rocprof": kernels[dom]["avg_ms"],
           "hbm_bytes_per_launch": kernels[dom]["hbm_bytes_per_launch"],
           "algorithmic_bytes_per_launch": int(algo_bytes), "kernels": kernels}
    json.dump(out, open(os.path.join(ROOT, "profiles", f"traffic_{tag}.json"), "w"), indent=1)
    print(json.dumps({k: out[k] for k in ("kernel", "avg_duration_ms_rocprof",
                                          "hbm_bytes_per_launch")}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4])
