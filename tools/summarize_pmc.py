"""Per-kernel summary of tools/pmc_probe.sh output (its trace + PMC passes): for the exact layer's
kernels, VGPRs / LDS, launches, average duration, every counter's per-launch average and the
derived shares (VALU instructions per wave; of the waves' cycles: parked = waiting on anything,
issue-stall = waiting to issue, active = issuing). FETCH/WRITE in KB.

    python tools/summarize_pmc.py gpurun_out/pmc_blk > profiles/rNN_pmc_exact_layer.txt
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

KEEP = ("k_layer", "k_emu_blocks", "k_emu_walk", "k_chain_rows", "k_score_topk")


def short(name):
    name = re.sub(r"^void ", "", name).replace("(anonymous namespace)::", "")
    return re.sub(r"\(.*$", "", name)


def main(d):
    meta = {}
    for f in glob.glob(os.path.join(d, "pass*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if not k.startswith(KEEP):
                continue
            m = meta.setdefault(k, {"vgpr": r["VGPR_Count"], "agpr": r.get("Accum_VGPR_Count", "0"),
                                    "lds": r["LDS_Block_Size"], "c": defaultdict(list)})
            m["c"][r["Counter_Name"]].append(float(r["Counter_Value"]))
    dur = defaultdict(list)
    for f in glob.glob(os.path.join(d, "trace", "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if k in meta:
                dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    print(f"# rocprofv3 --pmc passes under {d}, per kernel average over its launches; FETCH/WRITE "
          f"in KB; HBM bytes = (2*FETCH + WRITE)*1024 (gfx950 correction)")
    for k, m in sorted(meta.items()):
        c = {n: sum(v) / len(v) for n, v in m["c"].items()}
        ds = dur.get(k, [])
        line = (f"{k} vgpr={m['vgpr']} agpr={m['agpr']} lds={m['lds']} launches={len(ds)} "
                f"avg_ms={sum(ds) / len(ds) if ds else float('nan'):.3f} " +
                " ".join(f"{n}={v:.3g}" for n, v in sorted(c.items())))
        if c.get("SQ_WAVES") and c.get("SQ_WAVE_CYCLES"):
            cyc = c["SQ_WAVE_CYCLES"]
            line += (f" | valu/wave={c.get('SQ_INSTS_VALU', 0) / c['SQ_WAVES']:.0f} "
                     f"parked%={100 * c.get('SQ_WAIT_ANY', 0) / cyc:.0f} "
                     f"issue-stall%={100 * c.get('SQ_WAIT_INST_ANY', 0) / cyc:.0f} "
                     f"active%={100 * c.get('SQ_ACTIVE_INST_ANY', 0) / cyc:.0f}")
        print(line)


if __name__ == "__main__":
    main(sys.argv[1])
