"""Summarise rocprofv3 --pmc SQ_* passes into per-wave / per-launch figures.

usage: python scripts/sq_summary.py out.json gpurun_out/pmc_sq gpurun_out/pmc_sq2 ...
Averages every counter over the launches of each (kernel, grid) and derives
VALU instructions per wave; SQ_* cycle counters are summed over shader engines.
"""
import collections
import csv
import glob
import json
import sys


def main():
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in sys.argv[2:]:
        f = glob.glob(d + "/*counter_collection.csv")[0]
        for r in csv.DictReader(open(f)):
            if "rsm::" in r["Kernel_Name"]:
                acc[(r["Kernel_Name"], int(r["Grid_Size"]))][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = []
    for (name, grid), cs in sorted(acc.items()):
        c = {k: sum(v) / len(v) for k, v in cs.items()}
        waves = c.get("SQ_WAVES") or grid / 64
        row = {"kernel": name, "grid_threads": grid, "counters": c}
        if "SQ_INSTS_VALU" in c:
            row["valu_insts_per_wave"] = c["SQ_INSTS_VALU"] / waves
        if "SQ_INSTS_SALU" in c:
            row["salu_insts_per_wave"] = c["SQ_INSTS_SALU"] / waves
        out.append(row)
    json.dump({"method": "rocprofv3 --pmc SQ_* (separate passes, no tracing)", "launches": out},
              open(sys.argv[1], "w"), indent=1)
    for o in out:
        print(o["kernel"][:60], o["grid_threads"], {k: round(v) for k, v in o.items() if k.endswith("wave")})


if __name__ == "__main__":
    main()
