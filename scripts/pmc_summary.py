"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-launch HBM bytes.

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half the bytes of
a wide coalesced streaming read, so read bytes = 2 x FETCH_SIZE(KB) x 1024;
WRITE_SIZE(KB) x 1024 is exact for streaming stores.  Our encode kernels read
256 contiguous bytes per wave instruction (dword per lane); the corrected figure
matches the known compulsory bytes of each pass within ~2%.

usage: python scripts/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write out.json
"""
import collections
import csv
import glob
import json
import sys


def load(d, counter):
    """(kernel, grid) -> [value per dispatch, in dispatch order]"""
    f = glob.glob(d + "/*counter_collection.csv")[0]
    per = collections.defaultdict(float)
    key = {}
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == counter and "rsm::" in r["Kernel_Name"]:
            i = int(r["Dispatch_Id"])
            per[i] += float(r["Counter_Value"])
            key[i] = (r["Kernel_Name"], int(r["Grid_Size"]))
    acc = collections.defaultdict(list)
    for i in sorted(per):
        acc[key[i]].append(per[i])
    return acc


def main():
    fetch, write = load(sys.argv[1], "FETCH_SIZE"), load(sys.argv[2], "WRITE_SIZE")
    out = []
    # the two passes run the same program: pair the n-th dispatch of a (kernel, grid)
    # in one with the n-th in the other, then group dispatches of equal write volume
    # (persistent kernels launch every batch size on the same grid)
    for key in sorted(set(fetch) | set(write)):
        f, w = fetch.get(key, []), write.get(key, [])
        groups = collections.defaultdict(list)
        for n in range(max(len(f), len(w))):
            wr = (w[n] if n < len(w) else 0.0) * 1024
            rd = 2 * (f[n] if n < len(f) else 0.0) * 1024
            groups[round(wr / 2**20)].append((rd, wr))
        for _, g in sorted(groups.items()):
            rd = sum(x[0] for x in g) / len(g)
            wr = sum(x[1] for x in g) / len(g)
            out.append({"kernel": key[0], "grid_threads": key[1], "dispatches": len(g), "read_bytes": rd,
                        "write_bytes": wr, "traffic_bytes": rd + wr})
    json.dump({"method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE separate passes; read = 2*FETCH_SIZE*1024, "
                         "write = WRITE_SIZE*1024 (profiles/r03_calib16.json); dispatches paired in order and "
                         "grouped by write volume",
               "launches": out}, open(sys.argv[3], "w"), indent=1)
    for o in out:
        print(o)


if __name__ == "__main__":
    main()
