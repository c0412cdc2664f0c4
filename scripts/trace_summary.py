"""Per-(kernel, grid) duration summary of a rocprofv3 --kernel-trace CSV.

rocprofv3 --stats averages every launch of a kernel name together (the bench also
runs single-square Repair / roots launches of the same kernels); this splits them
by grid size so the batch launches the bench's HIP-event figures describe can be
compared one to one.
usage: python scripts/trace_summary.py gpurun_out/prof/run_kernel_trace.csv out.csv
"""
import collections
import csv
import sys


def main():
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(sys.argv[1])):
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        acc[(r["Kernel_Name"], grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    rows = sorted(acc.items(), key=lambda kv: -sum(kv[1]))
    with open(sys.argv[2], "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "grid_threads", "calls", "avg_us", "min_us", "max_us", "total_us"])
        for (name, grid), d in rows:
            w.writerow([name, grid, len(d), round(sum(d) / len(d), 2), round(min(d), 2), round(max(d), 2),
                        round(sum(d), 1)])
    for (name, grid), d in rows[:12]:
        print(f"{name[:70]:70s} {grid:>9d} {len(d):5d} {sum(d) / len(d):10.2f} us")


if __name__ == "__main__":
    main()
