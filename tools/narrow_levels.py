"""Per-level kernel times of narrow bit-parallel BFS traversals (jg_narrow.hip) from a rocprofv3
kernel_trace.csv: each traversal starts at nb_init_kernel, and a level is its five launches (bu, rest,
scan, td, td_apply).  Prints one block per traversal.
    python tools/narrow_levels.py gpurun_out/<tag>/tr/nb_kernel_trace.csv [traversal ...]
"""
import csv
import re
import sys


def main():
    path = sys.argv[1]
    rows = [r for r in csv.DictReader(open(path)) if "::nb_" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))

    def name(r):
        return re.search(r"nb_(\w+?)_kernel", r["Kernel_Name"]).group(1)

    def us(r):
        return (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0

    starts = [i for i, r in enumerate(rows) if name(r) == "init"] + [len(rows)]
    picks = [int(x) for x in sys.argv[2:]] or list(range(len(starts) - 1))
    for t in picks:
        seq = rows[starts[t] + 1:starts[t + 1]]
        seq = [r for r in seq if name(r) != "planes"]
        span = (int(seq[-1]["End_Timestamp"]) - int(rows[starts[t]]["Start_Timestamp"])) / 1000.0
        print(f"traversal {t}: {span:.1f} us from init to the last launch, {sum(us(r) for r in seq):.1f} us of kernels")
        for L in range(len(seq) // 5):
            lv = seq[L * 5:(L + 1) * 5]
            print(f"  level {L}: " + " ".join(f"{name(r)} {us(r):.1f}" for r in lv))


if __name__ == "__main__":
    main()
