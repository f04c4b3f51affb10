"""Per-kernel median durations of the PageRank superstep per pr_ab variant, from a rocprofv3 kernel
trace of `tools/pr_ab.py --rounds 1 <variants>` (dispatches are split evenly over the variants in
order).  Usage: python tools/trace_variants.py <kernel_trace.csv> name1 name2 ..."""
import collections
import csv
import sys


def main():
    path, names = sys.argv[1], sys.argv[2:]
    r = list(csv.DictReader(open(path)))
    r.sort(key=lambda x: int(x["Start_Timestamp"]))
    sel = [x for x in r if "PrOp" in x["Kernel_Name"] and any(
        k in x["Kernel_Name"] for k in ("pull_merge_kernel", "light_finalize", "fixup"))]
    per = len(sel) // len(names)
    for i, nm in enumerate(names):
        d = collections.defaultdict(list)
        k = 0
        for x in sel[i * per:(i + 1) * per]:
            n = x["Kernel_Name"]
            dur = (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1000
            if "pull_merge_kernel" in n:
                d["merge%d" % (k % 2)].append(dur)
                k += 1
            elif "fixup" in n:
                d["fixup"].append(dur)
            else:
                d["lightfin"].append(dur)
        med = {a: round(sorted(b)[len(b) // 2], 1) for a, b in d.items()}
        print(f"{nm:10s}", med, "sum", round(sum(med.values()), 1))


if __name__ == "__main__":
    main()
