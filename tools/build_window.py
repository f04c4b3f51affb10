"""Where one snapshot build goes, from a rocprofv3 kernel + memory-copy + HIP runtime trace of
tools/build_trace.py (diagnostic).  A build is the span between its BuildTimer's two hipEventRecord
calls; the last build of the trace is reported (the first pays code-object loading).

    python tools/build_window.py <dir> <prefix>"""
import collections
import csv
import sys


def main():
    d, pre = sys.argv[1], sys.argv[2]
    K = list(csv.DictReader(open(f"{d}/{pre}_kernel_trace.csv")))
    C = list(csv.DictReader(open(f"{d}/{pre}_memory_copy_trace.csv")))
    A = list(csv.DictReader(open(f"{d}/{pre}_hip_api_trace.csv")))
    rec = sorted(int(r["Start_Timestamp"]) for r in A if r["Function"] == "hipEventRecord")
    t0, t1 = rec[-2], rec[-1]
    print(f"build window {(t1 - t0) / 1e6:.2f} ms")
    gpu = collections.defaultdict(lambda: [0, 0])
    for r in K:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if t0 <= s and e <= t1 + 10**7:
            gpu["K " + r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:70]][0] += e - s
            gpu["K " + r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:70]][1] += 1
    for r in C:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if t0 <= s and e <= t1 + 10**7:
            gpu["C " + r["Direction"]][0] += e - s
            gpu["C " + r["Direction"]][1] += 1
    print(f"GPU busy {sum(v[0] for v in gpu.values()) / 1e6:.2f} ms")
    for k, v in sorted(gpu.items(), key=lambda x: -x[1][0])[:20]:
        print(f"  {v[0] / 1e6:8.3f} ms {v[1]:5d}  {k}")
    api = collections.defaultdict(lambda: [0, 0])
    for r in A:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if t0 <= s and e <= t1:
            api[r["Function"]][0] += e - s
            api[r["Function"]][1] += 1
    print("HIP API (host)")
    for k, v in sorted(api.items(), key=lambda x: -x[1][0])[:10]:
        print(f"  {v[0] / 1e6:8.3f} ms {v[1]:5d}  {k}")


if __name__ == "__main__":
    main()
