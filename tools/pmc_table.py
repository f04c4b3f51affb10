"""Per-kernel mean of every PMC counter over the passes of tools/pmc_variants.sh.
Kernels launched several times per superstep (one merge launch per split band) are told apart by
their launch order inside the superstep: name#0, name#1, ...
Usage: python tools/pmc_table.py <outdir> [--per-step N] [kernel-substring ...]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    args = sys.argv[1:]
    root = args.pop(0)
    per_step = {}
    if args and args[0] == "--per-step":
        args.pop(0)
        for kv in args.pop(0).split(","):
            k, v = kv.split("=")
            per_step[k] = int(v)
    subs = args or ["pull"]
    res = {}
    for vdir in sorted(glob.glob(os.path.join(root, "*"))):
        if not os.path.isdir(vdir):
            continue
        vals = defaultdict(lambda: defaultdict(list))
        for f in glob.glob(os.path.join(vdir, "p*", "**", "*counter_collection.csv"), recursive=True):
            order = defaultdict(list)  # kernel -> dispatch ids in order
            rows = list(csv.DictReader(open(f)))
            for r in rows:
                k = r["Kernel_Name"]
                if any(s in k for s in subs):
                    short = k.split("(")[0].replace("void ", "").replace("jg::", "")[:60]
                    did = int(r["Dispatch_Id"])
                    if did not in order[short]:
                        order[short].append(did)
            for r in rows:
                k = r["Kernel_Name"]
                if not any(s in k for s in subs):
                    continue
                short = k.split("(")[0].replace("void ", "").replace("jg::", "")[:60]
                ids = sorted(order[short])
                nper = next((v for kk, v in per_step.items() if kk in short), 1)
                tag = f"{short}#{ids.index(int(r['Dispatch_Id'])) % nper}" if nper > 1 else short
                vals[tag][r["Counter_Name"]].append(float(r["Counter_Value"]))
                vals[tag]["_us"].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        res[os.path.basename(vdir)] = {k: {c: sum(x) / len(x) for c, x in d.items()} for k, d in vals.items()}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
