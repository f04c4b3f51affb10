"""Per-kernel mean of every PMC counter over the passes of tools/pmc_variants.sh.
Usage: python tools/pmc_table.py <outdir> [kernel-substring ...]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    subs = sys.argv[2:] or ["pull"]
    res = {}
    for vdir in sorted(glob.glob(os.path.join(root, "*"))):
        if not os.path.isdir(vdir):
            continue
        vals = defaultdict(lambda: defaultdict(list))
        for f in glob.glob(os.path.join(vdir, "p*", "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"]
                if any(s in k for s in subs):
                    short = k.split("(")[0].replace("void ", "").replace("jg::", "")[:60]
                    vals[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
        res[os.path.basename(vdir)] = {k: {c: sum(x) / len(x) for c, x in d.items()} for k, d in vals.items()}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
