"""Dev tool: fold rocprofv3 --pmc passes (gpurun_out/<dir>/p*/run_counter_collection.csv)
into per-kernel averages per dispatch: python tools/pmc_fold.py <dir> [kernel substring ...]."""
import collections
import csv
import glob
import json
import sys


def short(name):
    n = name.replace("(anonymous namespace)::", "").split("(")[0].replace("pnr::", "").replace("void ", "")
    return n.strip()


def fold(src, want=()):
    sums = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(lambda: collections.defaultdict(set))
    for f in sorted(glob.glob(f"{src}/p*/**/run_counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if want and not any(w in k for w in want):
                continue
            c = r["Counter_Name"]
            sums[k][c] += float(r["Counter_Value"])
            disp[k][c].add(r["Dispatch_Id"])
    return {k: {c: v / len(disp[k][c]) for c, v in d.items()} for k, d in sums.items()}


if __name__ == "__main__":
    print(json.dumps(fold(sys.argv[1], sys.argv[2:]), indent=1))
