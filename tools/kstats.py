"""Dev tool: per-call kernel times from a rocprofv3 --stats csv, divided by a
repetition count: python tools/kstats.py <run_kernel_stats.csv> [reps]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
reps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
tot = 0.0
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    per = float(r["TotalDurationNs"]) / reps / 1e3
    tot += per
    name = r["Name"].replace("(anonymous namespace)::", "").split("(")[0]
    name = name.replace("void ", "").replace("pnr::", "")[-48:]
    print(f"{name:50s} calls/rep {int(r['Calls']) / reps:6.1f}  us/rep {per:9.1f}  avg_us {float(r['AverageNs']) / 1e3:8.2f}")
print(f"{'sum':50s} {'':17s}  us/rep {tot:9.1f}")
