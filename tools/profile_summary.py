"""Dev tool: fold a tools/prof_bench.sh run (gpurun_out/<dir>) into profiles/.

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --kernel-trace --stats),
profiles/<tag>_bench.json (the bench line) and profiles/<tag>_pmc_aggregate.json:
per aggregate launch (k_point_pre + k_pairs + k_color, one launch per frame)
the FETCH_SIZE / WRITE_SIZE bytes with the gfx950 correction of
MI355X_MICROARCH.md "HBM" (FETCH_SIZE counts 128-B reads at 64 B: x2),
MFMA busy fraction and effective clock.  bench.py reads hbm_bytes_per_launch.
"""
import csv
import collections
import json
import os
import shutil
import sys

AGG_BY_DTYPE = {"fp32": ("k_point_pre", "k_pairs", "k_color"),
                "fp32x3": ("k_point_pre", "k_pairs_x3", "k_color"),
                "fp32h2": ("k_point_pre_h2", "k_pairs_h2", "k_color_h2"),
                # (the last name runs once per aggregate launch: the per-launch divisor)
                "bf16": ("k_mark_used", "k_used_list", "k_point_pre_b", "k_bucket_hist", "k_bucket_scan",
                         "k_pairs_b", "k_bucket_scatter")}
MOPS = {"fp32": "SQ_INSTS_VALU_MFMA_MOPS_F32", "fp32x3": "SQ_INSTS_VALU_MFMA_MOPS_BF16",
        "fp32h2": "SQ_INSTS_VALU_MFMA_MOPS_F16",
        "bf16": "SQ_INSTS_VALU_MFMA_MOPS_BF16"}
AGG = AGG_BY_DTYPE["fp32"]


def short(name):
    n = name.replace("(anonymous namespace)::", "").split("(")[0].replace("pnr::", "").replace("void ", "")
    return n.split("<")[0]


def per_kernel(path, counters):
    """Counter values per aggregate launch: summed over a kernel's dispatches
    (the bf16 pairs stage is one dispatch per neighbour bucket), divided by the
    number of launches (dispatches of the list's last kernel, once per launch)."""
    sums = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        if k in AGG and r["Counter_Name"] in counters:
            sums[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
    launches = max(len(disp[AGG[-1]]), 1)
    return {k: {c: v / launches for c, v in d.items()} for k, d in sums.items()}


def main():
    global AGG
    src, tag = sys.argv[1], sys.argv[2]
    dtype = sys.argv[3] if len(sys.argv) > 3 else "fp32"
    AGG = AGG_BY_DTYPE[dtype]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prof = os.path.join(root, "profiles")
    os.makedirs(prof, exist_ok=True)
    shutil.copy(os.path.join(src, "stats", "run_kernel_stats.csv"), os.path.join(prof, f"{tag}_kernel_stats.csv"))
    bench = json.loads(open(os.path.join(src, "bench.json")).read().strip().splitlines()[-1])
    json.dump(bench, open(os.path.join(prof, f"{tag}_bench.json"), "w"), indent=1)
    # summed over a kernel's template instances (k_pairs_b<1/2/4/8>: one dispatch per bucket)
    stats = collections.defaultdict(lambda: {"Calls": 0, "TotalDurationNs": 0.0})
    for r in csv.DictReader(open(os.path.join(src, "stats", "run_kernel_stats.csv"))):
        st = stats[short(r["Name"])]
        st["Calls"] = max(st["Calls"], int(r["Calls"]))
        st["TotalDurationNs"] += float(r["TotalDurationNs"])
    fetch = per_kernel(os.path.join(src, "fetch", "run_counter_collection.csv"), {"FETCH_SIZE"})
    write = per_kernel(os.path.join(src, "write", "run_counter_collection.csv"), {"WRITE_SIZE"})
    mfma = per_kernel(os.path.join(src, "mfma", "run_counter_collection.csv"),
                      {"SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE", MOPS[dtype]})
    out = {"source": "tools/prof_bench.sh -> tools/profile_summary.py", "dtype": dtype, "kernels": {}}
    tot_bytes, tot_ns = 0.0, 0.0
    launches = max(int(stats[AGG[-1]]["Calls"]), 1) if AGG[-1] in stats else 1
    for k in AGG:
        if k not in stats:
            continue
        avg_ns = float(stats[k]["TotalDurationNs"]) / launches   # per aggregate launch
        fb = fetch.get(k, {}).get("FETCH_SIZE", 0.0) * 1024 * 2      # KB -> B, gfx950 x2 correction
        wb = write.get(k, {}).get("WRITE_SIZE", 0.0) * 1024
        m = mfma.get(k, {})
        gui = m.get("GRBM_GUI_ACTIVE", 0.0) / 8         # summed over 8 XCDs
        busy = m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / 1024   # per SIMD (256 CUs x 4)
        out["kernels"][k] = {"calls": int(stats[k]["Calls"]), "ms_per_launch": avg_ns / 1e6,
                             "fetch_bytes": fb, "write_bytes": wb,
                             "mfma_busy_frac": busy / gui if gui else None,
                             "eff_clock_ghz_profiled": gui / avg_ns if gui else None}
        tot_bytes += fb + wb
        tot_ns += avg_ns
    out["hbm_bytes_per_launch"] = tot_bytes
    out["avg_launch_ms_rocprof"] = tot_ns / 1e6
    out["avg_launch_ms_bench_events"] = bench["roofline"]["avg_launch_ms"]
    name = f"{tag}_pmc_aggregate.json" if dtype == "fp32" else f"{tag}_pmc_aggregate_{dtype.replace('fp32', '')}.json"
    json.dump(out, open(os.path.join(prof, name), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
