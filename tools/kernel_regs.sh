#!/bin/bash
# Dev tool: per-kernel register / spill / LDS metadata of one HIP source for
# gfx950 (device-only compile, code-object notes).  Usage:
#   tools/kernel_regs.sh pointnerf_amd/csrc/aggregate_x3.hip [extra hipcc flags] [| grep k_pairs_h2]
set -e
src=$1; shift
out=$(mktemp /tmp/kregs.XXXXXX.co)
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 --cuda-device-only --no-gpu-bundle-output -std=c++17 -munsafe-fp-atomics -Iinclude "$@" \
  -c "$src" -o "$out"
/opt/rocm/lib/llvm/bin/llvm-readelf --notes "$out" | python3 -c '
import sys, re
cur = {}
rows = []
# a kernel entry of amdhsa.kernels starts with "  - .<first key>" (keys in alphabetical
# order, so .agpr_count / .group_segment_fixed_size come BEFORE .name)
for line in sys.stdin:
    if re.match(r"\s+- \.", line):
        cur = {}
        rows.append(cur)
    m = re.match(r"\s+-?\s*\.(name|vgpr_count|agpr_count|vgpr_spill_count|sgpr_spill_count|private_segment_fixed_size|group_segment_fixed_size):\s+(\S+)", line)
    if not m:
        continue
    k, v = m.groups()
    if k == "name" and v.endswith(".kd"):
        continue
    cur[k] = v
rows = [r for r in rows if "name" in r]
for r in rows:
    print("%-60s vgpr %4s agpr %4s vspill %4s sspill %4s scratch %6s lds %6s" % (
        r["name"][:60], r.get("vgpr_count"), r.get("agpr_count"), r.get("vgpr_spill_count"),
        r.get("sgpr_spill_count"), r.get("private_segment_fixed_size"), r.get("group_segment_fixed_size")))
'
rm -f "$out"
