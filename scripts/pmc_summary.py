"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs (scripts/gpu_pmc.sh) into a per-kernel table:
HBM bytes read / written per dispatch (counters report KB) and the resulting bandwidth over the dispatch duration.

    python scripts/pmc_summary.py gpurun_out/pmc > profiles/r1_pmc.md
"""
import csv
import os
import re
import statistics
import sys
from collections import defaultdict


def short(name: str) -> str:
    m = re.match(r"void (pccl::hipk::k_\w+)(<[^()]*>)?", name)
    if m:
        args = (m.group(2) or "").replace("pccl::kernels::", "").replace("pccl::hipk::", "")
        return m.group(1).split("::")[-1] + args
    m = re.match(r"(?:void )?([\w:]+)", name)
    return (m.group(1) if m else name)[:60]


def load(path):
    per = defaultdict(list)  # kernel -> [(kb, ns)]
    with open(path) as f:
        for row in csv.DictReader(f):
            ns = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
            per[short(row["Kernel_Name"])].append((float(row["Counter_Value"]), ns))
    return per


def main(root):
    fetch = load(os.path.join(root, "FETCH_SIZE", "run_counter_collection.csv"))
    write = load(os.path.join(root, "WRITE_SIZE", "run_counter_collection.csv"))
    print("# HBM traffic per kernel dispatch (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, scripts/kernel_bench.py "
          "--mib 256)\n")
    print("FETCH_SIZE is derived from TCC->EA read requests assuming 64-byte requests; gfx950 streams 128-byte lines, so")
    print("it reports half of the bytes read (every streaming kernel below shows exactly 0.5x its logical read volume,")
    print("while WRITE_SIZE matches the logical writes). `read MB` is therefore 2 x FETCH_SIZE.\n")
    print("| kernel | dispatches | read MB | written MB | median us | read+write GB/s |")
    print("|---|---:|---:|---:|---:|---:|")
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k, []), write.get(k, [])
        if not f or not w:
            continue
        rd = 2 * statistics.median(x[0] for x in f) * 1024 / 1e6
        wr = statistics.median(x[0] for x in w) * 1024 / 1e6
        us = statistics.median([x[1] for x in f] + [x[1] for x in w]) / 1e3
        if us < 5:
            continue
        print(f"| `{k}` | {len(f)} | {rd:.1f} | {wr:.1f} | {us:.1f} | {(rd + wr) / us * 1e3:.0f} |")


if __name__ == "__main__":
    main(sys.argv[1])
