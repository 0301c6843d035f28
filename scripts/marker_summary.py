"""Summarise a rocprofv3 ``--kernel-trace --marker-trace --output-format csv`` run of pccl collectives.

usage: python scripts/marker_summary.py gpurun_out/prof_markers/bench > profiles/<name>.md

Every collective is a roctx range (``pccl all_reduce tag T bytes B``) on the thread that ran it, its protocol phases
are roctx markers on the same thread (``commence``, ``vote``, ``reduce_bcast`` ...), and its kernels are the
dispatches of that thread inside the range. Reported per op: range length, the time of each phase marker since the
range start, the summed kernel time, and the remainder (control path: master consensus, IPC barriers, launches).
"""
import csv
import statistics
import sys
from collections import defaultdict


def load(prefix):
    marks, ranges = defaultdict(list), defaultdict(list)
    with open(prefix + "_marker_api_trace.csv") as f:
        for r in csv.DictReader(f):
            tid, s, e, name = int(r["Thread_Id"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]
            (ranges if e > s or name.startswith("pccl ") else marks)[tid].append((s, e, name))
    kernels = defaultdict(list)
    with open(prefix + "_kernel_trace.csv") as f:
        for r in csv.DictReader(f):
            kernels[int(r["Thread_Id"])].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    return ranges, marks, kernels


def main(prefix):
    ranges, marks, kernels = load(prefix)
    rows, phase_t = [], defaultdict(list)
    for tid, rs in ranges.items():
        for s, e, name in rs:
            if not name.startswith("pccl all_reduce"):
                continue
            ks = [(ks_, ke) for ks_, ke, _ in kernels.get(tid, []) if s <= ks_ <= e]
            # kernels run asynchronously: count their GPU time, clipped to the range
            kt = sum(min(ke, e) - ks_ for ks_, ke in ks)
            for ms, _, mname in marks.get(tid, []):
                if s <= ms <= e:
                    phase_t[mname].append((ms - s) / 1e3)
            rows.append(((e - s) / 1e3, kt / 1e3, len(ks)))
    if not rows:
        print("no pccl all_reduce ranges found")
        return
    rows = rows[len(rows) // 5:]  # drop the warm-up share
    med = lambda xs: statistics.median(xs)
    print(f"# roctx view of `{prefix.split('/')[-1]}`: {len(rows)} all-reduce ranges (after warm-up)\n")
    print("| per op | median (us) | min (us) | max (us) |")
    print("|---|---:|---:|---:|")
    for label, idx in (("range (call to return)", 0), ("kernel time in range", 1)):
        xs = [r[idx] for r in rows]
        print(f"| {label} | {med(xs):.1f} | {min(xs):.1f} | {max(xs):.1f} |")
    ov = [r[0] - r[1] for r in rows]
    print(f"| control path (range - kernels) | {med(ov):.1f} | {min(ov):.1f} | {max(ov):.1f} |")
    print("\n| phase marker | median time since range start (us) |")
    print("|---|---:|")
    for name, ts in sorted(phase_t.items(), key=lambda kv: med(kv[1])):
        print(f"| `{name}` | {med(ts):.1f} |")


if __name__ == "__main__":
    main(sys.argv[1])
