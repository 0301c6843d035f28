"""Copy-engine / kernel occupancy timeline of a rocprofv3 CSV trace (``--kernel-trace --memory-copy-trace
--output-format csv``): per time bin, the fraction of the bin covered by host->device copies, device->host copies and
kernels (union of intervals, so concurrent copies on several queues count once), plus the moved GB/s.

usage: python scripts/copy_timeline.py <rocprofv3 output dir> [bin_ms=20] [skip_ms=0]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def _rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f, newline="") as fh:
            out.extend(csv.DictReader(fh))
    return out


def _col(row, *cands):
    for c in cands:
        for k in row:
            if k.lower() == c.lower():
                return row[k]
    return None


def _union(iv):
    iv = sorted(iv)
    out = []
    for a, b in iv:
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def _cover(iv, lo, hi):
    return sum(max(0, min(b, hi) - max(a, lo)) for a, b in iv)


def main(d, bin_ms=20.0, skip_ms=0.0):
    copies = _rows(os.path.join(d, "**", "*memory_copy_trace.csv"))
    kernels = _rows(os.path.join(d, "**", "*kernel_trace.csv"))
    if not copies and not kernels:
        sys.exit(f"no traces under {d}")
    if copies:
        print("memory copy columns:", ", ".join(copies[0].keys()))
    series = defaultdict(list)
    nbytes = defaultdict(int)
    for r in copies:
        a, b = int(_col(r, "Start_Timestamp")), int(_col(r, "End_Timestamp"))
        direction = (_col(r, "Direction", "Operation", "Kind") or "").upper()
        key = "H2D" if "HOST_TO_DEVICE" in direction else "D2H" if "DEVICE_TO_HOST" in direction else "copy:" + direction
        series[key].append((a, b))
        nbytes[key] += int(_col(r, "Size", "Bytes") or 0)
    for r in kernels:
        a, b = int(_col(r, "Start_Timestamp")), int(_col(r, "End_Timestamp"))
        name = _col(r, "Kernel_Name") or "?"
        low = name.lower()
        key = ("blit" if "rocclr" in low else "k_reduce_copy" if "reduce_copy" in name else
               "k_dq" if "k_dq_" in name else "k_q" if "k_q_" in name else "k_minmax" if "minmax" in name else
               "kernel:other")
        series[key].append((a, b))
    t0 = min(a for v in series.values() for a, _ in v) + int(skip_ms * 1e6)
    t1 = max(b for v in series.values() for _, b in v)
    keys = sorted(series)
    unions = {k: _union(series[k]) for k in keys}
    print(f"\nspan {(t1 - t0) / 1e6:.1f} ms; busy ms per series: " +
          ", ".join(f"{k} {_cover(unions[k], t0, t1) / 1e6:.1f}" for k in keys))
    for k in ("H2D", "D2H"):
        if k in nbytes and unions.get(k):
            busy = _cover(unions[k], t0, t1) / 1e9
            if nbytes[k] == 0:  # this rocprofv3 version's copy trace has no size column
                print(f"{k}: {len(series[k])} copies, {busy * 1e3:.1f} ms busy (sizes not in the trace)")
                continue
            print(f"{k}: {nbytes[k] / 2**30:.2f} GiB, {len(series[k])} copies, {nbytes[k] / 1e9 / max(busy, 1e-9):.1f} GB/s "
                  f"while busy")
    step = int(bin_ms * 1e6)
    print(f"\n| t (ms) | " + " | ".join(keys) + " |")
    print("|---:|" + "---:|" * len(keys))
    t = t0
    while t < t1:
        print(f"| {(t - t0) / 1e6:.0f} | " + " | ".join(f"{100 * _cover(unions[k], t, t + step) / step:.0f}%" for k in keys)
              + " |")
        t += step


if __name__ == "__main__":
    if len(sys.argv) < 2:
        sys.exit(__doc__)
    main(sys.argv[1], *(float(x) for x in sys.argv[2:4]))
