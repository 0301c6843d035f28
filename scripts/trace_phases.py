"""Median time of every PCCL_TRACE_OPS phase mark (us from op start) over the trace lines of a log, grouped by
(world, path); the first `skip` ops of each group are dropped (warmup).

usage: python scripts/trace_phases.py <stderr log> [skip=50]
"""
import json
import re
import statistics
import sys
from collections import defaultdict


def main(path, skip=50):
    groups = defaultdict(list)
    for ln in open(path, errors="replace"):
        if "[pccl-trace]" not in ln:
            continue
        m = re.search(r"world (\d+)(?: t0 -?\d+)? path (\S+) (ok|FAILED)(.*)", ln)
        if not m:
            continue
        marks = {k: int(v) for k, v in re.findall(r"(\w+) (\d+)us", m.group(4))}
        groups[(int(m.group(1)), m.group(2))].append(marks)
    for (world, p), ops in sorted(groups.items()):
        ops = ops[skip:] or ops
        keys = []
        for o in ops:
            for k in o:
                if k not in keys:
                    keys.append(k)
        med = {k: statistics.median([o[k] for o in ops if k in o]) for k in keys}
        print(json.dumps({"world": world, "path": p, "ops": len(ops), "median_mark_us": med}))


if __name__ == "__main__":
    main(sys.argv[1], *(int(x) for x in sys.argv[2:3]))
