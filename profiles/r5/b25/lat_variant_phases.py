"""Median PCCL_TRACE_OPS marks per call variant of a py_latency.py --trace-dir run (variants interleaved op by op, so
tag % len(variants) names the variant); the first `skip` ops per variant are dropped.

usage: python profiles/r5/b25/lat_variant_phases.py <peer stderr log> all_reduce,async,ready [skip=20]
"""
import json
import re
import statistics
import sys
from collections import defaultdict


def main(path, variants, skip=20):
    names = variants.split(",")
    groups = defaultdict(list)
    for ln in open(path, errors="replace"):
        m = re.search(r"\[pccl-trace\] tag (\d+) .* path (\S+) (ok|FAILED)(.*)", ln)
        if not m:
            continue
        marks = {k: int(v) for k, v in re.findall(r"(\w+) (\d+)us", m.group(4))}
        groups[names[int(m.group(1)) % len(names)]].append(marks)
    for v in names:
        ops = groups[v][skip:] or groups[v]
        keys = []
        for o in ops:
            keys += [k for k in o if k not in keys]
        print(json.dumps({"variant": v, "ops": len(ops),
                          "median_mark_us": {k: statistics.median([o[k] for o in ops if k in o]) for k in keys}}))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], *(int(x) for x in sys.argv[3:4]))
