#!/usr/bin/env python3
"""CPU mask A/B for the bench's one-process-per-peer TCP runs (bench.baseline_configs): full / spread / numa,
interleaved over passes; one JSON line per run on stdout."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--passes", type=int, default=2)
p.add_argument("--modes", default="full,spread,numa")
p.add_argument("--configs", default="config5_kill_rejoin_tcp,collocated_5ms_4peers,config3_wan_50ms")
a = p.parse_args()
spread = bench._cpu_spread()
os.environ["PCCL_BENCH_CONFIGS"] = a.configs
for k in range(a.passes):
    for mode in a.modes.split(","):
        os.environ["PCCL_BENCH_CONFIG_MASK"] = mode
        r = bench.baseline_configs(argparse.Namespace(mib=1024), 8)
        print(json.dumps({"pass": k + 1, "mask": mode, "spread": spread, "results": r}), flush=True)
