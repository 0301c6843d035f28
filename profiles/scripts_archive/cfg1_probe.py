"""Diagnostic: BASELINE config 1 latency (2 peers, 4 fp32 elements, host memory) the way bench.py measures it
(threaded peers of one process, bench.latency_cpu, full CPU mask); one JSON line."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

ba = argparse.Namespace(gpus=1, steps=1, warmup=0, peers=2, mib=1, pool=0, windows=1, quick=True, no_ipc_extra=True,
                        no_peer_curve=True, no_quant_extra=True, extras_child="")
job = bench.Job(ba)
print(json.dumps({"spin_us": os.environ.get("PCCL_MASTER_RX_SPIN_US", "default"), **bench.latency_cpu(job)}),
      flush=True)
