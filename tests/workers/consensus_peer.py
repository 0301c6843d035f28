"""Peer process for the idle-peer liveness test (tests/test_liveness.py::test_sigstopped_idle_peer_consensus).

usage: consensus_peer.py MASTER WORLD RANK [--duration S] [--step-sleep S]

Waits until WORLD peers are admitted, then loops until --duration passed: admit pending peers, a shared-state sync of
a small CPU state (revision + 1 each round: every accepted peer must vote), an all-reduce, then --step-sleep seconds
idle. One JSON line per round: {"t", "world", "sync", "ar"} with "error" instead when a call failed. A peer that
finds itself dropped by the master (MASTER_CONNECTED == 0) prints {"kicked": true} and exits 0.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import numpy as np  # noqa: E402

import pccl_amd as pccl  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("master")
    ap.add_argument("world", type=int)
    ap.add_argument("rank", type=int)
    ap.add_argument("--duration", type=float, default=12.0)
    ap.add_argument("--step-sleep", type=float, default=0.3)
    a = ap.parse_args()
    comm = pccl.Communicator(a.master, 0)
    comm.connect(n_attempts=60)
    deadline = time.time() + 60
    while comm.get_attribute(pccl.Attribute.GLOBAL_WORLD_SIZE) < a.world and time.time() < deadline:
        if comm.are_peers_pending():
            comm.update_topology()
        time.sleep(0.01)
    w = np.full(1024, 1.0, dtype=np.float32)
    st = pccl.SharedState([pccl.TensorInfo.from_numpy(w, "w")])
    x = np.full(4096, float(a.rank + 1), dtype=np.float32)
    y = np.empty_like(x)
    t_end = time.time() + a.duration
    tag = 0
    while time.time() < t_end:
        row = {"t": time.time()}
        try:
            if comm.are_peers_pending():
                comm.update_topology()
            st.revision += 1
            comm.sync_shared_state(st)
            row["sync"] = True
            tag += 1
            info = comm.all_reduce(x, y, op=pccl.ReduceOp.SUM, tag=tag)
            row["world"] = info.local_world_size
            row["ar"] = bool(np.all(y == y[0]))
        except pccl.PCCLError as e:
            row["error"] = str(e)[:120]
            if comm.get_attribute(pccl.Attribute.MASTER_CONNECTED) == 0:
                print(json.dumps({"t": time.time(), "kicked": True}), flush=True)
                return
            st.revision = max(0, st.revision - 1)
        print(json.dumps(row), flush=True)
        time.sleep(a.step_sleep)
    comm.destroy()


if __name__ == "__main__":
    main()
