"""Shared-state peer process for the same-host hand-off fault test (tests/test_fault_tolerance.py).

usage: ss_peer.py MASTER ROLE [--n N] [--shareable] [--device cuda:0|cpu] [--world 3] [--no-all-reduce]
  ROLE dist: holds w = 7.0 (n fp32 on cuda:0) at revision 5; admits the joiner, syncs (may serve), then all-reduces
  ROLE join: connects with w = 0 at revision 0, syncs (receives w), then all-reduces
Prints one JSON line per phase. A distributor started with PCCL_FAULT_INJECT=ss_serve:5 SIGKILLs itself while
serving; the joiner must still end with exact data and a working communicator. A failed sync prints its error and
time ({"phase": "sync", "error": ..., "sec": ...}) instead of the data checks.
"""
import argparse
import contextlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

import pccl_amd as pccl  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("master")
    ap.add_argument("role", choices=["dist", "join"])
    ap.add_argument("--n", type=int, default=1 << 26)
    ap.add_argument("--shareable", action="store_true")
    ap.add_argument("--extra-tensors", type=int, default=0, help="add K small tensors of odd sizes (packed staging)")
    ap.add_argument("--device", default="cuda:0")
    ap.add_argument("--world", type=int, default=3, help="peers the distributor admits before it syncs")
    ap.add_argument("--no-all-reduce", action="store_true", help="end after the sync")
    a = ap.parse_args()
    dev = torch.device(a.device)
    with pccl.memory.maybe_shareable(dev) if a.shareable else contextlib.nullcontext():
        w = torch.full((a.n,), 7.0 if a.role == "dist" else 0.0, device=dev)
        extra = [torch.full((1 + (k * 997) % 50000,), float(k % 13) if a.role == "dist" else -1.0, device=dev)
                 for k in range(a.extra_tensors)]
    st = pccl.SharedState([pccl.TensorInfo.from_torch(w, "w")] +
                          [pccl.TensorInfo.from_torch(t, f"x{k}") for k, t in enumerate(extra)])
    st.revision = 5 if a.role == "dist" else 0
    comm = pccl.Communicator(a.master, 0)
    comm.connect(n_attempts=60)
    if a.role == "dist":
        deadline = time.time() + 120
        while comm.get_attribute(pccl.Attribute.GLOBAL_WORLD_SIZE) < a.world and time.time() < deadline:
            if comm.are_peers_pending():
                comm.update_topology()
            time.sleep(0.01)
    t0 = time.perf_counter()
    try:
        info = comm.sync_shared_state(st)
    except pccl.PCCLError as e:
        print(json.dumps({"role": a.role, "phase": "sync", "error": str(e)[:120], "sec": time.perf_counter() - t0,
                          "t": time.time()}), flush=True)
        comm.destroy()
        return
    if dev.type == "cuda":
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    extra_ok = all(bool((t == float(k % 13)).all()) for k, t in enumerate(extra))
    print(json.dumps({"role": a.role, "phase": "sync", "rx": info.rx_bytes, "tx": info.tx_bytes, "sec": dt,
                      "lo": float(w.min()), "hi": float(w.max()), "revision": st.revision, "extra_ok": extra_ok}),
          flush=True)
    if a.no_all_reduce:
        comm.destroy()
        return
    g = torch.ones(1 << 20, device=dev)
    out = torch.empty_like(g)
    for attempt in range(100):  # the ring loses the killed distributor: retry until the new world completes
        try:
            r = comm.all_reduce(g, out, op=pccl.ReduceOp.SUM, tag=attempt)
            break
        except pccl.PCCLError:
            time.sleep(0.05)
            if comm.are_peers_pending():
                comm.update_topology()
    else:
        sys.exit(4)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    print(json.dumps({"role": a.role, "phase": "all_reduce", "world": r.local_world_size,
                      "lo": float(out.min()), "hi": float(out.max())}), flush=True)
    comm.destroy()


if __name__ == "__main__":
    main()
