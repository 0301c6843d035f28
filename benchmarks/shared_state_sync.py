"""BASELINE config 4: shared-state sync of a 1B-parameter fp32 state; a late-joining peer catches up from revision 0.

    python benchmarks/shared_state_sync.py [--params 1e9] [--tensors 8] [--device cuda:0|cpu] [--transport ipc|tcp]

Two peer processes and an in-process master on 127.0.0.1:
  * the *trainer* holds the state (random init, seeded) and advances it for a few revisions on its own
    (pcclSynchronizeSharedState with one peer), then admits the joiner at a topology update;
  * the *joiner* starts with zeros at revision 0 and calls pcclSynchronizeSharedState once: the master elects the
    trainer's content, the joiner pulls every tensor and re-hashes it.
Reported: the joiner's wall time for that call (hash + master election + transfer + verification) and the payload
throughput. ``--transport ipc`` (default on GPUs) hands HBM tensors over with HIP IPC (device-to-device copy);
``tcp`` streams them through pinned staging buffers over loopback TCP (the reference's only transport). The IPC
hand-off is fault-safe: the trainer's tensors are staged into VMM segments shared as fds unless ``--shareable`` puts
them in fd-shareable memory from the start (zero-copy).
The reference publishes no number for this configuration; its transfer path is the TCP stream.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _state(torch, pccl, n_params, n_tensors, device, fill, shareable=False):
    import contextlib
    per = n_params // n_tensors
    tensors = []
    for i in range(n_tensors):
        numel = per if i < n_tensors - 1 else n_params - per * (n_tensors - 1)
        with pccl.memory.maybe_shareable(device) if shareable else contextlib.nullcontext():
            t = torch.empty(numel, dtype=torch.float32, device=device)
        if fill == "random":
            g = torch.Generator(device=device).manual_seed(1234 + i)
            t.normal_(generator=g)
        else:
            t.zero_()
        tensors.append(t)
    st = pccl.SharedState([pccl.TensorInfo.from_torch(t, f"param{i}") for i, t in enumerate(tensors)])
    return tensors, st


def _hashes(tensors):
    """simplehash of every tensor (the library's content hash: HIP kernel for HBM tensors, host twin otherwise),
    computed by the benchmark after the sync, independently of the library's own per-entry verification."""
    from pccl_amd.ops import kernels as K
    return [int(K.simplehash(t)) for t in tensors]


def peer(a):
    import torch

    import pccl_amd as pccl
    dev = torch.device(a.device)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    comm = pccl.Communicator(a.master, 0)
    comm.connect(n_attempts=60)
    if a.role == "trainer":
        tensors, st = _state(torch, pccl, a.params, a.tensors, dev, "random", a.shareable)
        for rev in range(3):  # train alone for a few revisions
            st.revision = rev
            comm.sync_shared_state(st)
            for t in tensors:
                t.add_(1.0)
        print(json.dumps({"ready": True}), flush=True)
        deadline = time.time() + 300
        while comm.get_attribute(pccl.Attribute.GLOBAL_WORLD_SIZE) < 2:
            if comm.are_peers_pending():
                comm.update_topology()
            else:
                time.sleep(0.01)
            if time.time() > deadline:
                raise TimeoutError("joiner never arrived")
        st.revision = 3
        info = comm.sync_shared_state(st)
        sums = [float(t.double().sum()) for t in tensors]
        print(json.dumps({"role": "trainer", "tx_bytes": info.tx_bytes, "sums": sums, "hashes": _hashes(tensors)}),
              flush=True)
    else:
        tensors, st = _state(torch, pccl, a.params, a.tensors, dev, "zeros")
        st.revision = 0
        if dev.type == "cuda":
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        info = comm.sync_shared_state(st)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        sums = [float(t.double().sum()) for t in tensors]  # compared with the trainer's by the driver
        nbytes = sum(t.numel() * 4 for t in tensors)
        print(json.dumps({"role": "joiner", "seconds": dt, "rx_bytes": info.rx_bytes, "bytes": nbytes,
                          "revision": st.revision, "sums": sums, "hashes": _hashes(tensors)}), flush=True)
    comm.destroy()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", type=float, default=1e9)
    ap.add_argument("--tensors", type=int, default=8)
    ap.add_argument("--device", default="cuda:0")
    ap.add_argument("--transport", default="ipc", choices=["ipc", "tcp"])
    ap.add_argument("--role", default=None, choices=["trainer", "joiner"])
    ap.add_argument("--shareable", action="store_true", help="the trainer's state lives in fd-shareable memory "
                    "(pccl_amd.memory): the fault-safe IPC hand-off is zero-copy instead of staged")
    ap.add_argument("--master", default=None)
    a = ap.parse_args()
    a.params = int(a.params)
    if a.role:
        return peer(a)

    from pccl_amd.utils import local_master, spawn_python
    env = {"PCCL_SS_NO_IPC": "1"} if a.transport == "tcp" else {}
    common = ["--params", str(a.params), "--tensors", str(a.tensors), "--device", a.device] + \
        (["--shareable"] if a.shareable else [])
    with local_master() as addr:
        me = os.path.abspath(__file__)
        trainer = spawn_python([me, "--role", "trainer", "--master", addr, *common], env=env,
                               stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
        line = trainer.stdout.readline()  # {"ready": true} once the trainer advanced its state
        if not line:
            raise RuntimeError("trainer failed: " + trainer.stderr.read()[-3000:])
        joiner = spawn_python([me, "--role", "joiner", "--master", addr, *common], env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
        jo, je = joiner.communicate(timeout=900)
        to, te = trainer.communicate(timeout=120)
    if joiner.returncode != 0 or trainer.returncode != 0:
        raise RuntimeError(f"peer failed:\n{je[-3000:]}\n{te[-3000:]}")
    j = json.loads([x for x in jo.splitlines() if x.startswith("{")][-1])
    t = json.loads([x for x in to.splitlines() if x.startswith("{")][-1])
    print(json.dumps({
        "metric": "shared-state late-joiner catch-up", "config": "Shared-state sync: 1B-param fp32 state, "
        "late-joining peer catches up from rev 0", "params": a.params, "tensors": a.tensors, "device": a.device,
        "transport": a.transport, "shareable_state": a.shareable, "seconds": round(j["seconds"], 4), "bytes": j["bytes"],
        "GBps": round(j["bytes"] / j["seconds"] / 1e9, 3), "joiner_rx_bytes": j["rx_bytes"],
        "trainer_tx_bytes": t["tx_bytes"], "adopted_revision": j["revision"], "content_ok": j["sums"] == t["sums"],
        # the library re-hashes every received entry against the elected hash (a mismatch fails the sync); this is the
        # benchmark's own check of the same property
        "hash_verified": j["hashes"] == t["hashes"]}),
        flush=True)


if __name__ == "__main__":
    main()
