"""Elastic stress-test peer (reference python/tests/stress_tests/cross_step_async_reduces_test/stresstest_peer.py).

Loop: admit pending peers (after joining the background reduce of the previous step) -> sync shared state when the
topology changed -> launch this step's multi-tensor all-reduce in a background thread (it overlaps the next step's
"compute") -> join the previous step's reduce. Values are all ones, so every successful op must equal the world size
it ran with. Runs until <stop_file> exists, then leaves. Prints {"progress": n} after each successful step and one JSON
summary line at the end.
"""
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

import pccl_amd as pccl  # noqa: E402
from pccl_amd.parallel import all_reduce_multiple_with_retry  # noqa: E402


def main():
    import faulthandler
    import signal
    faulthandler.register(signal.SIGUSR1, all_threads=True)
    torch.set_num_threads(1)
    master, stop_file = sys.argv[1], sys.argv[2]
    n_tensors = int(sys.argv[3]) if len(sys.argv) > 3 else 6
    dev = torch.device(os.environ.get("STRESS_DEVICE", "cpu"))  # cuda:0 -> device tensors (xGMI/IPC path)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    comm = pccl.Communicator(master, 0, p2p_connection_pool_size=2)
    comm.connect(n_attempts=30)
    weights = torch.zeros(4096, device=dev)
    state = pccl.SharedState([pccl.TensorInfo.from_torch(weights, "weights")])
    grads = [torch.ones(64 * 64 * (k + 1) * (64 if dev.type == "cuda" else 1), device=dev) for k in range(n_tensors)]
    big_mib = int(os.environ.get("STRESS_BIG_MIB", "0"))  # one large tensor: kills land mid-pipeline
    if big_mib:
        grads.append(torch.ones(big_mib << 18, device=dev))
    bad, ok_ops, failed_ops, steps, syncs = 0, 0, 0, 0, 0
    reduce_thread = None
    result = {}

    def reduce_fn(tensors, tag_base):
        nonlocal bad, ok_ops, failed_ops
        res = all_reduce_multiple_with_retry(comm, tensors, pccl.ReduceOp.SUM, max_in_flight=4, tag_base=tag_base)
        if res.ok:
            ok_ops += 1
            print(json.dumps({"progress": ok_ops}), flush=True)  # the run's progress counts peers killed later too
            for t in tensors:
                if not torch.all(t == float(res.world_size)) and not torch.all(t == t[0]):
                    bad += 1
        else:
            failed_ops += 1

    it = 0
    while not os.path.exists(stop_file):
        topology_updated = it == 0
        if it > 0 and comm.are_peers_pending():
            if reduce_thread is not None:
                reduce_thread.join()
                reduce_thread = None
            try:
                comm.update_topology()
                topology_updated = True
            except pccl.PCCLError:
                result["kicked"] = True
                break
        it += 1
        if comm.get_attribute(pccl.Attribute.GLOBAL_WORLD_SIZE) < 2:
            if reduce_thread is not None:
                reduce_thread.join()
                reduce_thread = None
            time.sleep(0.05)
            continue
        if topology_updated:
            if reduce_thread is not None:
                reduce_thread.join()
                reduce_thread = None
            info = comm.sync_shared_state(state)
            state.revision += 1
            syncs += 1
            if syncs > 1 and info.rx_bytes and it > 2:
                pass  # a joiner may legitimately receive; drift on old peers is caught by equal final weights
        # the previous step's reduce overlaps this step's "compute" but must finish before we reuse its buffers
        for g in grads:
            g.fill_(1.0)
        if reduce_thread is not None:
            reduce_thread.join()
        snapshot = [g.clone() for g in grads]
        reduce_thread = threading.Thread(target=reduce_fn, args=(snapshot, 0))  # same tags on every peer
        reduce_thread.start()
        weights += 0.0
        steps += 1
        time.sleep(0.01)
    if reduce_thread is not None:
        reduce_thread.join()
    result.update({"steps": steps, "ok_ops": ok_ops, "failed_ops": failed_ops, "bad": bad, "syncs": syncs,
                   "revision": state.revision})
    print(json.dumps(result), flush=True)
    comm.destroy()


if __name__ == "__main__":
    main()
