"""MNIST with DiLoCo over PCCL (reference python/tests/end_to_end/mnist_diloco/mnist_diloco_peer.py).

Inner: ``--inner-steps`` Adam steps on local data. Outer: AVG all-reduce of the pseudo-gradients (fused HIP kernels
on GPU tensors) + SGD outer step. Shared state = outer params + outer step counter; late joiners catch up.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import pccl_amd as pccl  # noqa: E402
from pccl_amd.models.data import batches, load_mnist  # noqa: E402
from pccl_amd.models.mlp import MLP  # noqa: E402
from pccl_amd.ops import kernels as K  # noqa: E402
from pccl_amd.parallel import maybe_update_topology  # noqa: E402
from pccl_amd.parallel.diloco import DiLoCo  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--master", default=os.environ.get("PCCL_MASTER", "127.0.0.1:48148"))
    ap.add_argument("--rank", type=int, default=int(os.environ.get("RANK", "0")))
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--outer-steps", type=int, default=10)
    ap.add_argument("--inner-steps", type=int, default=8)
    ap.add_argument("--min-world", type=int, default=0)
    ap.add_argument("--start-world", type=int, default=int(os.environ.get("PCCL_START_WORLD", "2")),
                    help="train only once this many peers have formed the run (elastic afterwards)")
    a = ap.parse_args()
    torch.set_num_threads(1)
    torch.manual_seed(a.rank)
    dev = torch.device(a.device)
    model = MLP(hidden_sizes=(128,)).to(dev)
    inner = torch.optim.Adam(model.parameters(), lr=1e-3)
    comm = pccl.Communicator(a.master, 0)
    comm.connect(n_attempts=30)
    d = DiLoCo(model, comm, outer_lr=0.7)
    state = d.shared_state()
    x, y = load_mnist()
    data = batches(x, y, 32, seed=a.rank, device=dev)
    it, world_seen, losses = 0, 0, []
    while True:
        maybe_update_topology(comm, it)
        it += 1
        ws = comm.get_attribute(pccl.Attribute.GLOBAL_WORLD_SIZE)
        world_seen = max(world_seen, ws)
        if ws < 2 or world_seen < a.start_world:
            time.sleep(0.05)
            continue
        info = comm.sync_shared_state(state)
        state.revision += 1
        if info.rx_bytes or it == 1:
            d.load_outer_into_model()
        if int(d.outer_steps.item()) >= a.outer_steps:
            if a.min_world and world_seen < a.min_world:
                continue
            break
        for _ in range(a.inner_steps):
            xb, yb = next(data)
            loss = F.cross_entropy(model(xb), yb)
            inner.zero_grad()
            loss.backward()
            inner.step()
            losses.append(loss.item())
        d.outer_step()
    flat = torch.cat([o.reshape(-1) for o in d.outer]).cpu()
    print(json.dumps({"rank": a.rank, "outer_steps": int(d.outer_steps.item()), "hash": K.simplehash(flat),
                      "loss_first": losses[0] if losses else None,
                      "loss_last": sum(losses[-8:]) / max(1, len(losses[-8:])), "world": world_seen}), flush=True)
    comm.destroy()


if __name__ == "__main__":
    main()
