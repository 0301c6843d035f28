"""MNIST data-parallel peer with elastic membership (reference python/tests/end_to_end/mnist_ddp/mnist_peer.py).

Every iteration: admit pending peers -> sync shared state (params + Adam state, revision = step) -> local
forward/backward -> device-resident gradient all-reduce (AVG) -> optimizer step. A late joiner receives the current
state in its first shared-state sync. Prints one JSON summary line at the end (parameter hash, loss, revision).

env / args: --master 127.0.0.1:48148  --device cpu|cuda  --max-steps 256  --min-world 0 (DONT_EXIT_BEFORE_REACHED...)
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
from pccl_amd.parallel import DataParallel, init_optimizer_state, maybe_update_topology, shared_state_for  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--master", default=os.environ.get("PCCL_MASTER", "127.0.0.1:48148"))
    ap.add_argument("--rank", type=int, default=int(os.environ.get("RANK", "0")))
    ap.add_argument("--device", default="cuda" if os.environ.get("MNIST_USE_CUDA") == "1" else "cpu")
    ap.add_argument("--max-steps", type=int, default=int(os.environ.get("MAX_STEPS", "256")))
    ap.add_argument("--min-world", type=int, default=int(os.environ.get("DONT_EXIT_BEFORE_REACHED_WORLD_SIZE", "0")))
    ap.add_argument("--start-world", type=int, default=int(os.environ.get("PCCL_START_WORLD", "2")),
                    help="train only once this many peers have formed the run (elastic afterwards)")
    ap.add_argument("--batch-size", type=int, default=32)
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--hidden", type=int, nargs="+", default=[128])
    a = ap.parse_args()
    torch.set_num_threads(1)
    torch.manual_seed(a.rank)  # peers start from different weights: the first shared-state sync unifies them
    dev = torch.device(a.device)

    model = MLP(hidden_sizes=a.hidden).to(dev)
    opt = torch.optim.Adam(model.parameters(), lr=a.lr)
    init_optimizer_state(opt)
    comm = pccl.Communicator(a.master, 0)
    comm.connect(n_attempts=30)
    dp = DataParallel(model, comm)
    state = shared_state_for(model, opt)
    x, y = load_mnist()
    data = batches(x, y, a.batch_size, seed=a.rank, device=dev)

    it, losses, world_seen = 0, [], 0
    t0 = time.time()
    while True:
        maybe_update_topology(comm, it)
        it += 1
        ws = comm.get_attribute(pccl.Attribute.GLOBAL_WORLD_SIZE)
        world_seen = max(world_seen, ws)
        if ws < 2 or world_seen < a.start_world:
            time.sleep(0.05)
            continue
        comm.sync_shared_state(state)
        if state.revision >= a.max_steps:
            if a.min_world and world_seen < a.min_world:
                continue  # keep the run alive until the expected late joiner arrived
            break
        xb, yb = next(data)
        loss = F.cross_entropy(model(xb), yb)
        opt.zero_grad(set_to_none=False)
        loss.backward()
        res = dp.sync_gradients()
        if not res.ok:
            continue  # alone now: wait for peers
        opt.step()
        losses.append(float(loss))
        state.revision += 1
    flat = torch.cat([p.detach().reshape(-1).float().cpu() for p in model.parameters()])
    summary = {"rank": a.rank, "revision": state.revision, "steps_here": len(losses),
               "hash": K.simplehash(flat), "loss_first": losses[0] if losses else None,
               "loss_last": sum(losses[-10:]) / max(1, len(losses[-10:])), "world": world_seen,
               "seconds": round(time.time() - t0, 2)}
    print(json.dumps(summary), flush=True)
    comm.destroy()


if __name__ == "__main__":
    main()
