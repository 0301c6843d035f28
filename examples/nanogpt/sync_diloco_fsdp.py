"""nanoGPT DiLoCo with FSDP2 inside a node and PCCL across nodes (reference
python/examples/nanogpt_diloco/sync_diloco_fsdp.py).

    torchrun --nproc-per-node L sync_diloco_fsdp.py --master <pccl master ip:port>     (on every node)

Each node shards the model with FSDP2 (``fully_shard``; RCCL over xGMI inside the node). Local rank l of every node
joins PCCL peer group l, so shard l is averaged across nodes only with the other nodes' shard l: the L peer groups
run concurrently and each GPU moves 1/L of the pseudo-gradient over the network. The run starts once every node's
every rank is present (GLOBAL_WORLD_SIZE == L x LARGEST_PEER_GROUP_WORLD_SIZE, reference :419-420).
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from common import Timer, build, device_of, get_lr, parser  # noqa: E402

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
from torch.distributed.fsdp import fully_shard  # noqa: E402

import pccl_amd as pccl  # noqa: E402
from pccl_amd.parallel import init_optimizer_state, maybe_update_topology  # noqa: E402
from pccl_amd.parallel.diloco import DiLoCo  # noqa: E402


def main():
    ap = parser(__doc__)
    ap.add_argument("--inner-steps", type=int, default=8)
    ap.add_argument("--outer-lr", type=float, default=0.7)
    ap.add_argument("--nodes", type=int, default=2, help="expected number of nodes (peers per peer group)")
    a = ap.parse_args()
    device = device_of(a)
    if device.type == "cuda":
        torch.cuda.set_device(device)
    dist.init_process_group("nccl" if device.type == "cuda" else "gloo")
    L, l = dist.get_world_size(), dist.get_rank() % int(os.environ.get("LOCAL_WORLD_SIZE", dist.get_world_size()))
    cfg, model, _, data, ctx = build(a, device)
    for blk in model.h:
        fully_shard(blk)
    fully_shard(model)
    opt = torch.optim.AdamW(model.parameters(), lr=a.lr, weight_decay=a.weight_decay)
    init_optimizer_state(opt)
    shards = [p.to_local() for p in model.parameters()]
    comm = pccl.Communicator(a.master, peer_group=l)
    comm.connect(n_attempts=30)
    d = DiLoCo(model, comm, outer_lr=a.outer_lr, tensors=shards)
    state = d.shared_state()
    # Join phase. Every rank admits peers on its own until the whole run is present: a rank that is still waiting
    # for admission blocks inside connect(), so no intra-node collective may run before everyone is admitted.
    it_local, timer = 0, Timer()

    def run_complete() -> bool:
        ws = comm.get_attribute(pccl.Attribute.GLOBAL_WORLD_SIZE)
        largest = comm.get_attribute(pccl.Attribute.LARGEST_PEER_GROUP_WORLD_SIZE)
        return largest >= a.nodes and ws >= L * largest

    while not run_complete():
        maybe_update_topology(comm, it_local)
        it_local += 1
        time.sleep(0.05)
    dist.barrier()
    while True:
        info = comm.sync_shared_state(state)
        state.revision += 1
        if info.rx_bytes:
            d.load_outer_into_model()
        outer_it = int(d.outer_steps.item())
        if outer_it * a.inner_steps >= a.max_iters:
            break
        losses = []
        for s in range(a.inner_steps):
            for g in opt.param_groups:
                g["lr"] = get_lr(outer_it * a.inner_steps + s, a)
            opt.zero_grad(set_to_none=False)
            x, y = data.batch(a.batch_size, cfg.block_size, device)
            with ctx:
                _, loss = model(x, y)
            loss.backward()
            losses.append(loss.item())
            opt.step()
        res = d.outer_step()
        print(json.dumps({"rank": dist.get_rank(), "group": l, "outer": outer_it, "loss": round(sum(losses) / len(losses), 4),
                          "s": round(timer.lap(), 3), "reduce_tx": res.tx_bytes}), flush=True)
    flat = torch.cat([o.reshape(-1) for o in d.outer])
    print(json.dumps({"done": True, "group": l, "outer_steps": int(d.outer_steps.item()), "outer_sum": float(flat.sum())}),
          flush=True)
    comm.destroy()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
