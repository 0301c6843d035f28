"""nanoGPT data-parallel training over PCCL (reference python/examples/nanogptddp/train_pccl.py).

Single process per peer:          python train_pccl.py --master 127.0.0.1:48148
Hybrid (RCCL in node x PCCL across nodes, peer group per local rank):
                                  torchrun --nproc-per-node 8 train_pccl.py --master <master ip:port>
Gradients stay on the GPU (flat device buckets, device all-reduce). Shared state = params + AdamW state + iter.
"""
import contextlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from common import Timer, build, device_of, estimate_loss, get_lr, load_checkpoint, parser, save_checkpoint  # noqa

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import pccl_amd as pccl  # noqa: E402
from pccl_amd.parallel import DataParallel, init_optimizer_state, maybe_update_topology, shared_state_for  # noqa
from pccl_amd.parallel.hybrid import HierarchicalGradSync, local_peer_group  # noqa: E402
from pccl_amd.utils.profiler import Profiler  # noqa: E402


def main():
    ap = parser(__doc__)
    ap.add_argument("--overlap", action="store_true",
                    help="start each gradient bucket's all-reduce during backward (DataParallel(overlap=True))")
    a = ap.parse_args()
    hybrid = int(os.environ.get("WORLD_SIZE", "1")) > 1
    device = device_of(a)
    if device.type == "cuda":
        torch.cuda.set_device(device)
    if hybrid:
        dist.init_process_group("nccl" if device.type == "cuda" else "gloo")
    cfg, model, opt, data, ctx = build(a, device)
    init_optimizer_state(opt)
    start_iter = load_checkpoint(a, model, opt)
    iter_num = torch.tensor([start_iter], dtype=torch.int64)

    comm = pccl.Communicator(a.master, peer_group=local_peer_group() if hybrid else 0)
    comm.connect(n_attempts=30)
    sync = HierarchicalGradSync(model, comm) if hybrid else DataParallel(model, comm, overlap=a.overlap)
    state = shared_state_for(model, opt, extra={"iter_num": iter_num})
    state.revision = start_iter
    tokens_per_iter = a.batch_size * cfg.block_size * a.grad_accum

    it_local = 0
    timer = Timer()
    while True:
        prof = Profiler(sync_cuda=device.type == "cuda")  # phase times include the GPU work queued in them
        with prof.session("update_topology"):
            maybe_update_topology(comm, it_local)
        it_local += 1
        ws = comm.get_attribute(pccl.Attribute.GLOBAL_WORLD_SIZE)
        if ws < a.min_world:
            time.sleep(0.1)
            continue
        with prof.session("sync_shared_state"):
            info = comm.sync_shared_state(state)
        it = int(iter_num.item())
        if it >= a.max_iters:
            break
        for g in opt.param_groups:
            g["lr"] = get_lr(it, a)
        with prof.session("forward_backward"):
            opt.zero_grad(set_to_none=False)
            loss_acc = 0.0
            for micro in range(a.grad_accum):
                x, y = data.batch(a.batch_size, cfg.block_size, device)
                with ctx:
                    _, loss = model(x, y)
                last = micro == a.grad_accum - 1
                with sync.no_sync() if (a.overlap and not hybrid and not last) else contextlib.nullcontext():
                    (loss / a.grad_accum).backward()
                loss_acc += loss.item() / a.grad_accum
        with prof.session("all_reduce"):
            res = sync.sync_gradients()
        if res is not None and not res.ok:
            continue
        with prof.session("optimizer"):
            if a.grad_clip:
                torch.nn.utils.clip_grad_norm_(model.parameters(), a.grad_clip)
            opt.step()
        iter_num += 1
        state.revision += 1
        dt = timer.lap()
        phase_ms = {k: round(v * 1e3, 2) for k, v in prof.totals().items() if k in ("forward_backward", "all_reduce")}
        rec = {"iter": it, "loss": round(loss_acc, 4), "world": ws, "ms": round(dt * 1e3, 1), "phase_ms": phase_ms,
               "tok_s": round(tokens_per_iter / dt, 1), "mfu": round(model.estimate_mfu(tokens_per_iter, dt), 4),
               "ss_rx": info.rx_bytes, "ar_tx": res.tx_bytes if res else 0}
        if a.eval_interval and it % a.eval_interval == 0:
            rec["val_loss"] = round(estimate_loss(model, data, cfg, a, device, ctx), 4)
            save_checkpoint(a, model, opt, it)
        print(json.dumps(rec), flush=True)
    print(json.dumps({"done": True, "iter": int(iter_num.item()),
                      "param_sum": float(sum(p.detach().float().sum() for p in model.parameters()))}), flush=True)
    comm.destroy()
    if hybrid:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
