"""nanoGPT with synchronous DiLoCo over PCCL (reference python/examples/nanogpt_diloco/sync_diloco.py).

Every outer step: ``--inner-steps`` local AdamW steps, then the AVG all-reduce of the pseudo-gradients (device
path, optionally quantized with --quantize uint8|fp8) and a fused outer SGD step. Shared state = outer params,
outer momentum, inner AdamW state, outer step counter; a late joiner gets all of it in its first sync.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from common import Timer, build, device_of, get_lr, parser  # noqa: E402

import torch  # noqa: E402

import pccl_amd as pccl  # noqa: E402
from pccl_amd.parallel import init_optimizer_state, maybe_update_topology  # noqa: E402
from pccl_amd.parallel.diloco import AsyncDiLoCo, DiLoCo  # noqa: E402

QUANT = {"none": None,
         "uint8": pccl.QuantizationOptions(pccl.DataType.UINT8, pccl.QuantizationAlgorithm.MIN_MAX),
         "fp8": pccl.QuantizationOptions(pccl.DataType.FLOAT8_E4M3, pccl.QuantizationAlgorithm.MIN_MAX)}


def args():
    ap = parser(__doc__)
    ap.add_argument("--inner-steps", type=int, default=8)
    ap.add_argument("--outer-lr", type=float, default=0.7)
    ap.add_argument("--outer-momentum", type=float, default=0.0)
    ap.add_argument("--nesterov", action="store_true")
    ap.add_argument("--quantize", default="none", choices=sorted(QUANT))
    ap.add_argument("--async-outer", action="store_true", help="1-step-delayed (async) DiLoCo")
    return ap.parse_args()


def main():
    a = args()
    device = device_of(a)
    if device.type == "cuda":
        torch.cuda.set_device(device)
    cfg, model, opt, data, ctx = build(a, device)
    init_optimizer_state(opt)
    comm = pccl.Communicator(a.master, 0)
    comm.connect(n_attempts=30)
    cls = AsyncDiLoCo if a.async_outer else DiLoCo
    d = cls(model, comm, outer_lr=a.outer_lr, outer_momentum=a.outer_momentum, nesterov=a.nesterov,
            quantization=QUANT[a.quantize])
    state = d.shared_state(opt)
    tokens_per_outer = a.batch_size * cfg.block_size * a.grad_accum * a.inner_steps
    it_local, n_syncs, timer = 0, 0, Timer()
    while True:
        topology_updated = it_local == 0
        if it_local > 0 and comm.are_peers_pending():
            if a.async_outer:
                d.wait()  # no collectives may be in flight during the vote
            maybe_update_topology(comm, it_local)
            topology_updated = True
        it_local += 1
        ws = comm.get_attribute(pccl.Attribute.GLOBAL_WORLD_SIZE)
        if ws < a.min_world:
            time.sleep(0.1)
            continue
        if topology_updated or not a.async_outer:
            info = comm.sync_shared_state(state)
            state.revision += 1
            n_syncs += 1
            if info.rx_bytes or n_syncs == 1:
                d.load_outer_into_model()
        outer_it = int(d.outer_steps.item())
        if outer_it * a.inner_steps >= a.max_iters:
            break
        losses = []
        for s in range(a.inner_steps):
            for g in opt.param_groups:
                g["lr"] = get_lr(outer_it * a.inner_steps + s, a)
            opt.zero_grad(set_to_none=False)
            for _ in range(a.grad_accum):
                x, y = data.batch(a.batch_size, cfg.block_size, device)
                with ctx:
                    _, loss = model(x, y)
                (loss / a.grad_accum).backward()
            losses.append(loss.item())
            if a.grad_clip:
                torch.nn.utils.clip_grad_norm_(model.parameters(), a.grad_clip)
            opt.step()
        if a.async_outer:
            res = d.outer_step(topology_updated=topology_updated and outer_it > 0, shared_state=state,
                               joined_mid_run=topology_updated and outer_it > 0 and n_syncs == 1)
        else:
            res = d.outer_step()
        dt = timer.lap()
        print(json.dumps({"outer": outer_it, "loss": round(sum(losses) / len(losses), 4), "world": ws,
                          "s": round(dt, 3), "tok_s": round(tokens_per_outer / dt, 1),
                          "reduce_tx": res.tx_bytes if res else 0}), flush=True)
    if a.async_outer:
        d.close()
    flat = torch.cat([o.reshape(-1) for o in d.outer])
    print(json.dumps({"done": True, "outer_steps": int(d.outer_steps.item()), "outer_sum": float(flat.sum())}),
          flush=True)
    comm.destroy()


if __name__ == "__main__":
    main()
