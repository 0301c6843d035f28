"""Peer process of the wire-framing tests (tests/test_wire_compat.py): random inputs, SUM all-reduces, one JSON line
per op with a digest of the result (bit-identity across peers), its error against the fp64 sum of every peer's input
(regenerated from the shared seeds), the reduce path and the wire framing the op ran with.

usage: wire_peer.py MASTER WORLD RANK [--n N] [--dtype f32|bf16] [--device cpu|cuda:0] [--quant none|u8]
                    [--pool P] [--steps K]
The environment selects the peer's wire behaviour (PCCL_WIRE, PCCL_RING_STRIPES, PCCL_QUANT_LANES, ...).
"""
import argparse
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

import pccl_amd as pccl  # noqa: E402
from pccl_amd.utils import wait_for_world  # noqa: E402

DT = {"f32": torch.float32, "bf16": torch.bfloat16}


def _input(n, dtype, dev, rank, step):
    g = torch.Generator().manual_seed(1_000 * step + rank)
    return torch.randn(n, generator=g, dtype=torch.float32).to(dtype).to(dev)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("master")
    ap.add_argument("world", type=int)
    ap.add_argument("rank", type=int)
    ap.add_argument("--n", type=int, default=(1 << 20) + 37)
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--quant", default="none", choices=["none", "u8"])
    ap.add_argument("--pool", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device(a.device)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    dtype = DT[a.dtype]
    qopt = pccl.QuantizationOptions(pccl.DataType.UINT8, pccl.QuantizationAlgorithm.MIN_MAX) if a.quant == "u8" \
        else None
    comm = pccl.Communicator(a.master, 0, p2p_connection_pool_size=a.pool)
    comm.connect(n_attempts=30)
    wait_for_world(comm, a.world, timeout=120)
    for step in range(a.steps):
        x = _input(a.n, dtype, dev, a.rank, step)
        y = torch.empty_like(x)
        info = comm.all_reduce(x, y, op=pccl.ReduceOp.SUM, tag=step, quantization_options=qopt)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        want = sum(_input(a.n, dtype, torch.device("cpu"), r, step).double() for r in range(a.world))
        yc = y.cpu()
        print(json.dumps({"rank": a.rank, "step": step, "world": info.local_world_size,
                          "digest": hashlib.sha256(yc.view(torch.uint8).numpy().tobytes()).hexdigest(),
                          "max_err": float((yc.double() - want).abs().max()),
                          "path": comm.get_attribute(pccl.Attribute.LAST_REDUCE_PATH),
                          "framing": comm.get_attribute(pccl.Attribute.LAST_REDUCE_FRAMING),
                          "tx": info.tx_bytes, "rx": info.rx_bytes}), flush=True)
    comm.destroy()


if __name__ == "__main__":
    main()
