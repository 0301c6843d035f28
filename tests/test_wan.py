"""Emulated WAN (PCCL_SIM_WAN: latency + per-flow bandwidth caps on the P2P connections): quantized all-reduce moves
~4x fewer bytes and finishes correspondingly faster; striping over the connection pool multiplies the per-flow rate
(BASELINE config 3 shape: int8-quantized all-reduce over a 50 ms WAN). Runs peers as processes so the emulation
(read once per process) does not leak into other tests."""
import json
import os
import subprocess
import sys
import textwrap

import pytest

from pccl_amd.utils import DIAG_SIGNALS, communicate_all, local_master, spawn_python

PEER = textwrap.dedent(r"""
    import json, sys, time
    import torch
    import pccl_amd as pccl
    from pccl_amd.utils import wait_for_world
    addr, world, quant, pool = sys.argv[1], int(sys.argv[2]), sys.argv[3], int(sys.argv[4])
    c = pccl.Communicator(addr, 0, p2p_connection_pool_size=pool)
    c.connect(n_attempts=30)
    wait_for_world(c, world)
    g = torch.Generator().manual_seed(int(time.time() * 1e6) % 1000)
    x = torch.randn(1 << 22, generator=g)
    q = {"none": None, "uint8": pccl.QuantizationOptions(pccl.DataType.UINT8, pccl.QuantizationAlgorithm.MIN_MAX),
         "fp8": pccl.QuantizationOptions(pccl.DataType.FLOAT8_E4M3, pccl.QuantizationAlgorithm.MIN_MAX)}[quant]
    c.all_reduce(x[:1024].clone(), torch.empty(1024), op=pccl.ReduceOp.SUM, tag=1, quantization_options=q)  # warm
    t0 = time.perf_counter()
    info = c.all_reduce(x, torch.empty_like(x), op=pccl.ReduceOp.AVG, tag=0, quantization_options=q)
    print(json.dumps({"s": time.perf_counter() - t0, "tx": info.tx_bytes}), flush=True)
    c.destroy()
""")


def _timed(world, quant, pool, wan="10:400"):
    with local_master() as addr:
        ps = [spawn_python(["-c", PEER, addr, str(world), quant, str(pool)],
                           env={"PCCL_SIM_WAN": wan, "OMP_NUM_THREADS": "1", "PCCL_STRIPE_MIN_BYTES": str(1 << 20)},
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for _ in range(world)]
        outs = communicate_all(ps, 300, DIAG_SIGNALS)
    res = []
    for p, (o, e) in zip(ps, outs):
        assert p.returncode == 0, e[-2000:]
        res.append(json.loads(o.strip().splitlines()[-1]))
    return max(r["s"] for r in res), res[0]["tx"]


def test_quantization_pays_off_on_a_slow_link():
    t_fp32, tx_fp32 = _timed(3, "none", 1)
    t_u8, tx_u8 = _timed(3, "uint8", 1)
    assert tx_u8 < tx_fp32 / 3
    # a quarter of the bytes on a rate-limited link: ~0.3 of the time plus fixed latency terms; measured 0.4-0.52
    # while other tests load the CPUs
    assert t_u8 < 0.65 * t_fp32, (t_u8, t_fp32)


def test_striping_multiplies_per_flow_bandwidth():
    t1, _ = _timed(2, "none", 1)
    t4, _ = _timed(2, "none", 4)
    # ideal 0.25 plus fixed per-step costs; measured 0.35-0.62 across boxes and CPU load (e.g. 0.21 vs 0.35 s on a
    # GPU box), so the check only asks for a clear speed-up
    assert t4 < 0.75 * t1, (t4, t1)
