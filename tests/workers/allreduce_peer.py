"""Standalone peer process used by the multi-process tests (CPU and GPU).

usage: allreduce_peer.py MASTER WORLD RANK [--n N] [--dtype f32|bf16|f16|i32] [--device cpu|cuda:0] [--steps K]
                         [--die-at STEP] [--const] [--no-wait] [--inplace] [--op sum|avg|max] [--quant none|u8]
                         [--shareable] [--leave-when-alone]
Each step all-reduces a tensor and checks the result; prints one JSON line per attempt.
  default: x = rank + 1 + step, tag = step (all peers start together)
  --const: x = 1, tag 0, result must equal the op's world size (membership may change between steps)
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
from pccl_amd.utils import wait_for_world  # noqa: E402

DT = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16, "i32": torch.int32}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("master")
    ap.add_argument("world", type=int)
    ap.add_argument("rank", type=int)
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--die-at", type=int, default=-1)
    ap.add_argument("--const", action="store_true")
    ap.add_argument("--no-wait", action="store_true", help="do not wait for WORLD peers (late joiner)")
    ap.add_argument("--step-sleep", type=float, default=0.0)
    ap.add_argument("--inplace", action="store_true")
    ap.add_argument("--op", default="sum", choices=["sum", "avg", "max"])
    ap.add_argument("--quant", default="none", choices=["none", "u8"])
    ap.add_argument("--check-every", type=int, default=1, help="verify the result every k-th step only")
    ap.add_argument("--reuse", action="store_true", help="allocate x / y once (back-to-back ops, no refill)")
    ap.add_argument("--duration", type=float, default=0.0, help="run steps until this many seconds passed instead")
    ap.add_argument("--shareable", action="store_true", help="allocate x / y in fd-shareable memory (pccl_amd.memory)")
    ap.add_argument("--leave-when-alone", action="store_true",
                    help="exit 0 once every other peer has left after this one completed a step (a joiner whose "
                         "partners finished their run first cannot complete more steps)")
    ap.add_argument("--busy-threads", type=int, default=0,
                    help="extra threads that keep making syscalls (a SIGKILLed process with many live threads takes "
                         "longer to tear down: its group leader is a zombie while the other threads still exit)")
    ap.add_argument("--pool", type=int, default=0, help="P2P connection pool size (0: library default)")
    ap.add_argument("--max-failures", type=int, default=50, help="exit 3 after more failed ops than this")
    ap.add_argument("--report-mem", action="store_true", help="add the GPU's used bytes (all processes) to every line")
    ap.add_argument("--report-framing", action="store_true", help="add LAST_REDUCE_FRAMING to every line")
    ap.add_argument("--rejoin", action="store_true",
                    help="when the master drops this peer (MASTER_CONNECTED == 0, e.g. after it was stopped), print a "
                         "'kicked' line, destroy the communicator and join again as a new peer")
    ap.add_argument("--p2p-port", type=int, default=0, help="P2P listen port (0: library default)")
    ap.add_argument("--adv-port", type=int, default=0, help="advertised P2P port (a relay in front of --p2p-port)")
    ap.add_argument("--verify-restore-ms", type=int, default=-1,
                    help="in-place: after a failed op wait this long, then require the buffer to be bit-exactly the "
                         "input again (the abort restore must not be overwritten by a late peer write)")
    a = ap.parse_args()
    if a.busy_threads:
        import threading

        def _busy():
            while True:
                os.stat("/")
                time.sleep(0.002)
        for _ in range(a.busy_threads):
            threading.Thread(target=_busy, daemon=True).start()
    op = {"sum": pccl.ReduceOp.SUM, "avg": pccl.ReduceOp.AVG, "max": pccl.ReduceOp.MAX}[a.op]
    qopt = pccl.QuantizationOptions(pccl.DataType.UINT8, pccl.QuantizationAlgorithm.MIN_MAX) if a.quant == "u8" \
        else None
    dev = torch.device(a.device)
    t_start = time.perf_counter()
    def make_comm():
        kw = {"p2p_connection_pool_size": a.pool} if a.pool else {}
        if a.p2p_port:
            kw["p2p_listen_port"] = a.p2p_port
        if a.adv_port:
            kw["advertised_p2p_port"] = a.adv_port
        c = pccl.Communicator(a.master, 0, **kw)
        c.connect(n_attempts=30)
        return c

    comm = make_comm()
    if not a.no_wait:
        wait_for_world(comm, a.world, timeout=120)
    step, failures, first_ok = 0, 0, None
    it = 0
    t_loop = None
    while (step < a.steps) if a.duration <= 0 else (t_loop is None or time.perf_counter() - t_loop < a.duration):
        if t_loop is None:
            t_loop = time.perf_counter()
        try:
            if it > 0 and comm.are_peers_pending():
                comm.update_topology()
        except pccl.PCCLError:
            if comm.get_attribute(pccl.Attribute.MASTER_CONNECTED) != 0:
                raise
            print(json.dumps({"rank": a.rank, "step": step, "error": "dropped", "kicked": True, "t": time.time()}),
                  flush=True)
            if not a.rejoin:
                sys.exit(4)
            comm.destroy()
            comm = make_comm()
            it = 0  # a newcomer's first vote is the all-reduce, as the admitting peers' next one (no pending query)
            print(json.dumps({"rank": a.rank, "rejoined": True, "t": time.time()}), flush=True)
        it += 1
        ws = comm.get_attribute(pccl.Attribute.GLOBAL_WORLD_SIZE)
        if ws < 2:
            if a.leave_when_alone and step > 0:
                break
            time.sleep(0.05)
            continue
        val = 1.0 if a.const else float(a.rank + 1 + step)
        if not a.reuse or step == 0 or a.inplace:
            with pccl.memory.maybe_shareable(dev) if a.shareable else contextlib.nullcontext():
                x = torch.full((a.n,), val, dtype=DT[a.dtype], device=dev)
                y = x if a.inplace else torch.empty_like(x)
        if step == a.die_at:
            os._exit(17)  # simulated crash (no clean disconnect)
        t0 = time.perf_counter()
        try:
            info = comm.all_reduce(x, y, op=op, tag=0 if a.const else step, quantization_options=qopt)
        except pccl.PCCLError as e:
            rec = {"rank": a.rank, "step": step, "error": e.result.name, "t": time.time()}
            if comm.get_attribute(pccl.Attribute.MASTER_CONNECTED) == 0:
                rec["kicked"] = True
            if a.verify_restore_ms >= 0 and a.inplace:
                time.sleep(a.verify_restore_ms / 1e3)
                if dev.type == "cuda":
                    torch.cuda.synchronize()
                rec["restore_bad"] = not bool((x == val).all())
            if a.report_mem and dev.type == "cuda":
                free, total = torch.cuda.mem_get_info(dev)
                rec["hbm_used"] = total - free
                rec["ipc_bufs"] = pccl.memory.ipc_buffer_stats()
            print(json.dumps(rec), flush=True)
            failures += 1
            if failures > a.max_failures:
                sys.exit(3)
            if rec.get("kicked"):
                if not a.rejoin:
                    sys.exit(4)
                comm.destroy()  # dropped by the master: join again as a new peer
                comm = make_comm()
                it = 0
                print(json.dumps({"rank": a.rank, "rejoined": True, "t": time.time()}), flush=True)
            continue  # retry the step with the new world
        if dev.type == "cuda":
            torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if first_ok is None:
            first_ok = time.perf_counter() - t_start
        if step % a.check_every == 0 or step + 1 == a.steps or a.duration > 0 and step % 4 == 0:
            lo, hi = float(y.min().float()), float(y.max().float())
        else:
            lo = hi = float(info.local_world_size) if a.const else None
        rec = {"rank": a.rank, "step": step, "world": info.local_world_size, "lo": lo, "hi": hi,
               "path": comm.get_attribute(pccl.Attribute.LAST_REDUCE_PATH), "sec": dt, "tx": info.tx_bytes,
               "rx": info.rx_bytes, "first_ok_s": round(first_ok, 4), "t": time.time()}
        rec["staging"] = pccl.memory.staging_pool_stats()
        if a.report_framing:
            rec["framing"] = comm.get_attribute(pccl.Attribute.LAST_REDUCE_FRAMING)
        if dev.type == "cuda":
            rec["ipc_bufs"] = pccl.memory.ipc_buffer_stats()
            if a.report_mem:
                free, total = torch.cuda.mem_get_info(dev)
                rec["hbm_used"] = total - free
        if a.const and not (lo == hi == float(info.local_world_size)):
            rec["bad"] = True
        print(json.dumps(rec), flush=True)
        step += 1
        if a.step_sleep:
            time.sleep(a.step_sleep)
    comm.destroy()


if __name__ == "__main__":
    main()
