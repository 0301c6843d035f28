"""SIGKILL a peer while xGMI/IPC or device-ring all-reduce work is running (one GPU, separate processes).

    python scripts/ipc_kill_probe.py [--world 3] [--n 536870912] [--kill-after 3.0] [--duration 10] [--out DIR]
                                     [--disable-ipc] [--quant u8] [--inject POINT:SEQ[:STEP[:PHASE]]]

Spawns a master and WORLD peer processes on cuda:0 that run back-to-back bf16 all-reduces of `n` elements over the
IPC path (x = 1 everywhere, result must equal the world size; checked every 16th op). After `kill-after` seconds the
parent SIGKILLs peer 0 at an arbitrary point of its op loop (most of an op's time is kernel time at this size).
Survivors must see the loss, re-form the ring and finish all their steps with exact results. Each peer's stdout /
stderr (PCCL_LOG_LEVEL=DEBUG: the IPC mappings of every op) goes to DIR/peer<r>.{out,err}; a JSON summary is printed.
--disable-ipc runs every peer on the loopback-TCP device ring instead (PCCL_DISABLE_IPC=1); --inject ring:SEQ:STEP:PHASE
then kills the victim at a ring step (csrc/common/types.hpp).
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=3)
    ap.add_argument("--n", type=int, default=1 << 29)
    ap.add_argument("--kill-after", type=float, default=4.0)
    ap.add_argument("--duration", type=float, default=10.0, help="seconds each peer keeps running ops")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "ipc_kill"))
    ap.add_argument("--inplace", action="store_true")
    ap.add_argument("--shareable", action="store_true", help="peers allocate their buffers in fd-shareable memory "
                                                              "(zero-copy safe mode)")
    ap.add_argument("--log-level", default="INFO")
    ap.add_argument("--respawn", action="store_true", help="start a replacement peer after the kill (it joins the "
                                                            "running ring: new IPC arena with a fresh process)")
    ap.add_argument("--inject", default="", help="PCCL_FAULT_INJECT for the victim (e.g. ipc_kernel:200): it kills "
                                                 "itself at that protocol point instead of the parent's timed SIGKILL")
    ap.add_argument("--victim-threads", type=int, default=0, help="extra busy threads in the victim process")
    ap.add_argument("--disable-ipc", action="store_true", help="device TCP ring instead of the xGMI path")
    ap.add_argument("--quant", default="none", choices=["none", "u8"], help="quantized all-reduce (device ring)")
    ap.add_argument("--pool", type=int, default=0, help="P2P connection pool size of every peer (0: default)")
    ap.add_argument("--verify-restore-ms", type=int, default=-1,
                    help="survivors re-read an in-place buffer this long after an aborted op (must equal the input)")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    from pccl_amd.utils import local_master
    worker = os.path.join(ROOT, "tests", "workers", "allreduce_peer.py")
    env = dict(os.environ, PCCL_LOG_LEVEL=a.log_level, PCCL_DEBUG_BACKTRACE_SIGNAL="1")
    if a.disable_ipc:
        env["PCCL_DISABLE_IPC"] = "1"
    common = ["--quant", a.quant] + (["--pool", str(a.pool)] if a.pool else [])
    summary = {"world": a.world, "n": a.n, "kill_after_s": a.kill_after}
    with local_master() as addr:
        ps, files = [], []
        for r in range(a.world):
            fo = open(os.path.join(a.out, f"peer{r}.out"), "w")
            fe = open(os.path.join(a.out, f"peer{r}.err"), "w")
            files += [fo, fe]
            args = [sys.executable, "-u", worker, addr, str(a.world), str(r), "--const", "--n", str(a.n), "--dtype",
                    "bf16", "--duration", str(a.duration), "--device", "cuda:0", "--reuse", "--check-every", "16", *common]
            if a.inplace:
                args.append("--inplace")
            if a.shareable:
                args.append("--shareable")
            if r == 0 and a.victim_threads:
                args += ["--busy-threads", str(a.victim_threads)]
            if r != 0 and a.verify_restore_ms >= 0:
                args += ["--verify-restore-ms", str(a.verify_restore_ms)]
            penv = dict(env, PCCL_FAULT_INJECT=a.inject) if (r == 0 and a.inject) else env
            ps.append(subprocess.Popen(args, stdout=fo, stderr=fe, env=penv))
        # wait until the victim has completed a few ops, then kill it at an arbitrary point
        vic_out = os.path.join(a.out, "peer0.out")
        t0 = time.time()
        hung = False
        while True:
            if time.time() - t0 > 25:
                hung = True
                break
            try:
                with open(vic_out) as f:
                    if sum(1 for ln in f if ln.startswith("{")) >= 3:
                        break
            except OSError:
                pass
            if ps[0].poll() is not None:
                break
            time.sleep(0.05)
        if hung:  # no op completed at all: backtraces of every peer (PCCL_DEBUG_BACKTRACE_SIGNAL), then kill them
            summary["hung_before_kill"] = True
            for p in ps:
                os.kill(p.pid, signal.SIGUSR2)
            time.sleep(3.0)
            for p in ps:
                p.kill()
        elif a.inject:
            while ps[0].poll() is None and time.time() - t0 < 120:
                time.sleep(0.01)
        else:
            time.sleep(a.kill_after)
        killed_at = time.time()
        if ps[0].poll() is None:
            os.kill(ps[0].pid, signal.SIGKILL)
        try:
            summary["victim_rc"] = ps[0].wait(timeout=60)
        except subprocess.TimeoutExpired:
            summary["victim_rc"] = "timeout"
        if a.respawn and not summary.get("hung_before_kill"):
            r = a.world
            fo = open(os.path.join(a.out, f"peer{r}.out"), "w")
            fe = open(os.path.join(a.out, f"peer{r}.err"), "w")
            files += [fo, fe]
            args = [sys.executable, "-u", worker, addr, str(a.world), str(r), "--const", "--n", str(a.n), "--dtype",
                    "bf16", "--duration", str(max(2.0, a.duration / 2)), "--device", "cuda:0", "--reuse",
                    "--check-every", "16", "--no-wait", *common] + (["--inplace"] if a.inplace else []) + \
                (["--shareable"] if a.shareable else [])
            ps.append(subprocess.Popen(args, stdout=fo, stderr=fe, env=env))
        rcs = []
        deadline = time.time() + a.duration + 30
        for p in ps[1:]:
            try:
                rcs.append(p.wait(timeout=max(1.0, deadline - time.time())))
            except subprocess.TimeoutExpired:
                rcs.append("timeout")
        if "timeout" in rcs:  # hung: native backtraces of every live peer (PCCL_DEBUG_BACKTRACE_SIGNAL), then kill
            for p in ps:
                if p.poll() is None:
                    os.kill(p.pid, signal.SIGUSR2)
            time.sleep(2.0)
            for p in ps:
                if p.poll() is None:
                    p.kill()
                    p.wait()
        for f in files:
            f.close()
    summary["survivor_rcs"] = rcs
    for r in range(len(ps)):
        with open(os.path.join(a.out, f"peer{r}.out")) as f:
            lines = [json.loads(x) for x in f if x.startswith("{")]
        oks = [x for x in lines if "error" not in x]
        summary[f"peer{r}"] = {"ops_ok": len(oks), "errors": len(lines) - len(oks),
                               "bad": sum(1 for x in oks if x.get("bad")),
                               "worlds": sorted({x["world"] for x in oks}),
                               "ops_ok_by_world": {str(w): sum(1 for x in oks if x["world"] == w)
                                                   for w in sorted({x["world"] for x in oks})},
                               "paths": sorted({x["path"] for x in oks}),
                               "ipc_bufs": oks[-1].get("ipc_bufs") if oks else None,
                               "restore_checked": sum(1 for x in lines if "restore_bad" in x),
                               "restore_bad": sum(1 for x in lines if x.get("restore_bad"))}
        with open(os.path.join(a.out, f"peer{r}.err")) as f:
            err = f.read()
        summary[f"peer{r}"]["fault_lines"] = [ln for ln in err.splitlines() if "fault" in ln.lower()][:5]
    summary["killed_after_start_s"] = round(killed_at - t0, 2)
    print(json.dumps(summary), flush=True)
    ok = all(rc == 0 for rc in rcs) and all(summary[f"peer{r}"]["bad"] == 0 and summary[f"peer{r}"]["restore_bad"] == 0
                                            for r in range(1, len(ps)))
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
