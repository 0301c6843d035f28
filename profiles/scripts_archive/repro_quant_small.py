"""Repro harness: the quantized device ring with fewer elements than peers (tests/test_gpu_allreduce.py::
test_device_ring_fewer_elements_than_peers[True-1]), repeated in fresh sessions; on a hang (no progress for 30 s) it
prints every thread's native backtrace (PCCL_DEBUG_BACKTRACE_SIGNAL) and Python stacks, then exits 3."""
import faulthandler
import os
import signal
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("PCCL_DISABLE_IPC", "1")
os.environ.setdefault("PCCL_SMALL_ALLREDUCE_BYTES", "0")
os.environ["PCCL_DEBUG_BACKTRACE_SIGNAL"] = "1"
import torch  # noqa: E402

import pccl_amd as pccl  # noqa: E402
from pccl_amd.utils import local_master, run_threaded_peers  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
world = 4
qopt = pccl.QuantizationOptions(pccl.DataType.UINT8, pccl.QuantizationAlgorithm.MIN_MAX)
progress = [time.time()]


def watchdog():
    while True:
        time.sleep(1)
        if time.time() - progress[0] > 30:
            print("HANG: dumping stacks", flush=True)
            faulthandler.dump_traceback(all_threads=True)
            os.kill(os.getpid(), signal.SIGUSR2)
            time.sleep(3)
            os._exit(3)


threading.Thread(target=watchdog, daemon=True).start()
for rep in range(reps):
    def fn(rank, comm):
        x = (torch.arange(n, device="cuda", dtype=torch.float32) % 5 + rank).bfloat16()
        y = torch.full((n + 64,), -7.0, device="cuda", dtype=torch.bfloat16)
        for tag in range(2):
            comm.all_reduce(x, y[:n], op=pccl.ReduceOp.SUM, tag=tag, quantization_options=qopt)
            progress[0] = time.time()
        torch.cuda.synchronize()
        return y.cpu()
    with local_master() as addr:
        res = run_threaded_peers(world, fn, address=addr, timeout=60)
    print(f"rep {rep} ok {[r[:n].tolist() for r in res]}", flush=True)
print("all ok", flush=True)
