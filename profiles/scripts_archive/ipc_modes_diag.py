"""Repeat the threaded two-peer IPC all-reduce of tests/test_gpu_allreduce.py::test_device_ipc_modes and classify
every wrong result (stale zeros, the caller's original input, partial tiles).

    python profiles/scripts_archive/ipc_modes_diag.py [--iters 10] [--offset 777]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import pccl_amd as pccl  # noqa: E402
from pccl_amd.utils import local_master, run_threaded_peers  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--offset", type=int, default=777)
    ap.add_argument("--n", type=int, default=3_000_001)
    a = ap.parse_args()
    hip = torch.device("cuda:0")
    n, off = a.n, a.offset
    bad_total = 0
    for inplace in [(True, False), (False, True), (False, False), (True, True)]:
        for it in range(a.iters):
            big = [torch.randn(n + 1000 + off, device=hip) for _ in range(2)]
            orig = [b[off:off + n].clone() for b in big]
            expect = (orig[0] + orig[1]).clone()
            torch.cuda.synchronize()

            def fn(rank, comm):
                x = big[rank][off:off + n]
                y = x if inplace[rank] else torch.empty_like(x)
                comm.all_reduce(x, y, op=pccl.ReduceOp.SUM, tag=0)
                torch.cuda.synchronize()
                return y.clone()

            with local_master() as addr:
                res = run_threaded_peers(2, fn, address=addr, timeout=120)
            for rank, y in enumerate(res):
                wrong = (y != expect).nonzero().flatten()
                if wrong.numel() == 0:
                    continue
                bad_total += 1
                w = wrong
                rec = {"inplace": inplace, "iter": it, "rank": rank, "n_wrong": int(w.numel()),
                       "first": int(w[0]), "last": int(w[-1]),
                       "zeros": int((y[w] == 0).sum()),
                       "eq_own_input": int((y[w] == orig[rank][w]).sum()),
                       "eq_peer_input": int((y[w] == orig[1 - rank][w]).sum()),
                       "tiles_4k": sorted({int(i) * 4 // 4096 for i in w.tolist()[:100000]})[:16]}
                print(json.dumps(rec), flush=True)
        print(json.dumps({"inplace": inplace, "done": a.iters}), flush=True)
    print(json.dumps({"bad_results": bad_total}), flush=True)


if __name__ == "__main__":
    main()
