"""The BASELINE-config benchmark scripts (benchmarks/) at toy sizes: they must run end to end and report exact results.

CPU variants run everywhere; the `gpu` variants exercise the HBM paths (HIP IPC shared-state hand-off between two
processes, device ring with HIP quantization kernels under the WAN emulation, IPC all-reduce under fault injection).
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(script, *args, timeout=300, extra_env=None):
    env = dict(os.environ)
    env.update(extra_env or {})
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "benchmarks", script), *args], env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-3000:]
    return json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])


@pytest.mark.parametrize("device,transport", [("cpu", "tcp"), ("cpu", "ipc"),
                                              pytest.param("cuda:0", "ipc", marks=pytest.mark.gpu),
                                              pytest.param("cuda:0", "tcp", marks=pytest.mark.gpu)])
def test_shared_state_catch_up(device, transport):
    r = _run("shared_state_sync.py", "--params", "3000001", "--tensors", "3", "--device", device,
             "--transport", transport)
    assert r["content_ok"] and r["hash_verified"] and r["adopted_revision"] == 3
    assert r["joiner_rx_bytes"] == r["bytes"] == 3000001 * 4
    assert r["trainer_tx_bytes"] == r["bytes"]


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda:0", marks=pytest.mark.gpu)])
def test_shared_state_catch_up_crc32c(device):
    """PCCL_SHARED_STATE_HASH=crc32c: peers announce CRC-32C content hashes (HIP kernel for HBM tensors)."""
    r = _run("shared_state_sync.py", "--params", "1000003", "--tensors", "2", "--device", device,
             extra_env={"PCCL_SHARED_STATE_HASH": "crc32c"})
    assert r["content_ok"] and r["joiner_rx_bytes"] == r["bytes"]


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda:0", marks=pytest.mark.gpu)])
def test_basic_reduce(device):
    r = _run("basic_reduce.py", "--iters", "30", "--tensors", "4", "--numel", "65536", "--pool", "4",
             "--device", device)
    assert r["latency_us"]["median"] > 0
    assert r["multi_tensor"]["busbw_GBps"] > 0


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda:0", marks=pytest.mark.gpu)])
def test_wan_quantized(device):
    r = _run("wan_quantized.py", "--peers", "3", "--mib", "2", "--latency-ms", "5", "--flow-mbit", "2000",
             "--link-mbit", "8000", "--pool", "2", "--concurrent", "2", "--device", device,
             "--formats", "fp32,uint8,int8_zps")
    f = r["formats"]
    assert f["fp32"]["max_abs_err"] < 1e-5
    assert f["uint8"]["max_abs_err"] < 0.05 and f["int8_zps"]["max_abs_err"] < 0.05
    # quantized wire formats move ~4x fewer bytes than fp32
    assert f["uint8"]["ref_metric_rx_plus_tx_Gbit_per_peer"] * f["uint8"]["seconds"] < \
        0.35 * f["fp32"]["ref_metric_rx_plus_tx_Gbit_per_peer"] * f["fp32"]["seconds"]


@pytest.mark.parametrize("device,transport", [("cpu", "tcp"), pytest.param("cuda:0", "tcp", marks=pytest.mark.gpu),
                                              pytest.param("cuda:0", "ipc", marks=pytest.mark.gpu)])
def test_fault_tolerance(device, transport):
    """BASELINE config 5 at toy size: the victim SIGKILLs itself mid-op (fault injection), survivors abort with their
    in-place input restored, continue at W-1, admit a replacement process and re-solve the ring."""
    r = _run("fault_tolerance.py", "--peers", "3", "--mib", "4" if device == "cpu" else "64", "--device", device,
             "--transport", transport, "--kill-op", "4", "--post-ops", "3", "--timeout", "150", timeout=300)
    assert r["complete"] and r["all_results_exact"] and r["in_place_restore_exact"] and not r["peer_errors"], r
    assert r["failed_ops_per_survivor"] >= 1 and r["ops"]["w2"] >= 1 and r["ops"]["after_optimize"] >= 3 * 3, r
    assert r["optimize_ok"] and r["master_topology"]["solves"] == 1, r
    assert r["paths"] == [{"cpu": 1, "tcp": 2, "ipc": 3}["cpu" if device == "cpu" else transport]], r


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda:0", marks=pytest.mark.gpu)])
def test_py_latency(device):
    """One process per peer, both call variants, exact results (checked inside every peer)."""
    r = _run("py_latency.py", "--peers", "3", "--iters", "20", "--warmup", "3", "--sizes", "4096,262144",
             "--device", device)
    assert r["processes"] == "one per peer" and set(r["sizes"]) == {"4KiB", "256KiB"}
    for row in r["sizes"].values():
        assert row["path"] == ("host_ring" if device == "cpu" else "ipc")
        assert row["all_reduce"]["median_us"] > 0 and row["ready"]["median_us"] > 0
