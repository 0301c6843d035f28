"""Python API lifecycle tests (reference python/tests/unit_tests/pccl_test.py), using a free port per test instead of
the fixed 48148 so that tests can run side by side, plus the `import pccl` alias the reference's users write."""
import gc

import numpy as np
import pytest

from pccl_amd.utils import free_port


def test_import_lib():
    import pccl  # noqa: F401  (alias package: the reference's import name)
    import pccl_amd  # noqa: F401


def test_alias_exports_reference_names():
    import pccl
    for name in ("Communicator", "MasterNode", "SharedState", "TensorInfo", "ReduceOp", "Attribute", "DataType",
                 "DeviceType", "QuantizationAlgorithm", "QuantizationOptions", "ReduceDescriptor",
                 "ReduceOperandDescriptor", "ReduceOpDescriptor", "SharedStateSyncStrategy", "DistributionHint",
                 "PCCLError", "Result", "ReduceInfo", "AsyncReduceHandle", "SharedStateSyncInfo"):
        assert hasattr(pccl, name), name


def _master():
    import pccl
    addr = f"127.0.0.1:{free_port()}"
    m = pccl.MasterNode(listen_address=addr)
    m.run()
    return m, addr


def test_master_node_run():
    m, _ = _master()
    m.interrupt()
    m.await_termination()


def test_communicator():
    import pccl
    m, addr = _master()
    c = pccl.Communicator(addr, 0)
    c.connect()
    assert c.get_attribute(pccl.Attribute.GLOBAL_WORLD_SIZE) == 1
    c.destroy()
    m.interrupt()
    m.await_termination()


def test_communicator_destructor_with_connect():
    import pccl
    m, addr = _master()

    def connect():
        c = pccl.Communicator(addr, 0)
        c.connect()

    connect()
    gc.collect()
    m.interrupt()
    m.await_termination()


def test_communicator_destructor_without_connect():
    import pccl
    m, addr = _master()

    def create():
        pccl.Communicator(addr, 0)

    create()
    gc.collect()
    m.interrupt()
    m.await_termination()


def test_communicator_update_topology_without_connect():
    import pccl
    m, addr = _master()
    c = pccl.Communicator(addr, 0)
    with pytest.raises(pccl.PCCLError):
        c.update_topology()
    m.interrupt()
    m.await_termination()


def test_all_reduce_single_peer_too_few_peers():
    """numpy_only_test.py / pytorch_only_test.py: a lone peer's all-reduce raises PCCLError(TooFewPeers)."""
    import pccl
    m, addr = _master()
    c = pccl.Communicator(addr, 0)
    c.connect()
    x = np.ones(8, dtype=np.float32)
    with pytest.raises(pccl.PCCLError) as e:
        c.all_reduce(x, np.empty_like(x), op=pccl.ReduceOp.SUM)
    assert e.value.result == pccl.Result.TOO_FEW_PEERS
    c.destroy()
    m.interrupt()
    m.await_termination()


def test_build_info():
    import pccl
    info = pccl.build_info()
    assert "has_hip_support" in info and "has_cuda_support" in info


def test_profiler_nested_sessions_report_and_trace(tmp_path):
    """pccl_amd.utils.profiler (reference nanogptddp/profiler.py): nested sessions, totals, text report, Chrome
    trace export, and averages over a ProfilerCollection."""
    import json
    import time

    from pccl_amd.utils.profiler import Profiler, ProfilerCollection
    col = ProfilerCollection()
    for _ in range(2):
        p = Profiler()
        with p.session("step"):
            with p.session("forward"):
                time.sleep(0.002)
            with p.session("all_reduce"):
                time.sleep(0.001)
        col.add(p)
    t = col.profilers[0].totals()
    assert set(t) == {"step", "step/forward", "step/all_reduce"}
    assert t["step"] >= t["step/forward"] + t["step/all_reduce"] > 0
    rep = col.profilers[0].report()
    assert "forward" in rep and "all_reduce" in rep and "ms" in rep
    avg = col.averages()
    assert avg["step/forward"] >= 0.002
    path = tmp_path / "trace.json"
    col.chrome_trace(str(path))
    ev = json.loads(path.read_text())["traceEvents"]
    assert len(ev) == 6 and all(e["ph"] == "X" and e["dur"] > 0 for e in ev)


def test_shareable_memory_api_on_cpu():
    """pccl_amd.memory without a GPU: no shareable pool, CPU tensors are never shareable, the parallel modules fall
    back to ordinary allocations, and the IPC buffer counters are readable."""
    import contextlib

    import torch

    import pccl_amd as pccl
    assert not pccl.memory.is_shareable(torch.empty(16))
    assert isinstance(pccl.memory.maybe_shareable("cpu"), contextlib.nullcontext)
    st = pccl.memory.ipc_buffer_stats()
    assert set(st) == {"direct_in", "direct_out", "staged_in", "staged_out", "quarantined", "zombie_drains",
                       "preflight_failed", "preflight_passed", "reclaimed", "quarantine_freed"} and \
        all(v >= 0 for v in st.values())
    assert pccl.memory.live_bytes() >= 0
    if not torch.cuda.is_available():
        assert not pccl.memory.available()


def test_communicate_all_drains_every_pipe_concurrently():
    """A process blocked on a full stdout pipe must not stall the wait for another one (the sequential
    ``communicate()`` pattern deadlocks when the process waited on first needs the other one to progress)."""
    import subprocess
    import sys

    from pccl_amd.utils import communicate_all
    big = "import sys; sys.stdout.write('x' * (1 << 20)); sys.stdout.flush()"
    # the first process only exits once the second has written its megabyte (the file appears after the write)
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        flag = f"{d}/done"
        waiter = ("import os, time\nwhile not os.path.exists(%r): time.sleep(0.01)\nprint('ok')" % flag)
        writer = big + "; open(%r, 'w').close()" % flag
        ps = [subprocess.Popen([sys.executable, "-c", c], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
              for c in (waiter, writer)]
        outs = communicate_all(ps, 60)
    assert outs[0][0].strip() == "ok" and len(outs[1][0]) == 1 << 20


def test_communicate_all_deadline_reports_output():
    import subprocess
    import sys

    import pytest

    from pccl_amd.utils import communicate_all
    p = subprocess.Popen([sys.executable, "-c", "import time; print('started', flush=True); time.sleep(60)"],
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    with pytest.raises(TimeoutError, match="started"):
        communicate_all([p], 2.0)
    assert p.poll() is not None
