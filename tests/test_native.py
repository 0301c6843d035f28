"""Native (C/C++) tests: internal unit tests, C-API peers against the standalone ccoip_master executable
(reference tests/basic_reduce_test + tests/concurrent_reduce_test), C99 header compatibility, sanitizer build."""
import json
import os
import shutil
import subprocess
import sys

import pytest

from pccl_amd.utils import DIAG_SIGNALS, communicate_all, free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "build")
MASTER = os.path.join(ROOT, "pccl_amd", "lib", "ccoip_master")
STREAM_PEERS = os.path.join(BUILD, "tests", "pccl_stream_ordered_peers")
HOSTDEV = os.path.join(ROOT, "pccl_amd", "lib", "libpccl_hostdev.so")


def _ensure_built():
    need = [os.path.join(BUILD, "tests", "pccl_unit_tests"), os.path.join(BUILD, "tests", "pccl_reduce_peer"), MASTER]
    if not all(os.path.exists(p) for p in need + [STREAM_PEERS, HOSTDEV]):
        import __graft_entry__
        __graft_entry__.build()
    return need


def test_unit_tests():
    unit, _, _ = _ensure_built()
    r = subprocess.run([unit], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failure(s)" in r.stdout


@pytest.mark.parametrize("world,num_ops,n,pool,inflight", [(2, 4, 1 << 20, 1, 4), (3, 8, 100_003, 2, 3),
                                                           (4, 16, 65_536, 4, 16)])
def test_c_api_peers_with_standalone_master(world, num_ops, n, pool, inflight):
    _, peer, master = _ensure_built()
    port = free_port()
    m = subprocess.Popen([master, "--port", str(port)], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    try:
        assert "listening" in m.stdout.readline()
        peers = [subprocess.Popen([peer, str(port), str(world), "3", str(num_ops), str(n), str(pool), str(inflight)],
                                  stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for _ in range(world)]
        outs = communicate_all(peers, 180, DIAG_SIGNALS)
        for p, (o, e) in zip(peers, outs):
            assert p.returncode == 0, e[-2000:]
            steps = [json.loads(x) for x in o.splitlines() if x.startswith("{")]
            assert len(steps) == 3 and all(s["world"] == world for s in steps)
    finally:
        m.terminate()
        m.wait(timeout=30)
    assert m.returncode == 0  # SIGTERM -> clean interrupt + await termination


def _hostdev_env(plugin, **extra):
    # the host-emulated device backend: every pointer is "device" memory, streams are worker threads, no xGMI
    env = dict(os.environ)
    env.update(extra)
    env.update(PCCL_HIP_PLUGIN=plugin, PCCL_HOSTDEV_ALL_DEVICE="1", PCCL_DISABLE_IPC="1")
    env.pop("PCCL_DISABLE_HIP", None)
    return env


@pytest.mark.parametrize("peers,ops,n", [(2, 20, 1 << 20), (3, 12, 100_003)])
def test_stream_ordered_threaded_peers_hostdev(peers, ops, n):
    """Threaded peers of one process in the stream-ordered start path (pcclxAllReduce[Async]OnStream; the shared
    null stream and per-peer streams, producers that finish after the call returned) on the host-emulated device
    backend: exact sums on the device ring (docs/STREAM_QUERY_CRASH.md)."""
    _ensure_built()
    r = subprocess.run([STREAM_PEERS, str(peers), str(ops), str(n)], capture_output=True, text=True, timeout=300,
                       env=_hostdev_env(HOSTDEV))
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res == {"peers": peers, "ops": ops, "elements": n, "bad": 0}


EMULATED_DEVICE_SUITES = ["test_allreduce.py", "test_allreduce_matrix.py", "test_shared_state.py",
                          "test_shared_state_scenarios.py", "test_ddp_overlap.py", "test_diloco.py"]


def test_cpu_suites_on_emulated_device_rings():
    """The CPU all-reduce matrix, shared-state and DDP / DiLoCo suites with every buffer taken for device memory on
    the host-emulated backend: the same scenarios then run through the device rings (plain and quantized pipelines,
    OpSenders / RingRx / step slots, staging, the shared-state device paths) instead of the host ring."""
    _ensure_built()
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider", "-m", "not gpu",
                        *[os.path.join(ROOT, "tests", t) for t in EMULATED_DEVICE_SUITES]],
                       capture_output=True, text=True, timeout=900, cwd=ROOT, env=_hostdev_env(HOSTDEV))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]


def test_c99_header_compat(tmp_path):
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    src = os.path.join(ROOT, "tests", "native", "c99_compat.c")
    r = subprocess.run([cc, "-std=c99", "-pedantic", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include"),
                        "-c", src, "-o", str(tmp_path / "c99.o")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


@pytest.mark.skipif(os.environ.get("PCCL_TEST_SANITIZE") != "1", reason="set PCCL_TEST_SANITIZE=1 (slow build)")
def test_sanitizer_build_unit_and_peers():
    """ASan + UBSan build of the host library (reference PCCL_SANITIZE_TESTS); runs the unit tests and a 3-peer
    C-API reduce with the sanitized library."""
    bdir = os.path.join(ROOT, "build-asan")
    out = os.path.join(bdir, "lib")
    subprocess.run(["cmake", "-S", ROOT, "-B", bdir, "-G", "Ninja", "-DPCCL_SANITIZE=ON", "-DPCCL_BUILD_HIP_SUPPORT=OFF",
                    f"-DPCCL_OUTPUT_DIR={out}", "-DCMAKE_BUILD_TYPE=RelWithDebInfo"], check=True, capture_output=True)
    subprocess.run(["ninja", "-C", bdir, "-j", "8"], check=True, capture_output=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([os.path.join(bdir, "tests", "pccl_unit_tests")], capture_output=True, text=True, env=env,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    port = free_port()
    m = subprocess.Popen([os.path.join(out, "ccoip_master"), "--port", str(port)], stdout=subprocess.PIPE, text=True,
                         env=env)
    try:
        m.stdout.readline()
        peers = [subprocess.Popen([os.path.join(bdir, "tests", "pccl_reduce_peer"), str(port), "3", "3", "4",
                                   "200003", "2"], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
                 for _ in range(3)]
        for p in peers:
            o, e = p.communicate(timeout=300)
            assert p.returncode == 0, e[-3000:]
    finally:
        m.terminate()
        m.wait(timeout=60)


@pytest.mark.skipif(os.environ.get("PCCL_TEST_SANITIZE") != "1", reason="set PCCL_TEST_SANITIZE=1 (slow build)")
@pytest.mark.timeout(1800)
def test_tsan_build_unit_and_peers(tmp_path):
    """ThreadSanitizer build (-DPCCL_SANITIZE_THREAD=ON, ROCm's clang: GCC 11's libtsan does not intercept
    pthread_cond_clockwait, so every condition-variable wait looks like a lost unlock): the unit tests and a 3-peer
    C-API run with concurrent ops (master, RX threads, striped senders, collective workers) must report no races."""
    bdir = os.path.join(ROOT, "build-tsan")
    out = os.path.join(bdir, "lib")
    clang = "/opt/rocm/llvm/bin/clang"
    env_cc = dict(os.environ, CC=clang, CXX=clang + "++")
    subprocess.run(["cmake", "-S", ROOT, "-B", bdir, "-G", "Ninja", "-DPCCL_SANITIZE_THREAD=ON",
                    "-DPCCL_BUILD_HIP_SUPPORT=OFF", f"-DPCCL_OUTPUT_DIR={out}", "-DCMAKE_BUILD_TYPE=RelWithDebInfo"],
                   check=True, capture_output=True, env=env_cc)
    subprocess.run(["ninja", "-C", bdir, "-j", "8"], check=True, capture_output=True)
    logs = tmp_path / "tsan"
    env = dict(os.environ, TSAN_OPTIONS=f"halt_on_error=0 report_signal_unsafe=0 die_after_fork=0 log_path={logs}")
    r = subprocess.run([os.path.join(bdir, "tests", "pccl_unit_tests")], capture_output=True, text=True, env=env,
                       timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    port = free_port()
    m = subprocess.Popen([os.path.join(out, "ccoip_master"), "--port", str(port)], stdout=subprocess.PIPE, text=True,
                         env=env)
    try:
        m.stdout.readline()
        peers = [subprocess.Popen([os.path.join(bdir, "tests", "pccl_reduce_peer"), str(port), "3", "6", "4",
                                   "200003", "3"], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
                 for _ in range(3)]
        for p in peers:
            o, e = p.communicate(timeout=600)
            assert p.returncode == 0, e[-3000:]
    finally:
        m.terminate()
        m.wait(timeout=60)
    # two threaded peers in the stream-ordered start path on the host-emulated device backend (round-5 crash setup)
    r = subprocess.run([os.path.join(bdir, "tests", "pccl_stream_ordered_peers"), "2", "16", "262147"],
                       capture_output=True, text=True, timeout=900,
                       env=_hostdev_env(os.path.join(out, "libpccl_hostdev.so"), TSAN_OPTIONS=env["TSAN_OPTIONS"]))
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    # the Python-level scenarios (threaded peers in one process: all-reduce matrix, shared-state protocol; peer
    # processes stopped / black-holed mid-op: the liveness protocol's heartbeats, watchdog and teardown) against
    # the TSan library, with the clang TSan runtime preloaded into the (uninstrumented) interpreter
    import glob
    rt = sorted(glob.glob("/opt/rocm/llvm/lib/clang/*/lib/linux/libclang_rt.tsan-x86_64.so"))[-1]
    py_env = dict(env, PCCL_DISABLE_HIP="1", PCCL_LIBRARY=os.path.join(out, "libpccl.so"), LD_PRELOAD=rt,
                  TSAN_OPTIONS=env["TSAN_OPTIONS"] + " ignore_noninstrumented_modules=1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider", "-m", "not gpu",
                        os.path.join(ROOT, "tests", "test_allreduce.py"),
                        os.path.join(ROOT, "tests", "test_shared_state_scenarios.py"),
                        os.path.join(ROOT, "tests", "test_liveness.py")],
                       capture_output=True, text=True, env=py_env, timeout=900, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    # the same Python suites through the device rings of the host-emulated backend (TSan build of it)
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider", "-m", "not gpu",
                        *[os.path.join(ROOT, "tests", t) for t in EMULATED_DEVICE_SUITES]],
                       capture_output=True, text=True, timeout=1200, cwd=ROOT,
                       env=_hostdev_env(os.path.join(out, "libpccl_hostdev.so"), **py_env))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    # peer processes stopped / killed inside device ring steps on the emulated backend: the abort, drain and restore
    # paths of the plain and quantized device rings
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider", "-m", "not gpu", "-k",
                        "emulated", os.path.join(ROOT, "tests", "test_fault_tolerance.py"),
                        os.path.join(ROOT, "tests", "test_liveness.py")],
                       capture_output=True, text=True, timeout=1800, cwd=ROOT,
                       env=dict({k: v for k, v in py_env.items() if k != "PCCL_DISABLE_HIP"},
                                PCCL_TEST_HOSTDEV=os.path.join(out, "libpccl_hostdev.so"), PCCL_TEST_TIME_SCALE="3"))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    reports = [f.read_text() for f in tmp_path.glob("tsan*")]
    assert not any("WARNING: ThreadSanitizer" in t for t in reports), "\n".join(reports)[:5000]
