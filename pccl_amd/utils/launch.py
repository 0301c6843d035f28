"""Launch helpers for local PCCL runs: free ports, an in-process master, threaded and multi-process peers.

The reference drives its integration tests by spawning the master and peers as subprocesses on fixed ports
(`/root/reference/python/tests/end_to_end/test_end_to_end.py`); here every run picks free ports so that tests,
the bench and the smoke check can run side by side on one host.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import threading
import time
from contextlib import contextmanager
from typing import Callable, Dict, Iterator, List, Optional, Sequence

REPO_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# sent to peers that overran their deadline before they are killed: every thread's native backtrace on stderr
# (spawn_python turns on PCCL_DEBUG_BACKTRACE_SIGNAL)
DIAG_SIGNALS = (signal.SIGUSR2,)


def free_port(host: str = "127.0.0.1") -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((host, 0))
        return s.getsockname()[1]


def free_ports(n: int) -> List[int]:
    """n distinct free ports (held open together while probing so they cannot collide)."""
    socks, ports = [], []
    try:
        for _ in range(n):
            s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            s.bind(("127.0.0.1", 0))
            socks.append(s)
            ports.append(s.getsockname()[1])
    finally:
        for s in socks:
            s.close()
    return ports


def peer_ports(n_peers: int) -> List[Dict[str, int]]:
    """Per-peer listen ports (p2p / shared-state / benchmark); the library bumps a port that is taken anyway."""
    ports = free_ports(3 * n_peers)
    return [{"p2p_listen_port": ports[3 * i], "shared_state_listen_port": ports[3 * i + 1],
             "benchmark_listen_port": ports[3 * i + 2]} for i in range(n_peers)]


@contextmanager
def local_master(port: Optional[int] = None) -> Iterator[str]:
    """Runs a MasterNode on 127.0.0.1 in this process; yields its ``ip:port``."""
    from ..api import MasterNode
    port = port or free_port()
    master = MasterNode(f"127.0.0.1:{port}")
    master.run()
    try:
        yield f"127.0.0.1:{port}"
    finally:
        master.interrupt()
        master.await_termination()
        del master


def wait_for_world(comm, world_size: int, timeout: float = 60.0, poll: float = 0.02) -> None:
    """Accept pending peers until the run has ``world_size`` members (every existing peer must vote)."""
    from ..api import Attribute
    t0 = time.time()
    while comm.get_attribute(Attribute.GLOBAL_WORLD_SIZE) < world_size:
        if comm.are_peers_pending():
            comm.update_topology()
        else:
            time.sleep(poll)
        if time.time() - t0 > timeout:
            raise TimeoutError(f"world did not reach {world_size} peers in {timeout} s")


def run_threaded_peers(n: int, fn: Callable[[int, object], object], *, address: str, timeout: float = 120.0,
                       peer_group: int = 0, connect_stagger: float = 0.0,
                       comm_kwargs=None) -> List[object]:
    """Runs ``fn(rank, communicator)`` on n peers, one thread each, all connected to ``address``.

    ``comm_kwargs``: Communicator keyword arguments, a dict for every peer or a callable ``rank -> dict``.

    Each peer waits until the world has n members before calling ``fn``. Exceptions are re-raised in the caller.
    """
    from ..api import Communicator
    ports = peer_ports(n)
    results: List[object] = [None] * n
    errors: List[Optional[BaseException]] = [None] * n
    comms: List[object] = [None] * n

    def body(r: int):
        try:
            kw = comm_kwargs(r) if callable(comm_kwargs) else comm_kwargs
            c = Communicator(address, peer_group, **ports[r], **(kw or {}))
            comms[r] = c
            c.connect(n_attempts=10)
            wait_for_world(c, n, timeout=timeout)
            results[r] = fn(r, c)
        except BaseException as e:  # noqa: BLE001 - re-raised below
            errors[r] = e

    threads = [threading.Thread(target=body, args=(r,), daemon=True) for r in range(n)]
    for t in threads:
        t.start()
        if connect_stagger:
            time.sleep(connect_stagger)
    deadline = time.time() + timeout
    for t in threads:
        t.join(timeout=max(0.1, deadline - time.time()))
    try:
        if any(t.is_alive() for t in threads):
            raise TimeoutError(f"threaded peers did not finish within {timeout} s")
        for e in errors:
            if e is not None:
                raise e
        return results
    finally:
        if not any(t.is_alive() for t in threads):
            for c in comms:
                if c is not None:
                    c.destroy()


def spawn_python(args: Sequence[str], env: Optional[Dict[str, str]] = None, **kw) -> subprocess.Popen:
    """Starts ``python <args>`` with the repo on PYTHONPATH (and the IPC mode the box's driver needs)."""
    e = dict(os.environ)
    e["PYTHONPATH"] = REPO_ROOT + os.pathsep + e.get("PYTHONPATH", "")
    e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    e.setdefault("PCCL_DEBUG_BACKTRACE_SIGNAL", "1")
    if env:
        e.update(env)
    return subprocess.Popen([sys.executable, *args], env=e, **kw)


def communicate_all(procs: Sequence[subprocess.Popen], timeout: float,
                    diag_signals: Sequence[int] = ()) -> List[tuple]:
    """``communicate()`` on every process at once: each one's pipes are drained by its own thread, so a peer that
    writes more than a pipe buffer while another is being waited on cannot block (and stall the collective that the
    waited-on peer is in). On timeout the live processes get ``diag_signals`` (e.g. SIGUSR1 for a faulthandler
    dump, SIGUSR2 for PCCL_DEBUG_BACKTRACE_SIGNAL), then SIGKILL, and ``TimeoutError`` is raised with every
    process's output tail in its message."""
    outs: List[Optional[tuple]] = [None] * len(procs)

    def drain(k: int):
        outs[k] = procs[k].communicate()

    threads = [threading.Thread(target=drain, args=(k,), daemon=True) for k in range(len(procs))]
    for t in threads:
        t.start()
    deadline = time.time() + timeout
    for t in threads:
        t.join(timeout=max(0.0, deadline - time.time()))
    if any(t.is_alive() for t in threads):
        for sig in diag_signals:
            for p in procs:
                if p.poll() is None:
                    try:
                        p.send_signal(sig)
                    except OSError:
                        pass
            time.sleep(2.0)
        for p in procs:
            if p.poll() is None:
                p.kill()
        for t in threads:
            t.join(timeout=30)
        tails = []
        for k, o in enumerate(outs):
            o = o or ("", "")
            tails.append(f"--- process {k} (rc {procs[k].returncode}) stdout:\n{str(o[0])[-3000:]}\n"
                         f"--- stderr:\n{str(o[1])[-6000:]}")
        raise TimeoutError(f"processes did not finish within {timeout} s\n" + "\n".join(tails))
    return [o if o is not None else ("", "") for o in outs]
