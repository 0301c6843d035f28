"""Utilities: launch helpers (ports, local master, threaded / multi-process peers) and the profiler."""
from .launch import (DIAG_SIGNALS, communicate_all, free_port, free_ports, local_master, peer_ports,
                     run_threaded_peers, spawn_python, wait_for_world)

__all__ = ["DIAG_SIGNALS", "communicate_all", "free_port", "free_ports", "local_master", "peer_ports",
           "run_threaded_peers", "spawn_python", "wait_for_world"]
