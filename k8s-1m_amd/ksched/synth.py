"""Seeded kwok-shaped synthetic workloads (libksynth.so, include/ksynth.h)."""
from __future__ import annotations

import ctypes as C

from . import _abi

KWOK, HETERO, LABELED, ZONED = 1, 2, 4, 8


class Synth:
    """Owns one ksynth object (node or pod arrays + their strings)."""

    def __init__(self, handle):
        self.lib = _abi.ksynth_lib()
        self.h = handle
        n = C.c_uint32()
        self.nodes = self.lib.ksynth_node_array(self.h, C.byref(n))
        self.n_nodes = n.value
        self.pods = self.lib.ksynth_pod_array(self.h, C.byref(n))
        self.n_pods = n.value
        self.slot_ptr = self.lib.ksynth_slots(self.h, C.byref(n))
        self.n_slots = n.value

    def pods_at(self, start: int):
        """Pointer to pod `start` of the stream."""
        return C.cast(C.addressof(self.pods.contents) + start * C.sizeof(_abi.KsPod), C.POINTER(_abi.KsPod))

    def slots_at(self, start: int):
        return C.cast(C.addressof(self.slot_ptr.contents) + start * 4, C.POINTER(C.c_uint32))

    def close(self):
        if self.h:
            self.lib.ksynth_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def nodes(kind: int, n: int, seed: int) -> Synth:
    return Synth(_abi.ksynth_lib().ksynth_nodes(kind, n, seed))


def pods(kind: int, n: int, seed: int) -> Synth:
    return Synth(_abi.ksynth_lib().ksynth_pods(kind, n, seed))


def prefill(kind: int, n_nodes: int, nodes_seed: int, seed: int, max_fill: float = 0.5) -> Synth:
    return Synth(_abi.ksynth_lib().ksynth_prefill(kind, n_nodes, nodes_seed, seed, max_fill))


def besteffort_pods(n: int) -> Synth:
    return Synth(_abi.ksynth_lib().ksynth_besteffort_pods(n))


def spread_pods(n: int, n_apps: int, seed: int) -> Synth:
    return Synth(_abi.ksynth_lib().ksynth_spread_pods(n, n_apps, seed))


def deploy_pods(n: int, replicas: int, seed: int) -> Synth:
    return Synth(_abi.ksynth_lib().ksynth_deploy_pods(n, replicas, seed))


def deploy_dns_pods(n: int, replicas: int, seed: int) -> Synth:
    return Synth(_abi.ksynth_lib().ksynth_deploy_dns_pods(n, replicas, seed))


def affinity_pods(n: int, n_apps: int, seed: int) -> Synth:
    return Synth(_abi.ksynth_lib().ksynth_affinity_pods(n, n_apps, seed))


def slot_array(n: int, start: int = 0):
    return (C.c_uint32 * n)(*range(start, start + n))


def fnv64(buf, nbytes: int, seed: int = 0) -> int:
    return _abi.ksynth_lib().ksynth_fnv64(buf, nbytes, seed)
