"""The C-ABI boundary: libraries load, every symbol include/*.h declares is
exported, and the ctypes mirror matches the C struct layouts (no GPU needed:
only loads and layout checks, no compute calls)."""
import ctypes as C
import re
import subprocess
from pathlib import Path

import pytest

from ksched import _abi

ROOT = Path(__file__).resolve().parent.parent


def declared(header: str, prefix: str):
    text = (ROOT / "include" / header).read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(" + prefix + r"[a-z0-9_]+)\s*\(", text)))


def test_header_symbols_match_mirror():
    assert declared("ksched.h", "ks_") == sorted(_abi.KSCHED_SYMBOLS)
    assert declared("ksynth.h", "ksynth_") == sorted(_abi.KSYNTH_SYMBOLS)
    assert declared("ksgather.h", "ksg_") == sorted(_abi.KSGATHER_SYMBOLS)


def test_libksched_exports_every_declared_symbol():
    lib = _abi.ksched_lib()
    for name in declared("ksched.h", "ks_"):
        assert hasattr(lib, name), name
    assert lib.ks_abi_version() == 6


def test_libksgather_exports_every_declared_symbol():
    lib = _abi.ksgather_lib()
    for name in declared("ksgather.h", "ksg_"):
        assert hasattr(lib, name), name


def test_libksynth_exports_every_declared_symbol():
    lib = _abi.ksynth_lib()
    for name in declared("ksynth.h", "ksynth_"):
        assert hasattr(lib, name), name


def test_shared_objects_are_gfx950_and_link_rccl():
    so = ROOT / "k8s-1m_amd/ksched/lib/libksched.so"
    out = subprocess.run(["readelf", "-d", str(so)], capture_output=True, text=True).stdout
    assert "librccl" in out and "libamdhip64" in out
    blob = so.read_bytes()
    assert b"gfx950" in blob  # code object target


C_PROBE = r"""
#include <stdio.h>
#include <stddef.h>
#include "ksched.h"
#define S(t) printf(#t " %zu\n", sizeof(t));
#define O(t, f) printf(#t "." #f " %zu\n", offsetof(t, f));
int main(void) {
  S(ks_label) S(ks_taint) S(ks_toleration) S(ks_node) S(ks_container) S(ks_requirement) S(ks_term)
  S(ks_preferred_term) S(ks_pod) S(ks_event) S(ks_result) S(ks_node_score) S(ks_node_state) S(ks_config) S(ks_stats)
  S(ks_label_selector) S(ks_spread_constraint) S(ks_resource) S(ks_image) S(ks_pod_affinity_term)
  O(ks_pod, affinity_terms) O(ks_pod, n_namespace_labels) O(ks_pod_affinity_term, kind) O(ks_pod_affinity_term, weight)
  O(ks_config, hard_pod_affinity_weight) O(ks_node_score, affinity_pod_score) O(ks_result, flags)
  O(ks_node, extended) O(ks_node, n_extended) O(ks_container, extended) O(ks_container, n_extended)
  O(ks_pod, labels) O(ks_pod, spread) O(ks_pod, spread_defaulted) O(ks_spread_constraint, max_skew)
  O(ks_spread_constraint, node_taints_policy) O(ks_node_score, spread_score) O(ks_config, weight_topology_spread)
  O(ks_node, labels) O(ks_node, n_labels) O(ks_node, unschedulable)
  O(ks_pod, node_name) O(ks_pod, overhead_milli_cpu) O(ks_pod, n_containers) O(ks_pod, has_required)
  O(ks_pod, has_preferred) O(ks_pod, has_overhead)
  O(ks_result, total_score) O(ks_result, fail_counts) O(ks_result, flags)
  O(ks_event, pod) O(ks_event, node) S(ks_node_info) O(ks_node_info, generation) O(ks_node_info, node)
  O(ks_node_score, total_score) O(ks_config, weight_fit) O(ks_config, weight_image)
  O(ks_stats, sweep_ms) O(ks_stats, resolve_launches)
  O(ks_config, resolve_mode) O(ks_config, early_fix) O(ks_config, sync_timeout_ms) O(ks_config, spread_replica_runs)
  O(ks_stats, spread_pods) O(ks_stats, replica_pods) O(ks_stats, replica_ms)
  return 0;
}
"""


def test_struct_layouts_match_c(tmp_path):
    src = tmp_path / "probe.c"
    src.write_text(C_PROBE)
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-I", str(ROOT / "include"), str(src), "-o", str(exe)], check=True)
    lines = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n")
    got = dict(line.rsplit(" ", 1) for line in lines if line)
    for name, cls in _abi.STRUCTS.items():
        assert int(got[name]) == C.sizeof(cls), name
    for key, val in got.items():
        if "." in key:
            t, f = key.split(".")
            assert getattr(_abi.STRUCTS[t], f).offset == int(val), key


def test_open_without_device_fails_cleanly():
    # no HIP device in the CPU container: ks_open must return KS_ERR_DEVICE, not crash
    lib = _abi.ksched_lib()
    cfg = _abi.KsConfig()
    lib.ks_config_default(C.byref(cfg))
    ctx = C.c_void_p()
    st = lib.ks_open(C.byref(cfg), C.byref(ctx))
    if st == 0:
        lib.ks_close(ctx)
        pytest.skip("a GPU is present")
    assert st == 2
    assert not ctx.value


def test_invalid_configs_rejected():
    lib = _abi.ksched_lib()
    for field, value in (("node_capacity", 0), ("nodes_per_lane", 3), ("pods_per_round", 100000),
                         ("topk", 513), ("world_size", 2)):
        cfg = _abi.KsConfig()
        lib.ks_config_default(C.byref(cfg))
        setattr(cfg, field, value)
        if field == "world_size":
            cfg.rank = 5
        ctx = C.c_void_p()
        assert lib.ks_open(C.byref(cfg), C.byref(ctx)) == 1, field
