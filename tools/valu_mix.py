#!/usr/bin/env python3
"""Issue-cost model of the sweep kernels' VALU instruction mix.

The sweep is VALU-issue-bound, so its roofline peak is the SIMDs' issue rate
for ITS instruction mix, not a constant per instruction.  This tool:

  1. compiles ksched_kernels.hip for gfx950 (device code only) and
     disassembles it with llvm-objdump;
  2. for every sweep_kernel<NPL, EXT, LWU> instance takes its per-pod loop
     (the longest backward branch: the loop over the pods of a sweep block,
     nested clause loops counted once) and histograms its VALU opcodes;
  3. prices each opcode with the issue cost measured on MI355X at 4 waves per
     SIMD by tools/valu_issue.hip (profiles/valu_issue.jsonl); an opcode the
     microbenchmark does not cover takes its class's median (VOP1/VOP2
     32-bit moves / adds / logic ops: the 2-cycle class; everything else the
     4-cycle class), and the covered share is reported;
  4. writes profiles/valu_mix.json: per kernel the cost-weighted cycles per
     VALU wave-instruction, keyed by the hash bench.py uses for the kernel
     sources.

bench.py then prices the sweep at peak = 256 CUs x 4 SIMDs x 2.4 GHz /
(cycles per VALU instruction) wave-instructions per second.

  python3 tools/valu_mix.py            (no GPU needed; llvm-objdump from ROCm)
"""
from __future__ import annotations

import collections
import hashlib
import json
import re
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "k8s-1m_amd" / "csrc"
# the hash bench.py keys its per-configuration measurements by (bench.KERNEL_SOURCES)
def bench_kernel_sources(root):
    """bench.py's KERNEL_SOURCES, read from its text (one list for every hash)."""
    import ast
    tree = ast.parse((root / "bench.py").read_text())
    for node in tree.body:
        if isinstance(node, ast.Assign) and any(getattr(t, "id", None) == "KERNEL_SOURCES" for t in node.targets):
            return ast.literal_eval(node.value)
    raise RuntimeError("bench.py has no KERNEL_SOURCES")


KERNEL_SOURCES = bench_kernel_sources(ROOT)
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
HIPCC = "/opt/rocm/bin/hipcc"
WAVES = 4  # the sweep's occupancy: 4 waves per SIMD (5 for the EXT kernels; the costs barely differ)
FAST = re.compile(r"^v_(add|sub|subrev|and|or|xor|not|mov|ashrrev|lshrrev)_(u32|i32|b32|f32)(_e32|_e64)?$|"
                  r"^v_(add|mul)_f32(_e32)?$")


def kernel_src_hash() -> str:
    h = hashlib.sha256()
    for f in KERNEL_SOURCES:
        h.update((ROOT / f).read_bytes())
    return h.hexdigest()[:16]


def load_costs(path: Path):
    costs = {}
    for ln in path.read_text().splitlines():
        if not ln.startswith("{"):
            continue
        r = json.loads(ln)
        if r["waves_per_simd"] == WAVES:
            costs[r["instr"]] = r["cycles_per_instr"]
    return costs


def disassemble() -> list[str]:
    with tempfile.TemporaryDirectory() as d:
        obj = Path(d) / "k.o"
        subprocess.run([HIPCC, "-O3", "--offload-arch=gfx950", "-std=c++17", "-ffp-contract=off",
                        f"-I{ROOT / 'include'}", f"-I{CSRC}", "--cuda-device-only", "--no-gpu-bundle-output",
                        "-c", str(CSRC / "ksched_kernels.hip"), "-o", str(obj)], check=True)
        out = subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", str(obj)], check=True, capture_output=True,
                             text=True).stdout
    return out.splitlines()


def kernels(lines):
    """{mangled name: [(address, opcode, operands)]} for the sweep kernels."""
    out, cur = {}, None
    for ln in lines:
        m = re.match(r"^[0-9a-f]+ <(.*)>:$", ln)
        if m:
            cur = m.group(1) if "sweep_kernel" in m.group(1) else None
            if cur:
                out[cur] = []
            continue
        if cur:
            m = re.match(r"^\s*([a-z_0-9]+)(.*?)//\s*([0-9A-F]+):", ln)
            if m:
                out[cur].append((int(m.group(3), 16), m.group(1), m.group(2).strip()))
    return out


def pod_loop(ins):
    """[lo, hi) of the longest backward branch's loop."""
    best = None
    for a, op, args in ins:
        if not (op.startswith("s_cbranch") or op == "s_branch"):
            continue
        m = re.match(r"^(-?\d+)", args)
        if not m:
            continue
        off = int(m.group(1))
        if off >= 32768:
            off -= 65536
        if off >= 0:
            continue
        t = a + 4 + 4 * off
        if best is None or a - t > best[1] - best[0]:
            best = (t, a + 4)
    return best


def template_args(mangled: str) -> str:
    m = re.search(r"sweep_kernelILi(\d+)ELb(\d)ELi(\d+)E", mangled)
    return f"<{m.group(1)}, {'true' if m.group(2) == '1' else 'false'}, {m.group(3)}>"


SGPR_SRC = re.compile(r"^(s\d|s\[|vcc|exec|m0)")


def cost_of(op: str, costs: dict, fast_med: float, slow_med: float, args: str = ""):
    # the 2-cycle class needs VGPR (or inline-constant) sources: with an SGPR
    # source it issues like the 4-cycle class (tools/valu_issue.hip "(s, v)"
    # rows, profiles/r4/valu_vop.jsonl)
    if FAST.match(op) and any(SGPR_SRC.match(x.strip()) for x in args.split(",")[1:]):
        return slow_med, "v_add_u32 (s, v)" in costs
    base = re.sub(r"_e(32|64)$", "", op)
    for k in (op, base, base.replace("_dpp", "") + "_dpp" if op.endswith("_dpp") else base):
        if k in costs:
            return costs[k], True
    if base.startswith("v_cmp"):
        for k in costs:
            if k.startswith("v_cmp") and k.split("_")[-1] == base.split("_")[-1]:
                return costs[k], True
    return (fast_med if FAST.match(op) else slow_med), False


def main():
    costs = load_costs(ROOT / "profiles" / "valu_issue.jsonl")
    fast = sorted(v for k, v in costs.items() if FAST.match(k))
    slow = sorted(v for k, v in costs.items() if not FAST.match(k) and v < 8)
    fast_med, slow_med = fast[len(fast) // 2], slow[len(slow) // 2]
    res = {"kernel_src": kernel_src_hash(), "waves_per_simd": WAVES, "source": "profiles/valu_issue.jsonl",
           "class_median": {"fast_32bit": fast_med, "other": slow_med}, "kernels": {}}
    for name, ins in kernels(disassemble()).items():
        lo, hi = pod_loop(ins)
        loop = [(op, args) for a, op, args in ins if lo <= a < hi and op.startswith("v_")]
        hist = collections.Counter(op for op, _ in loop)
        n = len(loop)
        cyc = covered = 0.0
        for op, args in loop:
            v, ok = cost_of(op, costs, fast_med, slow_med, args)
            cyc += v
            covered += 1 if ok else 0
        res["kernels"][template_args(name)] = {
            "mangled": name, "loop_valu": n, "cycles_per_valu": round(cyc / n, 4),
            "measured_share": round(covered / n, 4),
            "hist": dict(hist.most_common())}
    out = ROOT / "profiles" / "valu_mix.json"
    out.write_text(json.dumps(res, indent=1) + "\n")
    for k, v in sorted(res["kernels"].items()):
        print(f"sweep_kernel{k}: {v['loop_valu']} VALU in the pod loop, {v['cycles_per_valu']} cycles each "
              f"(measured opcodes {v['measured_share']:.0%})")
    print("->", out.relative_to(ROOT))


if __name__ == "__main__":
    sys.exit(main())
