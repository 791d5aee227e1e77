#!/usr/bin/env python3
"""Summarise the rocprofv3 --pmc passes of tools/gpu.sh pmc into profiles/pmc/<key>.json.

    python tools/pmc_summary.py gpurun_out/pmc_r2c3 --tag r2c3 --out-dir profiles/pmc

<key> is the bench configuration (bench.py's extra.pmc_key, read from the
passes' own bench lines), and the file records the kernel-source hash it was
measured on (bench.py's roofline ignores a summary whose hash differs).

Main sweep dispatches only: the sweep kernel's dispatches with the largest
grid (FIX-mode re-sweeps of flagged pods use the same kernel on a smaller
grid).  Per evaluation (pod x node, evaluations per launch from the bench line):

* ``valu_wave_instr_per_eval`` = SQ_INSTS_VALU / evaluations (x 64 = lane-ops);
* ``hbm_bytes_per_eval`` = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 / evaluations:
  FETCH_SIZE / WRITE_SIZE are in KB; the x2 is MI355X_MICROARCH.md's gfx950
  correction (FETCH_SIZE tallies 128-B fabric reads at 64 B).  These are L2
  memory-side bytes (Infinity-Cache hits counted): an upper bound on HBM bytes;
* ``valu_cycles_per_instr`` = 4 x SQ_ACTIVE_INST_VALU / SQ_INSTS_VALU: cycles a
  wave64 VALU instruction occupies its SIMD (the counter is in quad-cycles);
* ``valu_busy`` = SQ_ACTIVE_INST_VALU / (GRBM_GUI_ACTIVE / 8 XCDs x 256 CUs x 4
  SIMDs / 4): the share of SIMD quad-cycles executing VALU;
* ``lds_bank_conflict_ratio`` = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE;
* ``clock_ghz`` = GRBM_GUI_ACTIVE / 8 XCDs / kernel duration.
"""
import argparse
import csv
import hashlib
import json
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
SWEEP = "sweep_kernel"
# the same list, in the same order, as bench.py's KERNEL_SOURCES (the bench
# uses a summary only when the hashes agree)
def bench_kernel_sources(root):
    """bench.py's KERNEL_SOURCES, read from its text (one list for every hash)."""
    import ast
    tree = ast.parse((root / "bench.py").read_text())
    for node in tree.body:
        if isinstance(node, ast.Assign) and any(getattr(t, "id", None) == "KERNEL_SOURCES" for t in node.targets):
            return ast.literal_eval(node.value)
    raise RuntimeError("bench.py has no KERNEL_SOURCES")


KERNEL_SOURCES = bench_kernel_sources(ROOT)


def kernel_src_hash() -> str:
    h = hashlib.sha256()
    for f in KERNEL_SOURCES:
        h.update((ROOT / f).read_bytes())
    return h.hexdigest()[:16]


def load(dirpath: Path):
    """kernel -> grid -> counter -> [values]; kernel -> grid -> [durations ms]."""
    per = defaultdict(lambda: defaultdict(lambda: defaultdict(list)))
    dur = defaultdict(lambda: defaultdict(list))
    for f in sorted(dirpath.rglob("*counter_collection.csv")):
        seen = set()
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k, g = row["Kernel_Name"], int(row["Grid_Size"])
                per[k][g][row["Counter_Name"]].append(float(row["Counter_Value"]))
                key = (f, row["Dispatch_Id"])
                if key not in seen:
                    seen.add(key)
                    dur[k][g].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-6)
    return per, dur


def bench_line(dirpath: Path):
    for f in sorted(dirpath.glob("p*.json")):
        for ln in f.read_text().splitlines():
            ln = ln.strip()
            if ln.startswith("{"):
                return json.loads(ln)
    raise SystemExit(f"no bench line under {dirpath}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--tag", required=True)
    ap.add_argument("--out-dir", required=True)
    a = ap.parse_args()
    d = Path(a.dir)
    line = bench_line(d)
    key = line["extra"]["pmc_key"]
    evals = line["roofline"]["evals_per_launch"]
    per, dur = load(d)
    kernels = {}
    for k, grids in per.items():
        name = k.split("(")[0]
        g = max(grids)  # the largest grid of this kernel
        ctrs = grids[g]
        kernels[name] = {c: sum(v) / len(v) for c, v in ctrs.items()}
        kernels[name]["grid"] = g
        kernels[name]["dispatches"] = max(len(v) for v in ctrs.values())
        ds = dur[k][g]
        kernels[name]["avg_ms_under_pmc"] = sum(ds) / len(ds) if ds else None
    out = {"tag": a.tag, "key": key, "kernel_src": kernel_src_hash(), "evals_per_launch": evals,
           "workload": line["config"]["workload"],
           "source": f"rocprofv3 --pmc passes (tools/gpu.sh pmc), {a.dir}", "kernels": kernels}
    sweep = {n: v for n, v in kernels.items() if SWEEP in n}
    if sweep:
        name, s = max(sweep.items(), key=lambda kv: kv[1].get("dispatches", 0))
        out["sweep_kernel"] = name
        if "SQ_INSTS_VALU" in s:
            out["valu_wave_instr_per_eval"] = s["SQ_INSTS_VALU"] / evals
            out["valu_lane_ops_per_eval"] = round(s["SQ_INSTS_VALU"] * 64 / evals, 2)
        if "SQ_INSTS_SALU" in s:
            out["salu_instr_per_valu_instr"] = round(s["SQ_INSTS_SALU"] / max(1.0, s.get("SQ_INSTS_VALU", 0)), 4)
        if "FETCH_SIZE" in s and "WRITE_SIZE" in s:
            b = 2 * s["FETCH_SIZE"] * 1024 + s["WRITE_SIZE"] * 1024
            out["hbm_bytes_per_launch"] = round(b)
            out["hbm_bytes_per_eval"] = b / evals
        if "SQ_LDS_BANK_CONFLICT" in s and s.get("SQ_LDS_IDX_ACTIVE"):
            out["lds_bank_conflict_ratio"] = round(s["SQ_LDS_BANK_CONFLICT"] / s["SQ_LDS_IDX_ACTIVE"], 5)
        if "GRBM_GUI_ACTIVE" in s and s.get("avg_ms_under_pmc"):
            out["clock_ghz"] = round(s["GRBM_GUI_ACTIVE"] / 8 / (s["avg_ms_under_pmc"] * 1e-3) / 1e9, 3)
        f64 = [s.get(c) for c in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                                  "SQ_INSTS_VALU_TRANS_F64")]
        if all(v is not None for v in f64) and s.get("SQ_INSTS_VALU"):
            n64 = sum(f64)
            out["valu_f64_share"] = round(n64 / s["SQ_INSTS_VALU"], 4)
            for c in ("SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64", "SQ_INSTS_VALU_CVT"):
                if c in s:
                    out[c.lower() + "_share"] = round(s[c] / s["SQ_INSTS_VALU"], 4)
        if "SQ_ACTIVE_INST_VALU" in s and s.get("SQ_INSTS_VALU"):
            # cycles a wave64 VALU instruction occupies its SIMD (quad-cycle counter x 4)
            out["valu_cycles_per_instr"] = round(4 * s["SQ_ACTIVE_INST_VALU"] / s["SQ_INSTS_VALU"], 3)
        if "SQ_ACTIVE_INST_VALU" in s and s.get("GRBM_GUI_ACTIVE"):
            simd_quads = s["GRBM_GUI_ACTIVE"] / 8 * 256 * 4 / 4
            out["valu_busy"] = round(s["SQ_ACTIVE_INST_VALU"] / simd_quads, 4)
    od = Path(a.out_dir)
    od.mkdir(parents=True, exist_ok=True)
    (od / f"{key}.json").write_text(json.dumps(out, indent=1, sort_keys=True) + "\n")
    print(json.dumps({k: v for k, v in out.items() if k != "kernels"}, indent=1))


if __name__ == "__main__":
    main()
