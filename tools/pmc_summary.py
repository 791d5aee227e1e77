#!/usr/bin/env python3
"""Summarise the rocprofv3 --pmc passes of tools/pmc.sh into profiles/<tag>_pmc.json.

    python tools/pmc_summary.py gpurun_out/pmc_r1e --tag r1e --out profiles/pmc_sweep.json

Per kernel (averaged over its dispatches): every collected counter, plus for
the sweep kernel the quantities bench.py's roofline reports:

* ``hbm_bytes_per_sweep_launch`` = 2 x FETCH_SIZE x 1024 + WRITE_SIZE x 1024.
  FETCH_SIZE / WRITE_SIZE are in KB.  The x2 is MI355X_MICROARCH.md's gfx950
  correction (FETCH_SIZE tallies 128-B fabric reads at 64 B); the sweep's
  loads are 8-B and 4-B per lane, outside the guide's calibrated 16-B case, so
  the script also checks it against the kernel's own known read volume
  (pod groups x node-table bytes), see ``fetch_calibration``.  These are L2
  memory-side bytes: Infinity-Cache hits are counted, so the figure is an
  upper bound on true HBM traffic (the 56 MB node table stays L3-resident).
* ``valu_lane_ops_per_eval`` = SQ_INSTS_VALU x 64 / evaluations per launch.
* ``lds_bank_conflict_ratio`` = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE.
* ``clock_ghz`` = GRBM_GUI_ACTIVE / 8 XCDs / kernel duration.
"""
import argparse
import csv
import json
from collections import defaultdict
from pathlib import Path

SWEEP = "sweep_kernel"


def load(dirpath: Path):
    per = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> values
    dur = defaultdict(list)
    for f in sorted(dirpath.rglob("*counter_collection.csv")):
        seen = set()
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row["Kernel_Name"]
                per[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
                key = (row["Dispatch_Id"], k)
                if key not in seen:
                    seen.add(key)
                    dur[k].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-6)
    return per, dur


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--tag", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--evals-per-launch", type=float, default=256 * 1_000_000,
                    help="(pod, node) evaluations per sweep launch of the profiled bench")
    ap.add_argument("--table-bytes", type=float, default=56 * 1_000_000, help="node-table bytes one pod group reads")
    ap.add_argument("--pod-groups", type=int, default=9, help="pod groups per sweep launch (host geometry)")
    a = ap.parse_args()
    per, dur = load(Path(a.dir))
    kernels = {}
    for k, ctrs in per.items():
        name = k.split("(")[0]
        kernels[name] = {c: sum(v) / len(v) for c, v in ctrs.items()}
        kernels[name]["dispatches"] = max(len(v) for v in ctrs.values())
        d = dur.get(k, [])
        kernels[name]["avg_ms_under_pmc"] = sum(d) / len(d) if d else None
    sweep = {n: v for n, v in kernels.items() if SWEEP in n}
    out = {"tag": a.tag, "source": f"rocprofv3 --pmc passes (tools/pmc.sh), {a.dir}", "kernels": kernels}
    if sweep:
        name, s = max(sweep.items(), key=lambda kv: kv[1].get("dispatches", 0))
        fetch = s.get("FETCH_SIZE")
        write = s.get("WRITE_SIZE")
        if fetch is not None and write is not None:
            out["hbm_bytes_per_sweep_launch"] = round(2 * fetch * 1024 + write * 1024)
            out["fetch_calibration"] = {
                "expected_read_bytes": a.pod_groups * a.table_bytes,
                "fetch_size_x2_bytes": 2 * fetch * 1024,
                "ratio": round(2 * fetch * 1024 / (a.pod_groups * a.table_bytes), 4),
            }
        if "SQ_INSTS_VALU" in s:
            out["valu_lane_ops_per_eval"] = round(s["SQ_INSTS_VALU"] * 64 / a.evals_per_launch, 2)
        if "SQ_LDS_BANK_CONFLICT" in s and s.get("SQ_LDS_IDX_ACTIVE"):
            out["lds_bank_conflict_ratio"] = round(s["SQ_LDS_BANK_CONFLICT"] / s["SQ_LDS_IDX_ACTIVE"], 5)
        if "GRBM_GUI_ACTIVE" in s and s.get("avg_ms_under_pmc"):
            out["clock_ghz"] = round(s["GRBM_GUI_ACTIVE"] / 8 / (s["avg_ms_under_pmc"] * 1e-3) / 1e9, 3)
        out["sweep_kernel"] = name
    Path(a.out).write_text(json.dumps(out, indent=1, sort_keys=True) + "\n")
    print(json.dumps({k: v for k, v in out.items() if k != "kernels"}, indent=1))


if __name__ == "__main__":
    main()
