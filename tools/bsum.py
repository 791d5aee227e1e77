"""One line per bench JSON (gpurun_out/bench_<tag>_*.json): value, resident, resolve ms / round, passes."""
import glob
import json
import sys

for f in sorted(glob.glob(f"gpurun_out/bench_{sys.argv[1]}_*.json")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(f, "unreadable:", e)
        continue
    x = d["extra"]
    rp = d.get("resolve_profile") or {}
    cyc = rp.get("cycles_per_round", {})
    print(f"{f.split('/')[-1]:38s} {d['value']:>10.0f} res {d.get('value_inputs_resident') or 0:>10.0f} "
          f"resolve {x.get('resolve_ms_per_round')} ms passes {x.get('parallel_commit_passes_per_round')} "
          f"cyc {cyc.get('total', 0):.0f}")
    if len(sys.argv) > 2 and cyc:
        print("   " + " ".join(f"{k}={v:.0f}" for k, v in cyc.items()))
