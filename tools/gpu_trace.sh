#!/bin/bash
# Kernel trace + stats of one bench configuration: tools/gpu_trace.sh TAG [bench args...]
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=$1
shift
mkdir -p gpurun_out/$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/$TAG/trace" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-resident --latency-calls 0 "$@" > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || exit $?
python3 - "$R/gpurun_out/$TAG" <<'PY'
import csv, json, sys
d = sys.argv[1]
b = json.load(open(d + "/bench.json"))
print("value", b["value"], "roofline", json.dumps({k: b["roofline"].get(k) for k in ("avg_launch_ms", "ms_per_pod", "frac")}), "resolve_ms", b["extra"]["resolve_ms_per_round"])
for r in list(csv.DictReader(open(d + "/trace/run_kernel_stats.csv")))[:12]:
    print(r["Name"][:70].ljust(70), r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
