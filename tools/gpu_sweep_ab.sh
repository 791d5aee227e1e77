#!/bin/bash
# Sweep-bound lines: C3 (default), C3 with 8 nodes per lane, C4 (EXT sweep)
mkdir -p gpurun_out
TAG=${1:-sw}
run() {
  name=$1; shift
  timeout -k 10 240 python -u bench.py --steps 6 --warmup 2 --no-resident --latency-calls 0 --no-cpu-baseline "$@" > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_$name.err || { tail -5 gpurun_out/${TAG}_$name.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_$name.json'));e=d['extra'];print('$name', d['value'], d['roofline']['avg_launch_ms'], e['resolve_ms_per_round'], e['pods_per_round_resolved'], e['speculated_rounds_wasted'])"
}
run c3
run c3npl8 --nodes-per-lane 8
run c4 --kind labeled
