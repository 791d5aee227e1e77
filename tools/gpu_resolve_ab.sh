#!/bin/bash
# Resolve-bound lines (C2 100k, one 8-GPU shard of C3 = 125k nodes) and the
# default C3 line, each printing pods/s, sweep / resolve ms, pods per round.
mkdir -p gpurun_out
TAG=${1:-ab}
run() {
  name=$1; shift
  timeout -k 10 240 python -u bench.py --steps 6 --warmup 2 --no-resident --latency-calls 0 --no-cpu-baseline "$@" > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_$name.err || { tail -5 gpurun_out/${TAG}_$name.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_$name.json'));e=d['extra'];print('$name', d['value'], d['roofline']['avg_launch_ms'], e['resolve_ms_per_round'], e['pods_per_round_resolved'], e['speculated_rounds_wasted'])"
}
run c3
run c2 --nodes 100000 --batch 100000 --steps 3 --warmup 1
run shard125k --nodes 125000
run c4 --kind labeled
run kwok512 --kind kwok --topk 512
