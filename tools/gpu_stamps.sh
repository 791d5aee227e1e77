#!/bin/bash
# Resolve stamps breakdown + a short default bench (diagnostics); extra env via caller.
export TMPDIR=/tmp
KSCHED_LIB_DIR=k8s-1m_amd/ksched/lib/stamps timeout -k 10 200 python -u tools/resolve_stamps.py 1000000 8192 > gpurun_out/stamps_$1.txt 2>&1
cat gpurun_out/stamps_$1.txt | tail -6
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 5 > gpurun_out/bench_$1.json 2>&1; cat gpurun_out/bench_$1.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['extra'])"
