#!/bin/bash
# Sweep geometry experiments at the default workload: nodes per lane x (block, pod-group) pairs.
export TMPDIR=/tmp
for npl in 4 8; do for sb in 8192 16384; do
  echo "== npl=$npl blocks=$sb"
  KS_SWEEP_BLOCKS=$sb timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 5 --nodes-per-lane $npl 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['avg_launch_ms'], d['extra']['resolve_ms_per_round'])" || exit 1
done; done
