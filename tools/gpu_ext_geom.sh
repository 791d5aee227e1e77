#!/bin/bash
# C4 (labeled) sweep geometry: EXT nodes per lane x (block, pod-group) target.
export TMPDIR=/tmp
for npl in 2 4; do for sb in 8192 16384; do
  echo "== ext npl=$npl blocks=$sb"
  KS_EXT_NPL=$npl KS_SWEEP_BLOCKS=$sb timeout -k 10 200 python -u bench.py --kind labeled --no-cpu-baseline --steps 5 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['avg_launch_ms'], d['extra']['resolve_ms_per_round'])" || exit 1
done; done
