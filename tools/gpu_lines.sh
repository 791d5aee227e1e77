#!/bin/bash
# Every bench line of BASELINE.json's configs on one box (1 GPU):
#   tools/gpu_lines.sh TAG   -> gpurun_out/bench_TAG_<line>.json
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-r2}
run() {
  local name=$1; shift
  timeout -k 10 420 python -u bench.py "$@" > gpurun_out/bench_${TAG}_$name.json 2> gpurun_out/bench_${TAG}_$name.err
  local rc=$?
  echo "$name rc=$rc $(python3 -c "import json;d=json.load(open('gpurun_out/bench_${TAG}_$name.json'));r=d['roofline'];print(d['value'], d.get('value_end_to_end'), r.get('frac'), r.get('avg_launch_ms', r.get('ms_per_pod')), d['extra']['pods_per_round_resolved'])" 2>/dev/null)"
  return $rc
}
mkdir -p gpurun_out
ONLY=${2:-}
if [ -n "$ONLY" ]; then
  for l in $ONLY; do
    case $l in
      c3) run c3 || exit $? ;;
      spread) run spread --kind zoned --pods spread --latency-calls 0 || exit $? ;;
      affinity) run affinity --kind zoned --pods affinity --latency-calls 0 || exit $? ;;
      c4) run c4 --kind labeled --no-cpu-baseline --latency-calls 0 || exit $? ;;
    esac
  done
  exit 0
fi
run c3 && \
run c4 --kind labeled --no-cpu-baseline --latency-calls 0 && \
run c2 --nodes 100000 --batch 20000 --steps 5 --no-cpu-baseline --latency-calls 0 && \
run kwok --kind kwok --topk 512 --no-cpu-baseline --latency-calls 0 && \
run kwokbe --kind kwok --pods besteffort --no-cpu-baseline --latency-calls 0 && \
run c5 --workload c5 --steps 5 --warmup 1 && \
run spread --kind zoned --pods spread --latency-calls 0 && \
run affinity --kind zoned --pods affinity --latency-calls 0
