#!/bin/bash
# Bench lines of BASELINE.json's configs on one box (1 GPU), a chosen subset:
#   tools/gpu_lines2.sh TAG "c3 c4 c2 kwok kwokbe c5 spread affinity prof"
# -> gpurun_out/bench_TAG_<line>.json; "prof" = rocprofv3 kernel trace + stats
# of a short default bench (gpurun_out/prof_TAG).
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-r2}
LINES=${2:-"c3 c4 c2 kwok kwokbe c5 spread affinity prof"}
mkdir -p gpurun_out
run() {
  local name=$1; shift
  timeout -k 10 420 python -u bench.py "$@" > gpurun_out/bench_${TAG}_$name.json 2> gpurun_out/bench_${TAG}_$name.err
  local rc=$?
  echo "$name rc=$rc $(python3 -c "import json;d=json.load(open('gpurun_out/bench_${TAG}_$name.json'));r=d['roofline'];print(d['value'], d.get('value_end_to_end'), r.get('frac'), r.get('avg_launch_ms', r.get('ms_per_pod')), d['extra']['pods_per_round_resolved'])" 2>/dev/null)"
  return $rc
}
for l in $LINES; do
  case $l in
    c3) run c3 || exit $? ;;
    c4) run c4 --kind labeled --no-cpu-baseline --latency-calls 0 || exit $? ;;
    c2) run c2 --nodes 100000 --batch 20000 --steps 5 --no-cpu-baseline --latency-calls 0 || exit $? ;;
    kwok) run kwok --kind kwok --topk 512 --no-cpu-baseline --latency-calls 0 || exit $? ;;
    kwokbe) run kwokbe --kind kwok --pods besteffort --no-cpu-baseline --latency-calls 0 || exit $? ;;
    c5) run c5 --workload c5 --steps 5 --warmup 1 --no-cpu-baseline || exit $? ;;
    spread) run spread --kind zoned --pods spread --latency-calls 0 || exit $? ;;
    affinity) run affinity --kind zoned --pods affinity --latency-calls 0 || exit $? ;;
    prof)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run --output-format csv -- python3 "$R/bench.py" --steps 4 --warmup 1 --no-cpu-baseline --no-resident --latency-calls 0 > gpurun_out/bench_prof_$TAG.json 2> gpurun_out/prof_$TAG.err
      rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc ;;
  esac
done
