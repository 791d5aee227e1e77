#!/bin/bash
# A/B: GPU parity tests on the default library, then the C3 (and C4) bench on
# the default library and on k8s-1m_amd/ksched/lib/alt.
export TMPDIR=/tmp
TAG=${1:-ab}
C4=${2:-0}
PX=${3:-0}  # 1: also a 125k-node run (one 8-GPU shard of C3: resolve-bound)
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/tests_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/tests_$TAG.log; if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/tests_$TAG.log | head; exit $rc; fi
for v in new alt new alt; do
  # ALT_ENV="VAR=value": the alt runs use the default library with that setting
  if [ $v = alt ]; then
    if [ -n "$ALT_ENV" ]; then export "$ALT_ENV"; else export KSCHED_LIB_DIR=k8s-1m_amd/ksched/lib/alt; fi
  else
    unset KSCHED_LIB_DIR; if [ -n "$ALT_ENV" ]; then unset "${ALT_ENV%%=*}"; fi
  fi
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 6 > gpurun_out/ab_${TAG}_$v.json 2> gpurun_out/ab_${TAG}_$v.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ab_${TAG}_$v.json')); print('$v C3', d['value'], d['roofline']['avg_launch_ms'], d['extra']['resolve_ms_per_round'])"
  if [ "$C4" = 1 ]; then
    timeout -k 10 200 python -u bench.py --kind labeled --no-cpu-baseline --steps 4 > gpurun_out/ab4_${TAG}_$v.json 2> gpurun_out/ab4_${TAG}_$v.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/ab4_${TAG}_$v.json')); print('$v C4', d['value'], d['roofline']['avg_launch_ms'], d['extra']['resolve_ms_per_round'])"
  fi
  if [ "$PX" = 1 ]; then
    timeout -k 10 200 python -u bench.py --nodes 125000 --no-cpu-baseline --steps 6 > gpurun_out/abp_${TAG}_$v.json 2> gpurun_out/abp_${TAG}_$v.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/abp_${TAG}_$v.json')); print('$v 125k', d['value'], d['roofline']['avg_launch_ms'], d['extra']['resolve_ms_per_round'])"
  fi
done
