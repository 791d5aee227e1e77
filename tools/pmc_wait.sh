#!/bin/bash
# Wave issue / wait breakdown of the sweep (one rocprofv3 --pmc pass per kind).
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-wait}
for KIND in hetero labeled; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_SMEM SQ_INSTS_SMEM -d "$R/gpurun_out/pmc_${TAG}_$KIND" -o run --output-format csv -- python3 "$R/bench.py" --kind $KIND --steps 2 --warmup 1 --no-cpu-baseline > "gpurun_out/pmc_${TAG}_$KIND.json" 2> "gpurun_out/pmc_${TAG}_$KIND.err"
  rc=$?; echo "$KIND rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "gpurun_out/pmc_${TAG}_$KIND.err"; exit $rc; fi
done
