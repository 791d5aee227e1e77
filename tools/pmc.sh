#!/bin/bash
# PMC passes for the sweep kernel (one counter group per rocprofv3 run, as the
# MI355X guide prescribes); summaries are parsed by tools/pmc_summary.py.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-r1}
ARGS="--steps 2 --warmup 1 --no-cpu-baseline"
# Counter collection serialises dispatches; cross-stream hand-offs by stream
# wait-value packets then stall behind it, so the PMC runs use event waits.
export KS_VALUE_SYNC=0
# rocprofv3 --pmc prints nothing until the end: keep the run visibly alive
( while sleep 30; do echo "pmc: alive"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAVES" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $ctr -d "$R/gpurun_out/pmc_$TAG/p$i" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "gpurun_out/pmc_${TAG}_p$i.json" 2> "gpurun_out/pmc_${TAG}_p$i.err"
  rc=$?; echo "pass $i ($ctr) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "gpurun_out/pmc_${TAG}_p$i.err"; exit $rc; fi
done
find gpurun_out/pmc_$TAG -name '*counter_collection*' | head
python3 tools/pmc_summary.py gpurun_out/pmc_$TAG --tag $TAG --out gpurun_out/pmc_$TAG/pmc_sweep.json
