#!/bin/bash
# Instruction-mix PMC passes of the sweep for one bench kind (default C3,
# "labeled" = C4): one counter group per rocprofv3 run.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-mix}
KIND=${2:-hetero}
ARGS="--kind $KIND --steps 2 --warmup 1 --no-cpu-baseline"
i=0
for ctr in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VALU SQ_INSTS_VALU_FMA_F64" \
           "SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_CVT SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr -d "$R/gpurun_out/pmc_$TAG/p$i" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "gpurun_out/pmc_${TAG}_p$i.json" 2> "gpurun_out/pmc_${TAG}_p$i.err"
  rc=$?; echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "gpurun_out/pmc_${TAG}_p$i.err"; exit $rc; fi
done
