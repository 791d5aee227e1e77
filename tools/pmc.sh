#!/bin/bash
# PMC passes for the sweep kernel of ONE bench configuration (one counter
# group per rocprofv3 run, as MI355X_MICROARCH.md prescribes), summarised into
# profiles/pmc/<key>.json, the file bench.py's roofline reads for that
# configuration (the key is printed by the bench itself: extra.pmc_key).
#   tools/pmc.sh TAG [bench args...]
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-r2}
shift
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-resident --latency-calls 0 $*"
# Counter collection serialises dispatches; cross-stream hand-offs by stream
# wait-value packets then stall behind it, so the PMC runs use event waits.
export KS_VALUE_SYNC=0
# rocprofv3 --pmc prints nothing until the end: keep the run visibly alive
( while sleep 30; do echo "pmc: alive"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
OUT="$R/gpurun_out/pmc_$TAG"
mkdir -p "$OUT"
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE GRBM_COUNT" "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT"; do
  i=$((i+1))
  timeout -s KILL 170 rocprofv3 --pmc $ctr -d "$OUT/p$i" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "$OUT/p$i.json" 2> "$OUT/p$i.err"
  rc=$?; echo "pass $i ($ctr) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.err"; exit $rc; fi
done
python3 tools/pmc_summary.py "$OUT" --tag "$TAG" --out-dir "$R/gpurun_out/pmc"
