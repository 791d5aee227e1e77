#!/bin/bash
# One driver for every GPU-box job of this repo (run through gpurun from the
# repo root).  Every GPU step has its own time limit; steps chain with && and
# the script stops at the first failure.
#
#   tools/gpu.sh tests TAG [pytest -k expr]   GPU parity suite (one process) + smoke()
#   tools/gpu.sh lines TAG "c3 c4 ..."        bench lines: c3 c4 c2 kwok kwokbe c5 spread deploy deploydns affinity
#                                             (each -> gpurun_out/bench_TAG_<line>.json)
#   tools/gpu.sh trace TAG [bench args]       rocprofv3 --kernel-trace --stats of a short bench run
#   tools/gpu.sh pmc TAG [bench args]         PMC passes of one configuration -> gpurun_out/pmc/<key>.json
#   tools/gpu.sh sq TAG [bench args]          SQ counters per kernel of one short bench run
#   tools/gpu.sh ab TAG [bench args]          A/B: default library vs lib/alt (or ALT_OPT="name=value": a
#                                             ks_config option of the alt arm), twice each
#   tools/gpu.sh variants TAG [bench args]    VARIANTS="default stamps ..." one configuration on several lib/<name> builds
#   tools/gpu.sh stamps TAG [kind]            resolve-phase stamps (make stamps stamps2 stamps3 first)
#   tools/gpu.sh valu                         VALU issue costs (tools/valu_issue, built by hipcc on the CPU side)
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
JOB=$1
TAG=${2:-run}
shift 2 2>/dev/null

line_args() {  # bench.py arguments of a named BASELINE.json configuration
  case $1 in
    c3) echo "" ;;
    c4) echo "--kind labeled --no-cpu-baseline --latency-calls 0" ;;
    c2) echo "--nodes 100000 --batch 20000 --steps 5 --no-cpu-baseline --latency-calls 0" ;;
    kwok) echo "--kind kwok --topk 512 --no-cpu-baseline --latency-calls 0" ;;
    kwokbe) echo "--kind kwok --pods besteffort --no-cpu-baseline --latency-calls 0" ;;
    c5) echo "--workload c5 --steps 20 --warmup 1 --no-cpu-baseline" ;;
    spread) echo "--kind zoned --pods spread --latency-calls 0" ;;
    deploy) echo "--kind zoned --pods deploy --latency-calls 0" ;;
    pct5) echo "--pct 5 --latency-calls 0" ;;
    deploydns) echo "--kind zoned --pods deploy-dns --latency-calls 0" ;;
    deploydnschain) echo "--kind zoned --pods deploy-dns --latency-calls 0 --no-cpu-baseline --opt spread_replica_runs=0" ;;
    deploychain) echo "--kind zoned --pods deploy --latency-calls 0 --no-cpu-baseline --opt spread_replica_runs=0" ;;
    affinity) echo "--kind zoned --pods affinity --latency-calls 0" ;;
    proxy) echo "--nodes 125000 --no-cpu-baseline --latency-calls 0" ;;
    c4proxy) echo "--nodes 125000 --kind labeled --no-cpu-baseline --latency-calls 0" ;;
    *) echo "unknown line $1" >&2; return 1 ;;
  esac
}

summary() {  # one line per bench json
  python3 -c "
import json, sys
d = json.load(open(sys.argv[1])); r = d['roofline']
print(sys.argv[2], d['value'], d.get('value_inputs_resident'), r.get('frac'), r.get('avg_launch_ms', r.get('ms_per_pod')),
      d['extra']['pods_per_round_resolved'], d['extra'].get('resolve_ms_per_round'))" "$1" "$2" 2>/dev/null
}

case $JOB in
  tests)
    timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout ${PYTEST_TIMEOUT:-600} --timeout-method thread \
      --durations=15 ${1:+-k "$1"} > gpurun_out/tests_gpu_$TAG.log 2>&1
    rc=$?; tail -5 gpurun_out/tests_gpu_$TAG.log; echo "tests rc=$rc"
    [ $rc -eq 0 ] || exit $rc
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
    rc=$?; cat gpurun_out/smoke_$TAG.log; exit $rc ;;
  lines)
    for l in ${1:-c3 c4 c2 kwok kwokbe c5 spread deploy deploydns affinity pct5}; do
      args=$(line_args $l) || exit 1
      timeout -k 10 420 python -u bench.py $args > gpurun_out/bench_${TAG}_$l.json 2> gpurun_out/bench_${TAG}_$l.err
      rc=$?; echo "$l rc=$rc $(summary gpurun_out/bench_${TAG}_$l.json $l)"
      [ $rc -eq 0 ] || { tail -3 gpurun_out/bench_${TAG}_$l.err; exit $rc; }
    done ;;
  trace)
    mkdir -p gpurun_out/trace_$TAG
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/trace_$TAG" -o run --output-format csv -- \
      python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-resident --latency-calls 0 "$@" \
      > gpurun_out/trace_$TAG/bench.json 2> gpurun_out/trace_$TAG/bench.err
    rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
    python3 - "$R/gpurun_out/trace_$TAG" <<'PY'
import csv, glob, json, sys
d = sys.argv[1]
b = json.load(open(d + "/bench.json"))
print("value", b["value"], "sweep avg ms (HIP events)", b["roofline"].get("avg_launch_ms"))
stats = glob.glob(d + "/**/*kernel_stats.csv", recursive=True)
for r in list(csv.DictReader(open(stats[0])))[:12]:
    print(r["Name"][:70].ljust(70), r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
    ;;
  pmc)
    # one counter group per rocprofv3 run (MI355X_MICROARCH.md); stream
    # wait-value hand-offs stall behind counter collection, so event waits
    ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-resident --latency-calls 0 --opt value_sync=0 --opt sync_timeout_ms=600000 $*"
    ( while sleep 30; do echo "pmc: alive"; done ) &
    HB=$!
    trap 'kill $HB 2>/dev/null' EXIT
    OUT="$R/gpurun_out/pmc_$TAG"
    mkdir -p "$OUT"
    i=0
    for ctr in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
               "SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE GRBM_COUNT" \
               "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT"; do
      i=$((i+1))
      timeout -s KILL 170 rocprofv3 --pmc $ctr -d "$OUT/p$i" -o run --output-format csv -- python3 "$R/bench.py" $ARGS \
        > "$OUT/p$i.json" 2> "$OUT/p$i.err"
      rc=$?; echo "pass $i ($ctr) rc=$rc"
      [ $rc -eq 0 ] || { tail -5 "$OUT/p$i.err"; exit $rc; }
    done
    python3 tools/pmc_summary.py "$OUT" --tag "$TAG" --out-dir "$R/gpurun_out/pmc" || exit 1
    # the raw counter CSVs (~16 MB per configuration) stay on the box unless
    # PMC_KEEP_RAW=1: gpurun merges at most 64 MiB of gpurun_out/ back
    [ "${PMC_KEEP_RAW:-0}" = 1 ] || rm -rf "$OUT"/p[0-9]* ;;
  sq)
    # SQ counters per kernel of one short bench run (e.g. the one-pod path:
    # tools/gpu.sh sq TAG --kind zoned --pods spread --batch 128); value sync
    # off as in pmc, small batches: per-dispatch collection slows every launch
    mkdir -p gpurun_out/sq_$TAG
    timeout -s KILL 170 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_WAVE_CYCLES \
      SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d "$R/gpurun_out/sq_$TAG/p1" -o run --output-format csv -- \
      python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --no-resident --latency-calls 0 --opt value_sync=0 --opt sync_timeout_ms=600000 "$@" \
      > gpurun_out/sq_$TAG/p1.json 2> gpurun_out/sq_$TAG/p1.err
    rc=$?; echo "sq rc=$rc"; exit $rc ;;
  ab)
    for v in new alt new alt; do
      EXTRA=""
      if [ $v = alt ]; then
        if [ -n "$ALT_OPT" ]; then EXTRA="--opt $ALT_OPT"; else export KSCHED_LIB_DIR=k8s-1m_amd/ksched/lib/alt; fi
      else
        unset KSCHED_LIB_DIR
      fi
      timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 6 --latency-calls 0 $EXTRA "$@" \
        > gpurun_out/ab_${TAG}_$v.json 2> gpurun_out/ab_${TAG}_$v.err || { tail -3 gpurun_out/ab_${TAG}_$v.err; exit 1; }
      summary gpurun_out/ab_${TAG}_$v.json $v
    done ;;
  variants)
    # one bench configuration on several library builds: VARIANTS="default stamps ..." (lib/<name>)
    for v in ${VARIANTS:-default}; do
      if [ "$v" = default ]; then unset KSCHED_LIB_DIR; else export KSCHED_LIB_DIR=k8s-1m_amd/ksched/lib/$v; fi
      timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 4 --warmup 1 --latency-calls 0 "$@" \
        > gpurun_out/var_${TAG}_$v.json 2> gpurun_out/var_${TAG}_$v.err || { tail -3 gpurun_out/var_${TAG}_$v.err; exit 1; }
      summary gpurun_out/var_${TAG}_$v.json $v
    done ;;
  stamps)
    KIND=${1:-hetero}
    for v in stamps stamps2 stamps3; do
      KSCHED_LIB_DIR=k8s-1m_amd/ksched/lib/$v timeout -k 10 200 python -u tools/resolve_stamps.py 1000000 8192 $KIND \
        > gpurun_out/${v}_$TAG.txt 2>&1 || exit $?
      cat gpurun_out/${v}_$TAG.txt
    done ;;
  valu)
    timeout -k 10 250 ./tools/valu_issue > gpurun_out/valu_issue.jsonl
    rc=$?; cat gpurun_out/valu_issue.jsonl; exit $rc ;;
  *)
    sed -n '2,16p' "$0"; exit 2 ;;
esac
