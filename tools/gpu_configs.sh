#!/bin/bash
# Bench lines for the other BASELINE.json configs (C2: 100k nodes; C4: 1M
# labeled nodes with taints / affinity; C5: bursts + event logs) at the default round geometry.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-r1}
timeout -k 10 300 python -u bench.py --kind labeled --no-cpu-baseline > gpurun_out/bench_c4_$TAG.json 2> gpurun_out/bench_c4_$TAG.err
rc=$?; echo "c4 rc=$rc"; cat gpurun_out/bench_c4_$TAG.json; tail -3 gpurun_out/bench_c4_$TAG.err
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --nodes 100000 --batch 20000 --steps 5 --no-cpu-baseline > gpurun_out/bench_c2_$TAG.json 2> gpurun_out/bench_c2_$TAG.err
rc=$?; echo "c2 rc=$rc"; cat gpurun_out/bench_c2_$TAG.json; tail -3 gpurun_out/bench_c2_$TAG.err
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --kind kwok --prefill 0 --no-cpu-baseline > gpurun_out/bench_kwok_$TAG.json 2> gpurun_out/bench_kwok_$TAG.err
rc=$?; echo "kwok rc=$rc"; cat gpurun_out/bench_kwok_$TAG.json; tail -3 gpurun_out/bench_kwok_$TAG.err
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --workload c5 --steps 5 --warmup 1 > gpurun_out/bench_c5_$TAG.json 2> gpurun_out/bench_c5_$TAG.err
rc=$?; echo "c5 rc=$rc"; cat gpurun_out/bench_c5_$TAG.json; tail -3 gpurun_out/bench_c5_$TAG.err
exit $rc
