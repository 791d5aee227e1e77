#!/bin/bash
# GPU parity tests, C3 + C4 benches and the resolve stamps breakdown.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-r1}
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/tests_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/tests_$TAG.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/tests_$TAG.log | head -20; exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json; tail -3 gpurun_out/bench_$TAG.err
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --kind labeled --no-cpu-baseline > gpurun_out/bench_c4_$TAG.json 2> gpurun_out/bench_c4_$TAG.err
rc=$?; echo "c4 rc=$rc"; cat gpurun_out/bench_c4_$TAG.json; tail -3 gpurun_out/bench_c4_$TAG.err
if [ $rc -ne 0 ]; then exit $rc; fi
KSCHED_LIB_DIR=k8s-1m_amd/ksched/lib/stamps timeout -k 10 200 python -u tools/resolve_stamps.py 1000000 8192 > gpurun_out/stamps_$TAG.txt 2>&1
rc=$?; echo "stamps rc=$rc"; cat gpurun_out/stamps_$TAG.txt | tail -8
exit $rc
