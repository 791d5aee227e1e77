#!/bin/bash
# One GPU pass: parity tests, default bench, rocprofv3 kernel trace of a short bench.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-r1}
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/tests_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/tests_$TAG.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 500 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json; tail -3 gpurun_out/bench_$TAG.err
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run --output-format csv -- python3 "$R/bench.py" --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/bench_prof_$TAG.json 2> gpurun_out/prof_$TAG.err
rc=$?; echo "prof rc=$rc"; cat gpurun_out/bench_prof_$TAG.json; find gpurun_out/prof_$TAG -name '*stats*' | head
