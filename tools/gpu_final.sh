#!/bin/bash
# Round-end evidence: GPU tests, the default bench line (with cpu_baseline),
# rocprofv3 kernel trace + stats of the same command, the other configs.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-final}
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/tests_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/tests_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json
if [ $rc -ne 0 ]; then tail -5 gpurun_out/bench_$TAG.err; exit $rc; fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline > gpurun_out/bench_under_rocprof_$TAG.json 2> gpurun_out/prof_$TAG.err
rc=$?; echo "prof rc=$rc"
if [ $rc -ne 0 ]; then tail -5 gpurun_out/prof_$TAG.err; exit $rc; fi
bash tools/gpu_configs.sh $TAG
