#!/bin/bash
# One bench line on the box: tools/gpu_bench.sh TAG [bench args...] -> gpurun_out/bench_TAG.json
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=$1
shift
mkdir -p gpurun_out
timeout -k 10 420 python -u bench.py "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench $TAG rc=$rc"; cat gpurun_out/bench_$TAG.json; tail -3 gpurun_out/bench_$TAG.err
exit $rc
