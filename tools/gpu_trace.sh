#!/bin/bash
# Kernel trace of a short bench (args after the tag are passed to bench.py).
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=$1; shift
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/trace_$TAG" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline "$@" > gpurun_out/trace_$TAG.json 2> gpurun_out/trace_$TAG.err
rc=$?; echo "trace rc=$rc"; cat gpurun_out/trace_$TAG.json; exit $rc
