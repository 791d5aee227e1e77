#!/bin/bash
# rocprofv3 kernel trace + stats of one bench run: tools/prof.sh TAG [KIND] [extra bench args]
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-r1}
KIND=${2:-hetero}
shift 2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run --output-format csv -- python3 "$R/bench.py" --kind $KIND --no-cpu-baseline "$@" > gpurun_out/bench_prof_$TAG.json 2> gpurun_out/prof_$TAG.err
rc=$?; echo "prof rc=$rc"; cat gpurun_out/bench_prof_$TAG.json; tail -3 gpurun_out/prof_$TAG.err
exit $rc
