#!/bin/bash
# rocprofv3 kernel trace of the C4 (labeled) bench
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-r1}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_c4_$TAG" -o run --output-format csv -- python3 "$R/bench.py" --kind labeled --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_prof_c4_$TAG.json 2> gpurun_out/prof_c4_$TAG.err
rc=$?; echo "prof rc=$rc"; cat gpurun_out/bench_prof_c4_$TAG.json; tail -3 gpurun_out/prof_c4_$TAG.err
exit $rc
