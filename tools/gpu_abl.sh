#!/bin/bash
# C4 sweep timing ablations (KS_ABL builds, results wrong) + a kernel trace of the real build.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-abl}
ARGS="--kind labeled --steps 3 --warmup 1 --no-cpu-baseline --no-resident --latency-calls 0"
mkdir -p gpurun_out/$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/$TAG/trace" -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/$TAG/real.json 2> gpurun_out/$TAG/real.err || exit $?
python3 -c "import json;d=json.load(open('gpurun_out/$TAG/real.json'));print('real', d['value'], d['roofline']['avg_launch_ms'])"
for m in 1 2 4 8 15; do
  KSCHED_LIB_DIR=$R/k8s-1m_amd/ksched/lib/abl$m timeout -k 10 200 python3 bench.py $ARGS > gpurun_out/$TAG/abl$m.json 2> gpurun_out/$TAG/abl$m.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/$TAG/abl$m.json'));print('abl$m', d['value'], d['roofline']['avg_launch_ms'])"
done
