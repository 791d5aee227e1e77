#!/bin/bash
# GPU parity suite on the box: every -m gpu test (one process), then smoke().
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-r2}
SEL=${2:-}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout ${PYTEST_TIMEOUT:-170} --timeout-method thread --durations=15 $SEL > gpurun_out/tests_gpu_$TAG.log 2>&1
rc=$?; tail -5 gpurun_out/tests_gpu_$TAG.log; echo "tests rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; cat gpurun_out/smoke_$TAG.log; exit $rc
