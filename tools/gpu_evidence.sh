#!/bin/bash
# Round-end evidence in one GPU call: parity tests, default bench (+ cpu_baseline),
# rocprofv3 kernel stats of a short bench, the PMC passes, the other configs.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-r1}
bash tools/gpu_round.sh "$TAG" && bash tools/gpu_configs.sh "$TAG" && bash tools/pmc.sh "$TAG"
