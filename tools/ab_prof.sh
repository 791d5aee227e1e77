#!/bin/bash
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
for d in ab_base cur; do
  if [ $d = cur ]; then L=$R/k8s-1m_amd/ksched/lib; else L=$R/k8s-1m_amd/ksched/lib/$d; fi
  KS_FUSE_START=0 KS_FUSE_GATHER=0 KSCHED_LIB_DIR=$L timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/ab_$d" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --steps 4 --warmup 1 > gpurun_out/ab_$d.json 2> gpurun_out/ab_$d.err || exit 1
done
