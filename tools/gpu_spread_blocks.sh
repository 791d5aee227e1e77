#!/bin/bash
# Spread-path block-cap A/B (KS_SPREAD_BLOCKS): ms per pod of the spread and
# affinity streams at 1M nodes for each cap.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/blocks
for b in ${BLOCKS:-256 512 1024}; do
  for kind in spread affinity; do
    KS_SPREAD_BLOCKS=$b timeout -k 10 200 python3 bench.py --kind zoned --pods $kind --steps 2 --warmup 1 --batch 1024 \
      --no-cpu-baseline --no-resident --latency-calls 0 > gpurun_out/blocks/${kind}_$b.json 2> gpurun_out/blocks/${kind}_$b.err || exit $?
    echo "$b $kind $(python3 -c "import json;d=json.load(open('gpurun_out/blocks/${kind}_$b.json'));print(d['value'], d['roofline']['ms_per_pod'])")"
  done
done
