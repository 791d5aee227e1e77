#!/bin/bash
# One rocprofv3 --pmc pass of one bench configuration, averaged per kernel:
#   tools/pmc_one.sh TAG "CTR1 CTR2 ..." [bench args...]
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=$1; CTRS=$2; shift 2
export KS_VALUE_SYNC=0
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
timeout -s KILL 170 rocprofv3 --pmc $CTRS -d "$OUT/p" -o run --output-format csv -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-resident --latency-calls 0 "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -5 "$OUT/bench.err"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, sys, collections
from pathlib import Path
d = Path(sys.argv[1])
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in d.rglob("*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = (r["Kernel_Name"].split("(")[0], int(r["Grid_Size"]))
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for (k, g), c in sorted(acc.items(), key=lambda kv: -len(next(iter(kv[1].values())))):
    if "sweep" in k or "resolve" in k or "patch" in k:
        print(k[:50], g, {n: round(sum(v) / len(v)) for n, v in c.items()})
PY
