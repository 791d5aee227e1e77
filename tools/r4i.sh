# round-4 GPU check: selected tests, then the proxy (profiled and not) and optional kwok-be modes
set -e
T=${T:-r4m}
PYTEST_TIMEOUT=200 tools/gpu.sh tests $T "${SEL:-resolve or stall or dedup or records}"
B="timeout -k 10 200 python -u bench.py --no-cpu-baseline --latency-calls 0 --steps 5"
$B --nodes 125000 --resolve-profile > gpurun_out/bench_${T}_proxy.json 2> gpurun_out/bench_${T}_proxy.err
$B --nodes 125000 > gpurun_out/bench_${T}_proxynp.json 2> gpurun_out/bench_${T}_proxynp.err
for m in ${MODES:-}; do
  $B --kind kwok --pods besteffort --opt resolve_mode=$m --resolve-profile > gpurun_out/bench_${T}_kwokbe_m$m.json 2> gpurun_out/bench_${T}_kwokbe_m$m.err
done
