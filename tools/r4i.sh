# round-4 GPU check: the resolve-mode tests, then the proxy / kwok-be benches per resolve mode
set -e
T=${T:-r4j}
PYTEST_TIMEOUT=200 tools/gpu.sh tests $T "${SEL:-resolve or stall or dedup}"
B="timeout -k 10 200 python -u bench.py --no-cpu-baseline --latency-calls 0 --steps 5"
$B --nodes 125000 --resolve-profile > gpurun_out/bench_${T}_proxy.json 2> gpurun_out/bench_${T}_proxy.err
for m in ${MODES:-0 1}; do
  $B --kind kwok --pods besteffort --opt resolve_mode=$m --resolve-profile > gpurun_out/bench_${T}_kwokbe_m$m.json 2> gpurun_out/bench_${T}_kwokbe_m$m.err
done
VALU_ONLY="(s, " timeout -k 10 120 ./tools/valu_issue > gpurun_out/valu_sgpr.jsonl
tools/gpu.sh trace r4j --nodes 125000
