set -e
T=${T:-r4w}
PYTEST_TIMEOUT=300 tools/gpu.sh tests $T "resolve or dedup or kwok or besteffort or records or stall"
B="timeout -k 10 300 python -u bench.py --no-cpu-baseline --latency-calls 0 --steps 6"
$B --kind kwok --pods besteffort > gpurun_out/bench_${T}_kwokbe.json 2> gpurun_out/bench_${T}_kwokbe.err
$B --kind kwok --pods besteffort --opt resolve_mode=1 > gpurun_out/bench_${T}_kwokbe_m1.json 2> gpurun_out/bench_${T}_kwokbe_m1.err
$B --nodes 125000 > gpurun_out/bench_${T}_proxy.json 2> gpurun_out/bench_${T}_proxy.err
