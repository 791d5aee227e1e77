set -e
T=${T:-r4v}
B="timeout -k 10 300 python -u bench.py --no-cpu-baseline --latency-calls 0"
$B --nodes 100000 --batch 20000 --steps 10 > gpurun_out/bench_${T}_c2.json 2> gpurun_out/bench_${T}_c2.err
$B --nodes 125000 --steps 6 > gpurun_out/bench_${T}_proxy.json 2> gpurun_out/bench_${T}_proxy.err
$B --steps 6 > gpurun_out/bench_${T}_c3.json 2> gpurun_out/bench_${T}_c3.err
PYTEST_TIMEOUT=300 tools/gpu.sh tests $T "stall or parity or fullsize_c3 or records"
