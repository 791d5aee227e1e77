# after the diag-stream fix: stall tests, then proxy / C3 / kwok-be per resolve mode
set -e
T=${T:-r4r}
PYTEST_TIMEOUT=200 tools/gpu.sh tests $T "stall or resolve"
B="timeout -k 10 300 python -u bench.py --no-cpu-baseline --latency-calls 0 --steps 6"
for m in 0 1; do
  $B --nodes 125000 --opt resolve_mode=$m > gpurun_out/bench_${T}_proxy_m$m.json 2> gpurun_out/bench_${T}_proxy_m$m.err
  $B --opt resolve_mode=$m > gpurun_out/bench_${T}_c3_m$m.json 2> gpurun_out/bench_${T}_c3_m$m.err
  $B --kind kwok --pods besteffort --opt resolve_mode=$m > gpurun_out/bench_${T}_kwokbe_m$m.json 2> gpurun_out/bench_${T}_kwokbe_m$m.err
done
$B --nodes 125000 --resolve-profile > gpurun_out/bench_${T}_proxy_prof.json 2> gpurun_out/bench_${T}_proxy_prof.err
