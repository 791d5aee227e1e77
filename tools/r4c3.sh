# C3 (1M nodes) per resolve mode, with the parallel commit's phase profile
set -e
T=${T:-r4o}
B="timeout -k 10 300 python -u bench.py --no-cpu-baseline --latency-calls 0 --steps 6"
for m in 0 1; do
  $B --opt resolve_mode=$m --resolve-profile > gpurun_out/bench_${T}_c3m$m.json 2> gpurun_out/bench_${T}_c3m$m.err
done
