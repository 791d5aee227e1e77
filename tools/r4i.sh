set -e
PYTEST_TIMEOUT=200 tools/gpu.sh tests r4i "resolve or stall or semantics or dedup or parity or boundary or solo"
B="timeout -k 10 200 python -u bench.py --no-cpu-baseline --latency-calls 0 --steps 5"
$B --nodes 125000 --resolve-profile > gpurun_out/bench_r4i_proxy.json 2> gpurun_out/bench_r4i_proxy.err
for m in 0 1 2; do
  $B --kind kwok --pods besteffort --opt resolve_mode=$m --resolve-profile > gpurun_out/bench_r4i_kwokbe_m$m.json 2> gpurun_out/bench_r4i_kwokbe_m$m.err
done
VALU_ONLY="f32" timeout -k 10 120 ./tools/valu_issue > gpurun_out/valu_vop.jsonl
