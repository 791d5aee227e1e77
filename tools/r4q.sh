# C3 regression hunt: SERIAL resolve, default library vs lib/alt (no diag stream), and 32,768-pod steps
set -e
T=${T:-r4q}
B="timeout -k 10 300 python -u bench.py --no-cpu-baseline --latency-calls 0 --steps 6 --opt resolve_mode=1"
$B > gpurun_out/bench_${T}_def.json 2> gpurun_out/bench_${T}_def.err
KSCHED_LIB_DIR=k8s-1m_amd/ksched/lib/alt $B > gpurun_out/bench_${T}_alt.json 2> gpurun_out/bench_${T}_alt.err
$B --batch 32768 > gpurun_out/bench_${T}_b32k.json 2> gpurun_out/bench_${T}_b32k.err
