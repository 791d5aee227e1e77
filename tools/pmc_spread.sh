set -o pipefail
export KS_VALUE_SYNC=0
mkdir -p gpurun_out/pmcsp
timeout -s KILL 170 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d gpurun_out/pmcsp/p1 -o run --output-format csv -- python3 bench.py --kind zoned --pods spread --steps 1 --warmup 1 --batch 128 --no-cpu-baseline --no-resident --latency-calls 0 > gpurun_out/pmcsp/p1.json 2> gpurun_out/pmcsp/p1.err
echo "rc=$?"
