# PMC summaries of every bench configuration (tools/gpu.sh pmc per line; run through gpurun
# from the repo root: `bash tools/pmc_all.sh`); the raw
# per-pass rocprof output is dropped after each summary (gpurun merges <= 64 MiB)
set -e
run() { tag=$1; shift; tools/gpu.sh pmc $tag "$@"; rm -rf gpurun_out/pmc_$tag; }
run r4c3
run r4c4 --kind labeled
run r4c2 --nodes 100000 --batch 20000
run r4kw --kind kwok --topk 512
run r4kb --kind kwok --pods besteffort
run r4c5 --workload c5 --steps 2 --warmup 1
