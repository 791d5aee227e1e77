# PMC summaries of the non-headline bench configurations (tools/gpu.sh pmc per line)
set -e
tools/gpu.sh pmc r4c4 --kind labeled
tools/gpu.sh pmc r4c2 --nodes 100000 --batch 20000
tools/gpu.sh pmc r4kw --kind kwok --topk 512
tools/gpu.sh pmc r4kb --kind kwok --pods besteffort
tools/gpu.sh pmc r4c5 --workload c5 --steps 2 --warmup 1
