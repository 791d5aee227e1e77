#!/bin/bash
# Resolve stamps: decider phases (stamps) and eval-wave phases (stamps2).
export TMPDIR=/tmp
TAG=${1:-r1}
KIND=${2:-hetero}
KSCHED_LIB_DIR=k8s-1m_amd/ksched/lib/stamps timeout -k 10 200 python -u tools/resolve_stamps.py 1000000 8192 $KIND > gpurun_out/stamps1_$TAG.txt 2>&1 &&
KSCHED_LIB_DIR=k8s-1m_amd/ksched/lib/stamps2 timeout -k 10 200 python -u tools/resolve_stamps.py 1000000 8192 $KIND > gpurun_out/stamps2_$TAG.txt 2>&1
rc=$?; [ $rc -eq 0 ] && KSCHED_LIB_DIR=k8s-1m_amd/ksched/lib/stamps3 timeout -k 10 200 python -u tools/resolve_stamps.py 1000000 8192 $KIND > gpurun_out/stamps3_$TAG.txt 2>&1; rc=$?
cat gpurun_out/stamps1_$TAG.txt gpurun_out/stamps2_$TAG.txt gpurun_out/stamps3_$TAG.txt; exit $rc
