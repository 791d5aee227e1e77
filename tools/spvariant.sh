#!/bin/bash
# Diagnostic builds of the one-pod path (ksched_spread.hip) with extra defines:
#   tools/spvariant.sh NAME "-DKS_..."  ->  k8s-1m_amd/ksched/lib/NAME/libksched.so
# (load with KSCHED_LIB_DIR; never used by tests / bench / smoke)
set -e
cd "$(dirname "$0")/../k8s-1m_amd"
make -s build/ksched_host.o build/ksched_kernels.o
NAME=$1; shift
mkdir -p ksched/lib/$NAME
F="-O3 --offload-arch=gfx950 -std=c++17 -fPIC -ffp-contract=off -Wall -I../include -Icsrc"
/opt/rocm/bin/hipcc $F "$@" -c csrc/ksched_spread.hip -o build/ksched_spread_$NAME.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ksched/lib/$NAME/libksched.so build/ksched_kernels.o \
  build/ksched_spread_$NAME.o build/ksched_host.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
