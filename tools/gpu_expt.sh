#!/bin/bash
# Resolve timing experiments (diagnostic builds under ksched/lib/x*): per-role stamps with roles disabled.
export TMPDIR=/tmp
for m in 1 2 4 7; do
  echo "== KS_EXPT=$m"; KSCHED_LIB_DIR=k8s-1m_amd/ksched/lib/x$m timeout -k 10 100 python -u tools/resolve_stamps.py 200000 4096 2>&1 | tail -6 || exit 1
done
