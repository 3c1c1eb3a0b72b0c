#!/bin/bash
# A/B the kernels of several library builds in one box session.
R=${GRAFT_REPO_ROOT:-$(pwd)}
for lib in "$@"; do
  echo "== $lib"
  P64GPU_LIB=$R/$lib timeout -k 10 120 python3 $R/tools/kbench.py --reps 10 2>&1 | grep -v amdgpu.ids
done
