#!/bin/bash
# phase timing of chain_fused_k (SDG_FU_SKIP; results are invalid in these runs, only kernel times matter)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/phases
for s in ${SKIPS:-0 4 8 1 2 3}; do
  SDG_FU_SKIP=$s timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/phases/skip$s.log 2>&1 || exit $?
  echo "skip=$s $(grep -o '"ms_chain_match": [0-9.]*' gpurun_out/phases/skip$s.log)"
done
