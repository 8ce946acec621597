#!/bin/bash
# gate/up slot-kernel experiment: profile_decode timings under DSOCR_DBG_GU knobs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS:-0 1 2 3}; do
  DSOCR_DBG_GU=$v timeout -k 10 300 python bench.py --steps 1 --warmup 0 --max-new-tokens 32 --no-cpu-baseline --roofline-iters 20 > gpurun_out/exp_gu_$v.log 2>&1 || exit $?
done
