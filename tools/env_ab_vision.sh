#!/bin/bash
# Vision / prefill switch A/B: tools/prof_vision.py (one 1024 px page, vision tower + prefill, no profiler) in
# separate processes, one per environment setting; prints each repetition's vision_compute_ms / decode_prefill_ms.
#   tools/env_ab_vision.sh "name:VAR=VAL,VAR2=VAL" ...     (name: alone = the default environment)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%:*}; vars=${spec#*:}
  envs=(); IFS=',' read -ra kv <<< "$vars"; for x in "${kv[@]}"; do [ -n "$x" ] && envs+=("$x"); done
  echo "== $name ${envs[*]}"
  env "${envs[@]}" timeout -k 10 180 python tools/prof_vision.py --reps ${AB_REPS:-4} 2>&1 | grep '"rep"' || exit 1
done
