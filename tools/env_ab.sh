#!/bin/bash
# Runtime-knob A/B: the same decode (tools/ab_trace.py, no profiler) in separate processes, one per environment
# setting (HIP runtime variables are read once at start-up); prints each process's per-generate decode ms.
#   tools/env_ab.sh "name:VAR=VAL,VAR2=VAL" ...     (name: alone = the default environment)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%:*}; vars=${spec#*:}
  envs=(); IFS=',' read -ra kv <<< "$vars"; for x in "${kv[@]}"; do [ -n "$x" ] && envs+=("$x"); done
  echo "== $name ${envs[*]}"
  env "${envs[@]}" timeout -k 10 180 python tools/ab_trace.py --tokens ${AB_TOKENS:-256} --rounds ${AB_ROUNDS:-3} \
      --variant "$name:" --out gpurun_out/envab_$name.json ${AB_EXTRA} 2>&1 | grep "\[ab\]" || exit 1
done
