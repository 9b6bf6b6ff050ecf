#!/bin/bash
# A/B of built libraries and knob settings on the GPU box, alternated over rounds:
#   bash tools/ab_variants.sh ROUNDS "name:lib[:tune,tune]" ... -- [bench args]
# lib is ab/<lib>.so (or "tree" for the in-tree libkdpt.so); tunes are NAME=VALUE knobs.  One line per run:
# name round value ms_per_step k_trace_avg_launch_ms.  Logs under gpurun_out/ab/.
ROUNDS=$1; shift
VARS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do VARS+=("$1"); shift; done
[ "$1" = "--" ] && shift
mkdir -p gpurun_out/ab
for r in $(seq 1 "$ROUNDS"); do
  for v in "${VARS[@]}"; do
    IFS=: read -r name lib tunes <<< "$v"
    lib_path=$PWD/ab/$lib.so
    [ "$lib" = "tree" ] && lib_path=$PWD/kdtreepathtraceroptimization_amd/libkdpt.so
    targs=()
    IFS=, read -ra TL <<< "$tunes"
    for t in "${TL[@]}"; do [ -n "$t" ] && targs+=(--tune "$t"); done
    log=gpurun_out/ab/${name}_$r.log
    KDPT_LIBRARY=$lib_path timeout -k 10 240 python -u bench.py --no-cpu-baseline "${targs[@]}" "$@" > "$log" 2>&1 \
      || { echo "$name round $r failed"; tail -5 "$log"; exit 1; }
    python -c "
import json; d=json.loads(open('$log').read().strip().splitlines()[-1])
print('$name', $r, d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], flush=True)"
  done
done
