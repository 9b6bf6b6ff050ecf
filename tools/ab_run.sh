#!/bin/bash
# A/B of (library, bench args) pairs, alternating, N rounds (GPU box, from the repo root):
#   bash tools/ab_run.sh ROUNDS "LABEL=LIB=bench args" "LABEL=LIB=bench args" ...
# LIB: a name under ab/ (ab/LIB.so), or "tree" for the in-tree libkdpt.so.  Each run is
# `bench.py --no-cpu-baseline --warmup 5` plus the args (add --steps); logs under gpurun_out/ab_run/.
# Prints label, round, Mrays/s, ms/step, k_trace avg launch ms.
ROUNDS=$1; shift
mkdir -p gpurun_out/ab_run
for r in $(seq 1 "$ROUNDS"); do
  for spec in "$@"; do
    label=${spec%%=*}; rest=${spec#*=}
    lib=${rest%%=*}; args=${rest#*=}
    log=gpurun_out/ab_run/${label}_$r.log
    if [ "$lib" = tree ]; then unset KDPT_LIBRARY; else export KDPT_LIBRARY=$PWD/ab/$lib.so; fi
    timeout -k 10 240 python -u bench.py --no-cpu-baseline --warmup 5 $args > "$log" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "$label round $r failed rc=$rc"; tail -5 "$log"; exit $rc; fi
    python -c "
import json; d=json.loads(open('$log').read().strip().splitlines()[-1])
print('$label', $r, d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], flush=True)"
  done
done
unset KDPT_LIBRARY
