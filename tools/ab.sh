#!/bin/bash
# A/B of built libraries on the GPU box: alternates the bench over ab/<name>.so (KDPT_LIBRARY), N rounds.
#   bash tools/ab.sh "base new" ROUNDS [bench args...]
# Prints value / ms_per_step / k_trace avg launch ms per run; logs under gpurun_out/ab/.
NAMES=$1; ROUNDS=${2:-3}; shift 2
mkdir -p gpurun_out/ab
for r in $(seq 1 "$ROUNDS"); do
  for n in $NAMES; do
    log=gpurun_out/ab/${n}_$r.log
    KDPT_LIBRARY=$PWD/ab/$n.so timeout -k 10 180 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 "$@" > "$log" 2>&1 \
      || { echo "$n round $r failed"; tail -5 "$log"; exit 1; }
    python -c "
import json; d=json.loads(open('$log').read().strip().splitlines()[-1])
print('$n', $r, d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
  done
done
