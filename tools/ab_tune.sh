#!/bin/bash
# A/B of tuning knobs on the in-tree library, alternating, N rounds (GPU box, from the repo root):
#   bash tools/ab_tune.sh ROUNDS "LABEL=bench args|LABEL=bench args|..."
# Prints value / ms_per_step / k_trace avg launch ms per run; logs under gpurun_out/ab_tune/.
ROUNDS=$1
IFS='|' read -ra SPECS <<< "$2"
mkdir -p gpurun_out/ab_tune
for r in $(seq 1 "$ROUNDS"); do
  for spec in "${SPECS[@]}"; do
    label=${spec%%=*}; args=${spec#*=}
    log=gpurun_out/ab_tune/${label}_$r.log
    timeout -k 10 180 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 $args > "$log" 2>&1 \
      || { echo "$label round $r failed"; tail -5 "$log"; exit 1; }
    python -c "
import json; d=json.loads(open('$log').read().strip().splitlines()[-1])
print('$label', $r, d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['config'].get('intersect'))"
  done
done
