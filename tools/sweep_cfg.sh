#!/bin/bash
# Bench configurations one after another (one process each): each argument is "NAME|bench args".
#   bash tools/sweep_cfg.sh "p8b4|--pipeline 8 --batch 4" "p4b8|--pipeline 4 --batch 8" ...
# KDPT_LIBRARY picks the library if set.  Prints value / ms_per_step / k_trace avg launch ms.
mkdir -p gpurun_out/sweep
for cfg in "$@"; do
  name=${cfg%%|*}; args=${cfg#*|}
  log=gpurun_out/sweep/$name.log
  timeout -k 10 180 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 $args > "$log" 2>&1 \
    || { echo "$name failed"; tail -5 "$log"; exit 1; }
  python -c "
import json; d=json.loads(open('$log').read().strip().splitlines()[-1])
print('$name', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['launch_grid_share'])"
done
