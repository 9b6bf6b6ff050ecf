#!/bin/bash
# Sweep a kdpt_set_tuning knob over bench.py runs (one process each); prints value / ms_per_step / k_trace avg.
# usage: tools/sweep_tune.sh NAME "v1 v2 ..." [bench args...]
NAME=$1; VALS=$2; shift 2
mkdir -p gpurun_out
for v in $VALS; do
  timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --tune "$NAME=$v" "$@" > gpurun_out/sweep.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/sweep.log; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/sweep.log').read().strip().splitlines()[-1])
print('$NAME=$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done
