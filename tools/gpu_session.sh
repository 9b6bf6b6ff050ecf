#!/bin/bash
# One GPU-box session (run from the repo root through gpurun):
#   bash tools/gpu_session.sh TAG "STEP;STEP;..."
# Steps: tests[:pytest args, shell-quoted] | smoke | bench:<args> | gloo2:<args> (two ranks sharing the GPU, gloo reduce) | py:<args> | sh:<cmd>
# Every step has its own time limit; a fault, abort, segfault or time-out ends the session there
# (pytest assertion failures, exit 1, do not).  Logs go to gpurun_out/<TAG>/.
# Presets (STEPS = the preset's name), the sessions earlier rounds wrote one script each for:
#   driver   the driver's bench command (with the CPU baseline) and the GPU tests
#   c5       C5: icosphere_8, 1600x1600, depth 16, cap 16, 30 steps
#   c4       C4's per-GPU frame shapes: 32-spp frames, 256-spp frames, --total-spp 256
#   trace    rocprofv3 kernel trace + stats of the driver's command (profiles/<round>_kernel_stats.csv)
#   pmc      tools/pmc_profile.sh on C3 (then tools/summarize_pmc.py); pmc5: the same on C5
#   dist1    bench.py under a one-rank RCCL process group (the library's ncclReduce per frame)
#   columns  tools/reference_columns.py (the reference's brute / bbox / kd / short-stack table)
TAG=${1:?tag}
STEPS=${2:-"tests;bench:--steps 20 --warmup 5"}
C5="--no-cpu-baseline --mesh icosphere_8 --res 1600 1600 --depth 16 --bounce-cap 16 --spp-per-step 64"
C4="--scene cornell8 --no-cpu-baseline"
case "$STEPS" in
  driver) STEPS="tests;smoke;bench:--steps 20 --warmup 5" ;;
  c5) STEPS="bench:$C5 --steps 30 --warmup 3" ;;
  c4) STEPS="bench:$C4 --spp-per-step 32 --steps 160 --warmup 20;bench:$C4 --spp-per-step 256 --steps 20 --warmup 3;bench:$C4 --total-spp 256 --steps 20 --warmup 3" ;;
  trace) STEPS="sh:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/trace -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline" ;;
  pmc) STEPS="sh:bash tools/pmc_profile.sh $TAG/pmc" ;;
  pmc5) STEPS="sh:bash tools/pmc_profile.sh $TAG/pmc5 $C5" ;;
  dist1) STEPS="sh:python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --force-dist --steps 20 --warmup 5 --no-cpu-baseline" ;;
  columns) STEPS="py:tools/reference_columns.py --out gpurun_out/$TAG/reference_columns.json" ;;
esac
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
n=0
IFS=';' read -ra LIST <<< "$STEPS"
for step in "${LIST[@]}"; do
  n=$((n + 1))
  kind=${step%%:*}
  args=${step#*:}
  [ "$args" = "$step" ] && args=""
  log="$OUT/$(printf %02d $n)_${kind}.log"
  echo "[session] step $n: $kind $args -> $log"
  case "$kind" in
    tests) eval "timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --maxfail 30 $args" > "$log" 2>&1 ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$log" 2>&1 ;;
    bench) timeout -k 10 600 python -u bench.py $args > "$log" 2>&1 ;;
    gloo2) timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
             --master-port 29533 bench.py --gpus 2 --dist-backend gloo $args > "$log" 2>&1 ;;
    py) timeout -k 10 600 python -u $args > "$log" 2>&1 ;;
    sh) timeout -k 10 600 bash -c "$args" > "$log" 2>&1 ;;
    *) echo "unknown step $kind"; exit 2 ;;
  esac
  rc=$?
  tail -3 "$log"
  echo "[session] step $n rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[session] stopping after rc=$rc"; exit $rc; fi
done
echo "[session] done"
