#!/bin/bash
# One GPU-box session (run from the repo root through gpurun):
#   bash tools/gpu_session.sh TAG "STEP;STEP;..."
# Steps: tests[:pytest args, shell-quoted] | smoke | bench:<args> | gloo2:<args> (two ranks sharing the GPU, gloo reduce) | py:<args> | sh:<cmd>
# Every step has its own time limit; a fault, abort, segfault or time-out ends the session there
# (pytest assertion failures, exit 1, do not).  Logs go to gpurun_out/<TAG>/.
TAG=${1:?tag}
STEPS=${2:-"tests;bench:--steps 20 --warmup 5"}
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
