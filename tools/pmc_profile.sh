#!/bin/bash
# rocprofv3 passes for the bench workload (run on the GPU box from the repo root, e.g. through
# tools/gpu_session.sh's sh: step):
#   bash tools/pmc_profile.sh TAG [extra bench.py args]
# 1. kernel trace + stats of the bench command as the driver runs it (concurrent launches);
# 2. PMC passes, one counter group each (rocprofv3 serialises dispatches while it counts, so these
#    launches run exclusively): SQ issue/wait counters, LDS counters, FETCH_SIZE, WRITE_SIZE.
# Outputs under gpurun_out/TAG/; summarise with tools/summarize_pmc.py.
TAG=${1:?tag}
shift
OUT=gpurun_out/$TAG
ROOT=$PWD
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH=(bench.py --no-cpu-baseline "$@")
# the fixed step counts come last (argparse: the last one wins), so workload args pass through but the PMC
# passes always count exactly the dispatches of the one timed step the summariser divides by
PMC_BENCH=(bench.py --no-cpu-baseline "$@" --steps 1 --warmup 0 --spp-per-step 16)
run() {  # name, then rocprofv3 args; a time-out or crash stops the script
  local name=$1
  shift
  timeout -s KILL 180 rocprofv3 "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[pmc] $name rc=$rc"
  tail -2 "$OUT/$name.log"
  if [ $rc -ge 124 ]; then exit $rc; fi
  return 0
}
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters_avail.txt" 2>&1
echo "[pmc] counter list rc=$?"
run trace --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 "${BENCH[@]}"
run pmc_sq_a --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
    SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT \
    --kernel-trace --output-format csv -d "$OUT/pmc_sq_a" -o run -- python3 "${PMC_BENCH[@]}"
run pmc_sq_b --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM \
    SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA \
    --kernel-trace --output-format csv -d "$OUT/pmc_sq_b" -o run -- python3 "${PMC_BENCH[@]}"
run pmc_fetch --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 "${PMC_BENCH[@]}"
run pmc_write --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_write" -o run -- python3 "${PMC_BENCH[@]}"
echo "[pmc] done"
