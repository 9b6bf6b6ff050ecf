#!/bin/bash
# Kernel trace + PMC passes for bench.py (run on the GPU box from the repo root).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/prof}
STEPS=${STEPS:-6}
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 bench.py --steps $STEPS --warmup 2 --no-cpu-baseline > "$OUT/bench_trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace --output-format csv -d "$OUT/pmc_sq" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/bench_pmc_sq.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/bench_pmc_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_write" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/bench_pmc_write.log" 2>&1
echo profile-done
