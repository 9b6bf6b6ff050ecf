#!/bin/bash
# Kernel trace + PMC passes for bench.py (run on the GPU box from the repo root):
#   bash tools/profile.sh gpurun_out/prof_r01
set -e
OUT=${1:-gpurun_out/prof}
STEPS=${STEPS:-10}
ROOT=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 bench.py --steps $STEPS --warmup 2 --no-cpu-baseline > "$OUT/bench_trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench_pmc_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_write" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench_pmc_write.log" 2>&1
echo profile-done
