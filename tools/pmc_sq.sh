#!/bin/bash
# SQ counters for the intersect kernel (issue vs wait), one PMC pass; run on the GPU box.
set -e
OUT=${1:-gpurun_out/pmc_sq}
ROOT=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --kernel-trace --output-format csv -d "$OUT/a" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/a.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d "$OUT/b" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/b.log" 2>&1
echo pmc-done
