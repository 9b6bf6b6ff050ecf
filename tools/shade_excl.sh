#!/bin/bash
# Exclusive fused-shading launch times: one batch in flight (--pipeline 1), so each dispatch runs alone;
# rocprofv3 kernel trace per library in ab/ (GPU box, repo root).   bash tools/shade_excl.sh TAG "lib1 lib2"
TAG=$1; LIBS=$2
for l in $LIBS; do
  d=gpurun_out/$TAG/excl_$l
  mkdir -p "$d"
  KDPT_LIBRARY=$PWD/ab/$l.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o run -- \
    python3 -u bench.py --no-cpu-baseline --steps 4 --warmup 1 --pipeline 1 --spp-per-step 16 > "$d/bench.log" 2>&1 || exit $?
  f=$(find "$d" -name '*kernel_stats.csv' | head -1)
  echo "$l"; grep -E "k_shade_fused_b|k_trace<true, false" "$f" | cut -d, -f1-5
done
