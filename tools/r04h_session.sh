# round-4 session h: kernel trace + PMC passes of the current build (C3, C5), the shading timeline, the driver's
# bench command
set -o pipefail
O=gpurun_out/r04h
mkdir -p $O
timeout -k 10 900 bash tools/pmc_profile.sh r04h_c3 --steps 4 --warmup 1 > $O/pmc_c3.txt 2>&1 || { cat $O/pmc_c3.txt; exit 1; }
cat $O/pmc_c3.txt
python tools/timeline.py gpurun_out/r04h_c3/trace/run_kernel_trace.csv --last-ms 1500 > $O/timeline_c3.txt 2>&1
cat $O/timeline_c3.txt
timeout -k 10 900 bash tools/pmc_profile.sh r04h_c5 --mesh icosphere_8 --res 1600 1600 --depth 16 --bounce-cap 16 \
  --spp-per-step 64 --steps 2 --warmup 1 > $O/pmc_c5.txt 2>&1 || { cat $O/pmc_c5.txt; exit 1; }
cat $O/pmc_c5.txt
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || exit $?
tail -c 300 $O/bench_driver.log
# wave profiles (counting kernel) of C3 and C5 at the bench's batch shape
timeout -k 10 300 python -u tools/batch_profile.py dragon_5 8x16 > $O/wave_c3.log 2>&1 || exit $?
KDPT_PROF_RES=1600x1600 KDPT_PROF_DEPTH=16 KDPT_PROF_CAP=16 timeout -k 10 300 python -u tools/batch_profile.py icosphere_8 4x16 > $O/wave_c5.log 2>&1 || exit $?
tail -2 $O/wave_c3.log $O/wave_c5.log | cut -c1-1500
# knob sweeps at batch 16 (C3)
bash tools/ab_run.sh 1 "ew16=tree=--steps 10 --tune early_walk=16" "ew32=tree=--steps 10 --tune early_walk=32" "el8=tree=--steps 10 --tune early_leaf=8" "gf20=tree=--steps 10 --tune trace_grid_frac=0.2" "gf30=tree=--steps 10 --tune trace_grid_frac=0.3" "p7=tree=--steps 10 --pipeline 7" "p9=tree=--steps 10 --pipeline 9" "def=tree=--steps 10" > $O/sweep.txt 2>&1
cat $O/sweep.txt
