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
