# round-4 final session 1: the full GPU suite and smoke on the final build, then the PMC passes (C3, C5) and
# the kernel-trace timeline of the shading
set -o pipefail
O=gpurun_out/r04z
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 bash tools/pmc_profile.sh r04z_c3 --steps 4 --warmup 1 > $O/pmc_c3.txt 2>&1 || { cat $O/pmc_c3.txt; exit 1; }
cat $O/pmc_c3.txt
python tools/timeline.py gpurun_out/r04z_c3/trace/run_kernel_trace.csv --last-ms 1500 > $O/timeline_c3.txt 2>&1
tail -20 $O/timeline_c3.txt
timeout -k 10 900 bash tools/pmc_profile.sh r04z_c5 --mesh icosphere_8 --res 1600 1600 --depth 16 --bounce-cap 16 \
  --spp-per-step 64 --steps 2 --warmup 1 > $O/pmc_c5.txt 2>&1 || { cat $O/pmc_c5.txt; exit 1; }
cat $O/pmc_c5.txt
