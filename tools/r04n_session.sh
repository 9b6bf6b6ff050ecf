# round-4 session n: triangle materials looked up once per ray (at its end) instead of per leaf phase
set -o pipefail
O=gpurun_out/r04n
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_stress_c5.py -m gpu -x -v \
  --timeout 300 --timeout-method thread -k "pipelined or tuning or fullsize or cluster_cull or c5 or c3" \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
C3="--spp-per-step 64 --steps 8"
C5="--spp-per-step 64 --mesh icosphere_8 --res 1600 1600 --depth 16 --bounce-cap 16 --steps 8"
bash tools/ab_run.sh 2 "c5_defer=tree=$C5" "c5_early=early=$C5" "c3_defer=tree=$C3" "c3_early=early=$C3" > $O/ab.txt 2>&1 || exit $?
cat $O/ab.txt
