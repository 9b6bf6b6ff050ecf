# round-4 session q: big-leaf threshold 32 (now the default) -- parity, then A/B against 64 and 48
set -o pipefail
O=gpurun_out/r04q
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_stress_c5.py -m gpu -x -v \
  --timeout 300 --timeout-method thread -k "pipelined or tuning or fullsize or cluster_cull or c3 or c5 or kd" \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
C3="--spp-per-step 64 --steps 8"
C5="--spp-per-step 64 --mesh icosphere_8 --res 1600 1600 --depth 16 --bounce-cap 16 --steps 8"
bash tools/ab_run.sh 3 "c3_bl32=tree=$C3" "c3_bl64=bl64=$C3" "c3_bl48=bl48=$C3" > $O/ab.txt 2>&1 || exit $?
bash tools/ab_run.sh 1 "c5_bl32=tree=$C5" "c5_bl64=bl64=$C5" >> $O/ab.txt 2>&1 || exit $?
cat $O/ab.txt
