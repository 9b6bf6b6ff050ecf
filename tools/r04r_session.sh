# round-4 session r: big-leaf threshold 48 (now the default) -- parity, then A/B against 64, 56, 40
set -o pipefail
O=gpurun_out/r04r
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_stress_c5.py -m gpu -x -v \
  --timeout 300 --timeout-method thread -k "pipelined or tuning or fullsize or cluster_cull or c3 or c5 or kd" \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
C3="--spp-per-step 64 --steps 8"
bash tools/ab_run.sh 3 "c3_bl48=tree=$C3" "c3_bl64=bl64=$C3" "c3_bl56=bl56=$C3" "c3_bl40=bl40=$C3" > $O/ab.txt 2>&1 || exit $?
cat $O/ab.txt
bash tools/r04s_session.sh || exit $?
