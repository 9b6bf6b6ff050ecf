# round-4 session o: the one-level cluster cull (C3's route) also tests the box survivors' oriented boxes
set -o pipefail
O=gpurun_out/r04o
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -v \
  --timeout 300 --timeout-method thread -k "pipelined or tuning or fullsize or cluster_cull or c3" \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
C3="--spp-per-step 64 --steps 8"
bash tools/ab_run.sh 3 "c3_fobb=tree=$C3" "c3_nofobb=tree=$C3 --tune flat_obb=0" > $O/ab.txt 2>&1 || exit $?
cat $O/ab.txt
timeout -k 10 300 python -u tools/batch_profile.py dragon_5 8x16 > $O/wave_c3.log 2>&1 || exit $?
tail -1 $O/wave_c3.log | cut -c1-1500
