# round-4 session l: candidate rays written in queue order (cray) -- parity, then A/B against the last commit
set -o pipefail
O=gpurun_out/r04l
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_sharded.py -m gpu -x -v \
  --timeout 300 --timeout-method thread -k "pipelined or tuning or fullsize or sharded or render_ or cluster_cull or c3 or c4" \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
C3="--spp-per-step 64 --steps 8"
C5="--spp-per-step 64 --mesh icosphere_8 --res 1600 1600 --depth 16 --bounce-cap 16 --steps 8"
bash tools/ab_run.sh 2 "c3_cray=tree=$C3" "c3_prev=prev=$C3" "c5_cray=tree=$C5" "c5_prev=prev=$C5" > $O/ab.txt 2>&1 || exit $?
cat $O/ab.txt
