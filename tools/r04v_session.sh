# round-4 session v: 40-byte cluster triangle records (C5's sweeps stream ~6 KB per ray from HBM) -- parity, A/B
set -o pipefail
O=gpurun_out/r04v
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_stress_c5.py -m gpu -x -v \
  --timeout 300 --timeout-method thread -k "pipelined or tuning or fullsize or cluster_cull or c3 or c5" \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
C3="--spp-per-step 64 --steps 8"
C5="--spp-per-step 64 --mesh icosphere_8 --res 1600 1600 --depth 16 --bounce-cap 16 --steps 8"
bash tools/ab_run.sh 3 "c5_tri40=tree=$C5" "c5_tri48=tri48=$C5" "c3_tri40=tree=$C3" "c3_tri48=tri48=$C3" > $O/ab.txt 2>&1 || exit $?
cat $O/ab.txt
