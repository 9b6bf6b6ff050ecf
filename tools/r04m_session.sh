# round-4 session m: cull records requested early (super slab before the box test, oriented boxes before the
# ray exchange) -- parity, then A/B
set -o pipefail
O=gpurun_out/r04m
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_stress_c5.py -m gpu -x -v \
  --timeout 300 --timeout-method thread -k "cluster_cull or tuning or c5 or pipelined" \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
C3="--spp-per-step 64 --steps 8"
C5="--spp-per-step 64 --mesh icosphere_8 --res 1600 1600 --depth 16 --bounce-cap 16 --steps 8"
bash tools/ab_run.sh 2 "c5_early=tree=$C5" "c5_nocl=nocl=$C5" "c5_prev=prev=$C5" "c3_early=tree=$C3" "c3_prev=prev=$C3" > $O/ab.txt 2>&1 || exit $?
cat $O/ab.txt
