# round-4 session w: the oriented-box cull by quarters (each cluster's four 16-triangle quarters' in-plane
# bounds) -- parity, A/B against the whole cluster's box, and the sweeps per ray
set -o pipefail
O=gpurun_out/r04w
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_stress_c5.py -m gpu -x -v \
  --timeout 300 --timeout-method thread -k "pipelined or tuning or fullsize or cluster_cull or c3 or c5" \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
C3="--spp-per-step 64 --steps 8"
C5="--spp-per-step 64 --mesh icosphere_8 --res 1600 1600 --depth 16 --bounce-cap 16 --steps 8"
bash tools/ab_run.sh 3 "c5_sub=tree=$C5" "c5_nosub=nosub=$C5" "c3_sub=tree=$C3" "c3_nosub=nosub=$C3" > $O/ab.txt 2>&1 || exit $?
cat $O/ab.txt
KDPT_PROF_RES=1600x1600 KDPT_PROF_DEPTH=16 KDPT_PROF_CAP=16 timeout -k 10 300 python -u tools/batch_profile.py icosphere_8 4x16 > $O/wave_c5.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/batch_profile.py dragon_5 8x16 > $O/wave_c3.log 2>&1 || exit $?
for f in wave_c5 wave_c3; do tail -2 $O/$f.log | head -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['per_ray']; print('$f', {k:p[k] for k in ['big_sweeps','big_pass','big_cycles','big_cull_cycles']})"; done
