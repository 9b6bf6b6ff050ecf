# round-4 session j: the super-clusters' slabs in the first cull level (knob super_slab) -- parity, then A/B
set -o pipefail
O=gpurun_out/r04j
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_stress_c5.py -m gpu -x -v \
  --timeout 300 --timeout-method thread -k "cluster_cull or tuning or derived_box or c5" \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
C5="--spp-per-step 64 --mesh icosphere_8 --res 1600 1600 --depth 16 --bounce-cap 16 --steps 8"
bash tools/ab_run.sh 2 "c5_sslab=tree=$C5" "c5_nosslab=tree=$C5 --tune super_slab=0" > $O/ab.txt 2>&1 || exit $?
cat $O/ab.txt
KDPT_PROF_RES=1600x1600 KDPT_PROF_DEPTH=16 KDPT_PROF_CAP=16 timeout -k 10 300 python -u tools/batch_profile.py icosphere_8 4x16 > $O/wave_c5.log 2>&1 || exit $?
tail -1 $O/wave_c5.log | cut -c1-600
