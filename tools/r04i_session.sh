# round-4 session i: the oriented-box second cull level (knob cluster_obb) -- parity, then A/B
set -o pipefail
O=gpurun_out/r04i
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_stress_c5.py tests/test_gpu_sharded.py -m gpu -x -v \
  --timeout 300 --timeout-method thread -k "cluster_cull or tuning or derived_box or c5 or sharded or render_" \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
C5="--spp-per-step 64 --mesh icosphere_8 --res 1600 1600 --depth 16 --bounce-cap 16 --steps 8"
bash tools/ab_run.sh 2 "c5_obb=tree=$C5" "c5_noobb=tree=$C5 --tune cluster_obb=0" "c5_head=head=$C5" > $O/ab.txt 2>&1 || exit $?
bash tools/ab_run.sh 1 "c3_tree=tree=--steps 10" "c3_head=head=--steps 10" >> $O/ab.txt 2>&1
cat $O/ab.txt
