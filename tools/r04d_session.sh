# round-4 session d: new cull margins + native multi-GPU entry points on the GPU (parity), C5 margin A/B
set -o pipefail
C5="--spp-per-step 64 --mesh icosphere_8 --res 1600 1600 --depth 16 --bounce-cap 16"
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded.py -m gpu -x -v --timeout 300 \
  --timeout-method thread -k "cluster_cull or tuning_knobs or derived_box or pipelined or render_" \
  > gpurun_out/r04d_tests.log 2>&1 || exit $?
bash tools/ab_run.sh 2 "c5_tree=tree=--steps 8 $C5" "c5_fast=tree=--steps 8 $C5 --tune cull_margin=1e-4" > gpurun_out/r04d_ab.txt 2>&1
