# round-4 session e: parity of the new pieces (cull margins, MAXB 16, native frames / sharded render),
# then the new bench defaults (C3), C4's per-GPU frame shape, C5 margin A/B
set -o pipefail
O=gpurun_out/r04e
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded.py -m gpu -x -v --timeout 300 \
  --timeout-method thread -k "cluster_cull or tuning_knobs or derived_box or pipelined or sharded or render_ or bench" \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/c3.log 2>&1 || exit $?
tail -c 400 $O/c3.log | head -c 0
C4="--scene cornell8 --no-cpu-baseline"
timeout -k 10 300 python -u bench.py $C4 --spp-per-step 32 --steps 160 --warmup 20 > $O/c4_32.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py $C4 --spp-per-step 256 --steps 20 --warmup 3 > $O/c4_256.log 2>&1 || exit $?
C5="--spp-per-step 64 --mesh icosphere_8 --res 1600 1600 --depth 16 --bounce-cap 16 --no-cpu-baseline --steps 8 --warmup 2"
C5AB="--spp-per-step 64 --mesh icosphere_8 --res 1600 1600 --depth 16 --bounce-cap 16 --steps 8"
timeout -k 10 300 python -u bench.py $C5 > $O/c5.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py $C5 --tune cull_margin=1e-4 > $O/c5_fast.log 2>&1 || exit $?
for f in c3 c4_32 c4_256 c5 c5_fast; do python -c "
import json; d=json.loads(open('$O/$f.log').read().strip().splitlines()[-1])
print('$f', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['config']['intersect'].get('cull_margin'), d['config']['intersect'].get('cull_exact'))"; done
# CLUSTER 32 (two (ray, cluster) pairs per sweep round) against the tree's 64, and the strict no-cull route
bash tools/ab_run.sh 2 "c3_tree=tree=--steps 10" "c3_c32=c32=--steps 10" > $O/ab_c32.txt 2>&1 || exit $?
bash tools/ab_run.sh 1 "c5_tree=tree=$C5AB" "c5_c32=c32=$C5AB" "c3_nocull=tree=--steps 4 --tune cluster_cull=0" >> $O/ab_c32.txt 2>&1
cat $O/ab_c32.txt
