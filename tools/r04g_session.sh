# round-4 session g: k_trace refill through an LDS pointer table (parity first), then A/B against HEAD
set -o pipefail
O=gpurun_out/r04g
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -v \
  --timeout 300 --timeout-method thread -k "sharded or render_ or bench or pipelined or tuning or entry_points or fullsize or iteration2 or counters or c3 or c4" \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/ab_run.sh 2 "head=head=--steps 10" "lt16=tree=--steps 10" "lt32=lt32=--steps 10 --batch 32 --pipeline 8" "lt32p6=lt32=--steps 10 --batch 32 --pipeline 6" > $O/ab.txt 2>&1 || exit $?
cat $O/ab.txt
C4="--scene cornell8 --no-cpu-baseline"
timeout -k 10 300 python -u bench.py $C4 --spp-per-step 32 --steps 160 --warmup 20 > $O/c4_32.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py $C4 --spp-per-step 256 --steps 20 --warmup 3 > $O/c4_256.log 2>&1 || exit $?
for f in c4_32 c4_256; do python -c "
import json; d=json.loads(open('$O/$f.log').read().strip().splitlines()[-1])
print('$f', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['k_trace_busy_share'])"; done
