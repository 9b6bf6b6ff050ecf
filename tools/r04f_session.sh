# round-4 session f: frames stay in flight across frames (slot groups in turn, reduces on their own stream):
# parity, C3/C4 benches, a pipeline sweep at batch 16, then the kernel trace + PMC passes of the default build
set -o pipefail
O=gpurun_out/r04f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 \
  --timeout-method thread -k "sharded or render_ or bench or pipelined or tuning or entry_points" \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/c3.log 2>&1 || exit $?
C4="--scene cornell8 --no-cpu-baseline"
timeout -k 10 300 python -u bench.py $C4 --spp-per-step 32 --steps 160 --warmup 20 > $O/c4_32.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py $C4 --spp-per-step 256 --steps 20 --warmup 3 > $O/c4_256.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py $C4 --spp-per-step 32 --steps 160 --warmup 20 --batch 8 > $O/c4_32_b8.log 2>&1 || exit $?
for f in c3 c4_32 c4_256 c4_32_b8; do python -c "
import json; d=json.loads(open('$O/$f.log').read().strip().splitlines()[-1])
print('$f', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['k_trace_busy_share'])"; done
bash tools/ab_run.sh 1 "p6=tree=--steps 10 --pipeline 6" "p10=tree=--steps 10 --pipeline 10" "p12=tree=--steps 10 --pipeline 12" "p8=tree=--steps 10 --pipeline 8" > $O/sweep.txt 2>&1 || exit $?
cat $O/sweep.txt
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > $O/trace.log 2>&1 || exit $?
python tools/timeline.py $O/trace/run_kernel_trace.csv --last-ms 1000 > $O/timeline.txt 2>&1; cat $O/timeline.txt
