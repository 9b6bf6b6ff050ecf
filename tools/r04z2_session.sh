# round-4 final session 2 (after the PMC summaries are committed): the driver's bench command with the CPU
# baseline, C5, C4's per-GPU frame shapes and strong-scaling split at N = 1, and the kernel trace of the
# driver's command for profiles/
set -o pipefail
O=gpurun_out/r04z2
mkdir -p $O
export TMPDIR=/tmp
# the zero fills moved onto the contexts' streams (host-side change): the multi-context and pipelined tests again
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 \
  --timeout-method thread -k "pipelined or sharded or render_ or bench or tuning" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || { tail -20 $O/bench_driver.log; exit 1; }
tail -c 400 $O/bench_driver.log; echo
timeout -k 10 300 python -u bench.py --no-cpu-baseline --mesh icosphere_8 --res 1600 1600 --depth 16 --bounce-cap 16 \
  --spp-per-step 64 --steps 12 --warmup 2 > $O/bench_c5.log 2>&1 || { tail -20 $O/bench_c5.log; exit 1; }
tail -c 300 $O/bench_c5.log; echo
C4="--scene cornell8 --no-cpu-baseline"
timeout -k 10 300 python -u bench.py $C4 --spp-per-step 32 --steps 160 --warmup 20 > $O/c4_32.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py $C4 --spp-per-step 256 --steps 20 --warmup 3 > $O/c4_256.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py $C4 --total-spp 256 --steps 20 --warmup 3 > $O/c4_strong.log 2>&1 || exit $?
for f in c4_32 c4_256 c4_strong; do python -c "
import json; d=json.loads(open('$O/$f.log').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d['scaling'])"; done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline \
  > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
tail -c 300 $O/trace.log; echo
