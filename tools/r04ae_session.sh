# round-4 session ae: bench.py also reports the HIP-event launch time (compare with rocprofv3's kernel trace)
set -o pipefail
O=gpurun_out/r04ae
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py -m gpu -x -v --timeout 300 --timeout-method thread -k "bench" \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
python -c "
import json; d=json.loads([l for l in open('$O/bench.log').read().splitlines() if l.startswith('{\"metric\"')][-1]); r=d['roofline']
print(d['value'], r['avg_launch_ms'], r['avg_launch_ms_hip_events'], r['launches'])"
