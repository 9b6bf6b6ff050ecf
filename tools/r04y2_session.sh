# round-4 closing measurements: the driver's command twice more (run-to-run spread), bench.py under a one-rank
# RCCL process group (the library's own ncclReduce per frame), and C5 over more steps
set -o pipefail
O=gpurun_out/r04y2
mkdir -p $O
for k in 1 2; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_driver_$k.log 2>&1 || { tail -20 $O/bench_driver_$k.log; exit 1; }
done
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 1 --force-dist --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_force_dist.log 2>&1 || { tail -20 $O/bench_force_dist.log; exit 1; }
timeout -k 10 400 python -u bench.py --no-cpu-baseline --mesh icosphere_8 --res 1600 1600 --depth 16 --bounce-cap 16 \
  --spp-per-step 64 --steps 30 --warmup 3 > $O/bench_c5.log 2>&1 || { tail -20 $O/bench_c5.log; exit 1; }
for f in bench_driver_1 bench_driver_2 bench_force_dist bench_c5; do python -c "
import json; d=json.loads([l for l in open('$O/$f.log').read().splitlines() if l.startswith('{\"metric\"')][-1])
print('$f', d['value'], d['ms_per_step'], d['config']['parallelism'], d['roofline'].get('chip_wide_frac'))"; done
