# round-4 session aa: super-cluster size 8 / 32 clusters against 16 on C5
set -o pipefail
O=gpurun_out/r04aa
mkdir -p $O
C5="--spp-per-step 64 --mesh icosphere_8 --res 1600 1600 --depth 16 --bounce-cap 16 --steps 8"
bash tools/ab_run.sh 3 "c5_s16=tree=$C5" "c5_s8=s8=$C5" "c5_s32=s32=$C5" > $O/ab.txt 2>&1 || exit $?
cat $O/ab.txt
for f in c5_s8_1 c5_s32_1 c5_s16_1; do python -c "
import json; d=json.loads(open('gpurun_out/ab_run/$f.log').read().strip().splitlines()[-1]); print('$f', d['config']['intersect'])"; done
