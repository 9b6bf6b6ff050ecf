# round-4 session k: super-cluster slabs in LDS (SUPER 32, 48-byte records) against the HBM slab and none
set -o pipefail
O=gpurun_out/r04k
mkdir -p $O
C5="--spp-per-step 64 --mesh icosphere_8 --res 1600 1600 --depth 16 --bounce-cap 16 --steps 8"
bash tools/ab_run.sh 2 "tree=tree=$C5" "tree_noss=tree=$C5 --tune super_slab=0" "s32r3=s32r3=$C5" "s32r3_noss=s32r3=$C5 --tune super_slab=0" > $O/ab.txt 2>&1 || exit $?
cat $O/ab.txt
for f in gpurun_out/ab_run/s32r3_1.log gpurun_out/ab_run/tree_1.log; do python -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['config']['intersect'])"; done
