# round-4 session ad: MAXB 32 (32 iterations per intersect launch) on C5, and its cost to C3 at batch 16
set -o pipefail
O=gpurun_out/r04ad
mkdir -p $O
C3="--spp-per-step 64 --steps 8"
C5="--spp-per-step 64 --mesh icosphere_8 --res 1600 1600 --depth 16 --bounce-cap 16 --steps 8"
bash tools/ab_run.sh 2 "c5_m16=tree=$C5" "c5_m32b32=m32=$C5 --batch 32" "c5_m32b32p4=m32=$C5 --batch 32 --pipeline 4" "c3_m16=tree=$C3" "c3_m32b16=m32=$C3" > $O/ab.txt 2>&1 || exit $?
cat $O/ab.txt
