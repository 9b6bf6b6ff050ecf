# round-4 session t: early_walk 16 / 12 / 8 against 24 on C5 and C3
set -o pipefail
O=gpurun_out/r04t
mkdir -p $O
C3="--spp-per-step 64 --steps 8"
C5="--spp-per-step 64 --mesh icosphere_8 --res 1600 1600 --depth 16 --bounce-cap 16 --steps 6"
bash tools/ab_run.sh 2 "c5_ew24=tree=$C5" "c5_ew16=tree=$C5 --tune early_walk=16" "c5_ew12=tree=$C5 --tune early_walk=12" \
  "c5_ew8=tree=$C5 --tune early_walk=8" "c5_ew16el8=tree=$C5 --tune early_walk=16 --tune early_leaf=8" > $O/ab.txt 2>&1 || exit $?
bash tools/ab_run.sh 3 "c3_ew24=tree=$C3" "c3_ew16=tree=$C3 --tune early_walk=16" "c3_ew20=tree=$C3 --tune early_walk=20" >> $O/ab.txt 2>&1 || exit $?
cat $O/ab.txt
