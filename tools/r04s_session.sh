# round-4 session s: the node/leaf hand-over thresholds on C5 (swept on C3 only so far)
set -o pipefail
O=gpurun_out/r04s
mkdir -p $O
C5="--spp-per-step 64 --mesh icosphere_8 --res 1600 1600 --depth 16 --bounce-cap 16 --steps 6"
bash tools/ab_run.sh 2 "def=tree=$C5" "ew16=tree=$C5 --tune early_walk=16" "ew32=tree=$C5 --tune early_walk=32" \
  "el8=tree=$C5 --tune early_leaf=8" "el16=tree=$C5 --tune early_leaf=16" "ew32el16=tree=$C5 --tune early_walk=32 --tune early_leaf=16" \
  "ew40=tree=$C5 --tune early_walk=40" > $O/ab.txt 2>&1 || exit $?
cat $O/ab.txt
