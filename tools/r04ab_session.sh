# round-4 session ab: C3's one-level cull requesting the oriented-box records together with the box (variant fe)
set -o pipefail
O=gpurun_out/r04ab
mkdir -p $O
C3="--spp-per-step 64 --steps 8"
bash tools/ab_run.sh 3 "c3_tree=tree=$C3" "c3_fe=fe=$C3" > $O/ab.txt 2>&1 || exit $?
cat $O/ab.txt
