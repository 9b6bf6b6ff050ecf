# round-4 session p: small-leaf triangles loaded two rounds ahead (variant pf2) against one round (tree);
# the big-leaf threshold re-checked with the one-level oriented-box cull (bl32, bl128)
set -o pipefail
O=gpurun_out/r04p
mkdir -p $O
C3="--spp-per-step 64 --steps 8"
bash tools/ab_run.sh 2 "c3_pf1=tree=$C3" "c3_pf2=pf2=$C3" "c3_bl32=bl32=$C3" "c3_bl128=bl128=$C3" > $O/ab.txt 2>&1 || exit $?
cat $O/ab.txt
