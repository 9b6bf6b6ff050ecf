# round-4 session u: C5's launch shape (pipeline depth, grid share, batch) -- swept on C3 only so far
set -o pipefail
O=gpurun_out/r04u
mkdir -p $O
C5="--spp-per-step 64 --mesh icosphere_8 --res 1600 1600 --depth 16 --bounce-cap 16 --steps 6"
bash tools/ab_run.sh 2 "def=tree=$C5" "p6=tree=$C5 --pipeline 6" "p10=tree=$C5 --pipeline 10" "p4=tree=$C5 --pipeline 4" \
  "gf30=tree=$C5 --tune trace_grid_frac=0.3" "gf20=tree=$C5 --tune trace_grid_frac=0.2" "b8=tree=$C5 --batch 8" > $O/ab.txt 2>&1 || exit $?
cat $O/ab.txt
C3="--spp-per-step 64 --steps 8"
bash tools/ab_run.sh 3 "c3_tree=tree=$C3" "c3_pre=pre=$C3" > $O/ab_pre.txt 2>&1 || exit $?
cat $O/ab_pre.txt
