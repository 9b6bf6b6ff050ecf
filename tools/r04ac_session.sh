# round-4 session ac: the max-memory-clause machine scheduler (all kernels) against max-ilp
set -o pipefail
O=gpurun_out/r04ac
mkdir -p $O
C3="--spp-per-step 64 --steps 8"
C5="--spp-per-step 64 --mesh icosphere_8 --res 1600 1600 --depth 16 --bounce-cap 16 --steps 8"
bash tools/ab_run.sh 2 "c3_ilp=tree=$C3" "c3_memcl=memcl=$C3" "c5_ilp=tree=$C5" "c5_memcl=memcl=$C5" > $O/ab.txt 2>&1 || exit $?
cat $O/ab.txt
