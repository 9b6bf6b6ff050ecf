# round-4 session x: k_trace compiled for 4 waves per SIMD (128 VGPRs, no spills) instead of 5 (96 VGPRs)
set -o pipefail
O=gpurun_out/r04x
mkdir -p $O
C3="--spp-per-step 64 --steps 8"
C5="--spp-per-step 64 --mesh icosphere_8 --res 1600 1600 --depth 16 --bounce-cap 16 --steps 8"
bash tools/ab_run.sh 3 "c5_w5=tree=$C5" "c5_w4=w4=$C5" "c3_w5=tree=$C3" "c3_w4=w4=$C3" > $O/ab.txt 2>&1 || exit $?
cat $O/ab.txt
