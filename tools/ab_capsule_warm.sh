set -e
mkdir -p gpurun_out
for k in 0.2 0.05 0.01 0.002; do for h in 0.5 0.2 0.05; do
 NMPC_AMD_WARM_KAPPA=$k NMPC_AMD_SIGMA_HI=$h timeout -k 10 60 build/capsule_latency 300 > gpurun_out/cwab_${k}_${h}.json 2>/dev/null
 echo "k=$k h=$h $(cat gpurun_out/cwab_${k}_${h}.json)"
done; done
