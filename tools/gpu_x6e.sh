mkdir -p gpurun_out
for c in diff1024 omni4 tric mixed; do for rep in 1 2; do
  timeout -k 10 300 python bench.py --config $c --steps 60 --no-cpu-baseline > gpurun_out/x6e_${c}_product$rep.json 2>> gpurun_out/x6e_err.log || exit 1
  timeout -k 10 300 python bench.py --config $c --steps 60 --no-cpu-baseline --ipm-rules acados > gpurun_out/x6e_${c}_acados$rep.json 2>> gpurun_out/x6e_err.log || exit 1
done; done
