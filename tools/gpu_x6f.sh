mkdir -p gpurun_out
for rep in 1 2; do
  for v in "p:" "thr:qp_thr0=0.5" "cold:qp_warm_start=0" "both:qp_thr0=0.5,qp_warm_start=0" "wi8:qp_warm_iter_max=8" "k1:qp_warm_kappa=1.0"; do
    n=${v%%:*}; q=${v#*:}
    if [ -z "$q" ]; then a=""; else a="--qp $q"; fi
    timeout -k 10 300 python bench.py --config metric --steps 60 --no-cpu-baseline $a > gpurun_out/x6f_metric_${n}$rep.json 2>> gpurun_out/x6f_err.log || exit 1
  done
done
