mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread -m gpu tests/test_gpu_fleet.py -k full_batch_replay > gpurun_out/x6d_tests.log 2>&1 || exit 1
for rep in 1 2; do
  timeout -k 10 300 python bench.py --config metric > gpurun_out/x6d_metric_product$rep.json 2> gpurun_out/x6d_err.log || exit 1
  timeout -k 10 300 python bench.py --config metric --ipm-rules acados > gpurun_out/x6d_metric_acados$rep.json 2>> gpurun_out/x6d_err.log || exit 1
done
