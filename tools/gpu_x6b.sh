mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_reference_wrappers.py tests/test_gpu_golden.py tests/test_gpu_split.py tests/test_gpu_seg.py > gpurun_out/x6b_tests.log 2>&1 || exit 1
timeout -k 10 200 python tools/tick_dump.py omni4 260 2 gpurun_out/tick_dump_omni4.npz > gpurun_out/x6b_dump.log 2>&1 || exit 1
timeout -k 10 200 python tools/tick_dump.py tric 260 2 gpurun_out/tick_dump_tric.npz >> gpurun_out/x6b_dump.log 2>&1
