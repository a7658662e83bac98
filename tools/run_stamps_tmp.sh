cd $GRAFT_REPO_ROOT
timeout -k 10 120 python tools/phase_stamps.py diff 4096 40 > gpurun_out/st_diff4096.txt 2>&1; echo "st rc=$?"
timeout -k 10 120 python tools/phase_stamps.py diff 1024 40 > gpurun_out/st_diff1024.txt 2>&1; echo "st rc=$?"
bash tools/pmc.sh r02p1_metric --config metric
