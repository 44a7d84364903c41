cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 600 python tools/sweep.py > gpurun_out/sweep.log 2>&1; echo sweep rc=$?; cat gpurun_out/sweep.log | grep case; \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o prof --output-format csv -- python bench.py --rows 125000000 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/bench_prof.json 2>&1; echo prof rc=$?; \
SKIP_BENCH=1 bash tools/gpu_check.sh
