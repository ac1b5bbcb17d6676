cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-c1 --no-cdr > gpurun_out/pipe_T.json 2> gpurun_out/pipe_T.err || exit $?
timeout -k 10 300 python bench.py --workload C3 --steps 20 --warmup 5 --no-cpu-baseline --no-c1 --no-cdr > gpurun_out/pipe_C3.json 2> gpurun_out/pipe_C3.err || exit $?
