cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./tools/mb_barrier > gpurun_out/mb_barrier.log 2>&1 && echo "mbb ok" >> gpurun_out/rc.log &&
DSOCR_CAPTURE_RELAXED=1 DSOCR_GRAPH_SYNC=16 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/gprof -o g --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/gprof.log 2>&1 && echo "gprof ok" >> gpurun_out/rc.log
