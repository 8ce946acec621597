cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread -k "gemv" > gpurun_out/kern.log 2>&1 && echo "kern ok" >> gpurun_out/rc.log &&
timeout -k 10 900 python -u -m pytest tests/test_full_parity.py -x -q -m gpu -p no:cacheprovider --timeout 600 --timeout-method thread -s -k batch8 > gpurun_out/par.log 2>&1 && echo "par ok" >> gpurun_out/rc.log &&
timeout -k 10 600 python bench.py --pages-per-gpu 8 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench8.log 2>&1 && echo "bench8 ok" >> gpurun_out/rc.log &&
DSOCR_DENSE_MM=0 timeout -k 10 600 python bench.py --pages-per-gpu 8 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench8_nodense.log 2>&1 && echo "bench8b ok" >> gpurun_out/rc.log
