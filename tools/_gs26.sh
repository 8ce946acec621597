cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
DSOCR_GEMM_NJ=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread -k "gemm_f32a" > gpurun_out/kg4.log 2>&1 && echo "kg4 ok" >> gpurun_out/rc.log &&
DSOCR_GEMM_NJ=4 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pv4 -o pv -- python tools/prof_vision.py --reps 3 > gpurun_out/pv4.log 2>&1 &&
timeout -k 10 300 python bench.py --pages-per-gpu 8 --steps 2 --warmup 1 --no-cpu-baseline --max-new-tokens 32 > gpurun_out/b8_nj2.log 2>&1 &&
DSOCR_GEMM_NJ=4 timeout -k 10 300 python bench.py --pages-per-gpu 8 --steps 2 --warmup 1 --no-cpu-baseline --max-new-tokens 32 > gpurun_out/b8_nj4.log 2>&1 && echo "ab ok" >> gpurun_out/rc.log
