cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread -k "gemm" > gpurun_out/kg.log 2>&1 && echo "kg ok" >> gpurun_out/rc.log &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_full_parity.py tests/test_golden.py -x -q -m gpu -p no:cacheprovider --timeout 500 --timeout-method thread > gpurun_out/model.log 2>&1 && echo "model ok" >> gpurun_out/rc.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pv -o pv -- python tools/prof_vision.py --reps 3 > gpurun_out/pv.log 2>&1 && echo "pv ok" >> gpurun_out/rc.log &&
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench1.log 2>&1 && echo "b1 ok" >> gpurun_out/rc.log &&
timeout -k 10 600 python bench.py --pages-per-gpu 8 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench8.log 2>&1 && echo "b8 ok" >> gpurun_out/rc.log
