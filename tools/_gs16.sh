cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread -k "gemm" > gpurun_out/kg.log 2>&1 && echo "kg ok" >> gpurun_out/rc.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pv -o pv -- python tools/prof_vision.py --reps 3 > gpurun_out/pv.log 2>&1 && echo "pv ok" >> gpurun_out/rc.log
