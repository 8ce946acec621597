cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread -k "attention" > gpurun_out/katt.log 2>&1 && echo "katt ok" >> gpurun_out/rc.log &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_full_parity.py tests/test_golden.py -x -q -m gpu -p no:cacheprovider --timeout 500 --timeout-method thread > gpurun_out/model.log 2>&1 && echo "model ok" >> gpurun_out/rc.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pv -o pv -- python tools/prof_vision.py --reps 3 > gpurun_out/pv.log 2>&1 && echo "pv ok" >> gpurun_out/rc.log
