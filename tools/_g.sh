cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -k "attention" > gpurun_out/t_att.log 2>&1; echo "rc=$?" >> gpurun_out/t_att.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -k "tiny or full_page or image" > gpurun_out/t_all.log 2>&1; echo "rc=$?" >> gpurun_out/t_all.log
timeout -k 10 300 python -u tools/prof_decode.py --tag rel --max-new 8 --iters 2 >> gpurun_out/prof.jsonl 2>gpurun_out/prof_err.log || exit $?
rm -rf gpurun_out/trv
DSOCR_NO_GRAPH=1 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/trv -o tr --output-format csv -- python -u tools/prof_decode.py --max-new 2 --iters 1 --tag trace > gpurun_out/trv.log 2>&1 || exit $?
