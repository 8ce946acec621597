cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_kernels.py -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1; echo "rc=$?" >> gpurun_out/t_all.log
DSOCR_SCREEN_STATS=1 timeout -k 10 300 python -u tools/prof_decode.py --tag stats --iters 2 > gpurun_out/stats.log 2>&1 || exit 1
rm -f gpurun_out/prof.jsonl
for f in 1 0; do DSOCR_SCREEN=$f timeout -k 10 300 python -u tools/prof_decode.py --tag scr$f >> gpurun_out/prof.jsonl 2>gpurun_out/prof_err.log || exit $?; done
