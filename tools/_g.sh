cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1; echo "rc=$?" >> gpurun_out/t_all.log
for f in 1 0; do DSOCR_GEMM_BF16=$f timeout -k 10 300 python -u tools/prof_decode.py --tag g16_$f --max-new 8 --iters 2 >> gpurun_out/prof.jsonl 2>gpurun_out/prof_err.log || exit $?; done
