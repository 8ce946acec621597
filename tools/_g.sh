cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for pf in 0 1 3 7 15 31 16; do DSOCR_FUSED_MOE=0 DSOCR_PF=$pf timeout -k 10 300 python -u tools/prof_decode.py --tag pf$pf >> gpurun_out/prof.jsonl 2>gpurun_out/prof_err.log || exit $?; done
DSOCR_FUSED_MOE=0 DSOCR_PF=15 timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -k "full" > gpurun_out/t_model.log 2>&1 || exit $?
