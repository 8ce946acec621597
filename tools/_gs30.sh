cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread -k "decode_attention" > gpurun_out/kat.log 2>&1 && echo "kat ok" >> gpurun_out/rc.log &&
KB_STAMPS=1 timeout -k 10 120 ./tools/kbench attn1 attn8 > gpurun_out/kb_p1.log 2>&1 &&
DSOCR_ATT_POLL=0 timeout -k 10 120 ./tools/kbench attn1 attn8 > gpurun_out/kb_p0.log 2>&1 && echo "kb ok" >> gpurun_out/rc.log
