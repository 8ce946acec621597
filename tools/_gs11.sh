cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread -k "decode_attention" > gpurun_out/kat.log 2>&1 && echo "kat ok" >> gpurun_out/rc.log &&
KB_STAMPS=1 timeout -k 10 120 ./tools/kbench attn1 attn8 > gpurun_out/kb_auto.log 2>&1 &&
DSOCR_ATT_NSUB=4 timeout -k 10 120 ./tools/kbench attn8 > gpurun_out/kb_n4.log 2>&1 &&
DSOCR_ATT_NSUB=1 timeout -k 10 120 ./tools/kbench attn8 > gpurun_out/kb_n1.log 2>&1 &&
DSOCR_ATT_EARLY=0 timeout -k 10 120 ./tools/kbench attn1 > gpurun_out/kb_e0.log 2>&1 && echo "kb ok" >> gpurun_out/rc.log
