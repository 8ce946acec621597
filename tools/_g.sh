cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
rm -rf gpurun_out/trv
DSOCR_NO_GRAPH=1 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/trv -o tr --output-format csv -- python -u tools/prof_decode.py --max-new 2 --iters 1 --tag trace > gpurun_out/trv.log 2>&1 || exit $?
