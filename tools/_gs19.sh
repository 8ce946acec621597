cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python bench.py --steps 1 --warmup 0 --max-new-tokens 16 --no-cpu-baseline --roofline-iters 2"
DSOCR_NO_GRAPH=1 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pf1 -o pmc --output-format csv -- $B > gpurun_out/pf1.log 2>&1 && echo "pf1 ok" >> gpurun_out/rc.log &&
DSOCR_NO_GRAPH=1 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pw1 -o pmc --output-format csv -- $B > gpurun_out/pw1.log 2>&1 && echo "pw1 ok" >> gpurun_out/rc.log &&
DSOCR_NO_GRAPH=1 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pf8 -o pmc --output-format csv -- $B --pages-per-gpu 8 > gpurun_out/pf8.log 2>&1 && echo "pf8 ok" >> gpurun_out/rc.log &&
DSOCR_NO_GRAPH=1 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pw8 -o pmc --output-format csv -- $B --pages-per-gpu 8 > gpurun_out/pw8.log 2>&1 && echo "pw8 ok" >> gpurun_out/rc.log &&
DSOCR_NO_GRAPH=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o b1 --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof1.log 2>&1 && echo "prof1 ok" >> gpurun_out/rc.log &&
DSOCR_NO_GRAPH=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof8 -o b8 --output-format csv -- python bench.py --pages-per-gpu 8 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof8.log 2>&1 && echo "prof8 ok" >> gpurun_out/rc.log
