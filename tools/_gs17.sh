cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS -d gpurun_out/pmcv -o pmc --output-format csv -- python tools/prof_vision.py --reps 2 > gpurun_out/pmcv.log 2>&1 && echo "pmc ok" >> gpurun_out/rc.log
