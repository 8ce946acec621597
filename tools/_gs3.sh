cd $GRAFT_REPO_ROOT
bash tools/gpu_session.sh dots
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -m gpu -rf -p no:cacheprovider --timeout 200 --timeout-method thread -k "attention_bf16 or moe_decode_full" > gpurun_out/k2.log 2>&1; echo "rc=$? k2" >> gpurun_out/rc.log
bash tools/gpu_session.sh benchdots bench
echo "session rc=$?" >> gpurun_out/rc.log
