mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bloom.py -q --maxfail=5 --timeout 300 --timeout-method thread -k "partitioned or skew or overflow or bloom or reused" > gpurun_out/t3.log 2>&1
rc=$?; tail -3 gpurun_out/t3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b3_c2.json 2> gpurun_out/b3_c2.err && \
timeout -k 10 300 python bench.py --config C2S --no-cpu-baseline > gpurun_out/b3_c2s.json 2> gpurun_out/b3_c2s.err && \
bash tools/gpu_prof2.sh c2v3 "--config C2" c2sv3 "--config C2S"
