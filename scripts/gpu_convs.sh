# conv-kernel iteration: numerics tests, per-shape conv timings, GEMM microbenchmark
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/conv && \
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/conv/tests.log 2>&1; rc=$?; tail -5 gpurun_out/conv/tests.log; \
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc, stopping"; exit $rc; fi; \
timeout -k 10 300 python scripts/bench_convs.py --torch 0 > gpurun_out/conv/convs.log 2>&1 && cat gpurun_out/conv/convs.log && \
timeout -k 10 300 python scripts/bench_gemm.py > gpurun_out/conv/gemm.log 2>&1; cat gpurun_out/conv/gemm.log
