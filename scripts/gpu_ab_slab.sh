cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ab && \
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/ab/slab1.log 2>&1 && tail -1 gpurun_out/ab/slab1.log | cut -c1-200 && \
MLC_WGRAD_SLAB=0 timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/ab/slab0.log 2>&1 && tail -1 gpurun_out/ab/slab0.log | cut -c1-200 && \
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/ab/slab1b.log 2>&1 && tail -1 gpurun_out/ab/slab1b.log | cut -c1-200 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab/prof -o resnet -- python3 bench.py --steps 6 --warmup 3 --graph 0 > gpurun_out/ab/prof.log 2>&1 && \
python scripts/prof_summary.py gpurun_out/ab/prof/resnet_kernel_stats.csv 9 > gpurun_out/ab/summary.txt && head -40 gpurun_out/ab/summary.txt
