set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/dmadg2
for i in 1 2; do for v in 0 1; do
  MLC_GEMM_DMA=$v timeout -k 10 300 python bench.py > gpurun_out/dmadg2/resnet_dma${v}_$i.log 2>&1 || exit 1
  echo "resnet dma=$v run $i: $(tail -1 gpurun_out/dmadg2/resnet_dma${v}_$i.log | cut -c60-100)"
done; done
