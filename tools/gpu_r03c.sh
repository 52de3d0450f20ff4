# Round 3, call 3: LDS-DMA issue cost beside an MFMA stream, by instruction form
# (tools/probe_dma_issue.hip; profiles/r03_dma_issue_probe.txt), then the device-buffer check
set -u
mkdir -p gpurun_out/r03c
timeout -k 10 120 tools/bin/probe_dma_issue > gpurun_out/r03c/probe.txt 2>&1; rc=$?
cat gpurun_out/r03c/probe.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -k "host_buffers or kmap" -x -v --timeout 120 --timeout-method thread > gpurun_out/r03c/t.log 2>&1; rc=$?
tail -3 gpurun_out/r03c/t.log; exit $rc
