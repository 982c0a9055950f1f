#!/bin/bash
# Round-6 session m: the batch renderer's GPU tests (the new sugar_shading mode against the per-view loop).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_batch_renderer.py -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r06m_tests.log 2>&1 || { tail -40 gpurun_out/r06m_tests.log; exit 1; }
tail -3 gpurun_out/r06m_tests.log
