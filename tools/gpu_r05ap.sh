#!/bin/bash
# bias solver at K = 37 (KP = 42 with padded rows) and K = 43 (KP = 44) against the CPU path
set -o pipefail
O=gpurun_out/r05ap; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_eigen.py -k "matches_reference_path or agree_on_pipeline" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
