#!/bin/bash
# Diagnose "no HIP device" from libcpg under pytest: which test module's import breaks it.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for m in conftest test_abi test_cli test_dist test_format test_oracle test_ref_constants test_gpu_c3 test_gpu_c5 test_gpu_cli test_gpu_general test_gpu_workspace test_gpu_parity; do
  timeout -k 5 60 python3 -c "
import sys; sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import importlib; importlib.import_module('$m')
import torch; torch.cuda.is_available()
from cpgisland_amd import Context
try:
    x = Context(0); print('$m ok'); x.close()
except Exception as e: print('$m FAIL', e)
" 2>&1 | grep -v amdgpu.ids | tail -1
done
timeout -k 5 120 python3 -m pytest tests/test_gpu_c3.py -m gpu -x -q -p no:cacheprovider 2>&1 | tail -2
