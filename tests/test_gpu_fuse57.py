"""The fused forward + traceback Viterbi kernel (k_vit_fwdtrace, opt-in: CPG_VIT_FUSE57=1,
read once per process) — run in a child process with the variable set, so that this
process's library keeps the default two-kernel path."""
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.gpu
def test_fused_forward_traceback_vs_oracle():
    env = dict(os.environ, CPG_VIT_FUSE57="1")
    r = subprocess.run([sys.executable, os.path.join(HERE, "fuse57_check.py")], env=env,
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "fuse57 ok" in r.stdout, (r.returncode, r.stdout[-2000:],
                                                           r.stderr[-4000:])
