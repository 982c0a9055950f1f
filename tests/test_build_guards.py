"""The product library cannot be built with a timing-experiment switch (GSR_EXP_*: parts of the blends compiled
out, wrong results by design): gsr_common.h refuses them unless GSR_DIAG_BUILD (`make exp`) is defined."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "threestudio-3dgs_amd", "csrc")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


def _preprocess(*defs):
    return subprocess.run([HIPCC, "-E", "-x", "hip", "--offload-arch=gfx950", "--cuda-device-only", *defs,
                           os.path.join(CSRC, "gsr_common.h"), "-o", os.devnull],
                          capture_output=True, text=True)


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
@pytest.mark.parametrize("exp", ["NOREPLAY", "NOMFMA", "FWD_NOC", "NOREACH"])
def test_experiment_switch_refused_in_product_build(exp):
    r = _preprocess(f"-DGSR_EXP_{exp}")
    assert r.returncode != 0 and "make exp" in r.stderr
    assert _preprocess(f"-DGSR_EXP_{exp}", "-DGSR_DIAG_BUILD").returncode == 0
    assert _preprocess().returncode == 0
