"""Host-side AddressSanitizer run of the MLP packer (SURVEY §5 debug aids; CPU only).

tools/asan/run.sh compiles the packer translation units with ASan on their host code and runs
tools/asan/pack_driver.cpp, which packs every MLP shape the path uses plus ragged corners.  With
no GPU visible nrt_mlp_create runs all of its host-side packing (fragment layouts, index maps,
weight programs) and stops at the first device allocation; an out-of-range host access aborts
with an ASan report and a non-zero exit."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc") and not shutil.which("hipcc"),
                    reason="hipcc not available")
def test_packer_host_code_is_asan_clean():
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "asan", "run.sh")], cwd=ROOT,
                       capture_output=True, text=True, timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "AddressSanitizer" not in out, out[-4000:]
    assert "all shapes packed cleanly" in out
