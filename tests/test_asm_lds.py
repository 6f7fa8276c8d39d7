"""The inline-asm LDS reads of k_stage1_q8m (and the stage-2 kernels) are only correct if no
compiler-inserted instruction reads their destination registers before the counted
s_waitcnt that ties them: a branch between a read and its wait once made the compiler copy
the registers ahead of the wait (whole-beam subbands wrong at ds 2).  This compiles the
kernels to gfx950 assembly (hipcc, no GPU) and runs scripts/asm_lds_check.py on them."""
import os
import re
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "pipeline2.0_amd", "csrc")
sys.path.insert(0, os.path.join(ROOT, "scripts"))
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not in this image")
@pytest.mark.parametrize("src,pattern", [("hd_q8m.hip", r"_ZN2hd12k_stage1_q8m\w*"),
                                         ("hd_stage2.hip", r"_ZN2hd1\dk_stage2_(?:qp|pair)\w*")])
def test_no_register_use_before_lds_wait(tmp_path, src, pattern):
    import asm_lds_check
    out = tmp_path / "k.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                    "-fhip-fp32-correctly-rounded-divide-sqrt", "--cuda-device-only", "-S", "-o", str(out),
                    os.path.join(CSRC, src)], check=True, cwd=CSRC, capture_output=True)
    text = out.read_text()
    syms = sorted(set(re.findall(r"^(" + pattern + r"):", text, re.M)))
    assert syms, "no kernels matched"
    for sym in syms:
        bad = asm_lds_check.check(str(out), sym)
        assert not bad, (sym, bad[:5])
