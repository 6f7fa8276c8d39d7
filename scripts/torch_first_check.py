"""GPU-box check for the multi-GPU bench path: torch (RCCL, its bundled HIP runtime) is
initialised first, then libhipdedisp.so runs a pass on the same device and must still be
bit-exact against the oracle."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pipeline2.0_amd"), os.path.join(ROOT, "oracle")]
assert torch.cuda.is_available(), "torch sees no GPU"
torch.cuda.set_device(0)
x = torch.ones(1 << 20, device="cuda")
print("torch ok:", float(x.sum()))
import __graft_entry__ as g  # noqa: E402
g.smoke()
