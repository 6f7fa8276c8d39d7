"""Host-side guards of the device code (CPU suite, no GPU):

* the DMA extent check (hd_plan_extents): for every pass of the C1, C2 and C4 plans, at 8, 4
  and 16 bits, padded and unpadded, and for subband counts whose k_stage2_qp tiles have an
  odd chunk count, the furthest byte any whole 1 KiB DMA piece of the stage-2 kernels can
  touch lies inside its buffer -- the subband block [nsub][sub_stride] and every per-chunk
  offset table (round 5's fault: k_stage2_qp's last offset block read past its table);
* the teardown order after a device fault: plans first, then the context, neither making a
  device call, both reporting HD_E_HIP as PrestoError instead of aborting the process
  (round 5: hd_close after an illegal memory access aborted in HIP's teardown).
"""
import os
import subprocess
import sys

import pytest

from hipdedisp import Opts, PassParams, plan
from hipdedisp.engine import plan_extents
from hipdedisp.synth import palfa_obs

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def pdev_passes(N):
    for d in plan.ddplans_for("pdev"):
        for i in range(d.numpasses):
            yield PassParams(subdm=float(d.subdmlist[i]), lodm=float(d.lodm_arg(i)), dmstep=float(d.dmstep_arg()),
                             numdms=d.dmsperpass, nsub=d.numsub, ds=d.sub_downsamp,
                             numout=plan.choose_N(N / d.downsamp))


def c4_passes(obs):
    for d in plan.ddplan2b_plans(obs.dt, 1375.5, 322.6, obs.nchan, 2048, 0.0, 10000.0, 96, 0.1):
        for i in range(d.numpasses):
            yield PassParams(subdm=float(d.subdmlist[i]), lodm=float(d.lodm_arg(i)), dmstep=float(d.dmstep_arg()),
                             numdms=d.dmsperpass, nsub=d.numsub, ds=d.sub_downsamp,
                             numout=plan.choose_N(obs.N / d.downsamp))


def check(obs, pp, opts=None, want_qp=True):
    ex = plan_extents(obs, opts or Opts(), pp)
    assert ex, pp
    for x in ex:
        assert 0 < x["reach"] <= x["size"], (pp, x)
        if x["region"] == "offsets":
            # a table carries only the tail its last piece needs (< one 1 KiB piece + the
            # rows of the pairs a smaller pairs-per-chunk launch leaves out)
            assert x["size"] - x["reach"] < 4, (pp, x)
    kernels = {x["kernel"] for x in ex}
    if want_qp:
        assert 9 in kernels, (pp, kernels)          # k_stage2_qp: the default stage-2 kernel
        assert {x["ppc"] for x in ex if x["kernel"] == 9 and x["region"] == "offsets"}
    return ex


@pytest.mark.parametrize("nbits", [8, 4, 16])
def test_extents_c2_every_pass(nbits):
    """C2 (configs[1]): every pass of the 57-pass DDplan at 2^22."""
    obs = palfa_obs(N=1 << 22, nbits=nbits)
    n = 0
    for pp in pdev_passes(obs.N):
        check(obs, pp)
        n += 1
    assert n == 57


def test_extents_c1_and_unpadded():
    """C1 (configs[0]): 2^20 spectra, every pass, padded to choose_N and unpadded (numout 0)."""
    obs = palfa_obs(N=1 << 20, nbits=8)
    for pp in pdev_passes(obs.N):
        check(obs, pp)
        pp.numout = 0
        check(obs, pp)


def test_extents_c4_every_pass():
    """C4 (configs[3]): the DDplan2b plan 0-10000 pc cm^-3 (93 passes, ds 1..64)."""
    obs = palfa_obs(N=1 << 22, nbits=8)
    n = sum(1 for pp in c4_passes(obs) if check(obs, pp))
    assert n == 93


@pytest.mark.parametrize("nsub", [60, 120])
def test_extents_odd_chunk_counts(nsub):
    """Subband counts whose quarter-layout tiles have an odd number of chunks (nsub / 2 / ppc
    odd): the kernel's running buffer parity differs from the table's on every other tile;
    the extents of all three offset tables must still hold."""
    obs = palfa_obs(N=(1 << 20) + 12345, nbits=8)
    for ds, lodm, step in ((1, 0.0, 0.1), (2, 212.8, 0.3), (5, 443.2, 0.5)):
        pp = PassParams(subdm=lodm + 20.0, lodm=lodm, dmstep=step, numdms=76, nsub=nsub, ds=ds, numout=0)
        ex = check(obs, pp)
        assert any(x["kernel"] == 9 and (nsub // 2 // x["ppc"]) % 2 == 1 for x in ex if x["region"] == "offsets"), nsub


def test_extents_cover_the_last_tile():
    """The subband reach is that of the last subband's window in the last tile: at least
    (nsub - 1) rows plus nvalid - T samples (T <= 1024), so the check is not vacuous."""
    obs = palfa_obs(N=1 << 22, nbits=8)
    for pp in pdev_passes(obs.N):
        nvalid = min(obs.N // pp.ds, pp.numout)
        for x in plan_extents(obs, Opts(), pp):
            if x["region"] == "subbands":
                stride = x["size"] // (2 * pp.nsub)
                assert x["reach"] >= 2 * ((pp.nsub - 1) * stride + nvalid - 1024), (pp, x)


def test_extents_sub_input_and_f32():
    obs = palfa_obs(N=1 << 18, nbits=8)
    # f32 subbands: no pair/DMA kernel applies
    pp = PassParams(subdm=71.0, lodm=65.0, dmstep=0.5, numdms=76, nsub=96, ds=1, numout=0)
    opts = Opts()
    opts.sub_dtype = 1
    assert plan_extents(obs, opts, pp) == []
    # no-subband pass (nsub = nchan)
    pp = PassParams(subdm=0.0, lodm=0.0, dmstep=0.1, numdms=64, nsub=obs.nchan, ds=1, numout=0)
    for x in plan_extents(obs, Opts(), pp):
        assert x["reach"] <= x["size"]


_TEARDOWN = r"""
import sys
sys.path[:0] = [%r]
from hipdedisp import Engine, Opts, PassParams, PrestoError, _lib
from hipdedisp.synth import palfa_obs
obs = palfa_obs(N=1 << 18, nbits=8)
pp = PassParams(subdm=71.0, lodm=65.0, dmstep=0.5, numdms=76, nsub=96, ds=1, numout=0)
# a clean host-only context: plans and context close without error
e = Engine(_lib.HD_HOST_ONLY)
e.set_obs(obs, Opts())
ps = [e.plan(pp) for _ in range(3)]
e.close()
assert all(not p._p for p in ps)
print("clean ok")
# faulted: the plans go first, then the context; no device call, HD_E_HIP as PrestoError
e = Engine(_lib.HD_HOST_ONLY)
e.set_obs(obs, Opts())
ps = [e.plan(pp) for _ in range(3)]
del ps[1]
e.debug_fault()
try:
    e.close()
except PrestoError as err:
    msg = str(err)
    assert "HD_E_HIP" in msg and "faulted" in msg, msg
    print("faulted ok:", msg)
else:
    raise SystemExit("close of a faulted context did not report HD_E_HIP")
assert all(not p._p for p in ps)
# the process carries on: a new context works
e = Engine(_lib.HD_HOST_ONLY)
e.set_obs(obs, Opts())
e.plan(pp).destroy()
e.close()
print("after ok")
"""


def test_teardown_after_fault_does_not_abort():
    code = _TEARDOWN % os.path.join(ROOT, "pipeline2.0_amd")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "clean ok" in out.stdout and "faulted ok" in out.stdout and "after ok" in out.stdout
