"""Teardown of a context marked faulted on a real device: after a sticky
HIP error the plans and the context release their host side only and report HD_E_HIP as
PrestoError -- the process stays alive and a new context on the same device works.  (The
fault is the hd_debug_fault flag; no kernel is made to fault.)  Reference failure path:
PALFA2_presto_search.py:123-128 raises PrestoError, job.py:140-165 retries the beam."""
import numpy as np
import pytest

import oracle as OR
from hipdedisp import Engine, Opts, PassParams, PrestoError
from hipdedisp.synth import host_spectra, palfa_obs, palfa_synth

pytestmark = pytest.mark.gpu


def run_small(eng):
    obs = palfa_obs(N=1 << 15, nbits=8)
    s = palfa_synth()
    eng.set_obs(obs, Opts())
    eng.synth_device(s)
    pp = PassParams(subdm=3.80, lodm=0.0, dmstep=0.1, numdms=76, nsub=96, ds=1, numout=0)
    p = eng.plan(pp)
    p.run_subband()
    got = p.run_dedisp()
    _, want = OR.run_pass(obs, Opts(), host_spectra(obs, s), pp)
    assert np.array_equal(got, want)
    return p


def test_faulted_context_closes_without_abort(engine):
    e = Engine(0)
    p = run_small(e)
    e.debug_fault()
    with pytest.raises(PrestoError, match="HD_E_HIP.*faulted"):
        e.close()
    assert not p._p
    e2 = Engine(0)
    try:
        run_small(e2).destroy()
    finally:
        e2.close()
