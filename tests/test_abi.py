"""The C-ABI library: loads without a GPU, exports every symbol include/hipdedisp.h declares,
reports errors through return codes, and its host-only pieces (delay tables, synthetic
generator) agree with the oracle.  No device compute here (CPU suite)."""
import ctypes
import os
import re

import numpy as np
import pytest

import oracle as OR
from hipdedisp import Opts, PassParams, _lib, plan
from hipdedisp.engine import plan_tables
from hipdedisp.synth import host_spectra, palfa_obs, palfa_synth

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "hipdedisp.h")


def declared_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(hd_[a-z_0-9]+)\s*\(", txt)))


def test_header_and_binding_agree():
    assert declared_functions() == sorted(_lib.EXPORTED)


def test_library_exports_every_declared_symbol():
    L = _lib.load()
    for name in declared_functions():
        assert hasattr(L, name), name
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (hd_\w+)", out))
    assert set(declared_functions()) <= exported
    # no C++ mangled names leak through the public surface
    assert not any(n.startswith("_Z") and "hd_" in n for n in re.findall(r" T (\S+)", out))


def test_version_and_defaults():
    L = _lib.load()
    assert L.hd_version().decode().startswith("hipdedisp")
    o = _lib.hd_opts()
    L.hd_opts_default(ctypes.byref(o))
    # the reference's commands: int16 .sub files, mean downsampling, first-DM padding, default
    # -clip 6 (no -noclip at PALFA2_presto_search.py:506-511), (short)(x + 0.5) rounding
    assert (o.sub_dtype, o.ds_mode, o.pad_mode, o.nibble_hi_first, o.be16, o.inf_roundtrip, o.sub_round) == \
        (0, 1, 2, 1, 1, 1, 0)
    assert o.clip_sigma == 6.0
    d = Opts()
    assert (d.ds_mode, d.pad_mode, d.clip_sigma, d.sub_round) == (o.ds_mode, o.pad_mode, o.clip_sigma, o.sub_round)


def test_errors_are_return_codes():
    L = _lib.load()
    assert L.hd_open(0, None) == _lib.HD_E_INVAL
    assert "NULL" in _lib.last_error()
    bad = palfa_obs(N=1024).to_c()
    bad.nbits = 3
    pp = PassParams(0, 0, 0.1, 4, 96, 1).to_c()
    assert L.hd_plan_tables(ctypes.byref(bad), None, ctypes.byref(pp), None, None, None, None, None) == _lib.HD_E_INVAL
    assert "nbits" in _lib.last_error()
    good = palfa_obs(N=1024).to_c()
    pp.nsub = 97
    assert L.hd_plan_tables(ctypes.byref(good), None, ctypes.byref(pp), None, None, None, None, None) == _lib.HD_E_INVAL
    assert "nsub" in _lib.last_error()


@pytest.mark.parametrize("backend", ["pdev", "wapp"])
def test_delay_tables_match_oracle_every_pass(backend):
    """Bit-exact integer delay tables for every pass of the reference's hard-coded plans."""
    obs = palfa_obs(N=1 << 22)
    opts = Opts()
    for p in plan.ddplans_for(backend):
        for i in range(p.numpasses):
            pp = PassParams(subdm=float(p.subdmlist[i]), lodm=float(p.lodm_arg(i)),
                            dmstep=float(p.dmstep_arg()), numdms=p.dmsperpass, nsub=p.numsub,
                            ds=p.sub_downsamp, numout=plan.choose_N((1 << 22) / p.downsamp))
            idd, off, (lof, bw, sdt) = plan_tables(obs, opts, pp)
            assert np.array_equal(idd, OR.chan_delays(obs, pp.nsub, pp.subdm))
            assert np.array_equal(off, OR.dm_offsets(obs, opts, pp.nsub, pp.ds, pp.lodm, pp.dmstep, pp.numdms))
            assert (lof, bw, sdt) == OR.sub_params(obs, opts, pp.nsub, pp.ds)


def test_sub_input_tables():
    obs = palfa_obs(N=1 << 20)
    opts = Opts()
    lof, bw, sdt = OR.sub_params(obs, opts, 96, 5)
    sobs = palfa_obs(N=(1 << 20) // 5, nchan=96)
    sobs.lofreq, sobs.df, sobs.dt, sobs.flip = lof, bw, sdt, False
    pp = PassParams(subdm=553.4, lodm=534.4, dmstep=0.5, numdms=76, nsub=96, ds=1, sub_input=True)
    idd, off, got = plan_tables(sobs, opts, pp)
    assert not idd.any() and got == (lof, bw, sdt)
    assert np.array_equal(off, OR.dm_offsets(obs, opts, 96, 5, 534.4, 0.5, 76))


@pytest.mark.parametrize("nbits", [4, 8, 16])
def test_host_synth_deterministic_and_shaped(nbits):
    obs = palfa_obs(N=8192, nbits=nbits)
    s = palfa_synth(nbits=nbits)
    a = host_spectra(obs, s)
    b = host_spectra(obs, s, start=1000, count=3000)
    assert np.array_equal(a[1000:4000], b)
    assert a.shape == (8192, obs.rowbytes)
    c = host_spectra(obs, palfa_synth(beam=1, nbits=nbits))
    assert not np.array_equal(a, c)


def test_host_synth_statistics():
    """8-bit beam: bandpass around base level, RFI channels hot, flip puts channel 0 last."""
    obs = palfa_obs(N=16384, nbits=8)
    s = palfa_synth()
    a = host_spectra(obs, s).astype(np.float64)[:, ::-1]     # ascending frequency
    lvl = a.mean(axis=0)
    rfi = [s.rfi_chan[i] for i in range(s.rfi_nchan)]
    quiet = np.setdiff1d(np.arange(obs.nchan), rfi)
    assert abs(lvl[quiet].mean() - s.base_level) < 2.0
    assert lvl[quiet][-1] > lvl[quiet][0]                    # positive bandpass slope
    assert (lvl[rfi] > lvl[quiet].mean() + 0.5 * s.rfi_amp).all()
    assert 0.8 * s.noise_sigma < a[:, quiet].std(axis=0).mean() < 1.3 * s.noise_sigma


def test_comm_without_rccl_is_an_error_code():
    """hd_comm_unique_id on a host without RCCL: HD_E_HIP and a message, not an abort
    (the loader's dlerror() is read once).  HD_TEST_NO_RCCL makes the library skip dlopen;
    a child process, since the loader runs once per process."""
    import subprocess
    import sys
    code = (
        "import ctypes, sys\n"
        "sys.path[:0] = %r\n"
        "from hipdedisp import _lib\n"
        "L = _lib.load()\n"
        "buf = (ctypes.c_uint8 * 128)()\n"
        "rc = L.hd_comm_unique_id(buf)\n"
        "print(rc, _lib.last_error())\n" % ([os.path.join(os.path.dirname(HEADER), "..", "pipeline2.0_amd")],))
    env = dict(os.environ, HD_TEST_NO_RCCL="1")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=120)
    assert out.returncode == 0, out.stderr
    rc, msg = out.stdout.strip().split(" ", 1)
    assert int(rc) == _lib.HD_E_HIP
    assert "librccl not found" in msg
