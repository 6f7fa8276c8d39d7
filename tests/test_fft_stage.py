"""CPU checks of the realfft/zapbirds/rednoise row: the library's host layouts
(hd_zap_ranges, hd_rednoise_blocks) equal the oracle's independent restatement, the zaplist
reader follows PRESTO's format, and the oracle's numeric steps behave as the tools are meant
to (white noise normalised to unit mean power, a red-noise slope flattened, birdies replaced
by the local level).  Parity with PRESTO itself is unpinned (not in this image)."""
import json
import math
import os

import numpy as np
import pytest

import fft_oracle as FO
from hipdedisp import PrestoError
from hipdedisp import fft_stage as FS

ZAPLIST = """# This file created automatically with makebirds.py
# Lines beginning with '#' are comments
# Lines beginning with 'B' are barycentric freqs (i.e. PSR freqs)
#                 Freq                 Width
# --------------------  --------------------
            0.07618684                 0.003
            0.08317989                 0.004

           60.0                         0.5
B          29.946923                    0.02
"""


def test_read_zaplist(tmp_path):
    p = tmp_path / "t.zaplist"
    p.write_text(ZAPLIST)
    birds = FS.read_zaplist(str(p))
    assert birds == [(0.07618684, 0.003, False), (0.08317989, 0.004, False), (60.0, 0.5, False),
                     (29.946923, 0.02, True)]
    lo, hi = FS.birdie_bins(birds, 100.0, baryv=1e-4)
    assert lo[2] == pytest.approx(5975.0) and hi[2] == pytest.approx(6025.0)
    f = 29.946923 / (1 + 1e-4)
    assert lo[3] == pytest.approx((f - 0.01) * 100.0) and hi[3] == pytest.approx((f + 0.01) * 100.0)


GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "palfa_zaplist.json")
REF_ZAPLIST = "/root/reference/lib/zaplists/PALFA.zaplist"


def palfa_birdies():
    return [(f, w, b) for f, w, b in json.load(open(GOLDEN))["birdies"]]


def test_palfa_zaplist_fixture_shape():
    """The reference's PALFA.zaplist (lib/zaplists/, the default zaplist of search_job,
    PALFA2_presto_search.py:472-474, 548-553) as committed: 226 lines, 5 comments, 221
    topocentric birdies -- the 0.0762/0.0832 Hz families and the 60 Hz mains comb."""
    g = json.load(open(GOLDEN))
    assert g["lines"] == 226 and g["comment_lines"] == 5
    birds = palfa_birdies()
    assert len(birds) == 221 and not any(b for _, _, b in birds)
    assert birds[0] == (0.07618684, 0.003, False) and birds[-1] == (300.0, 0.5, False)
    assert [(f, w) for f, w, _ in birds[-5:]] == [(60.0, 0.1), (120.0, 0.2), (180.0, 0.3), (240.0, 0.4), (300.0, 0.5)]


def test_read_zaplist_palfa(tmp_path):
    """read_zaplist on the reference's file (when the reference is present) and on the same
    lines rewritten from the fixture (with a 'B' line added) gives the fixture's birdies."""
    if os.path.exists(REF_ZAPLIST):
        assert FS.read_zaplist(REF_ZAPLIST) == palfa_birdies()
    p = tmp_path / "PALFA.zaplist"
    body = "".join("%22r%22r\n" % (f, w) for f, w, _ in palfa_birdies())
    p.write_text("# Freq Width\n" + body + "B 29.946923 0.02\n")
    assert FS.read_zaplist(str(p)) == palfa_birdies() + [(29.946923, 0.02, True)]


def test_palfa_zaplist_ranges_match_oracle():
    """The PALFA birdies of a C2 stage-0 series (2^22 x 65.476 us) and of a ds-10 series as
    merged bin ranges: library == oracle; the 60 Hz comb lands at its bins."""
    for n, dt in ((1 << 22, 65.476e-6), (419432, 654.76e-6)):
        T = n * dt
        lo, hi = FS.birdie_bins(palfa_birdies(), T, baryv=0.0)
        got = FS.zap_ranges(lo, hi, n // 2)
        assert np.array_equal(got, FO.zap_ranges(lo, hi, n // 2))
        k60 = int(math.floor((60.0 - 0.05) * T))
        assert any(r[0] <= k60 < r[1] for r in got)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_zap_ranges_match_oracle(seed):
    rng = np.random.default_rng(seed)
    nb = 50000
    c = rng.uniform(-10, nb + 10, 300)
    w = rng.exponential(3.0, 300)
    lo, hi = c - w, c + w
    lo[:5], hi[:5] = hi[:5], lo[:5]                      # reversed: dropped
    lo[5], hi[5] = 100.0, 100.0                          # empty after floor/ceil? [100, 100) dropped
    lo[6], hi[6] = 4000.0, 9000.0                        # wide: window side capped at 2048
    got = FS.zap_ranges(lo, hi, nb)
    want = FO.zap_ranges(lo, hi, nb)
    assert np.array_equal(got, want)
    assert np.all(got[1:, 0] > got[:-1, 1])              # merged: disjoint, not touching
    assert np.all((got[:, 0] >= 1) & (got[:, 1] <= nb))


def test_zap_ranges_empty():
    assert FS.zap_ranges([], [], 1000).shape == (0, 4)


@pytest.mark.parametrize("numbins,T", [(1 << 21, 274.9), (5000, 10.0), (300000, 1e4), (10, 1.0)])
def test_rednoise_blocks_match_oracle(numbins, T):
    got = FS.rednoise_blocks(numbins, T)
    want = FO.rednoise_blocks(numbins, T)
    assert np.array_equal(got, want)
    w = np.diff(got)
    assert got[0] == 1 and got[-1] == numbins and np.all(w >= 1) and np.all(w <= 100)
    assert np.all(np.diff(w[:-1]) >= 0)                  # widths never shrink (but the last)


def test_rednoise_blocks_rejects():
    with pytest.raises(PrestoError):
        FS.rednoise_blocks(1000, 10.0, endwidth=200)
    with pytest.raises(PrestoError):
        FS.rednoise_blocks(1000, 0.0)


def test_oracle_rednoise_normalises():
    rng = np.random.default_rng(3)
    n = 1 << 18
    T = n * 1e-3
    f = np.arange(n // 2) / T
    red = 1.0 + 50.0 / (1.0 + f) ** 1.5                  # red power spectrum
    z = (rng.normal(size=n // 2) + 1j * rng.normal(size=n // 2)) * np.sqrt(red / 2)
    F = z.astype(np.complex64)[None, :]
    G = FO.rednoise(F, FO.rednoise_blocks(n // 2, T))
    p = np.abs(G[0, 1:].astype(np.complex128)) ** 2
    assert G[0, 0] == 1.0
    for a, b in ((1, 200), (200, 5000), (5000, n // 2)):   # unit mean power everywhere
        assert p[a:b].mean() == pytest.approx(1.0, abs=0.15)


def test_oracle_zap_replaces_birdie():
    rng = np.random.default_rng(4)
    nb = 20000
    z = (rng.normal(size=nb) + 1j * rng.normal(size=nb)).astype(np.complex64)
    z[7000:7003] = 500.0
    r = FO.zap_ranges([6999.5], [7002.5], nb)
    assert r.tolist() == [[6999, 7003, 6949, 7053]]
    G = FO.zap(z[None, :], r)
    p = np.abs(z.astype(np.complex128)) ** 2
    w = np.concatenate([p[6949:6999], p[7003:7053]])
    a = np.float32(math.sqrt(np.sort(w)[(len(w) - 1) // 2] / math.log(2)))
    assert np.all(G[0, 6999:7003] == a) and np.array_equal(G[0, :6999], z[:6999])
    assert np.array_equal(G[0, 7003:], z[7003:])


def test_layout_edge_cases():
    # a spectrum of 2 bins: one block of one bin
    assert FS.rednoise_blocks(2, 1.0).tolist() == [1, 2]
    assert np.array_equal(FS.rednoise_blocks(7, 0.5), FO.rednoise_blocks(7, 0.5))
    # birdies wholly outside [1, numbins) or reversed vanish; one touching bin 0 is clamped
    r = FS.zap_ranges([-5.0, 2000.0, 10.0, -0.4], [-1.0, 2100.0, 9.0, 2.5], 1000)
    assert r.tolist() == [[1, 3, 1, 53]]
    assert np.array_equal(r, FO.zap_ranges([-5.0, 2000.0, 10.0, -0.4], [-1.0, 2100.0, 9.0, 2.5], 1000))
