"""PRESTO .inf metadata files [PRESTO-ext: writeinf/readinf of src/ioinf.c, restated].

The reference keeps every `<base>_DM<dm>.inf` (moved to the work dir at
PALFA2_presto_search.py:596-599, tarred into `_inf.tgz` at :708,716 and uploaded by
sp_candidates.py:358-363), and downstream PRESTO tools read the file by line
position, so the line order and labels below are the contract.
"""
from dataclasses import dataclass, field
from typing import List


@dataclass
class InfoData:
    name: str
    telescope: str = "Arecibo"
    instrument: str = "Mock"
    object: str = "SYNTH"
    ra: str = "19:00:00.0000"
    dec: str = "05:00:00.0000"
    observer: str = "hipdedisp"
    mjd: float = 56000.5          # epoch MJD
    bary: int = 0
    N: float = 0
    dt: float = 0.0
    onoff: List[float] = field(default_factory=list)   # flat list of (on, off) bin pairs
    band: str = "Radio"
    fov: float = 210.0            # beam diameter, arcsec
    dm: float = 0.0
    freq: float = 0.0             # centre freq of low channel, MHz
    freqband: float = 0.0         # total bandwidth, MHz
    num_chan: int = 1
    chan_wid: float = 0.0
    analyzer: str = "hipdedisp"
    notes: str = "Project ID P2030; dedispersed on MI355X by hipdedisp"


_LABELS = {
    "name": " Data file name without suffix          =  ",
    "telescope": " Telescope used                         =  ",
    "instrument": " Instrument used                        =  ",
    "object": " Object being observed                  =  ",
    "ra": " J2000 Right Ascension (hh:mm:ss.ssss)  =  ",
    "dec": " J2000 Declination     (dd:mm:ss.ssss)  =  ",
    "observer": " Data observed by                       =  ",
    "mjd": " Epoch of observation (MJD)             =  ",
    "bary": " Barycentered?           (1=yes, 0=no)  =  ",
    "N": " Number of bins in the time series      =  ",
    "dt": " Width of each time series bin (sec)    =  ",
    "breaks": " Any breaks in the data? (1=yes, 0=no)  =  ",
    "band": " Type of observation (EM band)          =  ",
    "fov": " Beam diameter (arcsec)                 =  ",
    "dm": " Dispersion measure (cm-3 pc)           =  ",
    "freq": " Central freq of low channel (Mhz)      =  ",
    "freqband": " Total bandwidth (Mhz)                  =  ",
    "num_chan": " Number of channels                     =  ",
    "chan_wid": " Channel bandwidth (Mhz)                =  ",
    "analyzer": " Data analyzed by                       =  ",
}


def format_inf(d: InfoData) -> str:
    L = _LABELS
    imjd = int(d.mjd)
    frac = "%.15f" % (d.mjd - imjd)
    lines = [L["name"] + d.name, L["telescope"] + d.telescope]
    if d.telescope != "None (Artificial Data Set)":
        lines += [L["instrument"] + d.instrument, L["object"] + d.object, L["ra"] + d.ra, L["dec"] + d.dec,
                  L["observer"] + d.observer, L["mjd"] + "%d%s" % (imjd, frac[1:]),
                  L["bary"] + "%d" % d.bary]
    lines.append(L["N"] + "%-11.0f" % d.N)
    lines.append(L["dt"] + "%.15g" % d.dt)
    npairs = len(d.onoff) // 2
    lines.append(L["breaks"] + "%d" % (1 if npairs > 1 else 0))
    if npairs > 1:
        for i in range(npairs):
            lines.append(" On/Off bin pair #%3d                   =  %-11.0f, %-11.0f"
                         % (i + 1, d.onoff[2 * i], d.onoff[2 * i + 1]))
    lines.append(L["band"] + d.band)
    if d.band == "Radio":
        lines += [L["fov"] + "%.0f" % d.fov, L["dm"] + "%.12g" % d.dm, L["freq"] + "%.12g" % d.freq,
                  L["freqband"] + "%.12g" % d.freqband, L["num_chan"] + "%d" % d.num_chan,
                  L["chan_wid"] + "%.12g" % d.chan_wid]
    lines.append(L["analyzer"] + d.analyzer)
    lines.append(" Any additional notes:")
    lines.append("    " + d.notes)
    return "\n".join(lines) + "\n\n"


def write_inf(path, d: InfoData):
    with open(path, "w") as f:
        f.write(format_inf(d))


def read_inf(path) -> InfoData:
    """Parse a .inf written by format_inf (or PRESTO's writeinf)."""
    vals, onoff = {}, []
    with open(path) as f:
        lines = f.read().splitlines()
    inv = {v[:40].strip(): k for k, v in _LABELS.items()}
    for ln in lines:
        # fixed layout: 40-character label, '=', value (labels may contain '=' themselves)
        if len(ln) > 40 and ln[40] == "=":
            lab, val = ln[:40].strip(), ln[41:].strip()
        elif "=" in ln:
            lab, _, val = ln.partition("=")
            lab, val = lab.strip(), val.strip()
        else:
            continue
        if lab.startswith("On/Off bin pair"):
            a, b = val.split(",")
            onoff += [float(a), float(b)]
            continue
        k = inv.get(lab)
        if k:
            vals[k] = val
    d = InfoData(name=vals.get("name", ""))
    for k in ("telescope", "instrument", "object", "ra", "dec", "observer", "band", "analyzer"):
        if k in vals:
            setattr(d, k, vals[k])
    for k in ("mjd", "N", "dt", "fov", "dm", "freq", "freqband", "chan_wid"):
        if k in vals:
            setattr(d, k, float(vals[k]))
    for k in ("bary", "num_chan"):
        if k in vals:
            setattr(d, k, int(vals[k]))
    d.onoff = onoff
    return d
