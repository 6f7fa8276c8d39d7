"""Phase split of k_stage2_qp from its in-kernel stamps (HD_S2_STAMPS=<file>, hd_stage2.hip
kStamp*): per chunk and wave the shader-clock cycles spent issuing the DMA, in the expand, in
the offsets read + sums, in the ring wait (vmcnt) and from there to the next chunk (barrier,
plus the flush at a tile's end).  Usage: python3 scripts/qp_stamps.py stamps.bin [nw]"""
import sys

import numpy as np

WG, CH, PH = 8, 32, 6
path = sys.argv[1]
nw = int(sys.argv[2]) if len(sys.argv) > 2 else 16
a = np.fromfile(path, dtype=np.uint32)
a = a[:WG * nw * CH * PH].reshape(WG, nw, CH, PH).astype(np.int64)
t = a.copy()
ok = np.ones((WG, nw, CH - 1), bool)
d = {
    "dma issue": t[:, :, :-1, 1] - t[:, :, :-1, 0],
    "expand": t[:, :, :-1, 2] - t[:, :, :-1, 1],
    "voff + sums": t[:, :, :-1, 3] - t[:, :, :-1, 2],
    "ring wait": t[:, :, :-1, 4] - t[:, :, :-1, 3],
    "barrier (+flush)": t[:, :, 1:, 0] - t[:, :, :-1, 4],
    "chunk": t[:, :, 1:, 0] - t[:, :, :-1, 0],
}
for k, v in d.items():
    v = v % (1 << 32)
    print("%-18s mean %8.0f  median %8.0f  p90 %8.0f cycles" % (k, v.mean(), np.median(v), np.percentile(v, 90)))
# skew: per (WG, chunk) the spread over waves of the sums' end
end = (t[:, :, :-1, 3]) % (1 << 32)
start = (t[:, :, :-1, 0]) % (1 << 32)
print("wave skew at sums end: mean %.0f cycles (max - min over the waves of a chunk)" % (end.max(1) - end.min(1)).mean())
print("wave skew at chunk start: mean %.0f cycles" % (start.max(1) - start.min(1)).mean())
