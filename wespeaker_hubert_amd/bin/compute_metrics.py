"""EER / minDCF — drop-in for wespeaker/bin/compute_metrics.py."""
from __future__ import annotations

import os
import sys

from ..scoring import compute_metrics
from . import _fire


def main(p_target=0.01, c_miss=1, c_fa=1, *scores_files):
    for f in scores_files:
        eer, min_dcf = compute_metrics(str(f), p_target, c_miss, c_fa)
        print("---- {} -----".format(os.path.basename(str(f))))
        print("EER = {0:.3f}".format(eer))
        print("minDCF (p_target:{} c_miss:{} c_fa:{}) = {:.3f}".format(p_target, c_miss, c_fa, min_dcf))


if __name__ == "__main__":
    pos, kw = _fire.parse(sys.argv[1:])
    main(kw.get("p_target", 0.01), kw.get("c_miss", 1), kw.get("c_fa", 1), *pos)
