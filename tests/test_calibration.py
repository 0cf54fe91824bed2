"""QMF score calibration (bin/score_calibration.py) against the reference's own
gather -> train -> infer run on the same synthetic AS-Norm side outputs
(tests/golden/calibration.npz, made by tests/golden/make_golden.py).  CPU only."""
import os

import numpy as np

from wespeaker_hubert_amd.bin import score_calibration as sc

GOLD = os.path.join(os.path.dirname(__file__), "golden", "calibration.npz")


def _write(path, lines):
    with open(path, "w") as f:
        f.write("\n".join(str(x) for x in lines) + "\n")


def test_calibration_matches_reference(tmp_path):
    z = np.load(GOLD, allow_pickle=False)
    dur, sn = tmp_path / "dur", tmp_path / "sn"
    fac, mdl, cal = tmp_path / "fac", tmp_path / "m.pt", tmp_path / "cal"
    _write(dur, z["dur_lines"])
    _write(sn, z["score_norm_lines"])
    sc.gather_calibration_factors(str(dur), float(z["max_dur"]), str(sn), str(fac))
    assert open(fac).read().splitlines() == [str(x) for x in z["factor_lines"]]
    sc.train_calibration_model(str(fac), str(mdl))
    import torch
    sd = torch.load(str(mdl), weights_only=True)
    np.testing.assert_allclose(sd["linear.weight"].numpy(), z["weight"], rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(sd["linear.bias"].numpy(), z["bias"], rtol=1e-9, atol=1e-12)
    sc.infer_calibration(str(fac), str(mdl), str(cal))
    got = [ln.split() for ln in open(cal).read().splitlines()]
    ref = [str(x).split() for x in z["calibrated_lines"]]
    assert [g[:2] + g[3:] for g in got] == [r[:2] + r[3:] for r in ref]
    np.testing.assert_allclose([float(g[2]) for g in got], [float(r[2]) for r in ref], rtol=1e-12, atol=1e-12)


def test_gather_drop_duration(tmp_path):
    z = np.load(GOLD, allow_pickle=False)
    sn, fac = tmp_path / "sn", tmp_path / "fac"
    _write(sn, z["score_norm_lines"][:5])
    sc.gather_calibration_factors("unused", 10.0, str(sn), str(fac), drop_duration=True)
    rows = [ln.split() for ln in open(fac).read().splitlines()]
    assert len(rows) == 5 and all(len(r) == 4 + 8 for r in rows)  # ids, label, score, mag x4, cmean x4
