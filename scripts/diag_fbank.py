"""Diagnostic (GPU box): where does the HIP fbank differ from the f64 oracle?"""
import os
import re
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import fbank_ref  # noqa: E402
from wespeaker_hubert_amd.frontend import compute_fbank  # noqa: E402
from wespeaker_hubert_amd.synthetic import synth_audio  # noqa: E402

hdr = open(os.path.join(os.path.dirname(__file__), "..", "wespeaker_hubert_amd", "csrc", "fbank_mel_table.h")).read()
vals = [float.fromhex(v[:-1]) for v in re.findall(r"0x[0-9a-fp.+-]+f", hdr)]
starts = [int(v) for v in re.search(r"kMelStart\[80\] = \{([^}]*)\}", hdr).group(1).split(",")]
lens = [int(v) for v in re.search(r"kMelLen\[80\] = \{([^}]*)\}", hdr).group(1).split(",")]
W = np.zeros((80, 257))
o = 0
for b in range(80):
    W[b, starts[b]:starts[b] + lens[b]] = vals[o:o + lens[b]]
    o += lens[b]
mb = fbank_ref.mel_banks().astype(np.float64)
print("table vs oracle mel_banks on this host: max |dw|", np.abs(W - mb).max(), "n diff", int((W != mb).sum()))
wav = synth_audio(11, 3, 80000)
got = compute_fbank(torch.from_numpy(wav).cuda(), scale=1.0, cmn=False).cpu().numpy()
ref = np.stack([fbank_ref.fbank(w) for w in wav])
d = np.abs(got - ref)
print("max", d.max(), "mean", d.mean())
idx = np.argsort(d.ravel())[::-1][:12]
for i in idx:
    u, t, b = np.unravel_index(i, d.shape)
    print(f"utt {u} frame {t} bin {b}: got {got[u, t, b]:.7f} ref {ref[u, t, b]:.7f} d {d[u, t, b]:.2e}")
print("per-bin max err:", np.round(d.max(axis=(0, 1)) * 1e6, 1).tolist())
print("per-frame count of err>1e-5 (first 20 frames):", (d > 1e-5).sum(axis=(0, 2))[:20].tolist())
