"""GPU box: average fbank + CMN launch time at the C2 shape (B = 256 x 5 s, PCM16-valued f32)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from wespeaker_hubert_amd.frontend import compute_fbank  # noqa: E402
from wespeaker_hubert_amd.synthetic import synth_audio  # noqa: E402

wav = torch.from_numpy(synth_audio(3, 256, 80000)).cuda()
for _ in range(3):
    compute_fbank(wav, scale=1.0, cmn=True)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    compute_fbank(wav, scale=1.0, cmn=True)
e1.record()
torch.cuda.synchronize()
print(f"fbank+CMN B=256 x 5 s: {e0.elapsed_time(e1) / 20:.4f} ms per call")
