import time, numpy as np, torch, sys
sys.path.insert(0, '.')
from wespeaker_hubert_amd.speaker_model import HipSpeakerModel
from wespeaker_hubert_amd.synthetic import synth_state_dict, synth_audio
from wespeaker_hubert_amd.batching import embed_utterances
from wespeaker_hubert_amd.frontend import compute_fbank
dev = torch.device('cuda', 0)
m = HipSpeakerModel('ECAPA_TDNN_c1024', feat_dim=80, embed_dim=192)
m.load_state_dict(synth_state_dict(1, m.state_dict_layout())); m.to(dev)
rng = np.random.default_rng(0)
lens = rng.integers(32000, 160000, 1024)  # 2..10 s, vox1-like
pcms = [synth_audio(i, 1, int(n))[0] for i, n in enumerate(lens)]
embed_utterances(m, pcms[:8], dev); torch.cuda.synchronize()
t = time.perf_counter(); e1 = embed_utterances(m, pcms, dev); torch.cuda.synchronize(); tr = time.perf_counter() - t
t = time.perf_counter()
e2 = []
for x in pcms[:256]:
    f = compute_fbank(torch.from_numpy(x[None]).to(dev), cmn=True)
    e2.append(m(f)[-1][0].cpu().numpy())
torch.cuda.synchronize(); t1 = (time.perf_counter() - t) * 4
d = max(np.abs(a - b).max() for a, b in zip(e1[:256], e2))
print(f"ragged: {len(pcms)/tr:.0f} utt/s ({lens.sum()/16000/tr:.0f} s audio/s); one-by-one: {1024/t1:.0f} utt/s; max diff {d:.2e}")
