"""`wespeaker` Python API mirror on the MI355X path.

Same surface as wespeaker/cli/speaker.py (Speaker 38-290, load_model 300,
load_model_pt 306-322, main 325-383) for the extraction / similarity tasks.
Differences, all deliberate and documented in DESIGN.md:
  * the default device is the current HIP device (the HIP library has no CPU
    path); `set_device('cuda:N')` selects another GPU;
  * `load_model(name)` never downloads (no network): the name must be a model
    directory (the reference's Hub path, cli/hub.py, is out of scope);
  * VAD (silero) and diarization are out of scope: `set_vad(True)` and
    `diarize*` raise NotImplementedError; the diarization embedding batcher
    `extract_embedding_feats` (+ diar.subsegment) is implemented.
"""
from __future__ import annotations

import argparse
import os
import sys
from typing import List, Optional, Tuple

import numpy as np
import torch
import yaml

from ..audio import load_wav
from ..batching import embed_utterances
from ..frontend import FbankArgs
from ..frontend import apply_cmn as _apply_cmn
from ..frontend import compute_fbank as _gpu_fbank
from ..kaldi_io import WriteHelper
from ..resample import resample as _resample
from ..speaker_model import get_speaker_model


def _default_device() -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError("no HIP device visible: the MI355X path has no CPU fallback")
    return torch.device("cuda", torch.cuda.current_device())


class Speaker:

    def __init__(self, model_dir: str):
        self.model = load_model_pt(model_dir)
        self.table = {}
        self.resample_rate = 16000
        self.apply_vad = False
        self.device = _default_device()
        self.wavform_norm = False
        self.window_type = 'hamming'
        self.model.to(self.device)

    # ------------------------------------------------------------ setters --
    def set_wavform_norm(self, wavform_norm: bool):
        self.wavform_norm = wavform_norm

    def set_window_type(self, window_type: str):
        # kaldi.fbank window_type: hamming / hanning / povey / rectangular / blackman
        # (an unknown name raises at the next fbank, as torchaudio does)
        self.window_type = window_type

    def set_resample_rate(self, resample_rate: int):
        self.resample_rate = resample_rate

    def set_vad(self, apply_vad: bool):
        if apply_vad:
            raise NotImplementedError("silero VAD is out of scope on the MI355X path")
        self.apply_vad = False

    def set_device(self, device: str):
        self.device = torch.device(device)
        if self.device.type != 'cuda':
            raise RuntimeError("the MI355X path runs on HIP devices only")
        self.model = self.model.to(self.device)

    def set_diarization_params(self, *args, **kwargs):
        pass  # diarization is out of scope; accepted for CLI compatibility

    # ------------------------------------------------------------ fbank --
    def compute_fbank(self, wavform, sample_rate=16000, num_mel_bins=80, frame_length=25,
                      frame_shift=10, cmn=True):
        """speaker.py:89-104 on the GPU; `wavform` (1, N) int16-valued."""
        args = FbankArgs(int(num_mel_bins), float(frame_length), float(frame_shift), int(sample_rate),
                         self.window_type)
        if isinstance(wavform, torch.Tensor):
            x = wavform.to(device=self.device, dtype=torch.float32)
        else:
            x = torch.as_tensor(np.asarray(wavform), dtype=torch.float32).to(self.device)
        if x.dim() == 2:
            x = x[:1]
        return _gpu_fbank(x, scale=1.0, cmn=cmn, args=args)[0]

    # -------------------------------------------------------- embeddings --
    def extract_embedding_feats(self, fbanks, batch_size: int, subseg_cmn: bool) -> np.ndarray:
        """speaker.py:106-121: embeddings of equal-length fbank windows (a list of
        (T, F) arrays, e.g. diar.subsegment output) in batches of `batch_size`;
        subseg_cmn subtracts each window's mean over frames first (wsp_cmn on the
        device).  Returns an (N, D) float32 array."""
        arr = np.ascontiguousarray(np.stack([np.asarray(f, dtype=np.float32) for f in fbanks]))
        feats = torch.from_numpy(arr).to(self.device)
        if subseg_cmn:
            _apply_cmn(feats)
        out = []
        with torch.no_grad():
            for i in range(0, feats.shape[0], batch_size):
                emb = self.model(feats[i:i + batch_size])
                emb = emb[-1] if isinstance(emb, tuple) else emb
                out.append(emb.detach().cpu().numpy())
        return np.vstack(out)

    def extract_embedding(self, audio_path: str):
        pcm, sample_rate = load_wav(audio_path, normalize=self.wavform_norm)
        return self.extract_embedding_from_pcm(torch.from_numpy(pcm), sample_rate)

    def extract_embedding_from_pcm(self, pcm: torch.Tensor, sample_rate: int):
        pcm = pcm.to(torch.float)
        if sample_rate != self.resample_rate:  # speaker.py:155-157, on the device
            pcm = _resample(pcm.to(self.device), sample_rate, self.resample_rate)
        feats = self.compute_fbank(pcm, sample_rate=self.resample_rate, cmn=True)
        feats = feats.unsqueeze(0)
        with torch.no_grad():
            outputs = self.model(feats)
            outputs = outputs[-1] if isinstance(outputs, tuple) else outputs
        return outputs[0].to(torch.device('cpu'))

    def extract_embedding_list(self, scp_path: str) -> Tuple[List[str], List[np.ndarray]]:
        """speaker.py:170-179; utterances are embedded in ragged batches
        (batching.embed_utterances: each result equals extract_embedding of that file)."""
        names, pcms = [], []
        with open(scp_path, 'r') as read_scp:
            for line in read_scp:
                if not line.strip():
                    continue
                name, wav_path = line.strip().split()
                pcm, sample_rate = load_wav(wav_path, normalize=self.wavform_norm)
                pcm = pcm[0].astype(np.float32)
                if sample_rate != self.resample_rate:
                    x = torch.from_numpy(pcm).to(self.device)
                    pcm = _resample(x, sample_rate, self.resample_rate).cpu().numpy()
                names.append(name)
                pcms.append(pcm)
        with torch.no_grad():
            embeddings = embed_utterances(self.model, pcms, self.device,
                                          fbank_args=FbankArgs(sample_rate=self.resample_rate,
                                                               window_type=self.window_type))
        return names, [np.asarray(e, dtype=np.float32) for e in embeddings]

    def compute_similarity(self, audio_path1: str, audio_path2: str) -> float:
        e1 = self.extract_embedding(audio_path1)
        e2 = self.extract_embedding(audio_path2)
        if e1 is None or e2 is None:
            return 0.0
        return self.cosine_similarity(e1, e2)

    def cosine_similarity(self, e1, e2):
        cosine_score = torch.dot(e1, e2) / (torch.norm(e1) * torch.norm(e2))
        return (cosine_score.item() + 1.0) / 2

    def register(self, name: str, audio_path: str):
        if name in self.table:
            print('Speaker {} already registered, ignore'.format(name))
        else:
            self.table[name] = self.extract_embedding(audio_path)

    def recognize(self, audio_path: str):
        q = self.extract_embedding(audio_path)
        best_score, best_name = 0.0, ''
        for name, e in self.table.items():
            score = self.cosine_similarity(q, e)
            if best_score < score:
                best_score, best_name = score, name
        return {'name': best_name, 'confidence': best_score}

    def diarize(self, *args, **kwargs):
        raise NotImplementedError("diarization is out of scope on the MI355X path")

    diarize_list = diarize


def load_or_download(model_name_or_path: str) -> str:
    if not os.path.isdir(model_name_or_path):
        raise FileNotFoundError(f"{model_name_or_path} is not a model directory "
                                "(hub downloads are not available offline)")
    return model_name_or_path


def load_model(model_name_or_path: str) -> Speaker:
    return Speaker(load_or_download(model_name_or_path))


def load_model_pt(model_name_or_path: str):
    """config.yaml + avg_model.pt -> HipSpeakerModel (speaker.py:306-322)."""
    model_dir = load_or_download(model_name_or_path)
    for file in ('config.yaml', 'avg_model.pt'):
        if not os.path.exists(os.path.join(model_dir, file)):
            raise FileNotFoundError(f"{file} not found in {model_dir}")
    with open(os.path.join(model_dir, 'config.yaml'), 'r') as f:
        config = yaml.safe_load(f)
    model = get_speaker_model(config['model'])(**config['model_args'])
    state = torch.load(os.path.join(model_dir, 'avg_model.pt'), map_location='cpu', weights_only=True)
    model.load_state_dict(state, strict=False)
    return model.eval()


def get_args(argv=None):
    """cli/utils.py:19-115 (extraction / similarity subset)."""
    p = argparse.ArgumentParser(description='MI355X speaker embedding toolkit')
    p.add_argument('-t', '--task', choices=['embedding', 'embedding_kaldi', 'similarity'],
                   default='embedding')
    p.add_argument('-p', '--pretrain', type=str, default='', help='model directory')
    p.add_argument('--device', type=str, default='cuda')
    p.add_argument('--audio_file', help='audio file')
    p.add_argument('--audio_file2', help='audio file2, used for similarity')
    p.add_argument('--wav_scp', help='path to wav.scp, for extract and saving kaldi-stype embeddings')
    p.add_argument('--resample_rate', type=int, default=16000)
    p.add_argument('--vad', action='store_true')
    p.add_argument('--output_file', default=None)
    return p.parse_args(argv)


def main(argv=None):
    args = get_args(argv)
    if not args.pretrain:
        print('a model directory (-p/--pretrain) is required offline', file=sys.stderr)
        sys.exit(2)
    model = load_model(args.pretrain)
    model.set_resample_rate(args.resample_rate)
    model.set_vad(args.vad)
    model.set_device(args.device)
    if args.task == 'embedding':
        embedding = model.extract_embedding(args.audio_file)
        if embedding is not None:
            np.savetxt(args.output_file, embedding.detach().numpy())
            print('Succeed, see {}'.format(args.output_file))
        else:
            print('Fails to extract embedding')
    elif args.task == 'embedding_kaldi':
        names, embeddings = model.extract_embedding_list(args.wav_scp)
        embed_ark = args.output_file + ".ark"
        embed_scp = args.output_file + ".scp"
        with WriteHelper('ark,scp:' + embed_ark + "," + embed_scp) as writer:
            for name, embedding in zip(names, embeddings):
                writer(name, embedding)
    elif args.task == 'similarity':
        print(model.compute_similarity(args.audio_file, args.audio_file2))


if __name__ == '__main__':
    main()
