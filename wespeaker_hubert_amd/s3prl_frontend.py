"""HuBERT-base SSL front end on the HIP path — mirror of
`wespeaker.frontend.s3prl.S3prlFrontend` (wespeaker/frontend/s3prl.py:23-93).

Same constructor arguments, `output_size()` and `forward(wavs, wavs_len) ->
(feats, feats_lens)` contract; the s3prl `hubert` upstream (fairseq HuBERT-base)
and the s3prl Featurizer run in libwsp_hip.so (`wsp_frontend_forward`).
Weights arrive under the reference checkpoint's names
(`frontend.upstream.upstream.model.<fairseq name>`, `frontend.featurizer.weights`;
the module-local form without the `frontend.` prefix is accepted too).

Implemented: upstream name `hubert_base` (alias `hubert`), normalize=False,
equal-length batches (what bin/extract.py:100-102 feeds), ragged batches of whole
utterances (`extract_segments`: every utterance computed as if alone — GroupNorm,
pos-conv padding, attention and featurizer all per utterance), multilayer_feature /
layer selection.  s3prl itself is absent offline, so its glue (length match,
Featurizer) is restated — see oracle/hubert_ref.py for the pinning status.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Tuple

import numpy as np
import torch

from . import _lib
from .arch import HUBERT_BASE, hubert_params
from .speaker_model import _HipHandle

SUPPORTED_UPSTREAMS = ("hubert_base", "hubert")


class S3prlFrontend(_HipHandle):
    """Speech pretrained representation front end (HuBERT-base on gfx950)."""

    _ignored_prefixes = (
        # fairseq HubertModel members the extraction forward never reads
        "frontend.upstream.upstream.model.mask_emb",
        "frontend.upstream.upstream.model.final_proj.",
        "frontend.upstream.upstream.model.label_embs_concat",
    )

    def __init__(self, upstream_args: dict, download_dir: str = "./s3prl_hub", multilayer_feature: bool = True,
                 layer: int = -1, frozen: bool = False, frame_shift: int = 20, frame_length: int = 20,
                 sample_rate: int = 16000):
        super().__init__()
        name = (upstream_args or {}).get("name", None)
        if name not in SUPPORTED_UPSTREAMS:
            raise NotImplementedError(f"s3prl upstream {name!r}: only {SUPPORTED_UPSTREAMS} run on the MI355X path")
        if (upstream_args or {}).get("normalize", False):
            raise NotImplementedError("upstream normalize=True is not implemented (HuBERT-base uses False)")
        if layer != -1 and multilayer_feature:
            raise AssertionError("multilayer_feature must be False if layer is specified")  # s3prl.py:60-61
        self.multilayer_feature = multilayer_feature
        self.layer = layer
        self.frozen = frozen
        self.download_dir = download_dir
        self.sample_rate = sample_rate
        self.downsample_rate = 320
        # s3prl.py:69: featurizer.downsample_rate == sample_rate * frame_shift // 1000
        assert self.downsample_rate == sample_rate * frame_shift // 1000
        self._layout = hubert_params()
        self._pre_finalize = ("layer",)
        if layer != -1:
            self._options["layer"] = int(layer)
        elif not multilayer_feature:
            self._options["layer"] = HUBERT_BASE["layers"]  # featurizer(feats[-1:]) = last hidden state
        else:
            self._options["layer"] = -1

    def _create_args(self):
        return "HuBERT_base", 1, HUBERT_BASE["hidden"], False, False

    def _canonical(self, key: str) -> str:
        return key if key.startswith("frontend.") else "frontend." + key

    def output_size(self) -> int:
        return HUBERT_BASE["hidden"]

    # ----------------------------------------------------------- forward --
    def out_frames(self, num_samples: int) -> int:
        self._need()
        t = ctypes.c_int()
        _lib.check(_lib.load().wsp_frontend_out_frames(self._handle, int(num_samples), ctypes.byref(t)),
                   "wsp_frontend_out_frames")
        return t.value

    def workspace_bytes(self, B: int, num_samples: int) -> int:
        self._need()
        b = ctypes.c_size_t()
        _lib.check(_lib.load().wsp_frontend_workspace_bytes(self._handle, B, num_samples, ctypes.byref(b)),
                   "wsp_frontend_workspace_bytes")
        return b.value

    def extract(self, wavs: torch.Tensor, cmn: bool = False, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """(B, W) float32 HIP tensor in [-1, 1] -> (B, ceil(W/320), 768); cmn=True fuses
        bin/extract.py:104-106's apply_cmvn(norm_mean=True)."""
        if not wavs.is_cuda:
            raise RuntimeError("S3prlFrontend runs on a HIP device tensor (no CPU fallback)")
        if self._handle is None or self._device != wavs.device.index:
            self.to(wavs.device)
        if wavs.dim() != 2:
            raise ValueError(f"expected (B, W) waveforms, got {tuple(wavs.shape)}")
        wavs = wavs.float().contiguous()
        B, W = wavs.shape
        T = self.out_frames(W)
        if out is None:
            out = torch.empty(B, T, self.output_size(), dtype=torch.float32, device=wavs.device)
        ws = self._workspace_tensor(self.workspace_bytes(B, W), wavs.device)
        stream = torch.cuda.current_stream(wavs.device).cuda_stream
        _lib.check(_lib.load().wsp_frontend_forward(self._handle, wavs.data_ptr(), B, W, out.data_ptr(), int(cmn),
                                                    ws.data_ptr(), ws.numel(), stream), "wsp_frontend_forward")
        return out

    def extract_segments(self, wavs, cmn: bool = False) -> Tuple[torch.Tensor, List[int]]:
        """Ragged batch of whole utterances (sequence of 1-D [-1, 1] waveforms, >= 1
        samples each) -> (feats [sum_b T_b][768] on the device, frame offsets [B+1]);
        rows of utterance b equal extract(wavs[b][None])[0]."""
        dev = torch.device("cuda", self._device if self._device is not None else torch.cuda.current_device())
        if self._handle is None:
            self.to(dev)
        lens = np.asarray([int(len(w)) for w in wavs], dtype=np.int32)
        cat = torch.cat([torch.as_tensor(w).reshape(-1).to(torch.float32) for w in wavs]).to(dev)
        nb = ctypes.c_size_t()
        lib = _lib.load()
        _lib.check(lib.wsp_frontend_workspace_bytes_segments(self._handle, len(lens), lens.ctypes.data,
                                                             ctypes.byref(nb)), "wsp_frontend_workspace_bytes_segments")
        total = int(sum((int(n) + 319) // 320 for n in lens))
        feats = torch.empty(total, self.output_size(), dtype=torch.float32, device=dev)
        offs = np.zeros(len(lens) + 1, dtype=np.int32)
        ws = self._workspace_tensor(nb.value, dev)
        stream = torch.cuda.current_stream(dev).cuda_stream
        _lib.check(lib.wsp_frontend_forward_segments(self._handle, cat.data_ptr(), len(lens), lens.ctypes.data,
                                                     feats.data_ptr(), offs.ctypes.data, int(cmn), ws.data_ptr(),
                                                     ws.numel(), stream), "wsp_frontend_forward_segments")
        return feats, offs.tolist()

    def forward(self, input: torch.Tensor, input_lengths: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """s3prl.py:80-93: (wavs (B, W), wavs_len (B,)) -> (feats (B, T, 768), feats_lens (B,))."""
        lens = torch.as_tensor(input_lengths).flatten().tolist()
        if any(int(n) != input.shape[1] for n in lens):
            raise NotImplementedError("padded (unequal-length) batches are not implemented; bin/extract.py "
                                      "always passes equal lengths")
        feats = self.extract(input)
        feats_lens = torch.full((input.shape[0],), feats.shape[1], dtype=torch.long, device=feats.device)
        return feats, feats_lens

    __call__ = forward
