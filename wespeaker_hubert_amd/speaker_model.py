"""Host-side mirror of the reference model registry and forward contract.

`get_speaker_model(name)(**model_args)` (wespeaker/models/speaker_model.py:30-57)
returns a `HipSpeakerModel` whose `load_state_dict(sd, strict=False)` accepts the
reference `avg_model.pt` state_dict (wespeaker/utils/checkpoint.py:20-27) and whose
`__call__(feats)` returns `(aux, embed)` like ECAPA_TDNN.forward / ResNet.forward
(ecapa_tdnn.py:227-234, resnet.py:192-204) — `outputs[-1]` is the embedding as in
cli/speaker.py:166 and bin/extract.py:115.  All compute runs in libwsp_hip.so.
"""
from __future__ import annotations

import ctypes
import logging
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from . import _lib
from .arch import ModelSpec, make_spec, param_list

logger = logging.getLogger(__name__)


def _to_numpy(v) -> np.ndarray:
    if isinstance(v, torch.Tensor):
        return v.detach().to("cpu").contiguous().numpy()
    a = np.asarray(v)
    return a if a.flags.c_contiguous else a.copy()  # (ascontiguousarray turns 0-d into 1-d)


class _HipHandle:
    """Weight intake + device handle shared by the speaker backbones and the
    SSL front end: reference state_dict names in, one `wsp_model` handle per
    device out.  Subclasses provide `_layout`, `_create_args()` and
    `_ignored_keys` (checkpoint entries the reference module holds but the
    extraction path never reads)."""

    _ignored_prefixes: Tuple[str, ...] = ()

    def __init__(self):
        self._host: Dict[str, np.ndarray] = {}
        self._handle: Optional[ctypes.c_void_p] = None
        self._device: Optional[int] = None
        self._ws: Optional[torch.Tensor] = None
        self._options: Dict[str, int] = {}
        self._pre_finalize: Tuple[str, ...] = ()

    # ----------------------------------------------------------- weights --
    def state_dict_layout(self) -> List[Tuple[str, Tuple[int, ...]]]:
        return list(self._layout)

    def _canonical(self, key: str) -> str:
        return key

    def load_state_dict(self, state_dict, strict: bool = False):
        """Mirror of `model.load_state_dict(checkpoint, strict=False)` + its warnings."""
        names = {n: s for n, s in self._layout}
        missing, unexpected = [], []
        for k, v in state_dict.items():
            key = self._canonical(k)
            if key not in names:
                if not any(key.startswith(p) for p in self._ignored_prefixes):
                    unexpected.append(k)
                continue
            arr = _to_numpy(v)
            if tuple(arr.shape) != tuple(names[key]):
                raise ValueError(f"size mismatch for {k}: {tuple(arr.shape)} vs {names[key]}")
            self._host[key] = arr
        for n, _ in self._layout:
            if n not in self._host:
                missing.append(n)
        for key in missing:
            logger.warning("missing tensor: %s", key)
        for key in unexpected:
            logger.warning("unexpected tensor: %s", key)
        if strict and (missing or unexpected):
            raise RuntimeError(f"strict load failed: missing={missing} unexpected={unexpected}")
        self._release()
        return missing, unexpected

    def eval(self):
        return self

    # ------------------------------------------------------------ device --
    def _release(self):
        if self._handle is not None:
            _lib.load().wsp_model_destroy(self._handle)
            self._handle = None
            self._ws = None

    def __del__(self):
        try:
            self._release()
        except Exception:
            pass

    def to(self, device):
        device = torch.device(device)
        if device.type != "cuda":
            raise RuntimeError(f"{type(self).__name__} runs only on a HIP device (no CPU fallback)")
        idx = device.index if device.index is not None else torch.cuda.current_device()
        if self._handle is None or self._device != idx:
            self._release()
            with torch.cuda.device(idx):
                self._build()
            self._device = idx
        return self

    def _build(self):
        lib = _lib.load()
        h = ctypes.c_void_p()
        arch, feat_dim, embed_dim, emb_bn, two_emb = self._create_args()
        _lib.check(lib.wsp_model_create(arch.encode(), feat_dim, embed_dim, int(emb_bn), int(two_emb),
                                        ctypes.byref(h)), "wsp_model_create")
        name = ctypes.c_char_p()
        ndim = ctypes.c_int()
        shape = (ctypes.c_int64 * 4)()
        try:
            for k in self._pre_finalize:
                _lib.check(lib.wsp_model_set_option(h, k.encode(), self._options[k]), "set_option " + k)
            n = lib.wsp_model_num_params(h)  # after the pre-finalize options (they may reshape the layout)
            for i in range(n):
                _lib.check(lib.wsp_model_param_info(h, i, ctypes.byref(name), ctypes.byref(ndim), shape),
                           "param_info")
                key = name.value.decode()
                want = tuple(shape[d] for d in range(ndim.value))
                if key.endswith("num_batches_tracked"):
                    continue
                if key not in self._host:
                    raise RuntimeError(f"parameter {key} was not loaded (shape {want})")
                arr = np.ascontiguousarray(self._host[key], dtype=np.float32)
                if tuple(arr.shape) != want:
                    raise RuntimeError(f"{key}: shape {arr.shape} != {want}")
                _lib.check(lib.wsp_model_set_param(h, i, arr.ctypes.data, arr.size), "set_param " + key)
            _lib.check(lib.wsp_model_finalize(h), "wsp_model_finalize")
            for k, v in self._options.items():
                if k not in self._pre_finalize:
                    _lib.check(lib.wsp_model_set_option(h, k.encode(), v), "set_option " + k)
        except Exception:
            lib.wsp_model_destroy(h)
            raise
        self._handle = h

    def _need(self):
        if self._handle is None:
            raise RuntimeError("model not on a HIP device: call .to('cuda') first")

    def _workspace_tensor(self, need: int, device) -> torch.Tensor:
        if self._ws is None or self._ws.numel() < need or self._ws.device != device:
            self._ws = torch.empty(need, dtype=torch.uint8, device=device)
        return self._ws

    def set_option(self, key: str, value: int):
        """Runtime option of the handle (include/wespeaker_amd.h lists them), e.g.
        'precision': 1 = bf16x3 split MFMA (default), 0 = exact f32 MFMA;
        'streams': utterance ranges forwarded on concurrent HIP streams."""
        self._options[key] = int(value)
        if key in self._pre_finalize:
            self._release()  # rebuilt with the option on the next .to()/forward
        elif self._handle is not None:
            _lib.check(_lib.load().wsp_model_set_option(self._handle, key.encode(), int(value)), "set_option")

    def get_option(self, key: str) -> int:
        """Value of a runtime option on the device handle (set or per-architecture default)."""
        self._need()
        v = ctypes.c_int(0)
        _lib.check(_lib.load().wsp_model_get_option(self._handle, key.encode(), ctypes.byref(v)), "get_option")
        return int(v.value)

    # ----------------------------------------------------------- profile --
    def profile(self, enable: bool):
        self._need()
        _lib.check(_lib.load().wsp_model_profile(self._handle, int(enable)), "profile")

    def profile_query(self, kernel_class: str):
        self._need()
        n = ctypes.c_int()
        ms = ctypes.c_double()
        fl = ctypes.c_double()
        _lib.check(_lib.load().wsp_model_profile_query(self._handle, kernel_class.encode(), ctypes.byref(n),
                                                       ctypes.byref(ms), ctypes.byref(fl)), "profile_query")
        return n.value, ms.value, fl.value


class HipSpeakerModel(_HipHandle):
    """ECAPA-TDNN / ResNet speaker backbone executed by hand-written gfx950 kernels."""

    def __init__(self, arch: str, **model_args):
        super().__init__()
        self.spec: ModelSpec = make_spec(arch, **model_args)
        self._layout = param_list(self.spec)
        if self.spec.family == "simam" and self.spec.m_channels != 64:
            self._options["in_planes"] = self.spec.m_channels  # before the weights (samresnet.py:124)
            self._pre_finalize = ("in_planes",)

    def _create_args(self):
        s = self.spec
        return s.arch, s.feat_dim, s.embed_dim, s.emb_bn, s.two_emb_layer

    # ----------------------------------------------------------- forward --
    def workspace_bytes(self, B: int, T: int) -> int:
        self._need()
        b = ctypes.c_size_t()
        _lib.check(_lib.load().wsp_model_workspace_bytes(self._handle, B, T, ctypes.byref(b)),
                   "workspace_bytes")
        return b.value

    def _workspace(self, B: int, T: int, device) -> torch.Tensor:
        return self._workspace_tensor(self.workspace_bytes(B, T), device)

    def embed(self, feats: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """(B, T, feat_dim) float32 cuda -> (B, embed_dim) float32 cuda."""
        if not feats.is_cuda:
            raise RuntimeError("feats must be a HIP device tensor")
        if self._handle is None or self._device != feats.device.index:
            self.to(feats.device)
        if feats.dim() != 3 or feats.shape[2] != self.spec.feat_dim:
            raise ValueError(f"expected (B, T, {self.spec.feat_dim}) features, got {tuple(feats.shape)}")
        feats = feats.float().contiguous()
        B, T, _ = feats.shape
        if out is None:
            out = torch.empty(B, self.spec.embed_dim, dtype=torch.float32, device=feats.device)
        ws = self._workspace(B, T, feats.device)
        stream = torch.cuda.current_stream(feats.device).cuda_stream
        _lib.check(_lib.load().wsp_model_forward(self._handle, feats.data_ptr(), B, T, out.data_ptr(),
                                                 ws.data_ptr(), ws.numel(), stream), "wsp_model_forward")
        return out

    def embed_segments(self, feats: torch.Tensor, frame_offsets: torch.Tensor,
                       out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Ragged batch (ECAPA-TDNN): utterance b = rows [off[b], off[b+1]) of feats
        [sum T_b][feat_dim]; frame_offsets = int32 [B+1] on the same device.  Each row of
        the result equals embed(feats_b[None])."""
        if not feats.is_cuda or not frame_offsets.is_cuda:
            raise RuntimeError("feats / frame_offsets must be HIP device tensors")
        if self._handle is None or self._device != feats.device.index:
            self.to(feats.device)
        if feats.dim() != 2 or feats.shape[1] != self.spec.feat_dim:
            raise ValueError(f"expected (rows, {self.spec.feat_dim}) features, got {tuple(feats.shape)}")
        feats = feats.float().contiguous()
        off = frame_offsets.to(torch.int32).contiguous()
        B, M = off.numel() - 1, feats.shape[0]
        if out is None:
            out = torch.empty(B, self.spec.embed_dim, dtype=torch.float32, device=feats.device)
        b = ctypes.c_size_t()
        _lib.check(_lib.load().wsp_model_workspace_bytes_segments(self._handle, B, M, ctypes.byref(b)),
                   "workspace_bytes_segments")
        ws = self._workspace_tensor(b.value, feats.device)
        stream = torch.cuda.current_stream(feats.device).cuda_stream
        _lib.check(_lib.load().wsp_model_forward_segments(self._handle, feats.data_ptr(), B, off.data_ptr(), M,
                                                          out.data_ptr(), ws.data_ptr(), ws.numel(), stream),
                   "wsp_model_forward_segments")
        return out

    @property
    def supports_segments(self) -> bool:
        return self.spec.family == "ecapa"

    def __call__(self, feats: torch.Tensor):
        # SimAM_ResNet*_ASP.forward returns the embedding itself (samresnet.py:135-143);
        # ECAPA / ResNet return (aux, embed)
        if self.spec.family == "simam":
            return self.embed(feats)
        return None, self.embed(feats)

    forward = __call__


def get_speaker_model(model_name: str):
    """speaker_model.py:30-57 — returns a constructor taking **model_args."""
    make_spec(model_name)  # raises KeyError for unknown names

    def ctor(**model_args):
        return HipSpeakerModel(model_name, **model_args)

    return ctor
