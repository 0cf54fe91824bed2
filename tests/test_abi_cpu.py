"""CPU-only checks of the C-ABI library: it loads without a GPU and exports
every symbol include/wespeaker_amd.h declares (no compute calls)."""
import ctypes
import os
import re

from wespeaker_hubert_amd import _lib

HDR = os.path.join(os.path.dirname(os.path.dirname(__file__)), "include", "wespeaker_amd.h")


def header_symbols():
    txt = open(HDR).read()
    return sorted(set(re.findall(r"\b(wsp_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    lib = ctypes.CDLL(_lib.LIB_PATH)
    syms = header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(_lib.SIGNATURES), set(syms) ^ set(_lib.SIGNATURES)


def test_pure_host_entry_points():
    lib = _lib.load()
    assert lib.wsp_abi_version() == 1
    assert lib.wsp_fbank_num_frames(80000, 400, 160) == 498
    assert lib.wsp_fbank_num_frames(399, 400, 160) == 0
    assert lib.wsp_fbank_num_frames(400, 400, 160) == 1
    # model creation / parameter layout is host-only until finalize()
    h = ctypes.c_void_p()
    assert lib.wsp_model_create(b"ECAPA_TDNN_c512", 80, 192, 0, 0, ctypes.byref(h)) == 0
    n = lib.wsp_model_num_params(h)
    from wespeaker_hubert_amd.arch import make_spec, param_list
    plist = param_list(make_spec("ECAPA_TDNN_c512", feat_dim=80, embed_dim=192))
    assert n == len(plist)
    name = ctypes.c_char_p()
    nd = ctypes.c_int()
    shp = (ctypes.c_int64 * 4)()
    for i, (pn, ps) in enumerate(plist):
        assert lib.wsp_model_param_info(h, i, ctypes.byref(name), ctypes.byref(nd), shp) == 0
        assert name.value.decode() == pn
        assert tuple(shp[d] for d in range(nd.value)) == tuple(ps)
    assert lib.wsp_model_forward(h, None, 1, 10, None, None, 0, None) != 0
    assert b"null" in lib.wsp_last_error()
    lib.wsp_model_destroy(h)


def test_hubert_handle_layout_matches_reference_names():
    """HuBERT_base handle (host-only until finalize): parameter names / shapes are the
    reference checkpoint's frontend.* entries (arch.hubert_params)."""
    from wespeaker_hubert_amd.arch import hubert_params
    lib = _lib.load()
    h = ctypes.c_void_p()
    assert lib.wsp_model_create(b"HuBERT_base", 1, 768, 0, 0, ctypes.byref(h)) == 0
    try:
        want = hubert_params()
        assert lib.wsp_model_num_params(h) == len(want)
        name, ndim, shape = ctypes.c_char_p(), ctypes.c_int(), (ctypes.c_int64 * 4)()
        for i, (n, s) in enumerate(want):
            assert lib.wsp_model_param_info(h, i, ctypes.byref(name), ctypes.byref(ndim), shape) == 0
            assert name.value.decode() == n and tuple(shape[d] for d in range(ndim.value)) == tuple(s)
        assert lib.wsp_model_set_option(h, b"layer", 13) != 0  # only -1..12
        assert lib.wsp_model_set_option(h, b"layer", 6) == 0
        t = ctypes.c_int()
        assert lib.wsp_frontend_out_frames(h, 80000, ctypes.byref(t)) == 0 and t.value == 250
        # s3prl MIN_SECOND: short inputs run zero-padded, output keeps len(range(0, W, 320))
        assert lib.wsp_frontend_out_frames(h, 399, ctypes.byref(t)) == 0 and t.value == 2
        assert lib.wsp_frontend_out_frames(h, 0, ctypes.byref(t)) != 0
        b = ctypes.c_size_t()
        assert lib.wsp_frontend_workspace_bytes(h, 4, 16000, ctypes.byref(b)) == 0 and b.value > 0
        assert lib.wsp_model_workspace_bytes(h, 4, 100, ctypes.byref(b)) != 0  # not a backbone handle
    finally:
        lib.wsp_model_destroy(h)
    assert lib.wsp_model_create(b"HuBERT_base", 1, 512, 0, 0, ctypes.byref(h)) != 0


def test_unknown_arch_is_an_error():
    lib = _lib.load()
    h = ctypes.c_void_p()
    assert lib.wsp_model_create(b"NOPE", 80, 192, 0, 0, ctypes.byref(h)) != 0


def test_resnet_feat_dim_must_be_a_multiple_of_8():
    """resnet.py:124 sizes seg_1 for int(feat_dim / 8) frequency rows while the convs keep
    ceil(feat_dim / 8): the reference only runs for multiples of 8, so the C-ABI refuses the rest."""
    lib = _lib.load()
    h = ctypes.c_void_p()
    assert lib.wsp_model_create(b"ResNet34", 60, 256, 0, 0, ctypes.byref(h)) != 0
    assert b"multiple of 8" in lib.wsp_last_error()
    assert lib.wsp_model_create(b"ResNet34", 72, 256, 0, 0, ctypes.byref(h)) == 0
    lib.wsp_model_destroy(h)


def test_option_defaults_and_streams_workspace():
    """Host-only: per-architecture option defaults (wsp_model_get_option) and the
    workspace of a split batch ("streams": one 256-B-granular slice per range)."""
    lib = _lib.load()
    v, b1, b2 = ctypes.c_int(), ctypes.c_size_t(), ctypes.c_size_t()
    for arch, feat, emb, want in ((b"ECAPA_TDNN_c512", 80, 192, 1), (b"ResNet34", 80, 256, 2),
                                  (b"HuBERT_base", 1, 768, 2)):
        h = ctypes.c_void_p()
        assert lib.wsp_model_create(arch, feat, emb, 0, 0, ctypes.byref(h)) == 0
        try:
            assert lib.wsp_model_get_option(h, b"streams", ctypes.byref(v)) == 0 and v.value == want
            assert lib.wsp_model_get_option(h, b"precision", ctypes.byref(v)) == 0 and v.value == 1
            assert lib.wsp_model_get_option(h, b"nope", ctypes.byref(v)) != 0
            assert lib.wsp_model_set_option(h, b"streams", 0) != 0
            if arch != b"HuBERT_base":
                assert lib.wsp_model_set_option(h, b"streams", 1) == 0
                assert lib.wsp_model_workspace_bytes(h, 6, 200, ctypes.byref(b1)) == 0
                assert lib.wsp_model_set_option(h, b"streams", 3) == 0
                assert lib.wsp_model_get_option(h, b"streams", ctypes.byref(v)) == 0 and v.value == 3
                assert lib.wsp_model_workspace_bytes(h, 6, 200, ctypes.byref(b2)) == 0
                # three 2-utterance slices: about the 6-utterance workspace (per-slice fixed parts)
                assert b1.value // 2 < b2.value <= b1.value + 3 * 65536
        finally:
            lib.wsp_model_destroy(h)


def test_fbank_host_tables_match_oracle():
    """The kernel's mel filters are computed by the library's own host code
    (fbank.hip fbank_mel_banks, torchaudio get_mel_banks' float32 arithmetic): bit-identical
    to the oracle's independent numpy restatement for every recipe configuration."""
    import numpy as np
    from oracle.fbank_ref import mel_banks
    from wespeaker_hubert_amd.frontend import FbankArgs
    for nb in (23, 40, 64, 72, 80, 128):
        for sr in (8000, 16000):
            a = FbankArgs(nb, sample_rate=sr)
            fl, fs, padded = a.geometry()
            assert (fl, fs, padded) == ((200, 80, 256) if sr == 8000 else (400, 160, 512))
            got = a.mel_banks()
            ref = mel_banks(nb, padded, float(sr))
            assert got.shape == ref.shape == (nb, padded // 2 + 1)
            assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), (nb, sr)


def test_fbank_geometry_rejects_unsupported():
    import pytest
    from wespeaker_hubert_amd.frontend import FbankArgs
    assert FbankArgs(frame_length=32).geometry() == (512, 160, 512)
    with pytest.raises(_lib.WspError, match="pad to 256 or 512"):
        FbankArgs(frame_length=40).geometry()
    with pytest.raises(_lib.WspError, match="num_mel_bins"):
        FbankArgs(num_mel_bins=3).geometry()
    with pytest.raises(_lib.WspError, match="too wide"):
        FbankArgs(num_mel_bins=8).geometry()
    with pytest.raises(ValueError, match="Invalid window type"):
        FbankArgs(window_type="triangle").geometry()
    for w in ("hamming", "hanning", "povey", "rectangular", "blackman"):
        assert FbankArgs(window_type=w).geometry() == (400, 160, 512)
