"""kaldi ark/scp byte format (kaldiio WriteHelper layout; parity with kaldiio
itself is unpinned — kaldiio is absent) and fire-style flag parsing."""
import struct

import numpy as np
import pytest

from wespeaker_hubert_amd.bin import _fire
from wespeaker_hubert_amd.kaldi_io import WriteHelper, load_ark, load_scp_sequential


def test_ark_scp_roundtrip_and_bytes(tmp_path):
    ark = str(tmp_path / "x.ark")
    scp = str(tmp_path / "x.scp")
    rng = np.random.default_rng(0)
    vecs = {f"utt{i}": rng.standard_normal(192).astype(np.float32) for i in range(5)}
    with WriteHelper(f"ark,scp:{ark},{scp}") as w:
        for k, v in vecs.items():
            w(k, v)
    raw = open(ark, "rb").read()
    head = b"utt0 \x00BFV \x04" + struct.pack("<i", 192)
    assert raw.startswith(head)
    assert raw[len(head):len(head) + 192 * 4] == vecs["utt0"].tobytes()
    assert len(raw) == 5 * (len(head) + 192 * 4)
    lines = open(scp).read().splitlines()
    assert lines[0] == f"utt0 {ark}:5"
    assert lines[1] == f"utt1 {ark}:{5 + len(head) - 5 + 192 * 4 + 5}"
    got = dict(load_scp_sequential(scp))
    for k, v in vecs.items():
        np.testing.assert_array_equal(got[k], v)
    assert [k for k, _ in load_ark(ark)] == list(vecs)


def test_fire_parse():
    pos, kw = _fire.parse(["--exp_dir", "e", "--cal_mean", "True", "--batch-size", "16", "--top_n=300", "t1", "t2"])
    assert pos == ["t1", "t2"]
    assert kw == {"exp_dir": "e", "cal_mean": True, "batch_size": 16, "top_n": 300}


# ----------------------------------------------------------- matrix reader --
# Layouts from Kaldi's published sources (kaldi-matrix.cc Matrix::Read,
# compressed-matrix.{h,cc}); the bytes below are written by hand, not by the reader.

def _fm(rows, cols, data, tok=b"FM ", dt="<f4"):
    return (b"\0B" + tok + b"\x04" + struct.pack("<i", rows) + b"\x04" + struct.pack("<i", cols)
            + np.asarray(data, dtype=dt).tobytes())


def test_load_mat_fm_dm_offsets_and_slices(tmp_path):
    from wespeaker_hubert_amd.kaldi_io import load_mat
    a = np.arange(12, dtype=np.float32).reshape(3, 4) * 0.5 - 1.0
    b = np.arange(6, dtype=np.float64).reshape(2, 3) / 3.0
    p = tmp_path / "m.ark"
    blob = b"k1 " + _fm(3, 4, a) + b"k2 " + _fm(2, 3, b, b"DM ", "<f8")
    p.write_bytes(blob)
    off2 = len(b"k1 " + _fm(3, 4, a)) + 3
    np.testing.assert_array_equal(load_mat(f"{p}:3"), a)
    got = load_mat(f"{p}:{off2}")
    assert got.dtype == np.float64
    np.testing.assert_array_equal(got, b)
    np.testing.assert_array_equal(load_mat(f"{p}:3[1:3]"), a[1:3])
    np.testing.assert_array_equal(load_mat(f"{p}:3[0:2,1:3]"), a[0:2, 1:3])
    np.testing.assert_array_equal(load_mat(str(p)), a)  # path alone: the first object after its key


def test_load_mat_compressed_formats(tmp_path):
    from wespeaker_hubert_amd.kaldi_io import load_mat
    p = tmp_path / "c.ark"
    # CM3 (kOneByte, row-major): min -1, range 255 -> increment (255 * (1/255.0)) = 1 exactly
    q3 = np.array([[0, 1, 2], [250, 255, 7]], dtype=np.uint8)
    cm3 = b"\0BCM3 " + struct.pack("<ffii", -1.0, 255.0, 2, 3) + q3.tobytes()
    # CM2 (kTwoByte, row-major): min 2, range 65535 -> increment 1
    q2 = np.array([[0, 65535], [12345, 7]], dtype="<u2")
    cm2 = b"\0BCM2 " + struct.pack("<ffii", 2.0, 65535.0, 2, 2) + q2.tobytes()
    # CM (kOneByteWithColHeaders): per-column u16 percentiles, bytes column-major;
    # min 0, range 65535: Uint16ToFloat(v) = 65535 * 1.52590218966964e-05f * v
    pct = np.array([[0, 100, 300, 1000], [10, 20, 30, 40]], dtype="<u2")
    byt = np.array([[0, 64, 128, 192, 255], [32, 96, 160, 224, 200]], dtype=np.uint8)  # [col][row]
    cm = b"\0BCM " + struct.pack("<ffii", 0.0, 65535.0, 5, 2) + pct.tobytes() + byt.tobytes()
    blob = b"a " + cm3 + b"b " + cm2 + b"c " + cm
    p.write_bytes(blob)
    o_b = 2 + len(cm3) + 2
    o_c = o_b + len(cm2) + 2
    np.testing.assert_array_equal(load_mat(f"{p}:2"), q3.astype(np.float32) - 1.0)
    np.testing.assert_array_equal(load_mat(f"{p}:{o_b}"), q2.astype(np.float32) + 2.0)
    got = load_mat(f"{p}:{o_c}")
    assert got.shape == (5, 2) and got.dtype == np.float32

    def char_to_float(p0, p25, p75, p100, v):  # compressed-matrix.cc CharToFloat (in doubles)
        if v <= 64:
            return p0 + (p25 - p0) * v / 64.0
        if v <= 192:
            return p25 + (p75 - p25) * (v - 64) / 128.0
        return p75 + (p100 - p75) * (v - 192) / 63.0
    scale = 65535.0 * 1.52590218966964e-05
    for c in range(2):
        pc = [scale * float(x) for x in pct[c]]
        for r in range(5):
            want = char_to_float(*pc, int(byt[c, r]))
            assert abs(got[r, c] - want) <= 1e-6 * max(1.0, abs(want)), (r, c, got[r, c], want)


def test_load_mat_text(tmp_path):
    from wespeaker_hubert_amd.kaldi_io import load_mat
    p = tmp_path / "t.ark"
    p.write_bytes(b"u1  [\n  1 2.5 -3\n  4 5 6 ]\n")
    np.testing.assert_array_equal(load_mat(f"{p}:4"), np.array([[1, 2.5, -3], [4, 5, 6]], np.float32))


def test_load_scp_matrix_equals_sequential_reader(tmp_path):
    """The vectorised scp reader (scoring CLIs) returns exactly the per-record reader's
    keys and values: fixed-stride arks (strided view), variable-length keys and several
    arks in shuffled scp order (gather), and mixed dims / types (fallback)."""
    from wespeaker_hubert_amd.kaldi_io import load_scp_matrix
    rng = np.random.default_rng(5)
    with WriteHelper(f"ark,scp:{tmp_path}/a.ark,{tmp_path}/a.scp") as w:
        for i in range(40):
            w(f"u{i:04d}", rng.standard_normal(16).astype(np.float32))
    with WriteHelper(f"ark,scp:{tmp_path}/b.ark,{tmp_path}/b.scp") as w:
        for i in range(25):
            w("k" * (1 + i % 5) + str(i), rng.standard_normal(16).astype(np.float32))
    with WriteHelper(f"ark,scp:{tmp_path}/c.ark,{tmp_path}/c.scp") as w:
        w("d0", rng.standard_normal(16))  # float64 (DV)
        w("f0", rng.standard_normal(8).astype(np.float32))
    lines = open(tmp_path / "a.scp").read().splitlines() + open(tmp_path / "b.scp").read().splitlines()
    rng.shuffle(lines)
    (tmp_path / "m.scp").write_text("\n".join(lines) + "\n\n")
    for name in ("a.scp", "b.scp", "m.scp"):
        keys, mat = load_scp_matrix(str(tmp_path / name))
        ref = list(load_scp_sequential(str(tmp_path / name)))
        assert keys == [k for k, _ in ref] and mat.dtype == np.float32
        np.testing.assert_array_equal(mat, np.stack([v for _, v in ref]))
    with pytest.raises(ValueError):  # mixed dims cannot form one matrix
        load_scp_matrix(str(tmp_path / "c.scp"))
