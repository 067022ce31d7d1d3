"""TensorFlow tensor-bundle checkpoint I/O, CPU only.

No TensorFlow and no reference checkpoint exist offline, so the format is
pinned by published known answers (CRC-32C check values, the leveldb footer
magic), byte-level expectations of the protobuf / table encoding, round trips
and a strict reader (checksums of every block and tensor are verified)."""
import os
import struct

import numpy as np
import pytest

from lcn_amd import checkpoint as ckpt
from lcn_amd import tf_bundle as T


def test_crc32c_known_answers():
    # RFC 3720 B.4 / the CRC catalogue check value
    assert T.crc32c(b"123456789") == 0xE3069283
    assert T.crc32c(bytes(32)) == 0x8A9136AA
    assert T.crc32c(bytes([0xFF] * 32)) == 0x62A8AB43
    assert T.crc32c(bytes(range(32))) == 0x46DD794E
    assert T.crc32c(bytes(range(31, -1, -1))) == 0x113FDB5C
    data = np.random.default_rng(0).bytes(100003)
    assert T.crc32c(data[777:], T.crc32c(data[:777])) == T.crc32c(data)


def test_crc_mask_roundtrip():
    for c in (0, 1, 0xE3069283, 0xFFFFFFFF, 0x12345678):
        assert T.unmask_crc(T.mask_crc(c)) == c
    # leveldb crc32c::Mask of the check value
    assert T.mask_crc(0xE3069283) == ((((0xE3069283 >> 15) | (0xE3069283 << 17)) & 0xFFFFFFFF)
                                      + 0xA282EAD8) & 0xFFFFFFFF


def test_protobuf_encodings():
    # BundleHeaderProto{num_shards: 1, version{producer: 1}}
    assert T.encode_header() == bytes([0x08, 0x01, 0x1A, 0x02, 0x08, 0x01])
    e = T.encode_entry(T.DT_FLOAT, (34, 1088), 0, 34 * 1088 * 4, 0xE3069283)
    # dtype 1; shape{dim{size 34} dim{size 1088}}; size; fixed32 crc
    assert e[:2] == bytes([0x08, 0x01])
    assert e[2:13] == bytes([0x12, 0x09, 0x12, 0x02, 0x08, 34, 0x12, 0x03, 0x08, 0xC0, 0x08])
    d = T.decode_entry(e)
    assert d["dtype"] == 1 and d["shape"] == (34, 1088) and d["offset"] == 0
    assert d["size"] == 34 * 1088 * 4 and T.unmask_crc(d["crc32c"]) == 0xE3069283
    s = T.decode_entry(T.encode_entry(T.DT_INT32, (), 12, 4, 7))
    assert s["shape"] == () and s["offset"] == 12
    assert T.encode_entry(T.DT_INT32, (), 0, 4, 7)[2:4] == bytes([0x12, 0x00])  # scalar: empty shape


def test_table_layout_and_roundtrip(tmp_path):
    items = sorted((f"k{i:04d}".encode(), os.urandom(i % 50)) for i in range(300))
    p = str(tmp_path / "t.index")
    T.write_table(p, items)
    raw = open(p, "rb").read()
    assert struct.unpack("<Q", raw[-8:])[0] == 0xDB4775248B80FB57
    assert T.read_table(p) == items
    # a flipped byte in a block is caught by its checksum
    bad = bytearray(raw)
    bad[10] ^= 0x40
    open(p, "wb").write(bytes(bad))
    with pytest.raises(T.BundleError):
        T.read_table(p)


def test_table_with_many_blocks(tmp_path, monkeypatch):
    monkeypatch.setattr(T, "BLOCK_SIZE", 512)
    items = sorted((f"name/{i:05d}/x".encode(), bytes([i % 256]) * 40) for i in range(500))
    p = str(tmp_path / "m.index")
    T.write_table(p, items)
    assert T.read_table(p) == items


def test_separators():
    assert T._shortest_separator(b"abcdef", b"abzzz") == b"abd"
    assert T._shortest_separator(b"abc", b"abd") == b"abc"
    assert T._shortest_separator(b"ab", b"abc") == b"ab"
    assert T._short_successor(b"abc") == b"b"
    assert T._short_successor(b"\xff\xffa") == b"\xff\xffb"


def test_bundle_roundtrip(tmp_path):
    rng = np.random.default_rng(1)
    t = {"linear_model/w1": rng.standard_normal((34, 1088)).astype(np.float32),
         "linear_model/b1": rng.standard_normal(1088).astype(np.float32),
         "global_step": np.int32(1234).reshape(()),
         "beta1_power": np.float32(0.9 ** 5).reshape(()),
         "mask": rng.standard_normal((17, 17)).astype(np.float32),
         "x/f64": rng.standard_normal((3, 4, 5))}
    prefix = str(tmp_path / "model-7")
    T.write_bundle(prefix, t)
    assert os.path.exists(prefix + ".index") and os.path.exists(prefix + ".data-00000-of-00001")
    ent = T.list_bundle(prefix)
    assert list(ent) == sorted(t)
    back = T.read_bundle(prefix)
    for k, v in t.items():
        assert back[k].dtype == np.asarray(v).dtype and back[k].shape == np.asarray(v).shape
        np.testing.assert_array_equal(back[k], v)
    # data corruption is detected per tensor
    with open(prefix + ".data-00000-of-00001", "r+b") as f:
        f.seek(ent["linear_model/b1"]["offset"] + 5)
        f.write(b"\x00\x01")
    with pytest.raises(T.BundleError):
        T.read_bundle(prefix, names={"linear_model/b1"})
    T.read_bundle(prefix, names={"mask"})


class _FakeNet:
    """Host stand-in with the Network checkpoint surface (no GPU)."""

    def __init__(self, layout, n):
        self._layout, self.n_params = layout, n
        rng = np.random.default_rng(3)
        self.p = rng.standard_normal(n).astype(np.float32)
        self.m = rng.standard_normal(n).astype(np.float32)
        self.v = rng.random(n).astype(np.float32)
        self.state = (42, np.float32(0.9 ** 43), np.float32(0.999 ** 43))

    def param_layout(self):
        return self._layout

    def get_params(self):
        return self.p.copy()

    def set_params(self, f):
        self.p = np.asarray(f, np.float32).copy()

    def get_optimizer_state(self):
        return (self.m.copy(), self.v.copy()) + self.state

    def set_optimizer_state(self, m, v, gs, b1p, b2p):
        self.m, self.v = np.asarray(m, np.float32).copy(), np.asarray(v, np.float32).copy()
        self.state = (gs, np.float32(b1p), np.float32(b2p))


def _layout(F=64, L=2, in_F=2):
    import lcn_oracle as O
    cfg = O.Config(F=F, in_F=in_F, num_layers=L, neighbour=O.neighbour_matrix(2))
    out, off = [], 0
    for name, shape in O.param_specs(cfg):
        out.append((name, off, tuple(shape)))
        off += int(np.prod(shape))
    return out, off


def test_variable_names_follow_the_reference_graph():
    layout, _ = _layout(L=2)
    names = {ours: tf for ours, tf, _, _ in ckpt.tf_name_map(layout)}
    assert names["mask"] == "mask"
    assert names["w1"] == "linear_model/w1" and names["b4"] == "linear_model/b4"
    assert names["w2_1"] == "linear_model/two_linear_1/w2_1"
    assert names["bn0_gamma"] == "linear_model/batch_normalization/gamma"
    assert names["bn11_beta"] == "linear_model/two_linear_1/batch_normalization11/beta"
    assert names["bn20_gamma"] == "linear_model/two_linear_0/batch_normalization20/gamma"


def test_save_restore_roundtrip(tmp_path):
    layout, n = _layout(L=2)
    a = _FakeNet(layout, n)
    prefix = str(tmp_path / "final" / "model")
    out = ckpt.save(a, prefix, 42, {"regularization": False}, loss_ema=[0.3, 5])
    assert out.endswith("model-42")
    assert open(tmp_path / "final" / "checkpoint").read().startswith('model_checkpoint_path: "model-42"')
    names = T.list_bundle(out)
    for k in ("mask/Adam", "mask/Adam_1", "linear_model/w1/Adam_1", "beta1_power", "beta2_power",
              "global_step", "linear_model/batch_normalization/moving_variance",
              "loss/add/ExponentialMovingAverage",
              "loss/mse_loss/Mean/ExponentialMovingAverage"):
        assert k in names, k
    # zero_debias is off in the reference's EMA: no debias companions
    assert not [k for k in names if k.endswith("/biased") or k.endswith("/local_step")]
    assert names["global_step"]["dtype"] == T.DT_INT32
    b = _FakeNet(layout, n)
    b.p[:] = 0
    ema = ckpt.restore(b, ckpt.latest_checkpoint(str(tmp_path / "final")))
    np.testing.assert_array_equal(b.p, a.p)
    np.testing.assert_array_equal(b.m, a.m)
    np.testing.assert_array_equal(b.v, a.v)
    assert b.state[0] == 42 and b.state[1] == a.state[1] and b.state[2] == a.state[2]
    assert ema == (np.float32(0.3), 0)
    # max_to_keep=1: a later save replaces the files
    ckpt.save(a, prefix, 50)
    left = sorted(os.listdir(tmp_path / "final"))
    assert left == ["checkpoint", "model-50.data-00000-of-00001", "model-50.index"]


def test_latest_checkpoint_with_foreign_absolute_path(tmp_path):
    layout, n = _layout(L=1)
    a = _FakeNet(layout, n)
    d = tmp_path / "best"
    ckpt.save(a, str(d / "model"), 9)
    # the reference's Kaggle files name another machine's absolute path (README.md:84)
    (d / "checkpoint").write_text('model_checkpoint_path: "/kaggle/working/x/best/model-9"\n')
    assert ckpt.latest_checkpoint(str(d)) == str(d / "model-9")


def test_shape_mismatch_is_an_error(tmp_path):
    layout, n = _layout(L=1)
    ckpt.save(_FakeNet(layout, n), str(tmp_path / "model"), 1)
    layout2, n2 = _layout(L=1, F=128)
    with pytest.raises(ValueError):
        ckpt.restore(_FakeNet(layout2, n2), str(tmp_path / "model-1"))
