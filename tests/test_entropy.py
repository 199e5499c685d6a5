"""CPU: the native range coder behind cabac_compression (libic2ops.so ic2_rc_*; host code, no GPU).

The reference's CABAC (cabac_compression.py:60-406) raises on encode, so there is no reference
output to pin against; the contract tested is the one its cabac_encode/cabac_decode pair promises: lossless
round trips of [B, num_ws, w_dim] codebook indices, plus determinism and real compression of skewed codes.
"""
import numpy as np
import pytest

from image_compression_2_amd import cabac_compression as cc


def _round_trip(codes, n_symbols=256, threads=0):
    cm = cc.ContextModel(n_symbols=n_symbols)
    cm.n_threads = threads
    blob = cc.cabac_encode(codes, cm)
    back = cc.cabac_decode(blob, cm, codes.shape)
    assert back.dtype == np.int32 and back.shape == codes.shape
    assert np.array_equal(back, codes)
    return blob


@pytest.mark.parametrize("shape", [(4, 16, 512), (1, 1, 1), (3, 1, 7), (2, 5, 1), (1, 16, 512)])
def test_uniform_codes_round_trip(shape):
    rng = np.random.default_rng(0)
    codes = rng.integers(0, 256, size=shape, dtype=np.int32)
    blob = _round_trip(codes)
    # incompressible input: at most a few percent above 8 bits per symbol plus per-stream framing
    assert len(blob) <= codes.size * 1.04 + 24 + 4 * shape[0] + 8 * shape[0]


def test_skewed_latent_codes_compress():
    """Codes shaped like quantized encoder means (concentrated around the codebook centre, correlated along
    the w vector) compress well below 8 bits per symbol."""
    rng = np.random.default_rng(1)
    base = rng.normal(0, 0.15, size=(8, 1, 512))
    z = np.clip(base + rng.normal(0, 0.05, size=(8, 16, 512)), -1, 1)
    codes = np.rint((z + 1) * 0.5 * 255).astype(np.int32)
    blob = _round_trip(codes)
    bits_per_symbol = 8 * len(blob) / codes.size
    # order-0 entropy of the symbols
    p = np.bincount(codes.ravel(), minlength=256) / codes.size
    h0 = -(p[p > 0] * np.log2(p[p > 0])).sum()
    assert bits_per_symbol < 0.8 * 8
    assert bits_per_symbol < h0 + 0.5


@pytest.mark.parametrize("n_symbols", [2, 5, 17, 128, 256])
def test_alphabet_sizes(n_symbols):
    rng = np.random.default_rng(n_symbols)
    codes = rng.integers(0, n_symbols, size=(3, 4, 33), dtype=np.int32)
    _round_trip(codes, n_symbols=n_symbols)


def test_constant_codes_collapse():
    codes = np.full((2, 16, 512), 200, dtype=np.int32)
    blob = _round_trip(codes)
    assert len(blob) < codes.size / 25   # ~0.2 bit per symbol: 8 decisions at the 31/2048 probability floor


def test_deterministic_and_thread_independent():
    rng = np.random.default_rng(2)
    codes = rng.integers(0, 64, size=(16, 16, 512), dtype=np.int32)
    a = _round_trip(codes, threads=1)
    b = _round_trip(codes, threads=8)
    c = _round_trip(codes, threads=0)
    assert a == b == c
    # streams are independent: image 5 alone encodes to the same stream bytes
    one = cc.cabac_encode(codes[5:6], cc.ContextModel())
    sizes = np.frombuffer(a[24:24 + 4 * 16], dtype="<u4")
    start = 24 + 4 * 16 + int(sizes[:5].sum())
    assert one[28:] == a[start:start + int(sizes[5])]


def test_out_of_range_and_corrupt_input_fail_loudly():
    cm = cc.ContextModel(n_symbols=16)
    with pytest.raises(RuntimeError, match="outside"):
        cc.cabac_encode(np.array([[[3, 16]]], dtype=np.int32), cm)
    with pytest.raises(RuntimeError, match="outside"):
        cc.cabac_encode(np.array([[[-1]]], dtype=np.int32), cm)
    blob = cc.cabac_encode(np.zeros((1, 2, 8), dtype=np.int32), cm)
    with pytest.raises(ValueError):
        cc.cabac_decode(b"XXXX" + blob[4:], cm)
    with pytest.raises(ValueError):
        cc.cabac_decode(blob[:-3], cm)
    with pytest.raises(ValueError):
        cc.cabac_decode(blob, cc.ContextModel(n_symbols=256))
    with pytest.raises(ValueError):
        cc.cabac_decode(blob, cm, (1, 2, 9))


def test_untrusted_header_cannot_force_a_huge_allocation():
    """ADVICE r2 (decompression bomb): a ~256 KiB file must not make cabac_decode allocate b * num_ws * w_dim int32
    codes far beyond what its payload can hold -- the total is capped, and each stream's size must be able to
    hold its symbols (>= 5 bytes, <= 64 symbols per byte: the coder's probability floor allows ~45)."""
    import struct
    cm = cc.ContextModel(n_symbols=256)
    b, num_ws, w_dim = 65536, 16, 1 << 20          # 2^24 symbols per stream, 2^40 in total
    head = struct.pack("<4s5I", b"IC2R", 1, b, num_ws, w_dim, 256) + struct.pack(f"<{b}I", *([0] * b))
    with pytest.raises(ValueError, match="implausible"):
        cc.cabac_decode(head, cm)
    b, num_ws, w_dim = 16, 16, 1 << 20              # within the total cap, but zero-length streams
    head = struct.pack("<4s5I", b"IC2R", 1, b, num_ws, w_dim, 256) + struct.pack(f"<{b}I", *([0] * b))
    with pytest.raises(ValueError, match="implausible"):
        cc.cabac_decode(head, cm)
    # 5-byte streams claiming 2^24 symbols each: more than 5 bytes can decode to
    head = struct.pack("<4s5I", b"IC2R", 1, b, num_ws, w_dim, 256) + struct.pack(f"<{b}I", *([5] * b)) + bytes(5 * b)
    with pytest.raises(ValueError, match="implausible"):
        cc.cabac_decode(head, cm)
    # the densest genuine stream (constant codes) is still accepted
    codes = np.full((1, 16, 4096), 7, dtype=np.int32)
    assert np.array_equal(cc.cabac_decode(cc.cabac_encode(codes, cm), cm), codes)
