"""Entropy-coded codebook compression: drop-in for /root/reference/cabac_compression.py's codec classes.

The reference's CABAC (``ContextModel`` :60-162, ``ArithmeticCoder`` :166-311, ``cabac_encode`` / ``cabac_decode``
:315-406) cannot encode: ``high`` overflows 32 bits after ``_handle_underflow`` (:210) and ``bytes([...])`` raises
at :197.  Here the same stage is a context-adaptive binary range coder in native host code
(``ic2_rc_encode`` / ``ic2_rc_decode`` in libic2ops.so, ``csrc/entropy.hip``) with the reference's context
definition (previous symbol of the w vector, same position of the previous w vector; :78-117), one independent
stream per image, streams coded on parallel threads.  Round trips are lossless by construction and tested.

Byte format of ``cabac_encode`` (little-endian): ``b"IC2R"``, u32 version (1), u32 n_streams, u32 num_ws,
u32 w_dim, u32 n_symbols, u32 size[n_streams], then the streams.  ``.cabac`` files keep the reference's layout
(u32 metadata length, metadata, payload) but the metadata is JSON, not a pickle, so loading executes nothing.
The codes come from the GPU path (encoder + exact codebook argmin); only the entropy stage runs on the host.
"""
from __future__ import annotations

import ctypes
import json
import struct

import numpy as np
import torch

from . import _native as nv
from .gumbel_softmax_compression import GumbelSoftmaxDiscretization, check_codes, codebook_argmin, codebook_lookup

_MAGIC = b"IC2R"
_VERSION = 1
_MAX_SYMBOLS_PER_STREAM = 1 << 24   # an untrusted header may not ask for more than this per image ...
_MAX_STREAMS = 1 << 16
_MAX_TOTAL_SYMBOLS = 1 << 26        # ... nor for more than this in total (256 MiB of int32 codes)
# The coder's probabilities saturate at 2017/2048 (11 bits, shift-5 update), so a binary decision costs >= 0.022
# bits and a symbol (8 decisions) >= 0.176 bits: a stream cannot hold more than ~45 symbols per byte.  Its flush
# writes 5 bytes, so a genuine stream is never shorter.
_MAX_SYMBOLS_PER_BYTE = 64
_MIN_STREAM_BYTES = 5


class ContextModel:
    """Parameters of the coder's context model (ref :60-76).  The reference's float EMA tables
    (``adaptation_rate``) are replaced by 11-bit binary probabilities with a 1/32 update in the native coder;
    ``context_size`` / ``adaptation_rate`` are kept for signature compatibility."""

    def __init__(self, n_symbols=256, context_size=5, adaptation_rate=0.05):
        if not 2 <= n_symbols <= 256:
            raise ValueError(f"n_symbols must be in [2, 256], got {n_symbols}")
        self.n_symbols = n_symbols
        self.context_size = context_size
        self.adaptation_rate = adaptation_rate
        self.n_threads = 0    # native default: hardware concurrency, capped at 16


def _as_codes(data):
    a = data.detach().cpu().numpy() if isinstance(data, torch.Tensor) else np.asarray(data)
    if a.ndim == 2:
        a = a[None]
    if a.ndim != 3:
        raise ValueError(f"codes must be [batch, num_ws, w_dim], got shape {a.shape}")
    return np.ascontiguousarray(a, dtype=np.int32)


def cabac_encode(data, context_model):
    """codes [B, num_ws, w_dim] (ints in [0, n_symbols)) -> bytes (ref :315-360)."""
    codes = _as_codes(data)
    b, num_ws, w_dim = codes.shape
    lib = nv.load()
    cap = int(lib.ic2_rc_bound(b, num_ws * w_dim))
    out = np.empty(cap, dtype=np.uint8)
    sizes = np.empty(b, dtype=np.int64)
    nv.call("ic2_rc_encode", codes.ctypes.data_as(ctypes.c_void_p), b, num_ws, w_dim, context_model.n_symbols,
            out.ctypes.data_as(ctypes.c_void_p), cap, sizes.ctypes.data_as(ctypes.c_void_p), context_model.n_threads)
    head = struct.pack("<4s5I", _MAGIC, _VERSION, b, num_ws, w_dim, context_model.n_symbols)
    head += struct.pack(f"<{b}I", *[int(s) for s in sizes])
    return head + out[: int(sizes.sum())].tobytes()


def cabac_decode(encoded_bytes, context_model, shape=None):
    """bytes -> int32 codes [B, num_ws, w_dim] (ref :363-406).  ``shape``, when given, is checked."""
    buf = memoryview(encoded_bytes)
    if len(buf) < 24 or bytes(buf[:4]) != _MAGIC:
        raise ValueError("not an IC2R entropy-coded stream")
    _, version, b, num_ws, w_dim, n_symbols = struct.unpack_from("<4s5I", buf, 0)
    if version != _VERSION:
        raise ValueError(f"unsupported IC2R version {version}")
    # the header is untrusted: bound the allocation it asks for before making it -- per stream, in total, and by
    # what the payload bytes can possibly decode to
    per = num_ws * w_dim
    if not (0 < b <= _MAX_STREAMS and 0 < num_ws and 0 < w_dim and per <= _MAX_SYMBOLS_PER_STREAM
            and b * per <= _MAX_TOTAL_SYMBOLS):
        raise ValueError(f"implausible IC2R header: {b} streams of {num_ws} x {w_dim} symbols")
    if len(buf) < 24 + 4 * b:
        raise ValueError("truncated IC2R header")
    if n_symbols != context_model.n_symbols:
        raise ValueError(f"stream has {n_symbols} symbols, context model {context_model.n_symbols}")
    if shape is not None and tuple(shape) != (b, num_ws, w_dim):
        raise ValueError(f"stream shape {(b, num_ws, w_dim)} != expected {tuple(shape)}")
    off = 24 + 4 * b
    sizes = np.array(struct.unpack_from(f"<{b}I", buf, 24), dtype=np.int64)
    if (sizes < _MIN_STREAM_BYTES).any() or (per > _MAX_SYMBOLS_PER_BYTE * sizes).any():
        raise ValueError(f"implausible IC2R stream sizes for {per} symbols per stream")
    payload = np.frombuffer(buf, dtype=np.uint8, offset=off)
    if payload.size < int(sizes.sum()):
        raise ValueError("truncated IC2R stream")
    payload = np.ascontiguousarray(payload)
    codes = np.empty((b, num_ws, w_dim), dtype=np.int32)
    nv.call("ic2_rc_decode", payload.ctypes.data_as(ctypes.c_void_p), sizes.ctypes.data_as(ctypes.c_void_p), b,
            num_ws, w_dim, n_symbols, codes.ctypes.data_as(ctypes.c_void_p), context_model.n_threads)
    return codes


class CABACCompressor:
    """HVAE encoder + codebook quantizer + entropy coder + frozen generator (ref :409-588)."""

    def __init__(self, encoder, generator, discretization=None, n_embeddings=256, training_resolution=None):
        self.encoder = encoder
        self.generator = generator
        self.training_resolution = training_resolution
        if discretization is None:
            dev = next(encoder.parameters()).device
            discretization = GumbelSoftmaxDiscretization(latent_dim=encoder.w_dim, n_embeddings=n_embeddings).to(dev)
        self.discretization = discretization
        self.context_model = ContextModel(n_symbols=self.discretization.n_embeddings)

    def encode(self, x, deterministic=True):
        w_plus, means, _ = self.encoder(x)
        w_discrete, _, _ = self.discretization(means if deterministic else w_plus, hard=True)
        return w_discrete

    def compress(self, x, use_cabac=True):
        """-> (bytes, metadata) with the reference's metadata keys (ref :451-495)."""
        with torch.no_grad():
            w_plus, means, _ = self.encoder(x)
            indices = codebook_argmin(means, self.discretization.codebook)
            batch_size, num_ws, w_dim = w_plus.shape
            codes = indices.reshape(batch_size, num_ws, w_dim).cpu().numpy().astype(np.int32)
        orig_size = codes.size * np.log2(self.discretization.n_embeddings) / 8
        encoded = cabac_encode(codes, self.context_model) if use_cabac else codes.tobytes()
        comp_size = len(encoded)
        metadata = {"shape": list(codes.shape), "n_embeddings": int(self.discretization.n_embeddings),
                    "use_cabac": bool(use_cabac), "orig_size": float(orig_size), "comp_size": int(comp_size),
                    "compression_ratio": float(orig_size / comp_size)}
        return encoded, metadata

    def decompress(self, encoded_bytes, metadata, noise_mode="const"):
        shape = tuple(metadata["shape"])
        if metadata.get("use_cabac", True):  # the reference's default (ref :512)
            codes = cabac_decode(encoded_bytes, self.context_model, shape)
        else:
            codes = np.frombuffer(encoded_bytes, dtype=np.int32).reshape(shape)
        with torch.no_grad():
            dev = self.discretization.codebook.device
            w, flag = codebook_lookup(torch.from_numpy(codes.astype(np.int64)).to(dev), self.discretization.codebook)
            check_codes(flag, self.discretization.n_embeddings)
            return self.generator.synthesis(w, noise_mode=noise_mode)

    def save_compressed(self, x, filename, use_cabac=True):
        encoded, metadata = self.compress(x, use_cabac=use_cabac)
        meta = json.dumps(metadata).encode()
        with open(filename, "wb") as f:
            f.write(struct.pack("I", len(meta)))
            f.write(meta)
            f.write(encoded)
        return metadata["orig_size"], metadata["comp_size"], metadata["compression_ratio"]

    def load_compressed(self, filename, noise_mode="const"):
        with open(filename, "rb") as f:
            n = struct.unpack("I", f.read(4))[0]
            metadata = json.loads(f.read(n).decode())
            encoded = f.read()
        return self.decompress(encoded, metadata, noise_mode=noise_mode), metadata["compression_ratio"]
