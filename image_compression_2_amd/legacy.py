"""SG3 network-pickle loader that executes nothing from the file.

The reference loads its generator with ``pickle.load(f)['G_ema']`` (``gumbel_softmax_compression.py:390-391``,
``cabac_compression.py:638-639``; ``stylegan3_hvae_full.py`` receives ``G`` the same way from its caller).  An SG3
pickle stores every network as a ``torch_utils.persistence`` record: ``_reconstruct_persistent_obj(meta)`` where
``meta = {type, version, module_src, class_name, state}`` and ``module_src`` is Python source that a plain
``pickle.load`` would ``exec``.  Here that source is never run:

* ``find_class`` resolves only a fixed allow-list (the persistence reconstructor, tensor / parameter / storage
  rebuilders, ``collections.OrderedDict``, torch dtypes, ``dnnlib.EasyDict``, numpy's scalar / array
  reconstructors); every other global becomes an inert
  placeholder whose construction records its arguments and runs nothing;
* storages are decoded with ``torch.load(..., weights_only=True)`` instead of torch's ``_load_from_bytes``
  (which uses ``weights_only=False``);
* persistent records become ``PersistentRecord`` objects (class name + the module ``__dict__`` state) from which
  the parameters / buffers are walked into a flat state dict with SG3's key names.

``load_network_pkl(f)`` returns ``{'G_ema': Generator, ...}`` (other top-level entries as raw records) so
``load_network_pkl(f)['G_ema']`` is the drop-in for the reference line.  The generator is this package's
``Generator`` (SG3-T only; radial filters, i.e. SG3-R, are rejected), built from the record's ``_init_kwargs`` and
filled with ``load_state_dict(strict=True)``.

Parity: unpinned against a real NVlabs pickle (none is available offline); tests build pickles
with the same record layout and check the round trip, the allow-list and that injected globals never run.
"""
from __future__ import annotations

import collections
import io
import pickle

import numpy as np
import torch

try:  # numpy >= 2 keeps the reconstructors in numpy._core (numpy.core is a deprecated alias)
    from numpy._core import multiarray as _np_ma
except ImportError:  # pragma: no cover - numpy 1.x
    from numpy.core import multiarray as _np_ma

__all__ = ["PersistentRecord", "SafeUnpickler", "load_network_pkl", "record_state_dict", "generator_from_record"]


class PersistentRecord:
    """Inert stand-in for a ``torch_utils.persistence`` object: the decorated class name and its pickled state."""

    def __init__(self, meta):
        if not isinstance(meta, dict) or meta.get("type") != "class":
            raise pickle.UnpicklingError(f"unsupported persistent record: {type(meta).__name__}")
        self.class_name = str(meta.get("class_name"))
        self.version = meta.get("version")
        self.state = meta.get("state") or {}
        self.module_src_len = len(meta.get("module_src") or "")   # kept for diagnostics, never executed

    @property
    def init_kwargs(self):
        return dict(self.state.get("_init_kwargs") or {})

    @property
    def init_args(self):
        return tuple(self.state.get("_init_args") or ())

    def __repr__(self):
        return f"PersistentRecord({self.class_name})"


class _Opaque:
    """Placeholder for any global outside the allow-list: construction and state-setting only record data."""

    _qualname = "?"

    def __new__(cls, *args, **kwargs):
        return object.__new__(cls)

    def __init__(self, *args, **kwargs):
        self.args, self.kwargs = args, kwargs

    def __setstate__(self, state):
        self.state = state

    def __repr__(self):
        return f"<opaque {self._qualname}>"


def _opaque(module, name):
    return type(f"Opaque[{module}.{name}]", (_Opaque,), {"_qualname": f"{module}.{name}"})


def _load_storage(b):
    if not isinstance(b, (bytes, bytearray)):
        raise pickle.UnpicklingError("storage payload is not bytes")
    return torch.load(io.BytesIO(b), weights_only=True, map_location="cpu")


def _rebuild_tensor(storage, offset, size, stride, requires_grad=False, backward_hooks=None, metadata=None):
    if not isinstance(storage, (torch.TypedStorage, torch.UntypedStorage)):
        raise pickle.UnpicklingError(f"tensor storage of type {type(storage).__name__}")
    t = torch.empty(0, dtype=storage.dtype)
    t.set_(storage._untyped_storage if isinstance(storage, torch.TypedStorage) else storage,
           int(offset), tuple(int(s) for s in size), tuple(int(s) for s in stride))
    return t


def _rebuild_parameter(data, requires_grad=False, backward_hooks=None, state=None):
    if not isinstance(data, torch.Tensor):
        raise pickle.UnpicklingError("parameter data is not a tensor")
    return torch.nn.Parameter(data, requires_grad=bool(requires_grad))


class _EasyDict(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e


_ALLOWED = {
    ("torch_utils.persistence", "_reconstruct_persistent_obj"): PersistentRecord,
    ("torch.storage", "_load_from_bytes"): _load_storage,
    ("torch._utils", "_rebuild_tensor_v2"): _rebuild_tensor,
    ("torch._utils", "_rebuild_tensor"): _rebuild_tensor,
    ("torch._utils", "_rebuild_parameter"): _rebuild_parameter,
    ("torch._utils", "_rebuild_parameter_with_state"): _rebuild_parameter,
    ("collections", "OrderedDict"): collections.OrderedDict,
    ("dnnlib.util", "EasyDict"): _EasyDict,
    ("dnnlib", "EasyDict"): _EasyDict,
    ("builtins", "set"): set,
    ("builtins", "frozenset"): frozenset,
    ("builtins", "slice"): slice,
    ("torch", "Size"): torch.Size,
    # SG3 layers keep numpy scalars / arrays as attributes (sizes, sampling rates): data-only constructors
    ("numpy", "dtype"): np.dtype,
    ("numpy", "ndarray"): np.ndarray,
    ("numpy.core.multiarray", "scalar"): _np_ma.scalar,
    ("numpy._core.multiarray", "scalar"): _np_ma.scalar,
    ("numpy.core.multiarray", "_reconstruct"): _np_ma._reconstruct,
    ("numpy._core.multiarray", "_reconstruct"): _np_ma._reconstruct,
}
_DTYPES = {n for n in dir(torch) if isinstance(getattr(torch, n, None), torch.dtype)}


class SafeUnpickler(pickle.Unpickler):
    """Resolves only the allow-list; every other global is an inert ``_Opaque`` subclass (names kept in ``opaque``)."""

    def __init__(self, f):
        super().__init__(f)
        self.opaque = []

    def find_class(self, module, name):
        fn = _ALLOWED.get((module, name))
        if fn is not None:
            return fn
        if module == "torch" and name in _DTYPES:
            return getattr(torch, name)
        self.opaque.append(f"{module}.{name}")
        return _opaque(module, name)

    def persistent_load(self, pid):
        raise pickle.UnpicklingError("persistent ids are not used by SG3 network pickles")


def record_state_dict(rec, prefix=""):
    """Flatten a PersistentRecord module tree (``_parameters`` / ``_buffers`` / ``_modules``) into SG3 keys."""
    out = collections.OrderedDict()
    st = rec.state if isinstance(rec, PersistentRecord) else getattr(rec, "state", None)
    if not isinstance(st, dict):
        raise pickle.UnpicklingError(f"module record at '{prefix}' has no state")
    for group in ("_parameters", "_buffers"):
        for k, v in (st.get(group) or {}).items():
            if v is not None:
                out[prefix + k] = v.detach() if isinstance(v, torch.Tensor) else v
    for k, child in (st.get("_modules") or {}).items():
        if child is not None:
            out.update(record_state_dict(child, prefix + k + "."))
    return out


def _generator_kwargs(rec):
    kw = rec.init_kwargs
    if not kw:   # positional construction: Generator(z_dim, c_dim, w_dim, img_resolution, img_channels, ...)
        names = ["z_dim", "c_dim", "w_dim", "img_resolution", "img_channels"]
        kw = dict(zip(names, rec.init_args))
    st = rec.state
    for k in ("z_dim", "c_dim", "w_dim", "img_resolution", "img_channels"):
        if k not in kw and k in st:
            kw[k] = st[k]
    syn = dict(kw.pop("synthesis_kwargs", {}) or {})
    kw.update(syn)
    if kw.pop("use_radial_filters", False):
        raise NotImplementedError("StyleGAN3-R (radial filters) is out of scope (DESIGN.md (f)); use an SG3-T pickle")
    return kw


def generator_from_record(rec, precision="fp32", device="cuda"):
    """Build this package's ``Generator`` from a G/G_ema record and load its weights (strict key match)."""
    from .networks_stylegan3 import Generator
    if not isinstance(rec, PersistentRecord) or rec.class_name != "Generator":
        raise ValueError(f"expected a persistent Generator record, got {rec!r}")
    kw = _generator_kwargs(rec)
    G = Generator(precision=precision, **kw)
    sd = record_state_dict(rec)
    G.load_state_dict(sd, strict=True)
    return G.to(device).eval().requires_grad_(False)


def load_network_pkl(f, precision="fp32", device="cuda"):
    """``legacy.load_network_pkl`` / ``pickle.load(f)`` mirror: ``{'G_ema': Generator, 'G': ..., ...}``.

    ``f`` is a path or a binary file object.  ``G_ema`` (and ``G`` when present) become ``Generator`` modules on
    ``device``; other entries (``D``, ``augment_pipe``, ``training_set_kwargs``) are returned as inert records."""
    if isinstance(f, (str, bytes)) or hasattr(f, "__fspath__"):
        with open(f, "rb") as fh:
            return load_network_pkl(fh, precision=precision, device=device)
    data = SafeUnpickler(f).load()
    if not isinstance(data, dict) or "G_ema" not in data:
        raise ValueError("not an SG3 network pickle (no 'G_ema' entry)")
    out = dict(data)
    for k in ("G_ema", "G"):
        if isinstance(out.get(k), PersistentRecord):
            out[k] = generator_from_record(out[k], precision=precision, device=device)
    return out
