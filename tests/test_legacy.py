"""CPU: the SG3 network-pickle loader (image_compression_2_amd/legacy.py) executes nothing from the file.

The reference does ``pickle.load(f)['G_ema']`` (gumbel_softmax_compression.py:390-391).  No NVlabs pickle exists
offline, so these tests write pickles with the same record layout as
``torch_utils.persistence`` (``_reconstruct_persistent_obj(meta)``, ``meta = {type, version, module_src,
class_name, state}``, ``state`` = the module ``__dict__``) from a seeded Generator and check the round trip.
Parity against a real trained pickle: unpinned.
"""
import io
import os
import pickle
import sys
import types

import pytest
import torch

from image_compression_2_amd import legacy
from image_compression_2_amd.networks_stylegan3 import Generator


def _install_fake_persistence():
    """A stand-in ``torch_utils.persistence`` so pickle can name the reconstructor while WRITING fixtures."""
    mod = types.ModuleType("torch_utils.persistence")

    def _reconstruct_persistent_obj(meta):   # never called by the loader under test
        raise AssertionError("the loader must not call the pickled reconstructor")
    _reconstruct_persistent_obj.__module__ = "torch_utils.persistence"
    _reconstruct_persistent_obj.__qualname__ = "_reconstruct_persistent_obj"
    mod._reconstruct_persistent_obj = _reconstruct_persistent_obj
    pkg = sys.modules.get("torch_utils") or types.ModuleType("torch_utils")
    pkg.persistence = mod
    return {"torch_utils": pkg, "torch_utils.persistence": mod}


class _Rec:
    def __init__(self, meta):
        self.meta = meta

    def __reduce__(self):
        return (sys.modules["torch_utils.persistence"]._reconstruct_persistent_obj, (self.meta,))


class _Evil:
    """Pickles as a call to os.system: the loader must neutralise it."""

    def __init__(self, path):
        self.path = path

    def __reduce__(self):
        return (os.system, (f"touch {self.path}",))


def _module_record(m, init_kwargs=None, extra=None):
    st = {"training": False,
          "_parameters": dict(m._parameters), "_buffers": dict(m._buffers),
          "_modules": {k: _module_record(c) for k, c in m._modules.items()}}
    for k, v in vars(m).items():
        if not k.startswith("_") and isinstance(v, (int, float, str, bool)):
            st[k] = v
    if init_kwargs is not None:
        st["_init_args"] = ()
        st["_init_kwargs"] = init_kwargs
    st.update(extra or {})
    return _Rec(dict(type="class", version=4, module_src="raise SystemExit('module_src must not run')\n",
                     class_name=type(m).__name__, state=st))


def _write_pkl(G, init_kwargs, extra=None, evil_path=None):
    saved = {k: sys.modules.get(k) for k in ("torch_utils", "torch_utils.persistence")}
    sys.modules.update(_install_fake_persistence())
    try:
        top = {"G": None, "D": None, "G_ema": _module_record(G, init_kwargs, extra),
               "augment_pipe": None, "training_set_kwargs": {"resolution": G.img_resolution}}
        if evil_path is not None:
            top["augment_pipe"] = _Evil(evil_path)
        return pickle.dumps(top, protocol=4)
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v


def _sg3_kwargs(res):
    # the shape of SG3's train.py G_kwargs for stylegan3-t (training/training_loop.py passes c_dim/res/channels)
    return dict(z_dim=512, w_dim=512, mapping_kwargs={"num_layers": 2}, channel_base=32768, channel_max=512,
                magnitude_ema_beta=0.5 ** (32 / (20 * 1e3)), c_dim=0, img_resolution=res, img_channels=3)


@pytest.mark.parametrize("res", [256, 1024])
def test_pickle_round_trip_reproduces_every_tensor(res):
    torch.manual_seed(3)
    G = Generator(img_resolution=res)
    with torch.no_grad():
        for k, b in G.named_buffers():
            if k.endswith("magnitude_ema"):
                b.fill_(0.37)      # trained pickles carry non-default EMA buffers
        G.mapping.w_avg.normal_()
    blob = _write_pkl(G, _sg3_kwargs(res))
    out = legacy.load_network_pkl(io.BytesIO(blob), device="cpu")
    G2 = out["G_ema"]
    assert isinstance(G2, Generator)
    assert G2.img_resolution == res and G2.num_ws == G.num_ws
    sd, sd2 = G.state_dict(), G2.state_dict()
    assert list(sd) == list(sd2)
    for k in sd:
        assert torch.equal(sd[k], sd2[k]), k
    assert [n for n, _ in G2.synthesis.named_children()] == [n for n, _ in G.synthesis.named_children()]
    assert out["training_set_kwargs"] == {"resolution": res}


def test_loader_never_executes_pickled_code(tmp_path):
    torch.manual_seed(0)
    G = Generator(img_resolution=256)
    marker = tmp_path / "pwned"
    blob = _write_pkl(G, _sg3_kwargs(256), evil_path=str(marker))
    assert b"system" in blob
    up = legacy.SafeUnpickler(io.BytesIO(blob))
    data = up.load()
    assert not marker.exists()
    assert any(n.endswith(".system") for n in up.opaque)
    assert isinstance(data["G_ema"], legacy.PersistentRecord)
    assert data["G_ema"].module_src_len > 0          # the source is carried, not run
    out = legacy.load_network_pkl(io.BytesIO(blob), device="cpu")
    assert not marker.exists()
    assert "pwned" not in repr(out["augment_pipe"]) or isinstance(out["augment_pipe"], legacy._Opaque)


def test_rejects_radial_and_non_generator_records():
    torch.manual_seed(0)
    G = Generator(img_resolution=256)
    kw = _sg3_kwargs(256)
    kw.update(use_radial_filters=True, conv_kernel=1)
    with pytest.raises(NotImplementedError):
        legacy.load_network_pkl(io.BytesIO(_write_pkl(G, kw)), device="cpu")
    with pytest.raises(ValueError):
        legacy.load_network_pkl(io.BytesIO(pickle.dumps({"G": 1})), device="cpu")


def test_missing_or_extra_tensors_fail_strictly():
    torch.manual_seed(0)
    G = Generator(img_resolution=256)
    rec = _module_record(G, _sg3_kwargs(256))
    del rec.meta["state"]["_modules"]["mapping"].meta["state"]["_buffers"]["w_avg"]
    saved = {k: sys.modules.get(k) for k in ("torch_utils", "torch_utils.persistence")}
    sys.modules.update(_install_fake_persistence())
    try:
        blob = pickle.dumps({"G_ema": rec}, protocol=4)
    finally:
        for k, v in saved.items():
            sys.modules.pop(k, None) if v is None else sys.modules.__setitem__(k, v)
    with pytest.raises(RuntimeError, match="w_avg"):
        legacy.load_network_pkl(io.BytesIO(blob), device="cpu")


def test_easydict_kwargs_as_written_by_sg3_train():
    """SG3's train.py passes mapping_kwargs as a dnnlib.EasyDict; the loader maps that class to a plain dict."""
    mod = types.ModuleType("dnnlib.util")

    class EasyDict(dict):
        pass
    EasyDict.__module__ = "dnnlib.util"
    EasyDict.__qualname__ = "EasyDict"
    mod.EasyDict = EasyDict
    pkg = types.ModuleType("dnnlib")
    pkg.util = mod
    saved = {k: sys.modules.get(k) for k in ("dnnlib", "dnnlib.util")}
    sys.modules.update({"dnnlib": pkg, "dnnlib.util": mod})
    try:
        torch.manual_seed(4)
        G = Generator(img_resolution=256)
        kw = _sg3_kwargs(256)
        kw["mapping_kwargs"] = EasyDict(num_layers=2)
        blob = _write_pkl(G, kw)
    finally:
        for k, v in saved.items():
            sys.modules.pop(k, None) if v is None else sys.modules.__setitem__(k, v)
    up = legacy.SafeUnpickler(io.BytesIO(blob))
    rec = up.load()["G_ema"]
    assert not up.opaque
    assert rec.init_kwargs["mapping_kwargs"]["num_layers"] == 2
    G2 = legacy.generator_from_record(rec, device="cpu")
    assert all(torch.equal(a, b) for a, b in zip(G.state_dict().values(), G2.state_dict().values()))
