"""Out-of-bounds write hunt: every torch.empty / empty_like / zeros / zeros_like / full on the GPU made while the path
runs returns the leading view of a larger buffer whose tail (GUARD elements) holds a sentinel; after the run every
tail is compared and the allocation sites (file:line) of changed tails are printed.  Runs the f16 training step
(C5 config at a small batch, GradScaler), the C2 inference path and the C4 inference path.
    python tools/oob_guard.py [c5|c2|c4 ...]"""
import os
import sys
import traceback

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GUARD = 4096
_guards = []
_orig = {}


def _site():
    for fr in reversed(traceback.extract_stack()[:-2]):
        if "image_compression_2_amd" in fr.filename or "bench" in fr.filename:
            return f"{os.path.basename(fr.filename)}:{fr.lineno}"
    return "?"


def _shape(size):
    if len(size) == 1 and isinstance(size[0], (list, tuple, torch.Size)):
        return tuple(size[0])
    return tuple(size)


def _guarded(shape, dtype, device, fill=None):
    n = 1
    for s in shape:
        n *= int(s)
    base = _orig["empty"](n + GUARD, dtype=dtype, device=device)
    tail = base[n:]
    if dtype.is_floating_point:
        tail.fill_(-1234.5)
    else:
        tail.fill_(0x5A)
    _guards.append((tail, tail.clone(), _site(), tuple(shape), dtype))
    out = base[:n].view(shape)
    if fill is not None:
        out.fill_(fill)
    return out


def _is_gpu(device):
    return device is not None and torch.device(device).type == "cuda"


def install():
    _orig.update(empty=torch.empty, zeros=torch.zeros, empty_like=torch.empty_like, zeros_like=torch.zeros_like,
                 full=torch.full)

    def empty(*size, dtype=None, device=None, **kw):
        if not _is_gpu(device) or kw.get("out") is not None:
            return _orig["empty"](*size, dtype=dtype, device=device, **kw)
        return _guarded(_shape(size), dtype or torch.get_default_dtype(), device)

    def zeros(*size, dtype=None, device=None, **kw):
        if not _is_gpu(device) or kw.get("out") is not None:
            return _orig["zeros"](*size, dtype=dtype, device=device, **kw)
        return _guarded(_shape(size), dtype or torch.get_default_dtype(), device, 0)

    def full(size, value, dtype=None, device=None, **kw):
        if not _is_gpu(device):
            return _orig["full"](size, value, dtype=dtype, device=device, **kw)
        return _guarded(tuple(size), dtype or torch.get_default_dtype(), device, value)

    def empty_like(t, dtype=None, device=None, **kw):
        dev = device if device is not None else t.device
        if not _is_gpu(dev) or kw.get("memory_format") not in (None, torch.contiguous_format, torch.preserve_format):
            return _orig["empty_like"](t, dtype=dtype, device=device, **kw)
        return _guarded(tuple(t.shape), dtype or t.dtype, dev)

    def zeros_like(t, dtype=None, device=None, **kw):
        dev = device if device is not None else t.device
        if not _is_gpu(dev):
            return _orig["zeros_like"](t, dtype=dtype, device=device, **kw)
        return _guarded(tuple(t.shape), dtype or t.dtype, dev, 0)

    torch.empty, torch.zeros, torch.full, torch.empty_like, torch.zeros_like = empty, zeros, full, empty_like, zeros_like


def check(label):
    torch.cuda.synchronize()
    bad = {}
    for tail, ref, site, shape, dt in _guards:
        if not torch.equal(tail, ref):
            k = (site, shape, str(dt))
            nz = (tail != ref).nonzero()
            bad[k] = max(bad.get(k, 0), int(nz.max().item()) + 1 if nz.numel() else 0)
    print(f"[{label}] {len(_guards)} guarded allocations, {len(bad)} with writes past the end", flush=True)
    for (site, shape, dt), ext in sorted(bad.items()):
        print(f"   OOB  {site}  shape {shape} {dt}  (tail written up to element {ext})", flush=True)
    _guards.clear()
    return len(bad)


def run_c5(dev, ic2, ict):
    torch.manual_seed(0)
    enc = ic2.HVAE_VGG_Encoder(img_resolution=1024).to(dev)
    G = ic2.Generator(img_resolution=256).to(dev).eval().requires_grad_(False)
    comp = ic2.StyleGAN3Compressor(enc, G)
    scaler = ict.make_f16(comp)
    opt = ict.make_optimizer(enc)
    w_avg = G.mapping.w_avg.view(1, 1, -1)
    x = torch.rand(4, 3, 256, 256, generator=torch.Generator().manual_seed(1)).to(dev) * 2 - 1
    for _ in range(2):
        out = ict.train_step(comp, x, opt, w_avg, perceptual_weight=0.0, scaler=scaler)
    print("[c5] losses", {k: round(float(v), 5) for k, v in out.items()}, flush=True)


def run_c2(dev, ic2, res=256, n=4):
    """The bench's inference path: HVAE_VGG_Encoder(1024) in bf16x3 -> 8-bit quantizer -> SG3-T-<res> in f16."""
    torch.manual_seed(0)
    enc = ic2.HVAE_VGG_Encoder(img_resolution=1024, precision="bf16x3").to(dev).eval().requires_grad_(False)
    G = ic2.Generator(img_resolution=res, precision="f16").to(dev).eval()
    comp = ic2.StyleGAN3Compressor(enc, G)
    x = torch.rand(n, 3, res, res, generator=torch.Generator().manual_seed(2)).to(dev) * 2 - 1
    with torch.no_grad():
        img = comp.decompress(comp.compress(x, quantization_bits=8, deterministic=True))
    print(f"[c2 {res}] image", tuple(img.shape), float(img.float().abs().mean()), flush=True)


def main():
    which = sys.argv[1:] or ["c5", "c2", "c4"]
    import image_compression_2_amd as ic2
    from image_compression_2_amd import training as ict
    dev = torch.device("cuda", 0)
    install()
    bad = 0
    for w in which:
        if w == "c5":
            run_c5(dev, ic2, ict)
        elif w == "c2":
            run_c2(dev, ic2)
        elif w == "c4":
            run_c2(dev, ic2, res=1024, n=2)
        bad += check(w)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
