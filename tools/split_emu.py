"""CPU emulation of the encoder precision candidates against the fp32 oracle: each conv computed
in fp64 on operands rounded / split as a mode would store them, conv outputs f32; 8-bit index flips vs the oracle.
    python tools/split_emu.py B mode [mode ...]   (modes: fp64 bf16 f16 split_bf16 split_f16 x2_* w2_* mixK tailK hmixK)"""
import sys, torch, torch.nn.functional as F, time
sys.path.insert(0, '/root/repo')
import image_compression_2_amd as ic2
from oracle import encoder as oe
torch.set_num_threads(8)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
torch.manual_seed(0)
enc = ic2.HVAE_VGG_Encoder(img_resolution=1024)
sd = {k: v.detach() for k, v in enc.state_dict().items()}
RES = int(__import__("os").environ.get("RES", "256"))
x = torch.rand(B, 3, RES, RES, generator=torch.Generator().manual_seed(1000)) * 2 - 1
torch.manual_seed(5)
lin = torch.nn.Linear(128, 256); fc1 = (lin.weight.detach(), lin.bias.detach())
with torch.no_grad():
    _, m_ref, _ = oe.encoder_forward(sd, x, fine_fc1=fc1)

def rnd(t, dt): return t.to(dt).to(torch.float64)
def split(t, dt):
    hi = t.to(dt).to(torch.float64); lo = (t.double() - hi).to(dt).to(torch.float64); return hi, lo

CONV_IDX = [0]


def make_conv(mode):
    base = mode
    if mode.startswith('mix') or mode.startswith('tail') or mode.startswith('hmix') or mode.startswith('hy'):
        # mixK: the first K convs (from_rgb = 0, block i conv1 = 1 + 2i, conv2 = 2 + 2i) in bf16, the rest split;
        # tailK: the convs from index K on in bf16, the ones before split
        k = int(mode[4:] if mode.startswith('hmix') else mode[2:] if mode.startswith('hy') else mode[3:] if mode.startswith('mix') else mode[4:])
    def conv(x, w, b):
        mode = base
        if base.startswith('mix'):
            mode = 'bf16' if CONV_IDX[0] < k else 'split_bf16'
            CONV_IDX[0] += 1
        elif base.startswith('hmix'):
            mode = 'w2_f16' if 0 < CONV_IDX[0] < k else 'split_bf16'
            CONV_IDX[0] += 1
        elif base.startswith('hy'):  # hmixK with those convs' outputs stored f16 as well
            mode = 'w2_f16' if 0 < CONV_IDX[0] < k else 'split_bf16'
            y16 = 0 < CONV_IDX[0] < k
            CONV_IDX[0] += 1
        elif base.startswith('tail'):
            mode = 'bf16' if CONV_IDX[0] >= k else 'split_bf16'
            CONV_IDX[0] += 1
        if mode == 'fp64':
            y = F.conv2d(x.double(), w.double(), b.double(), padding=1)
        elif mode in ('bf16', 'f16'):
            dt = torch.bfloat16 if mode == 'bf16' else torch.float16
            y = F.conv2d(rnd(x, dt), rnd(w, dt), b.double(), padding=1)
        else:
            dt = torch.bfloat16 if 'bf16' in mode else torch.float16
            xh, xl = split(x, dt); wh, wl = split(w, dt)
            y = F.conv2d(xh, wh, b.double(), padding=1) + F.conv2d(xh, wl, None, padding=1) + F.conv2d(xl, wh, None, padding=1)
            if mode.startswith('w2'):
                y = F.conv2d(xh, wh, b.double(), padding=1) + F.conv2d(xh, wl, None, padding=1)
            if mode.startswith('x2'):
                y = F.conv2d(xh, wh, b.double(), padding=1) + F.conv2d(xl, wh, None, padding=1)
            if mode.endswith('4'):
                y = y + F.conv2d(xl, wl, None, padding=1)
        y = y.float()
        if base.startswith('hy') and y16:
            y = y.half().float()
        if mode in ('bf16',):
            y = y.to(torch.bfloat16).float()
        return y
    return conv

def enc_forward(mode):
    CONV_IDX[0] = 0
    conv = make_conv(mode)
    store = (lambda t: t.to(torch.bfloat16).float()) if mode == 'bf16' else (lambda t: t)
    if mode.startswith('mix'):  # activations stored bf16 while the convs consuming them are bf16
        k = int(mode[3:])
        store = lambda t: t.to(torch.bfloat16).float() if CONV_IDX[0] < k else t
    if mode.startswith('hmix') or mode.startswith('hy'):  # convs 1 .. K-1 (block 0 = 1, 2) x f16, w split f16; their inputs stored f16
        k = int(mode[4:] if mode.startswith('hmix') else mode[2:])
        store = lambda t: t.to(torch.float16).float() if 0 < CONV_IDX[0] < k else t
    if mode.startswith('tail'):
        k = int(mode[4:])
        store = lambda t: t.to(torch.bfloat16).float() if CONV_IDX[0] >= k else t
    h = store(conv(x, sd['from_rgb.weight'], sd['from_rgb.bias']))
    feats = {}
    for i in range(10):
        if h.shape[2] <= 1: break
        p = f'blocks.{i}.'
        c = sd[p + 'conv1.weight'].shape[0]; g = min(32, c)
        y = conv(h, sd[p+'conv1.weight'], sd[p+'conv1.bias'])
        h = store(F.leaky_relu(F.group_norm(y, g, sd[p+'norm1.weight'], sd[p+'norm1.bias'], 1e-5), 0.2))
        y = conv(h, sd[p+'conv2.weight'], sd[p+'conv2.bias'])
        h = F.leaky_relu(F.group_norm(y, g, sd[p+'norm2.weight'], sd[p+'norm2.bias'], 1e-5), 0.2)
        if h.shape[2] > 1: h = F.avg_pool2d(h, 2, 2)
        h = store(h)
        if i == 1: feats['fine'] = h
        elif i == 4: feats['medium'] = h
    feats['global'] = h
    g = oe.projector(sd, 'global_projector.', feats['global'], 5)
    m = oe.projector(sd, 'medium_projector.', feats['medium'], 7)
    f = oe.projector(sd, 'fine_projector.', feats['fine'], 4, fc1=fc1)
    return torch.cat([g[1], m[1], f[1]], 1)

i_ref = oe.uniform_indices(m_ref, 8)
u = (m_ref.double() + 1) * 0.5 * 255
hs = (u - u.floor() - 0.5).abs() * 2 / 255
for mode in sys.argv[2:]:
    t0 = time.time()
    with torch.no_grad():
        m = enc_forward(mode)
    i = oe.uniform_indices(m, 8)
    mism = i != i_ref
    err = (m - m_ref).abs()
    print(f"{mode:10s} max|dm| {err.max():.3e} mean|dm| {err.mean():.3e} flips {int(mism.sum())}/{mism.numel()} = {mism.float().mean():.2e}"
          f" max halfstep-dist of flip {hs[mism].max().item() if mism.any() else 0:.2e}  ({time.time()-t0:.1f}s)", flush=True)
