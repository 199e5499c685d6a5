"""Batch-sharded data parallelism: one process per GPU, contiguous batch slices,
no data-path collective; one all_reduce(SUM) of a small fp64 metric vector per batch over RCCL
(backend "nccl" on ROCm) -- gloo on CPU for tests.  The reference has no distributed code.

Training (BASELINE C5, data parallel): each rank backpropagates its own batch slice and the encoder's
gradients are averaged with ``allreduce_gradients`` -- bucketed flat all_reduce(SUM) / world, the only
collective of the step (the generator is frozen and has no gradients)."""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def env_rank_world():
    return int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)), int(os.environ.get("LOCAL_RANK", 0))


def init(backend=None):
    """Initialise the default process group from torchrun's env (no-op for world size 1)."""
    rank, world, local = env_rank_world()
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, local


def shard(n_total, rank, world):
    """Contiguous slice [start, stop) of a global batch for `rank` (sizes differ by at most 1)."""
    base, rem = divmod(n_total, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def metric_vector(sse_sum, n_values, n_images, hist=None, extra=()):
    """[sum SSE_uint8, n_pixels, n_images, *extra, *hist] as float64 (the all-reduced record)."""
    parts = [torch.tensor([float(sse_sum), float(n_values), float(n_images), *map(float, extra)], dtype=torch.float64)]
    if hist is not None:
        parts.append(hist.detach().to("cpu", torch.float64).reshape(-1))
    return torch.cat(parts)


def allreduce_sum(vec, device=None):
    """all_reduce(SUM) of a small fp64 vector (identity when not distributed)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return vec
    t = vec.to(device) if device is not None else vec
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.to(vec.device)


def allreduce_max(value, device=None):
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def allgather_floats(value, device=None):
    """[value of rank 0, value of rank 1, ...] (a one-element list when not distributed)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [float(value)]
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [float(o.item()) for o in out]


def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _spawned(local_rank, world, port, fn, args):
    os.environ.update({"RANK": str(local_rank), "LOCAL_RANK": str(local_rank), "WORLD_SIZE": str(world),
                       "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    fn(*args)


def launch(world, fn, *args):
    """One process per GPU without torchrun: spawn `world` fresh interpreters (start method 'spawn', so no
    child inherits a parent's GPU state and nothing exec's after a GPU call -- the parent never touches the
    device), each with torchrun's env (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT),
    running fn(*args).  Raises if any rank fails."""
    import torch.multiprocessing as mp
    # free_port() releases the port before rank 0's store binds it; if another process takes it in between, the
    # rendezvous fails with "address already in use": retry on a fresh port
    for attempt in range(4):
        try:
            mp.start_processes(_spawned, args=(world, free_port(), fn, args), nprocs=world, join=True,
                               start_method="spawn")
            return
        except Exception as e:  # torch.multiprocessing.ProcessRaisedException carries the rank's traceback text
            msg = str(e).lower()
            if attempt == 3 or not ("address already in use" in msg or "eaddrinuse" in msg):
                raise


def broadcast_params(module, src=0):
    """Copy `module`'s parameters from rank `src` to every rank (in place; no-op when not distributed).  Used for
    the fine projector's fc1, which the reference re-creates from each process's CPU generator on every call
    (stylegan3_hvae_full.py:225-230): without it the ranks of a data-parallel step would run -- and average the
    gradients of -- different weights."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return
    with torch.no_grad():
        for p in module.parameters():
            dist.broadcast(p.data, src)


def barrier(device=None):
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        if device is not None and device.type == "cuda":
            dist.barrier(device_ids=[device.index])
        else:
            dist.barrier()


def allreduce_gradients(params, world=None, bucket_bytes=64 << 20):
    """Average the .grad of ``params`` over ranks in place: grads are packed into flat f32 buckets of about
    ``bucket_bytes`` (one all_reduce per bucket: the encoder's 37.5 M gradients are three RCCL calls, large
    enough to run at xGMI ring bandwidth) and copied back divided by the world size.  Parameters without a
    gradient are skipped; every rank runs the same module graph, so the bucket layout agrees across ranks."""
    if world is None:
        world = dist.get_world_size() if dist.is_initialized() else 1
    grads = [p.grad for p in params if p.grad is not None]
    if world <= 1 or not grads:
        return 0
    buckets, cur, size = [], [], 0
    for g in grads:
        cur.append(g)
        size += g.numel() * 4
        if size >= bucket_bytes:
            buckets.append(cur)
            cur, size = [], 0
    if cur:
        buckets.append(cur)
    for b in buckets:
        flat = torch.cat([g.reshape(-1).to(torch.float32) for g in b])
        dist.all_reduce(flat, op=dist.ReduceOp.SUM)
        flat.div_(world)
        off = 0
        for g in b:
            k = g.numel()
            g.copy_(flat[off:off + k].view_as(g))
            off += k
    return len(buckets)


class GradReducer:
    """The gradient average of ``allreduce_gradients``, overlapped with backward: every parameter gets a
    post-accumulate-grad hook; a bucket (parameters packed to about ``bucket_bytes`` in the order backward produces
    their gradients) is flattened and its all_reduce(SUM) launched asynchronously (RCCL runs it on its own stream
    behind the flatten) as soon as its last gradient is accumulated, while backward continues with the layers below.
    Buckets launch strictly in index order (a completed bucket waits for the ones before it), so every rank issues
    the same collective sequence.  ``finish()`` waits for the handles, writes the averages back into .grad, and
    reduces what no hook covered: parameters created after the reducer (the reference's per-call fc1,
    stylegan3_hvae_full.py:225-230) and buckets with a parameter that got no gradient this step (the same on every
    rank: one module graph).

    Bucket order.  The first step's buckets follow reverse registration order.  That order is wrong for the
    reference's C5 encoder (img_resolution=1024 on 256^2 input): the 1x1 break (stylegan3_hvae_full.py:129-131)
    skips blocks 8-9, whose parameters register last, get no gradient, and would hold bucket 0 -- and with it every
    later bucket -- back until finish().  So the first step records the order the hooks actually fired in; rank 0's
    record is broadcast (every rank then buckets identically, as DDP's rebuild_buckets) and the buckets are rebuilt
    from it, leaving out the parameters that got no gradient.  From the second step on every bucket launches during
    backward.  A parameter left out that later does get a gradient is reduced by finish()'s leftover pass.

    Usage per step: ``r.start(); loss.backward(); r.finish()``.  Autograd sums every use of a parameter before its
    AccumulateGrad node runs, so a hook fires once per backward even with the training step's two encoder passes."""

    def __init__(self, module, world=None, bucket_bytes=25 << 20):
        self.world = world if world is not None else (dist.get_world_size() if dist.is_initialized() else 1)
        self.params = [p for p in module.parameters() if p.requires_grad]
        self.index = {id(p): i for i, p in enumerate(self.params)}
        self.module = module
        self.bucket_bytes = bucket_bytes
        self.rebuilt = False
        self._fired = []
        self._set_buckets(list(reversed(self.params)))
        self.active = False
        self._handles = []
        if self.world > 1:
            for p in self.params:
                self._handles.append(p.register_post_accumulate_grad_hook(self._hook))

    def _set_buckets(self, order):
        self.buckets = []
        cur, size = [], 0
        for p in order:
            cur.append(p)
            size += p.numel() * 4
            if size >= self.bucket_bytes:
                self.buckets.append(cur)
                cur, size = [], 0
        if cur:
            self.buckets.append(cur)
        self.slot = {}
        for bi, b in enumerate(self.buckets):
            for p in b:
                self.slot[id(p)] = bi

    def _rebuild(self):
        """Buckets from the recorded hook order, rank 0's copy broadcast (a collective every rank issues once, after
        the first step's reductions)."""
        n = len(self.params)
        rec = torch.full((n + 1,), -1, dtype=torch.int64)
        rec[0] = len(self._fired)
        rec[1:1 + len(self._fired)] = torch.tensor(self._fired, dtype=torch.int64)
        if dist.is_available() and dist.is_initialized():
            dev = self.params[0].device if self.params and dist.get_backend() == "nccl" else torch.device("cpu")
            t = rec.to(dev)
            dist.broadcast(t, 0)
            rec = t.cpu()
        k = int(rec[0])
        self._set_buckets([self.params[i] for i in rec[1:1 + k].tolist()])
        self.rebuilt = True

    def remove(self):
        for h in self._handles:
            h.remove()
        self._handles = []

    def start(self):
        """Arm the hooks for one backward.  A parameter the module no longer holds (re-created since the reducer
        was built) counts as ready, so its bucket does not wait for it."""
        current = {id(p) for p in self.module.parameters()}
        self.live = [[p for p in b if id(p) in current] for b in self.buckets]
        self.ready = [len(b) - len(lv) for b, lv in zip(self.buckets, self.live)]
        self.flat = [None] * len(self.buckets)
        self.work = [None] * len(self.buckets)
        self.next_launch = 0
        self.active = self.world > 1
        if self.active:
            self._advance()

    def _advance(self):
        while self.next_launch < len(self.buckets) and self.ready[self.next_launch] == len(self.buckets[self.next_launch]):
            self._launch(self.next_launch)
            self.next_launch += 1

    def _hook(self, p):
        if not self.active:
            return
        if not self.rebuilt:
            i = self.index.get(id(p))
            if i is not None:
                self._fired.append(i)
        bi = self.slot.get(id(p))
        if bi is None:
            return
        self.ready[bi] += 1
        self._advance()

    def _launch(self, bi):
        b = self.live[bi]
        if not b:
            return
        flat = torch.cat([p.grad.reshape(-1).to(torch.float32) for p in b])
        self.flat[bi] = flat
        self.work[bi] = dist.all_reduce(flat, op=dist.ReduceOp.SUM, async_op=True)

    def finish(self):
        """-> number of collectives issued (bucketed + leftover)."""
        if not self.active:
            return 0
        self.active = False
        n = 0
        for bi, b in enumerate(self.live):
            if self.work[bi] is None:
                continue
            self.work[bi].wait()
            flat = self.flat[bi].div_(self.world)
            off = 0
            for p in b:
                k = p.numel()
                p.grad.copy_(flat[off:off + k].view_as(p.grad))
                off += k
            n += 1
        done = {id(p) for bi, b in enumerate(self.live) if self.work[bi] is not None for p in b}
        rest = [p for p in self.module.parameters() if p.grad is not None and id(p) not in done]
        n += allreduce_gradients(rest, self.world)
        if not self.rebuilt:
            self._rebuild()
        self.flat = [None] * len(self.buckets)
        self.work = [None] * len(self.buckets)
        return n
