"""Multi-GPU frame rendering: image-row bands across ranks + one gather (RCCL over xGMI).

One process per GPU (torch.distributed, backend "nccl" = RCCL on ROCm).  Rays are
independent and the reference has no early termination, so equal row bands balance exactly;
the only exchange is the final gather of [rgb, depth, acc] (20 B/ray) to the destination rank
-- at 640x480 over 8 GPUs 768 KB per rank.
"""
import weakref

import torch
import torch.distributed as dist


def band(H, W, rank, world):
    """Pixel range [p0, p0 + n) of rank's row band; bands have ceil(H/world) rows (the last may
    be short or empty).  Returns (p0, n, n_max) with n_max the padded per-rank payload."""
    rows = -(-H // world)
    r0 = min(rank * rows, H)
    r1 = min(r0 + rows, H)
    return r0 * W, (r1 - r0) * W, rows * W


def assemble(parts, H, W):
    """Concatenate per-rank padded payloads (world, n_max, C) into the (H*W, C) frame."""
    world = len(parts)
    out = []
    for rank, part in enumerate(parts):
        _, n, _ = band(H, W, rank, world)
        out.append(part[:n])
    return torch.cat(out, 0)


def gather_frame(local, H, W, dst=0, group=None):
    """Gather every rank's band payload (n_max, C) to `dst` -> (H*W, C) there, None elsewhere."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = local.device
    if local.is_cuda and dist.get_backend(group) == "gloo":
        local = local.cpu()  # gloo is a host transport (CPU-only gather); RCCL gathers in HBM
    parts = [torch.empty_like(local) for _ in range(world)] if rank == dst else None
    dist.gather(local, parts, dst=dst, group=group)
    return assemble(parts, H, W).to(dev) if rank == dst else None


def render_frame_sharded(model, c2w, H, W, focal, near=2.0, far=6.0, white_bkgd=True, dst=0,
                         group=None, gather=True, timers=None):
    """Render this rank's band of the frame and gather the frame to `dst`.

    Returns (frame or None, local payload).  frame: (H*W, 5) = [rgb(3), depth, acc].
    """
    from .render import render_frame

    ddp = dist.is_initialized()
    world = dist.get_world_size(group) if ddp else 1
    rank = dist.get_rank(group) if ddp else 0
    p0, n, n_max = band(H, W, rank, world)
    local = torch.zeros((n_max, 5), device=torch.device("cuda", torch.cuda.current_device()))
    if n > 0:
        local[:n] = render_frame(model, c2w, H, W, focal, near, far, white_bkgd, p0, n, timers=timers)
    if not ddp or not gather:  # (a process group of one still runs the gather)
        return (local[:n] if world == 1 else None), local
    return gather_frame(local, H, W, dst, group), local


# ---------------------------------------------------------------------------- training (DDP)
class GradAllReduce:
    """Data-parallel gradient averaging for the training step (run.py:109/151 trains with
    Lightning DDP: every rank draws its own ray batch, gradients are averaged).

    The gradients are packed into ONE flat buffer (vanilla NeRF: 1,191,688 values = 4.77 MB in
    fp32) and averaged by all-reduce (RCCL over xGMI), then unpacked into each ``.grad``.

    ``buckets`` (optional): a partition of ``params`` into groups, in the order their gradients
    complete in the backward -- e.g. ``[fine_mlp params, coarse_mlp params]``: autograd runs the
    fine level's backward first (its node was created last), so the fine bucket's all-reduce is
    issued from a post-accumulate-grad hook as soon as its last gradient lands and runs on RCCL's
    stream while the coarse level's backward runs; the LAST bucket is always reduced in
    ``__call__``.  Autograd sums a parameter's contributions from several uses (latent codes
    both levels read) before its gradient lands, once per backward, so such a parameter simply
    completes its bucket late; a gradient landing again in a bucket already in flight (a second
    backward before ``__call__``: gradient accumulation) raises.
    One bucket (the default) is one collective at ``__call__``: at 2-5 MB the ring is latency-,
    not link-bound, so more buckets only pay where they overlap compute.

    ``dtype=torch.bfloat16`` (for C5's bf16 mode) halves the bytes (2.38 MB):
    each rank's gradients are rounded to bf16, summed by the collective in bf16 (RCCL's ring
    rounds every partial sum to bf16: world - 1 roundings), then widened to fp32 and divided by
    the world size.  Relative error per value <= ~world x 2^-8 of the largest magnitude summed
    into it; the fp32 master weights and Adam state are unchanged.  On a gloo group a device
    buffer is staged through the host (no early launch there).

    The early-launch hooks belong to this object: ``close()`` (or leaving a ``with`` block, or
    garbage collection) removes them, and a hook only holds a weak reference, so a second
    GradAllReduce over the same parameters (one per epoch or per bench leg) never sees the first
    one's hooks fire.
    """

    def __init__(self, params, group=None, dtype=torch.float32, buckets=None):
        if dtype not in (torch.float32, torch.bfloat16):
            raise ValueError("GradAllReduce: dtype must be torch.float32 or torch.bfloat16")
        self.params = [p for p in params if p.requires_grad]
        if buckets is None:
            buckets = [self.params]
        buckets = [[p for p in b if p.requires_grad] for b in buckets]
        order = [p for b in buckets for p in b]
        if sorted(map(id, order)) != sorted(map(id, self.params)):
            raise ValueError("GradAllReduce: buckets must partition the parameters")
        self.params = order  # bucket order: each bucket one contiguous slice of the buffer
        self.group = group
        self.dtype = dtype
        self.sizes = [p.numel() for p in self.params]
        spans, off = [], 0
        for b in buckets:
            n = sum(p.numel() for p in b)
            spans.append((off, off + n, len(b)))
            off += n
        self.spans = spans  # (start, end, parameter count) per bucket
        self.bucket_of = {}
        k = 0
        for bi, b in enumerate(buckets):
            for p in b:
                self.bucket_of[id(p)] = (bi, k)
                k += 1
        self.flat = None
        self.flat32 = None
        self.calls = 0  # collectives issued (bench.py records them with the DDP step)
        self._seen = [set() for _ in buckets]
        self._works = [None] * len(buckets)
        self._hooks = []
        self._closed = False
        if len(buckets) > 1:
            ref = weakref.ref(self)

            def hook(p):
                me = ref()
                if me is not None and not me._closed:
                    me._landed(p)

            for p in self.params:
                self._hooks.append(p.register_post_accumulate_grad_hook(hook))

    def close(self):
        """Remove the gradient hooks and drain a collective still in flight (idempotent)."""
        for h in self._hooks:
            h.remove()
        self._hooks = []
        if not self._closed:
            for w in self._works:
                if w is not None and w is not True:
                    w.wait()
        self._closed = True
        self._works = [None] * len(self.spans)
        self._seen = [set() for _ in self.spans]

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

    def __del__(self):
        try:
            for h in self._hooks:
                h.remove()
        except Exception:  # noqa: BLE001 (interpreter shutdown)
            pass

    def _ensure(self, dev):
        if self.flat is None or self.flat.device != dev:
            n = sum(self.sizes)
            self.flat = torch.empty(n, dtype=self.dtype, device=dev)
            self.flat32 = self.flat if self.dtype == torch.float32 else torch.empty(n, device=dev)

    def _staged(self):
        return self.flat.is_cuda and dist.get_backend(self.group) == "gloo"

    def _landed(self, p):
        # post-accumulate-grad hook: launch a bucket (not the last) once all its gradients landed
        if not dist.is_initialized():
            return
        bi, _ = self.bucket_of[id(p)]
        if self._works[bi] is not None:
            raise RuntimeError("GradAllReduce: a gradient landed in a bucket already in flight "
                               "(a second backward before the all-reduce; call it per backward)")
        self._seen[bi].add(id(p))
        if bi < len(self.spans) - 1 and len(self._seen[bi]) == self.spans[bi][2]:
            self._ensure(p.device)
            if not self._staged():
                self._launch(bi)

    def _launch(self, bi):
        a, b, _ = self.spans[bi]
        if a == b:  # an empty bucket: nothing to reduce
            self._works[bi] = True
            return
        off = a
        for p, n in zip(self.params, self.sizes):
            if self.bucket_of[id(p)][0] != bi:
                continue
            if p.grad is None:
                raise RuntimeError("GradAllReduce: a parameter has no gradient")
            self.flat[off:off + n].copy_(p.grad.reshape(-1))  # (rounds to bf16 in that mode)
            off += n
        self.calls += 1
        seg = self.flat[a:b]
        if self._staged():
            host = seg.cpu()
            dist.all_reduce(host, op=dist.ReduceOp.SUM, group=self.group)
            seg.copy_(host)
            self._works[bi] = True
        else:
            self._works[bi] = dist.all_reduce(seg, op=dist.ReduceOp.SUM, group=self.group,
                                              async_op=True)

    def __call__(self):
        if self._closed:
            raise RuntimeError("GradAllReduce: closed")
        if not dist.is_initialized():  # (a process group of one still runs the all-reduce)
            return
        world = dist.get_world_size(self.group)
        self._ensure(self.params[0].device)
        for bi in range(len(self.spans)):
            if self._works[bi] is None:
                self._launch(bi)
        for w in self._works:
            if w is not True:
                w.wait()  # (RCCL: the current stream waits for the collective's)
        self._works = [None] * len(self.spans)
        self._seen = [set() for _ in self.spans]
        if self.flat32 is not self.flat:
            self.flat32.copy_(self.flat)
        self.flat32.div_(world)
        off = 0
        for p, n in zip(self.params, self.sizes):
            p.grad.copy_(self.flat32[off:off + n].view_as(p.grad))
            off += n
