"""Multi-process (world_size 2, gloo on CPU) checks of the row-band sharding and the frame gather
used by bench.py on N GPUs (aonerf/parallel.py).  The GPU render is replaced by a payload that
encodes the pixel index, so the test checks exactly the partition + gather + re-assembly."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from aonerf.parallel import assemble, band, gather_frame


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def fake_payload(H, W, rank, world):
    p0, n, n_max = band(H, W, rank, world)
    out = torch.zeros((n_max, 5))
    pix = torch.arange(p0, p0 + n, dtype=torch.float32)
    out[:n, 0] = pix
    out[:n, 1] = pix // W
    out[:n, 2] = pix % W
    out[:n, 3] = rank
    out[:n, 4] = 1.0
    return out


def _worker(rank, world, port, H, W, q):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        frame = gather_frame(fake_payload(H, W, rank, world), H, W, dst=0)
        if rank == 0:
            # numpy: pickled by value (a torch CPU tensor crosses the queue as a shared-memory
            # handle that dies with this process if the parent has not mapped it yet)
            q.put(frame.numpy())
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("H,W", [(480, 640), (7, 5), (3, 4)])
def test_band_partition_covers_frame(H, W):
    for world in (1, 2, 3, 4, 8):
        covered = []
        for r in range(world):
            p0, n, n_max = band(H, W, r, world)
            assert 0 <= n <= n_max and p0 % W == 0
            covered.extend(range(p0, p0 + n))
        assert covered == list(range(H * W))


def test_assemble_single_process():
    H, W, world = 9, 4, 4
    parts = [fake_payload(H, W, r, world) for r in range(world)]
    frame = assemble(parts, H, W)
    assert torch.equal(frame[:, 0], torch.arange(H * W, dtype=torch.float32))


@pytest.mark.parametrize("H,W", [(48, 64), (7, 5)])
def test_gather_frame_gloo_world2(H, W):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, H, W, q)) for r in range(world)]
    for p in procs:
        p.start()
    frame = torch.from_numpy(q.get(timeout=120))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert frame.shape == (H * W, 5)
    assert torch.equal(frame[:, 0], torch.arange(H * W, dtype=torch.float32))
    assert torch.equal(frame[:, 1] * W + frame[:, 2], frame[:, 0])
    assert torch.all(frame[:, 4] == 1.0)
    # rank r rendered rows [r * ceil(H/2), ...)
    rows = -(-H // world)
    assert torch.equal(frame[:, 3], (frame[:, 1] // rows).float())


def _ddp_worker(rank, world, port, q):
    from aonerf.parallel import GradAllReduce

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        ps = [torch.zeros(s, requires_grad=True) for s in ((4, 3), (5,), (1,))]
        for i, p in enumerate(ps):
            p.grad = torch.full(p.shape, float(rank + 1) * (i + 1))
        GradAllReduce(ps)()
        q.put((rank, [p.grad.numpy().copy() for p in ps]))  # by value (see _worker)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_grad_allreduce_gloo_world2():
    """Training DDP step: the flat-bucket all-reduce averages every parameter's gradient."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ddp_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for _, grads in got:
        for i, gr in enumerate(grads):
            gr = torch.from_numpy(gr)
            assert torch.equal(gr, torch.full(gr.shape, 1.5 * (i + 1)))


def _ddp_bucket_worker(rank, world, port, q):
    """Two 'levels' (fine built last, so autograd runs its backward first) and a code shared by
    both: buckets [fine, coarse + shared] launch the fine all-reduce from the gradient hooks
    before __call__, and average exactly as one bucket does; a second backward before __call__
    (its gradients would land in a bucket already in flight) raises."""
    from aonerf.parallel import GradAllReduce

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(7)  # same weights on both ranks, different inputs
        coarse = torch.nn.Linear(6, 4)
        fine = torch.nn.Linear(6, 4)
        shared = torch.nn.Parameter(torch.randn(4, generator=g))
        for m in (coarse, fine):
            for t in m.parameters():
                t.data.copy_(torch.randn(t.shape, generator=g))
        x = torch.randn(5, 6, generator=torch.Generator().manual_seed(100 + rank))

        def backward():
            for t in [*coarse.parameters(), *fine.parameters(), shared]:
                t.grad = None
            yc = coarse(x) * shared
            yf = fine(x) * shared  # created last: its backward runs first
            ((yc ** 2).sum() + (yf ** 3).sum()).backward()

        params = [*coarse.parameters(), *fine.parameters(), shared]
        one = GradAllReduce(params)
        backward()
        one()
        ref = [t.grad.clone() for t in params]
        two = GradAllReduce(params, buckets=[list(fine.parameters()),
                                             [*coarse.parameters(), shared]])
        backward()
        early = two._works[0] is not None and two._works[1] is None and two.calls == 1
        two()
        same = all(torch.equal(t.grad, r) for t, r in zip(params, ref))
        two.close()  # its hooks go with it
        assert two._hooks == [] and two.calls == 2
        # a sync re-created per epoch while the old one is merely dropped: the dropped object's
        # (weakly referenced) hooks never fire, so the new one's first bucket is not disturbed
        with GradAllReduce(params, buckets=[list(fine.parameters()),
                                            [*coarse.parameters(), shared]]) as three:
            backward()
            three()
        del three
        import gc

        gc.collect()
        four = GradAllReduce(params, buckets=[list(fine.parameters()),
                                              [*coarse.parameters(), shared]])
        backward()
        four()
        recreated = (four.calls == 2
                     and all(torch.equal(t.grad, r) for t, r in zip(params, ref)))
        four.close()
        bad = GradAllReduce(params, buckets=[list(fine.parameters()), [*coarse.parameters(), shared]])
        backward()
        try:
            backward()  # gradient accumulation without the all-reduce in between
            raised = False
        except RuntimeError as e:
            raised = "already in flight" in str(e)
        bad.close()  # drains the bucket still in flight
        q.put((rank, early, same and recreated, two.calls, raised))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_grad_allreduce_buckets_overlap_gloo_world2():
    """GradAllReduce buckets: the first bucket's all-reduce is issued from the gradient hooks
    (before __call__, i.e. overlapping the rest of the backward); results bit-equal to the one
    bucket; a parameter accumulating after its bucket launched is refused."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ddp_bucket_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for rank, early, same, calls, raised in got:
        assert early, rank
        assert same, rank
        assert calls == 2 and raised, rank


def _ddp_bf16_worker(rank, world, port, q):
    from aonerf.parallel import GradAllReduce

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(rank)
        ps = [torch.zeros(s, requires_grad=True) for s in ((64, 3), (257,), (1,))]
        for p in ps:
            p.grad = torch.randn(p.shape, generator=g) * 10.0 ** torch.randint(-6, 2, p.shape, generator=g)
        sent = [p.grad.clone() for p in ps]
        GradAllReduce(ps, dtype=torch.bfloat16)()
        q.put((rank, [x.numpy() for x in sent], [p.grad.numpy().copy() for p in ps]))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_grad_allreduce_bf16_gloo_world2():
    """The bf16 bucket (half the bytes): every rank holds (bf16(g0) + bf16(g1))
    rounded to bf16, / 2, exactly -- i.e. within the bf16 rounding bound (3 roundings of 2^-9
    relative to the summed magnitudes) of the fp32 average."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ddp_bf16_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {r: (s, a) for r, s, a in (q.get(timeout=120) for _ in range(world))}
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for i in range(3):
        g0, g1 = (torch.from_numpy(got[r][0][i]) for r in range(world))
        want = (g0.bfloat16().float() + g1.bfloat16().float()).bfloat16().float() / 2
        mag = (g0.abs() + g1.abs()) / 2
        for r in range(world):
            avg = torch.from_numpy(got[r][1][i])
            assert torch.equal(avg, want), i
            assert torch.all((avg - (g0 + g1) / 2).abs() <= 3 * 2.0 ** -9 * mag + 1e-30)
