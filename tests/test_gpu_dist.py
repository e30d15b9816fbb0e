"""The multi-GPU paths with the real HIP kernels: two processes on the one GPU of the test box
(gloo process group; on a node, bench.py / tools/bench_train.py run one process per GPU over
RCCL with the same code).  (1) The row-band frame render + gather (aonerf.parallel,
BASELINE config C4) equals the single-process render bit for bit.  (2) A DDP training step
(tools/bench_train.py): after GradAllReduce every rank holds the average of the two ranks'
gradients, bit for bit as computed from each batch alone.  (3) The RCCL branch itself (backend
"nccl", a process group of one on the box's GPU -- RCCL refuses two ranks on one device): the
640x480 frame (config C4's size) gathered device-resident and the flat-bucket gradient
all-reduce, both equal to the single-process results bit for bit.  (4) Config C4's own partition:
8 ranks (gloo, all on the box's one GPU) each render their 60-row band of the 640x480 frame
with the HIP kernels and gather_frame assembles it on rank 0, bit-equal to a single-process
render_frame.  (5) interface.test_epoch at world 2 returns the single-rank stats exactly."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

H, W = 24, 32


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _net(train_precision="f16x3"):
    from aonerf.model import NeRF
    from aonerf.synthetic import init_like_reference

    return init_like_reference(NeRF(train_precision=train_precision)).cuda()


def _batch(seed, n=96):
    from aonerf.ray_utils import frame_rays
    from aonerf.render import create_spheric_poses, sapien_focal

    rays = frame_rays(torch.as_tensor(create_spheric_poses(4.0)[3 + seed]), H, W, sapien_focal(H))
    g = torch.Generator().manual_seed(seed)
    idx = torch.randperm(H * W, generator=g)[:n].cuda()
    b = {k: v[idx].contiguous() for k, v in rays.items()}
    b["target"] = torch.rand(n, 3, generator=g).cuda()
    u = (torch.rand(n, 65, generator=g).cuda(), torch.rand(n, 128, generator=g).cuda())
    return b, u


def _grads(net, seed):
    from aonerf import train

    b, (uc, uf) = _batch(seed)
    for p in net.parameters():
        p.grad = None
    loss, _ = train.training_step(net, b, True, True, 2.0, 6.0, u_coarse=uc, u_fine=uf)
    loss.backward()
    return [p.grad.clone() for p in net.parameters()]


def _worker(rank, world, port, q):
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        from aonerf.parallel import GradAllReduce, render_frame_sharded
        from aonerf.render import create_spheric_poses, sapien_focal

        net = _net()
        frame, _ = render_frame_sharded(net, create_spheric_poses(4.0)[7], H, W, sapien_focal(H))
        grads = _grads(net, rank)
        GradAllReduce(net.parameters())()
        # numpy arrays: pickled by value (a tensor would travel as a shared-memory handle that
        # dies with this process)
        q.put((rank, frame.cpu().numpy() if frame is not None else None,
               [p.grad.cpu().numpy() for p in net.parameters()]))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_sharded_render_and_ddp_step_two_ranks():
    from aonerf.render import create_spheric_poses, render_frame, sapien_focal

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict((r, (f, g)) for r, f, g in (q.get(timeout=240) for _ in range(world)))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    # (1) frame: bands of 12 rows rendered by two processes == one process, bit for bit
    net = _net()
    ref = render_frame(net, create_spheric_poses(4.0)[7], H, W, sapien_focal(H)).cpu()
    assert got[0][0] is not None and got[1][0] is None
    np.testing.assert_array_equal(got[0][0], ref.numpy())
    # (2) DDP: every rank holds (g_rank0 + g_rank1) / 2 of the single-batch gradients
    g0, g1 = _grads(net, 0), _grads(net, 1)
    for r in range(world):
        for a, b, c in zip(got[r][1], g0, g1):
            np.testing.assert_array_equal(a, ((b + c) / 2).cpu().numpy())


def _worker_rccl(port, q):
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        from aonerf import parallel
        from aonerf.render import create_spheric_poses, sapien_focal

        assert dist.get_backend() == "nccl"
        staged = []
        real_gather = dist.gather

        def spy(t, *a, **k):  # the payload must reach RCCL in HBM, not staged through the host
            staged.append(t.device.type)
            return real_gather(t, *a, **k)

        dist.gather = spy
        try:
            net = _net()
            Hf, Wf = 480, 640
            frame, _ = parallel.render_frame_sharded(net, create_spheric_poses(4.0)[7], Hf, Wf,
                                                     sapien_focal(Hf))
        finally:
            dist.gather = real_gather
        assert staged == ["cuda"] and frame.is_cuda
        grads = _grads(net, 0)
        parallel.GradAllReduce(net.parameters())()
        torch.cuda.synchronize()
        q.put((frame.cpu().numpy(), [g.cpu().numpy() for g in grads],
               [p.grad.cpu().numpy() for p in net.parameters()]))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_rccl_gather_and_allreduce_world1():
    """C4's code path over RCCL: device-resident gather of a 640x480 frame and the DDP
    all-reduce on an nccl process group (world 1), bit-identical to one process without one."""
    from aonerf.render import create_spheric_poses, render_frame, sapien_focal

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker_rccl, args=(_free_port(), q))
    p.start()
    frame, g_before, g_after = q.get(timeout=240)
    p.join(timeout=120)
    assert p.exitcode == 0
    net = _net()
    ref = render_frame(net, create_spheric_poses(4.0)[7], 480, 640, sapien_focal(480)).cpu()
    np.testing.assert_array_equal(frame, ref.numpy())
    g_ref = _grads(net, 0)
    for a, b, c in zip(g_after, g_before, g_ref):
        np.testing.assert_array_equal(a, b)  # all-reduce over one rank / 1 is the identity
        np.testing.assert_array_equal(b, c.cpu().numpy())


def _worker_c4(rank, world, port, q):
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        from aonerf import parallel
        from aonerf.render import create_spheric_poses, sapien_focal

        net = _net()
        p0, n, n_max = parallel.band(480, 640, rank, world)
        frame, local = parallel.render_frame_sharded(net, create_spheric_poses(4.0)[7], 480, 640,
                                                     sapien_focal(480))
        q.put((rank, p0, n, n_max, local.shape[0],
               frame.cpu().numpy() if frame is not None else None))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _spawn(target, world, extra=()):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + tuple(extra)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        got = [q.get(timeout=300) for _ in range(world)]
    finally:
        for p in procs:
            p.join(timeout=120)
    for p in procs:
        assert p.exitcode == 0
    return got


def test_c4_eight_row_bands_full_frame():
    """BASELINE config C4's partition at its size: 8 ranks x 60 rows of the 640x480 frame
    (38,400 rays each), rendered with the HIP kernels and gathered to rank 0 (interface.py:31-51 /
    run.py:109-111 shard the test set across DDP ranks; here the frame's rows are the shards)."""
    from aonerf.render import create_spheric_poses, render_frame, sapien_focal

    world = 8
    got = {r[0]: r[1:] for r in _spawn(_worker_c4, world)}
    for rank in range(world):
        p0, n, n_max, n_local, frame = got[rank]
        assert (p0, n, n_max, n_local) == (rank * 60 * 640, 60 * 640, 60 * 640, 60 * 640)
        assert (frame is None) == (rank != 0)
    net = _net()
    ref = render_frame(net, create_spheric_poses(4.0)[7], 480, 640, sapien_focal(480)).cpu().numpy()
    assert got[0][4].shape == ref.shape == (480 * 640, 5)
    np.testing.assert_array_equal(got[0][4], ref)


def _mini_dataset():
    from aonerf.datasets import SapienDataset

    root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "data", "sapien_mini")
    split = "test" if os.path.isdir(os.path.join(root, "test")) else "val"
    return SapienDataset(root, split, img_wh=(32, 24), white_back=True)


def _epoch_net():
    from aonerf.model import NeRF
    from oracle import weights as W

    net = NeRF().cuda().requires_grad_(False)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in W.nerf_state_dict(0).items()})
    return net


def _worker_epoch(rank, world, port, q, out_dir):
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        from aonerf.interface import test_epoch

        stats = test_epoch(_epoch_net(), _mini_dataset(), out_dir=out_dir if rank == 0 else None)
        q.put((rank, stats))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_epoch_world2_equals_single_rank(tmp_path):
    """interface.test_epoch (LitNeRF test loop + test_epoch_end, model.py:459-507,
    interface.py:31-51) with its images rendered in row bands by 2 ranks and gathered: rank 0
    returns exactly the single-rank PSNR / object-PSNR stats and writes the same images."""
    from aonerf.interface import test_epoch

    got = dict(_spawn(_worker_epoch, 2, (str(tmp_path / "w2"),)))
    assert got[1] is None
    single = test_epoch(_epoch_net(), _mini_dataset(), out_dir=str(tmp_path / "w1"))
    assert got[0] == single, (got[0], single)
    names = sorted(os.listdir(tmp_path / "w1"))
    assert names == sorted(os.listdir(tmp_path / "w2")) and "results.json" in names
    for nm in names:
        assert open(tmp_path / "w1" / nm, "rb").read() == open(tmp_path / "w2" / nm, "rb").read(), nm


def test_bench_spawns_two_ranks_gloo(tmp_path):
    """bench.py --gpus 2 launches its own two ranks (aonerf.launch; verdict r03 #1) -- gloo, so
    both share the box's one GPU.  Exactly one JSON line, n_gpus 2; the gathered frame of the
    row-band render equals the single-process render bit for bit; every C5 record ran the
    gradient all-reduce in every step (the ranks draw different batches, so their parameters
    agree after Adam only if the gradients were averaged)."""
    import json
    import subprocess
    import sys

    from aonerf.render import create_spheric_poses, render_frame, sapien_focal

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    dump = tmp_path / "frame.npy"
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2",
                        "--backend", "gloo", "--steps", "2", "--warmup", "1",
                        "--no-cpu-baseline", "--dump-frame", str(dump)],
                       env=env, capture_output=True, text=True, timeout=600, cwd=root)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["backend"] == "gloo" and rec["steps"] == 2
    assert rec["config"]["parallelism"].startswith("row-band x2")
    frame = np.load(dump)
    net = _net()
    ref = render_frame(net, create_spheric_poses(4.0)[7], 480, 640, sapien_focal(480)).cpu().numpy()
    np.testing.assert_array_equal(frame, ref)
    for key in ("train_step", "train_step_bf16", "train_step_art", "train_step_art_bf16"):
        d = rec[key]["ddp"]
        assert rec[key]["n_gpus"] == 2 and d["world"] == 2 and d["backend"] == "gloo", key
        assert d["calls"] == 3 * d["buckets"] == 6, (key, d)  # warm-up + timed steps, 2 buckets
        assert d["params_identical_across_ranks"], (key, d)
        assert d["bucket_dtype"] == ("bf16" if key.endswith("bf16") else "fp32")


def _c5_batch(rank, n=4096):
    from aonerf.ray_utils import frame_rays
    from aonerf.render import create_spheric_poses, sapien_focal

    rays = frame_rays(torch.as_tensor(create_spheric_poses(4.0)[5 * rank + 1]), 480, 640,
                      sapien_focal(480))
    g = torch.Generator().manual_seed(100 + rank)
    idx = torch.randperm(480 * 640, generator=g)[:n].cuda()
    b = {k: v[idx].contiguous() for k, v in rays.items()}
    b["target"] = torch.rand(n, 3, generator=g).cuda()
    u = (torch.rand(n, 65, generator=g).cuda(), torch.rand(n, 128, generator=g).cuda())
    return b, u


def _c5_bf16_grads(net, rank):
    from aonerf import train

    b, (uc, uf) = _c5_batch(rank)
    assert net.train_numerics.precision == "bf16"
    for p in net.parameters():
        p.grad = None
    loss, _ = train.training_step(net, b, True, True, 2.0, 6.0, u_coarse=uc, u_fine=uf)
    loss.backward()
    return [p.grad.clone() for p in net.parameters()]


def _worker_c5_bf16(rank, world, port, q):
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        from aonerf.parallel import GradAllReduce

        net = _net("bf16")
        _c5_bf16_grads(net, rank)
        GradAllReduce(net.parameters(), dtype=torch.bfloat16)()
        q.put((rank, [p.grad.cpu().numpy() for p in net.parameters()]))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _worker_rccl_buckets(port, q):
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        from aonerf.parallel import GradAllReduce

        net = _net("bf16")
        ref = _c5_bf16_grads(net, 0)  # no collective
        fine = list(net.fine_mlp.parameters())
        coarse = list(net.coarse_mlp.parameters())
        sync = GradAllReduce(net.parameters(), dtype=torch.bfloat16, buckets=[fine, coarse])
        got = _c5_bf16_grads(net, 0)  # the hooks issue the fine bucket inside the backward
        early = sync._works[0] is not None and sync._works[1] is None and sync.calls == 1
        sync()
        sync.close()
        torch.cuda.synchronize()
        q.put((early, sync.calls, [g.cpu().numpy() for g in ref], [g.cpu().numpy() for g in got],
               [p.grad.cpu().numpy() for p in net.parameters()]))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_rccl_bucketed_allreduce_overlaps_backward_world1():
    """GradAllReduce's buckets on RCCL (world 1): C5's bf16 step with [fine, coarse] buckets --
    the fine MLP's all-reduce is issued from the gradient hooks on autograd's device thread,
    before the backward returns (it then runs beside the coarse level's backward), and the
    gradients come back as bf16(g) exactly (one rank: the sum is the value), the same as
    without buckets."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker_rccl_buckets, args=(_free_port(), q))
    p.start()
    early, calls, ref, got, after = q.get(timeout=240)
    p.join(timeout=120)
    assert p.exitcode == 0
    assert early and calls == 2
    for r, g, a in zip(ref, got, after):
        np.testing.assert_array_equal(g, r)  # the backward itself is unchanged by the hooks
        rb = torch.from_numpy(r).to(torch.bfloat16).float().numpy()
        np.testing.assert_array_equal(a, rb)


def test_c5_bf16_ddp_step_two_ranks():
    """Config C5's bf16 step at its size (4,096 rays per rank, 64c+128f, randomized) on two ranks
    through GradAllReduce's bf16 bucket (verdict r03 #6, run.py:151): every rank's gradient is
    exactly bf16(bf16(g0) + bf16(g1)) / 2 of the two single-rank gradients."""
    world = 2
    got = dict(_spawn(_worker_c5_bf16, world))
    net = _net("bf16")
    g0, g1 = _c5_bf16_grads(net, 0), _c5_bf16_grads(net, 1)
    for a, b in zip(g0, g1):
        assert not torch.equal(a, b)  # different batches: the average is not trivial
    for r in range(world):
        for a, b, c in zip(got[r], g0, g1):
            want = (b.bfloat16().float() + c.bfloat16().float()).bfloat16().float() / 2
            np.testing.assert_array_equal(a, want.cpu().numpy())
