"""One process per GPU, started by the benchmark itself (run.py:101-111: the reference's
launcher takes ``devices=hparams.num_gpus`` and Lightning's DDPPlugin spawns that many ranks).

``spawn_ranks`` re-runs the calling script N times as fresh child processes with RANK /
LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set, waits for them and returns the worst
exit status.  It must run BEFORE anything touches the GPU: the parent only parses arguments
(and a child is started with ``subprocess``, never ``exec``, so no GPU-initialised process is
replaced).  If one rank fails, the others are terminated rather than left waiting in a
collective.  Under an external ``torchrun`` (WORLD_SIZE already set) nothing is spawned.

``init_rank`` is the child side: device selection and the process group.  Backend ``nccl``
(RCCL over xGMI) needs one device per local rank; ``gloo`` lets several ranks share one device
(the one-GPU test box rehearses the N-rank path that way -- RCCL refuses two ranks on one
device).
"""
import os
import socket
import subprocess
import sys
import time


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launched_externally():
    return "WORLD_SIZE" in os.environ


def spawn_ranks(script, argv, world, env_extra=None, poll_s=0.2):
    """Run ``python script *argv`` as `world` ranks on this node; return the max exit status
    (the first failing rank's status if any rank fails)."""
    port = str(_free_port())
    procs = []
    for r in range(world):
        env = dict(os.environ)
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(world),
                    "LOCAL_WORLD_SIZE": str(world), "GROUP_RANK": "0",
                    "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": port})
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if env_extra:
            env.update(env_extra)
        procs.append(subprocess.Popen([sys.executable, script] + list(argv), env=env))
    failed = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad and not failed:
                failed = bad[0]
                for p in procs:  # a dead rank leaves the others blocked in a collective
                    if p.poll() is None:
                        p.terminate()
            if all(c is not None for c in codes):
                break
            time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return failed or max(p.returncode for p in procs)


def init_rank(backend, expect_world=None):
    """Child side: (world, rank, local_rank, device).  Sets the device and, for world > 1,
    initialises the process group; asserts the world size matches ``expect_world``."""
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if expect_world is not None and world != expect_world:
        raise RuntimeError(f"--gpus {expect_world} but the launcher started {world} ranks")
    ndev = torch.cuda.device_count()
    if backend == "nccl":
        if local_rank >= ndev:
            raise RuntimeError(f"backend nccl needs one GPU per rank: local rank {local_rank}, "
                               f"{ndev} visible device(s) (use --backend gloo to share one)")
        dev_index = local_rank
    else:
        dev_index = local_rank % max(ndev, 1)
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
        got = dist.get_world_size()
        if got != world:
            raise RuntimeError(f"process group has {got} ranks, expected {world}")
    return world, rank, local_rank, dev


def max_over_ranks(x):
    """max of a host float over the ranks (a CPU tensor: gloo and RCCL both reduce it; RCCL
    needs a device tensor, so it goes through the current device there)."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(x)
    on_dev = dist.get_backend() == "nccl"
    t = torch.tensor([float(x)], dtype=torch.float64,
                     device=torch.device("cuda", torch.cuda.current_device()) if on_dev else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
