"""Host logic of the fp16x3 range guard's bookkeeping (aonerf._lib register_pack /
check_pending, aonerf.train's global optimizer step pre-hook), on CPU stand-in buffers whose
last 16 bytes play the packed stream's status block (include/aonerf.h aon_mlp_read_status).
No kernel runs: the status words are set by hand."""
import pytest
import torch


def _buf(status=0):
    b = torch.zeros(64, dtype=torch.float32)
    b.view(torch.int32)[-4] = status
    return b


@pytest.fixture
def L():
    from aonerf import _lib

    for d in (_lib.PENDING_PACKS, _lib._STICKY, _lib.PACK_PARAMS, _lib.SNAPSHOTS):
        d.clear()
    yield _lib
    for d in (_lib.PENDING_PACKS, _lib._STICKY, _lib.PACK_PARAMS, _lib.SNAPSHOTS):
        d.clear()


class _Event:
    def __init__(self):
        self.waited = False

    def synchronize(self):
        self.waited = True


def test_snapshot_read_from_host(L):
    """A pack with a snapshot (snapshot_pack: the status word copied to host memory after its
    last reader) is judged by the host copy once the snapshot's event has passed -- the device
    word is not read (no device sync) -- and a re-pack drops the snapshot (the old status then
    reaches the check through the sticky device word)."""
    b = _buf(0)
    L.register_pack(("train", "fwd65"), b)
    ev = _Event()
    L.SNAPSHOTS[("train", "fwd65", "cpu")] = (torch.tensor([1], dtype=torch.int32), ev)
    assert L.check_pending({"cpu"}) is True and ev.waited
    assert not L.SNAPSHOTS and not L.PENDING_PACKS
    # a clean snapshot: False, though the (stand-in) device word says otherwise -- it is not read
    L.register_pack(("train", "fwd65"), _buf(1))
    L.SNAPSHOTS[("train", "fwd65", "cpu")] = (torch.tensor([0], dtype=torch.int32), _Event())
    assert L.check_pending({"cpu"}) is False
    # re-pack of a pending pack: its snapshot is dropped, its device word goes sticky
    L.register_pack(("train", "fwd65"), _buf(1))
    L.SNAPSHOTS[("train", "fwd65", "cpu")] = (torch.tensor([0], dtype=torch.int32), _Event())
    L.register_pack(("train", "fwd65"), _buf(0))
    assert not L.SNAPSHOTS
    assert L.check_pending({"cpu"}) is True


def test_pending_consumed_once(L):
    L.register_pack(("train", "fwd65"), _buf(1))
    assert L.check_pending({"cpu"}) is True
    assert L.check_pending({"cpu"}) is False  # consumed
    L.register_pack(("train", "fwd65"), _buf(0))
    assert L.check_pending(None) is False


def test_repack_keeps_status_sticky(L):
    b = _buf(1)
    L.register_pack(("train", "fwd65"), b)
    L.register_pack(("train", "fwd65"), b)  # called before the re-pack: the 1 is kept
    b.view(torch.int32)[-4] = 0          # what the re-pack then does to the status word
    assert any(sk[0] == "cpu" for sk in L._STICKY)
    assert L.check_pending({"cpu"}) is True
    assert not L._STICKY and not L.PENDING_PACKS


def test_other_device_untouched(L):
    L.register_pack(("train", "fwd65"), _buf(1))
    assert L.check_pending({"cuda:0"}) is False
    assert L.PENDING_PACKS  # still pending for its own device


def test_torch_optimizer_hook_refuses(L):
    from aonerf import train

    p = torch.nn.Parameter(torch.ones(3))
    p.grad = torch.ones(3)
    opt = torch.optim.SGD([p], lr=0.1)
    L.register_pack(("train", "fwd65"), _buf(1))
    with pytest.raises(FloatingPointError):
        opt.step()
    assert torch.equal(p.detach(), torch.ones(3))
    opt.step()  # consumed: the next step goes through
    assert torch.allclose(p.detach(), torch.full((3,), 0.9))


def test_hook_limited_to_packed_parameters(L):
    """an optimizer over parameters no pending pack was packed from neither raises
    nor consumes the overflow; the model's own optimizer then still refuses its step."""
    from aonerf import train  # noqa: F401  (installs the hook)

    mine = torch.nn.Parameter(torch.ones(3))
    other = torch.nn.Parameter(torch.ones(3))
    for p in (mine, other):
        p.grad = torch.ones(3)
    L.register_pack(("train", "fwd65"), _buf(1), [mine])
    torch.optim.SGD([other], lr=0.1).step()  # unrelated model: goes through
    assert torch.allclose(other.detach(), torch.full((3,), 0.9))
    assert L.PENDING_PACKS  # not consumed
    with pytest.raises(FloatingPointError):
        torch.optim.SGD([mine], lr=0.1).step()
    assert torch.equal(mine.detach(), torch.ones(3))


def test_sticky_keeps_its_parameters(L):
    from aonerf import train  # noqa: F401

    mine = torch.nn.Parameter(torch.ones(3))
    other = torch.nn.Parameter(torch.ones(3))
    for p in (mine, other):
        p.grad = torch.ones(3)
    b = _buf(1)
    L.register_pack(("train", "fwd65"), b, [mine])
    L.register_pack(("train", "fwd65"), b, [mine])  # re-pack: the 1 goes to the sticky word
    b.view(torch.int32)[-4] = 0
    torch.optim.SGD([other], lr=0.1).step()
    assert L._STICKY
    with pytest.raises(FloatingPointError):
        torch.optim.SGD([mine], lr=0.1).step()
    assert not L._STICKY and not L.PENDING_PACKS


def test_two_models_repack_before_either_steps(L):
    """model A (no overflow) and model B (overflow) each re-pack before either steps.
    Their status goes to separate sticky words (per parameter set): A's optimizer steps, B's
    refuses -- a shared per-device word would have made A refuse and B go through."""
    from aonerf import train  # noqa: F401

    a = torch.nn.Parameter(torch.ones(3))
    b = torch.nn.Parameter(torch.ones(3))
    for p in (a, b):
        p.grad = torch.ones(3)
    ba, bb = _buf(0), _buf(1)
    L.register_pack(("train", "fwdA"), ba, [a])
    L.register_pack(("train", "fwdA"), ba, [a])   # re-pack: A's 0 goes sticky
    L.register_pack(("train", "fwdB"), bb, [b])
    L.register_pack(("train", "fwdB"), bb, [b])   # re-pack: B's 1 goes sticky
    bb.view(torch.int32)[-4] = 0                  # what B's re-pack does to its word
    assert len(L._STICKY) == 2
    torch.optim.SGD([a], lr=0.1).step()           # A: no overflow of its own
    assert torch.allclose(a.detach(), torch.full((3,), 0.9))
    with pytest.raises(FloatingPointError):
        torch.optim.SGD([b], lr=0.1).step()
    assert torch.equal(b.detach(), torch.ones(3))
