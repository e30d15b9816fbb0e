"""CPU check of the summation-order model the HIP kernels use to round like the reference's
torch CPU sums (csrc/torch_sum.hpp): the wave-parallel decomposition (`wave_row_sums`: <=16-term
left folds on separate lanes, then a per-sum combine) is restated here in numpy float32 and
compared bit-for-bit with torch.sum on the shapes the reference reduces (helper.py:176-181,
:207): a contiguous last-dim sum and the stride-3 (B,S,3) -> (B,3) sum."""
import numpy as np
import pytest
import torch

f32 = np.float32


def fold(vals):
    acc = f32(0.0)
    for v in vals:
        acc = f32(acc + v)
    return acc


def wave_row_sum(x, n):
    """wave_row_sums for one spec: chunk folds C[c][k], leftovers L[k], combine."""
    sil = n >> 2
    nch = sil >> 4
    C = [[fold(x[4 * (16 * c + s) + k] for s in range(16)) for k in range(4)] for c in range(nch)]
    L = [fold(x[4 * i + k] for i in range(16 * nch, sil)) for k in range(4)]
    p = []
    for k in range(4):
        a1 = fold(C[c][k] for c in range(nch))
        p.append(f32(f32(f32(L[k] + a1) + f32(0)) + f32(0)))
    for e in range(4 * sil, n):
        p[0] = f32(p[0] + x[e])
    return f32(f32(f32(p[0] + p[1]) + p[2]) + p[3])


def inner_sum(x):
    n = len(x)
    if n < 8:
        return wave_row_sum(x, n)
    m = n // 8
    s = fold(x[8 * m:])
    for c in range(8):
        s = f32(s + wave_row_sum(x[c::8][:m], m))
    return s


LENGTHS = list(range(1, 70)) + [96, 127, 128, 129, 191, 192, 193, 255, 256, 257, 383, 448, 511, 512, 513, 777, 1000, 1023]


@pytest.mark.parametrize("n", LENGTHS)
def test_inner_sum_matches_torch(n):
    rng = np.random.default_rng(n)
    for scale in (1.0, 1e-3):
        x = (rng.random(n, dtype=np.float32) * scale).astype(np.float32)
        want = torch.from_numpy(x[None]).sum(-1).numpy()[0]
        assert inner_sum(x) == want


@pytest.mark.parametrize("n", LENGTHS)
def test_strided_rgb_sum_matches_torch(n):
    rng = np.random.default_rng(1000 + n)
    x = rng.random((1, n, 3), dtype=np.float32)
    want = torch.from_numpy(x).sum(-2).numpy()[0]
    got = [wave_row_sum(x[0, :, ch], n) for ch in range(3)]
    assert np.array_equal(np.array(got, np.float32), want)
