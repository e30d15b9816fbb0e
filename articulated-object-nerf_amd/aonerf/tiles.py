"""The 16-row tiled layout of the tensors the fused training kernels keep for the backward
(include/aonerf.h, "Kept tensors"; csrc/mlp_f16x3_core.hpp act_base): for N rows of width W,
element (row, f) at (row // 16) * 16 W + 256 (f // 16) + 16 (row % 16) + f % 16, i.e.
contiguous row-major 16 x 16 tiles (one MFMA output fragment each), so the kernels' epilogue
stores are contiguous.  Buffers hold rows(N) = N rounded up to 16.  These helpers convert for
the layer-by-layer path (row-major) and for inspection in tests."""
import torch


def rows(n):
    """Rows a tiled buffer of n logical rows holds."""
    return (n + 15) // 16 * 16


def untile(x, n):
    """Row-major (n, W) copy of a tiled (rows(n), W) tensor ([block][tile][row][col] storage)."""
    W = x.shape[-1]
    return x.reshape(-1, W // 16, 16, 16).permute(0, 2, 1, 3).reshape(-1, W)[:n].contiguous()


def tile(x):
    """Tiled (rows(n), W) copy of a row-major (n, W) tensor (padding rows zero)."""
    n, W = x.shape
    pad = torch.zeros((rows(n), W), dtype=x.dtype, device=x.device)
    pad[:n] = x
    return pad.reshape(-1, 16, W // 16, 16).permute(0, 2, 1, 3).reshape(-1, W).contiguous()


def untile_masks(m, n):
    """Row-major (n, 8) int32 view order of tiled ReLU' words (rows(n), 8): word (row, g) at
    (row // 16) * 64 + 16 g + row % 16."""
    return m.reshape(-1, 4, 16, 2).permute(0, 2, 1, 3).reshape(-1, 8)[:n].contiguous()
