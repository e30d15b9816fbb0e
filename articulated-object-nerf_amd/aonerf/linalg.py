"""Layer products on aon_gemm (the f16x3 MFMA GEMM, gemm_f16x3.hip) shared by the
layer-by-layer paths: the training forward/backward (train.py) and the articulated
NeRF_AE_Art MLP (model_autodecoder.py).  Operands are tensor views passed as pointers +
leading dimensions; workspace for split reductions is cached per device and stream."""
import contextlib
import ctypes

import torch

from . import _lib as L

# power-of-two operand prescales of the fp16 hi/lo split (exact): activations at 2^-8 (fp16
# range up to 1.6e7, as the fused forward), gradients at 2^10 (dL/d* of a mean loss are small;
# this keeps their hi parts out of fp16's subnormal range), weights unscaled.
ACT_SCALE, GRAD_SCALE, W_SCALE = 2.0 ** -8, 2.0 ** 10, 1.0

_ws = {}


def _workspace(nbytes, device):
    # one per device AND stream: products on two streams (TrainNumerics.overlap_dweight) run
    # concurrently
    key = (str(device), torch.cuda.current_stream(device).cuda_stream)
    buf = _ws.get(key)
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8, device=device)
        _ws[key] = buf
    return buf


def gemm(C, A, B, M, N, K, *, lda, a_kc, ldb, b_kc, ldc, A2=None, lda2=0, K1=0, a2_rdiv=1,
         b_rdiv=1, bias=None, mask=None, ldm=0, relu=False, accumulate=False, a_scale=1.0,
         b_scale=1.0, k_splits=0, rowsum=None, a_amax=None, mma_bf16=False, a_tiled=False,
         b_tiled=False, n_store=0, exact_fp32=False, c_trans=False, f16_single=False):
    """aon_gemm on tensor views (each operand's data_ptr carries its own offset); a_amax: a
    device word with the bits of max |A| (per-call gradient scale, include/aonerf.h);
    mma_bf16: the bf16 mode (bf16 MFMA; torch.bfloat16 operands are read as bf16);
    a_tiled / b_tiled: a reduction-major operand in the fused training kernels' 16-row tiled
    layout (tiles.py); n_store: columns of C written (0: all N; a zero-padded bf16 B);
    exact_fp32: a tiny product in exact fp32 (include/aonerf.h); c_trans: C written transposed
    and rowsum = B's column sums (the bf16 skinny path, include/aonerf.h); f16_single: the
    caller's licence for the single-accumulator fp16x3 kernel (operands range-guarded at their
    scales, include/aonerf.h)."""
    a = L.AonGemmArgs(M=M, N=N, K=K, A=A.data_ptr(), lda=lda, a_kc=int(a_kc),
                      A2=A2.data_ptr() if A2 is not None else None, lda2=lda2, K1=K1,
                      a2_rdiv=a2_rdiv, B=B.data_ptr(), ldb=ldb, b_kc=int(b_kc), b_rdiv=b_rdiv,
                      C=C.data_ptr(), ldc=ldc, bias=bias.data_ptr() if bias is not None else None,
                      mask=mask.data_ptr() if mask is not None else None, ldm=ldm,
                      relu=int(relu), accumulate=int(accumulate), a_scale=a_scale,
                      b_scale=b_scale, k_splits=k_splits,
                      rowsum=rowsum.data_ptr() if rowsum is not None else None,
                      a_amax=a_amax.data_ptr() if a_amax is not None else None,
                      mma_bf16=int(bool(mma_bf16)), a_bf16=int(A.dtype == torch.bfloat16),
                      b_bf16=int(B.dtype == torch.bfloat16), a_tiled=int(bool(a_tiled)),
                      b_tiled=int(bool(b_tiled)), n_store=n_store,
                      exact_fp32=int(bool(exact_fp32)), c_trans=int(bool(c_trans)),
                      f16_single=int(bool(f16_single)))
    if _small is not None:
        Cw = C[:M, :(n_store or N)] if C.dim() == 2 else C
        writes = [_span(Cw)]
        reads = [_span(A), _span(B)] + [_span(t) for t in (A2, bias, mask, a_amax) if t is not None]
        if accumulate:
            reads.append(_span(Cw))
        if exact_fp32:
            # deferred to one aon_gemm_small_batch launch (small_batched); operands kept alive.
            # The library itself orders products on one C chain and refuses any other
            # dependency between the items of one launch
            _small.append((a, C.device, (A, B, C, bias), writes, reads))
            return
        if _small and any(_overlaps(w, it[3]) or _overlaps(w, it[4]) or _overlaps(r, it[3])
                          for it in _small for w in writes for r in reads):
            # a product that runs at once inside small_batched(): it must not read
            # what a deferred tiny product writes, nor write what one reads or writes -- launch
            # the deferred ones first, in issue order
            _flush_small(_small)
            _small.clear()
    bf = mma_bf16 and A.dtype == torch.bfloat16 and B.dtype == torch.bfloat16
    f16 = (not mma_bf16 and A.dtype == torch.float32 and B.dtype == torch.float32 and not a_kc
           and not b_kc and A2 is None and bias is None and mask is None and not relu
           and not exact_fp32 and n_store in (0, N))
    if (_batch is not None and (bf or f16) and M % 128 == 0 and N % 128 == 0 and K >= 8192
            and not k_splits and b_rdiv == 1):
        # operands kept alive until the flush; class: bf16 one 256 x 256 tile, bf16 128 x 128
        # tiles, or fp16x3
        cls = "f16" if f16 else 256 if M == 256 and N == 256 else 128
        if cls != 128 or _batch128:
            # what the product writes of C: its M x (n_store or N) corner, not the whole view (a
            # dW passed whole while a K-concat segment fills its later columns must not count
            # as overlapping that segment's product: a needless flush split the level's batch)
            Cw = C[:M, :(n_store or N)] if C.dim() == 2 else C
            writes = [_span(Cw)] + ([_span(rowsum)] if rowsum is not None else [])
            reads = [_span(A), _span(B)] + ([_span(a_amax)] if a_amax is not None else [])
            if any(_overlaps(w, it[4]) or _overlaps(w, it[5]) or _overlaps(r, it[4])
                   for it in _batch for w in writes for r in reads):
                # a pending product writes what this one reads or writes, or reads what it
                # writes (incl. accumulate into a pending C): run the pending ones first
                _flush(_batch)
                _batch.clear()
            # every operand (a_amax too: a temporary scale word must not be recycled by the
            # caching allocator before the flush) stays alive until the product runs
            _batch.append((a, C.device, cls, (A, B, C, rowsum, a_amax), writes, reads))
            return
    if _batch:
        # a product that runs at once inside batched(): it must not read what a
        # deferred product writes, nor write what one reads or writes -- launch those first
        Cw = C[:M, :(n_store or N)] if C.dim() == 2 else C
        writes = [_span(Cw)] + ([_span(rowsum)] if rowsum is not None else [])
        reads = [_span(A), _span(B)] + [_span(t) for t in (A2, bias, mask, a_amax) if t is not None]
        if accumulate:
            reads.append(_span(Cw))
        if any(_overlaps(w, it[4]) or _overlaps(w, it[5]) or _overlaps(r, it[4])
               for it in _batch for w in writes for r in reads):
            _flush(_batch)
            _batch.clear()
    nbytes = L.lib().aon_gemm_workspace_bytes(ctypes.byref(a))
    ws = _workspace(nbytes, C.device) if nbytes else None
    L.call("aon_gemm", ctypes.byref(a), L.ptr(ws), nbytes, L.stream(C.device))


# the deferral state of the innermost batched() / small_batched() context (None: outside one)
_batch = None
_batch128 = True
_small = None


@contextlib.contextmanager
def small_batched():
    """Defer the exact_fp32 tiny products issued inside (the articulated bf16 step's latent-code
    terms and folded biases) to aon_gemm_small_batch launches at exit, in issue order --
    GEMM_SMALL_BATCH_MAX per launch, bit-identical to launching them one by one (products on one
    C chain in order; the library refuses any other dependency between them).  An aon_gemm that
    runs at once inside the context and touches a deferred product's output (or writes its
    inputs) first launches the deferred ones; torch ops inside the context see no such check, so
    callers read a deferred output only after the context exits."""
    global _small
    outer, _small = _small, []
    try:
        yield
        items = _small
    finally:
        _small = outer
    _flush_small(items)


def _flush_small(items):
    for i in range(0, len(items), L.GEMM_SMALL_BATCH_MAX):
        chunk = items[i:i + L.GEMM_SMALL_BATCH_MAX]
        arr = (L.AonGemmArgs * len(chunk))(*[it[0] for it in chunk])
        L.call("aon_gemm_small_batch", arr, len(chunk), L.stream(chunk[0][1]))
@contextlib.contextmanager
def batched(enabled=True, tiles128=True):
    """Defer the weight-gradient products in whole 128-column tiles issued inside (dW = dZ^T X
    of pts_linears / bottleneck / views_linear.0, the bf16 enc-column products) to
    aon_gemm_batch launches -- bf16 256 x 256, other bf16, and fp16x3 ones, up to
    GEMM_BATCH_MAX products of equal K per launch -- flushed at exit; every other product runs
    at once.  The deferred products only read kept tensors and write their own dW / db (callers
    flush before reading a deferred db), so the reordering is safe.  enabled False: nothing is
    deferred (A/B of aon_gemm_batch against separate launches, same bits); tiles128 False: only
    the 256 x 256 products are (A/B of the 128-tile class) -- the caller's TrainNumerics
    (batch_dweights / batch_128) passes both."""
    global _batch, _batch128
    if not enabled:
        yield
        return
    outer, _batch = _batch, []
    outer128, _batch128 = _batch128, bool(tiles128)
    try:
        yield
        items = _batch
    finally:
        _batch, _batch128 = outer, outer128
    _flush(items)


def _span(t):
    """What a product may touch of a tensor view: (start, end) bytes, and for a 2-D view with
    unit column stride also (storage base, row pitch, first row, rows, first byte in the row,
    bytes per row), so that column slices of one dW tensor do not count as overlapping."""
    if t.numel() == 0:
        return (0, 0, None)
    es = t.element_size()
    last = sum((n - 1) * st for n, st in zip(t.shape, t.stride()))
    start = t.data_ptr()
    grid = None
    if t.dim() == 2 and t.stride(1) == 1 and t.stride(0) >= t.shape[1]:
        base = t.untyped_storage().data_ptr()
        pitch = t.stride(0) * es
        off = start - base
        grid = (base, pitch, off // pitch, t.shape[0], off % pitch, t.shape[1] * es)
    return (start, start + (last + 1) * es, grid)


def _overlaps(x, ys):
    for y in ys:
        if not (x[0] < y[1] and y[0] < x[1]):
            continue
        gx, gy = x[2], y[2]
        if (gx is not None and gy is not None and gx[:2] == gy[:2]
                and gx[4] + gx[5] <= gx[1] and gy[4] + gy[5] <= gy[1]):
            rows = gx[2] < gy[2] + gy[3] and gy[2] < gx[2] + gx[3]
            cols = gx[4] < gy[4] + gy[5] and gy[4] < gx[4] + gx[5]
            if not (rows and cols):
                continue
        return True
    return False


def _flush(items):
    """Launch deferred products grouped by class and K, GEMM_BATCH_MAX per aon_gemm_batch."""
    groups = {}
    for it in items:
        groups.setdefault((it[2], it[0].K, str(it[1])), []).append(it)
    for grp in groups.values():
        for i in range(0, len(grp), L.GEMM_BATCH_MAX):
            chunk = grp[i:i + L.GEMM_BATCH_MAX]
            arr = (L.AonGemmArgs * len(chunk))(*[it[0] for it in chunk])
            dev = chunk[0][1]
            nbytes = L.lib().aon_gemm_batch_workspace_bytes(arr, len(chunk))
            ws = _workspace(nbytes, dev) if nbytes else None
            L.call("aon_gemm_batch", arr, len(chunk), L.ptr(ws), nbytes, L.stream(dev))


def colsum(out, X, M, N, ldx, accumulate=False):
    nbytes = L.lib().aon_colsum_workspace_bytes(M, N)
    ws = _workspace(nbytes, X.device)
    L.call("aon_colsum", L.ptr(X), ldx, M, N, int(accumulate), L.ptr(out), L.ptr(ws), nbytes,
           L.stream(X.device))


def linear_fwd(out, X, Kx, W, b, *, ldx=None, ldo=None, relu=False, X2=None, K2=0, ld2=0, rdiv2=1,
               accumulate=False):
    """out (R x N) (+)= [X | X2] W^T + b (+ReLU); W is the nn.Linear weight (N x (Kx+K2))."""
    R, N = out.shape[0], W.shape[0]
    gemm(out, X, W, R, N, Kx + K2, lda=ldx or Kx, a_kc=True, ldb=W.shape[1], b_kc=True,
         ldc=ldo or out.shape[1], A2=X2, lda2=ld2, K1=Kx if X2 is not None else 0, a2_rdiv=rdiv2,
         bias=b, relu=relu, accumulate=accumulate, a_scale=ACT_SCALE, b_scale=W_SCALE)


