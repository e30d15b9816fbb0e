"""linalg.batched() deferral bookkeeping (CPU): deferred products keep every operand
alive (a_amax included) and a product that reads or writes what a pending product writes (or
writes what one reads, or accumulates into a pending C) flushes the pending ones first; column
slices of one dW tensor do not count as overlapping.  No kernel runs: _flush is recorded."""
import torch

from aonerf import linalg


def _rec(monkeypatch):
    log = []
    monkeypatch.setattr(linalg, "_flush", lambda items: log.append([it[3][2] for it in items]))
    return log


def _dw(C, A, B, **kw):
    M, N, K = C.shape[0], C.shape[1], A.shape[0]
    linalg.gemm(C, A, B, M, N, K, lda=A.shape[1], a_kc=False, ldb=B.shape[1], b_kc=False,
                ldc=C.stride(0), mma_bf16=True, **kw)


def test_disjoint_products_share_one_flush(monkeypatch):
    log = _rec(monkeypatch)
    K = 8192
    A = torch.zeros(K, 256, dtype=torch.bfloat16)
    B = torch.zeros(K, 512, dtype=torch.bfloat16)
    C = torch.zeros(256, 512)
    with linalg.batched():
        _dw(C[:, :256], A, B[:, :256])
        _dw(C[:, 256:], A, B[:, 256:])  # other columns of the same dW: no conflict
    assert len(log) == 1 and len(log[0]) == 2


def test_accumulate_into_pending_output_flushes_first(monkeypatch):
    log = _rec(monkeypatch)
    K = 8192
    A = torch.zeros(K, 256, dtype=torch.bfloat16)
    B = torch.zeros(K, 256, dtype=torch.bfloat16)
    C = torch.zeros(256, 256)
    with linalg.batched():
        _dw(C, A, B)
        _dw(C, A, B, accumulate=True)
    assert [len(g) for g in log] == [1, 1]


def test_read_after_pending_write_flushes_first(monkeypatch):
    log = _rec(monkeypatch)
    K = 8192
    A = torch.zeros(K, 256)
    buf = torch.zeros(K, 256)  # fp16x3 class: fp32 operands
    with linalg.batched():
        linalg.gemm(buf[:256], A, A, 256, 256, K, lda=256, a_kc=False, ldb=256, b_kc=False, ldc=256)
        other = torch.zeros(256, 256)
        linalg.gemm(other, A, torch.zeros(K, 256), 256, 256, K, lda=256, a_kc=False, ldb=256,
                    b_kc=False, ldc=256)
        assert log == []  # independent
        linalg.gemm(torch.zeros(256, 256), A, buf, 256, 256, K, lda=256, a_kc=False, ldb=256,
                    b_kc=False, ldc=256)  # reads what the first writes
        assert [len(g) for g in log] == [2]
    assert [len(g) for g in log] == [2, 1]


def test_a_amax_kept_alive(monkeypatch):
    seen = []
    monkeypatch.setattr(linalg, "_flush", lambda items: seen.extend(items))
    K = 8192
    A = torch.zeros(K, 256)
    B = torch.zeros(K, 256)
    C = torch.zeros(256, 256)
    amax = torch.zeros(1, dtype=torch.int32)
    with linalg.batched():
        linalg.gemm(C, A, B, 256, 256, K, lda=256, a_kc=False, ldb=256, b_kc=False, ldc=256,
                    a_amax=amax)
    assert len(seen) == 1 and seen[0][3][4] is amax


def test_whole_dw_view_with_concat_segment_one_flush(monkeypatch):
    """The fused backward passes pts_linears.5's dW WHOLE (256 x 319) for its 256 main columns and
    dW[:, 256:] for the skip segment's (63 stored of a 128-wide bf16 operand, n_store): the first
    product writes only its M x N corner, so the two share one flush (a flush between them split
    the level's 256 x 256 batch in two launches)."""
    log = _rec(monkeypatch)
    K = 8192
    A = torch.zeros(K, 256, dtype=torch.bfloat16)
    B = torch.zeros(K, 256, dtype=torch.bfloat16)
    E = torch.zeros(K, 128, dtype=torch.bfloat16)
    dW = torch.zeros(256, 319)
    with linalg.batched():
        linalg.gemm(dW, A, B, 256, 256, K, lda=256, a_kc=False, ldb=256, b_kc=False, ldc=319,
                    mma_bf16=True)
        linalg.gemm(dW[:, 256:], A, E, 256, 128, K, lda=256, a_kc=False, ldb=128, b_kc=False,
                    ldc=319, mma_bf16=True, n_store=63)
    assert len(log) == 1 and len(log[0]) == 2


def test_immediate_product_reading_pending_output_flushes_first(monkeypatch):
    """a product that runs at once inside batched() (here K < 8192, as the latent
    terms' tiny products) and reads a deferred product's bias gradient launches after it."""
    events = []
    monkeypatch.setattr(linalg, "_flush", lambda items: events.append(("flush", len(items))))
    monkeypatch.setattr(linalg.L, "call", lambda name, *a: events.append((name,)))
    monkeypatch.setattr(linalg.L, "stream", lambda device=None: None)  # (no GPU here)
    monkeypatch.setattr(linalg, "_workspace", lambda nbytes, device: None)
    K = 8192
    A = torch.zeros(K, 256, dtype=torch.bfloat16)
    B = torch.zeros(K, 256, dtype=torch.bfloat16)
    C, db = torch.zeros(256, 256), torch.zeros(256)
    lat = torch.zeros(1, 128)
    with linalg.batched():
        _dw(C, A, B, rowsum=db)
        other = torch.zeros(1, 128)
        linalg.gemm(other, lat, torch.zeros(256, 128), 1, 128, 16, lda=16, a_kc=True, ldb=128,
                    b_kc=False, ldc=128)  # independent: no flush
        assert events == [("aon_gemm",)]
        dl = torch.zeros(1, 128)
        linalg.gemm(dl, db[None, :], torch.zeros(256, 128), 1, 128, 256, lda=256, a_kc=True,
                    ldb=128, b_kc=False, ldc=128)  # reads the pending db
        assert events == [("aon_gemm",), ("flush", 1), ("aon_gemm",)]
    assert events[-1] == ("flush", 0) or events[-1] == ("aon_gemm",)


def _log_calls(monkeypatch):
    events = []
    monkeypatch.setattr(linalg, "_flush", lambda items: events.append(("flush", len(items))))
    monkeypatch.setattr(linalg.L, "call", lambda name, *a: events.append(
        (name, a[1]) if name == "aon_gemm_small_batch" else (name,)))
    monkeypatch.setattr(linalg.L, "stream", lambda device=None: None)  # (no GPU here)
    monkeypatch.setattr(linalg, "_workspace", lambda nbytes, device: None)
    return events


def _tiny(C, A, B, **kw):
    # (1 x n) = (1 x k) (k x n), the latent-term shape; exact_fp32 ones are deferred
    linalg.gemm(C, A, B, 1, C.shape[1], A.shape[1], lda=A.shape[1], a_kc=True, ldb=B.shape[1],
                b_kc=False, ldc=C.shape[1], **kw)


def test_small_batched_immediate_reader_flushes_first(monkeypatch):
    """inside small_batched(), an aon_gemm that runs at once (not exact_fp32) and
    reads a deferred tiny product's output launches after the deferred ones; an independent one
    does not split the batch."""
    events = _log_calls(monkeypatch)
    lat, W = torch.zeros(1, 16), torch.zeros(16, 128)
    fold = torch.zeros(1, 128)
    with linalg.small_batched():
        _tiny(fold, lat, W, exact_fp32=True)
        _tiny(torch.zeros(1, 128), lat, W, exact_fp32=True)
        _tiny(torch.zeros(1, 128), lat, W)  # independent, immediate
        assert events == [("aon_gemm",)]
        _tiny(torch.zeros(1, 8), fold[:, :16], torch.zeros(16, 8))  # reads the deferred fold
        assert events == [("aon_gemm",), ("aon_gemm_small_batch", 2), ("aon_gemm",)]
        _tiny(torch.zeros(1, 128), lat, W, exact_fp32=True)
    assert events[-1] == ("aon_gemm_small_batch", 1)


def test_small_batched_immediate_writer_of_deferred_input_flushes_first(monkeypatch):
    events = _log_calls(monkeypatch)
    lat, W = torch.zeros(1, 16), torch.zeros(16, 128)
    with linalg.small_batched():
        _tiny(torch.zeros(1, 128), lat, W, exact_fp32=True)
        _tiny(lat, torch.zeros(1, 4), torch.zeros(4, 16))  # overwrites the deferred input
        assert events == [("aon_gemm_small_batch", 1), ("aon_gemm",)]
    assert events == [("aon_gemm_small_batch", 1), ("aon_gemm",)]


def test_batched_disabled_defers_nothing(monkeypatch):
    """batched(enabled=False) (TrainNumerics.batch_dweights False): every product at once."""
    events = _log_calls(monkeypatch)
    K = 8192
    A = torch.zeros(K, 256, dtype=torch.bfloat16)
    with linalg.batched(False):
        _dw(torch.zeros(256, 256), A, A)
        assert events == [("aon_gemm",)]
    assert events == [("aon_gemm",)]


def test_batched_without_128_tiles(monkeypatch):
    """batched(tiles128=False): the 128-column-tile class runs at once, the 256 x 256 one is
    deferred; the flag does not leak out of the context."""
    events = _log_calls(monkeypatch)
    K = 8192
    A = torch.zeros(K, 256, dtype=torch.bfloat16)
    A128 = torch.zeros(K, 128, dtype=torch.bfloat16)
    with linalg.batched(True, False):
        _dw(torch.zeros(256, 256), A, A)
        _dw(torch.zeros(128, 256), A128, A)
        assert events == [("aon_gemm",)]
    assert events == [("aon_gemm",), ("flush", 1)]
    assert linalg._batch128 is True and linalg._batch is None
