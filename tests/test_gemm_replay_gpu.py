"""MFMA GEMM layers and the replay ring/sampler vs references — GPU only."""
import ctypes as C

import numpy as np
import pytest
import torch

from oracle import replay as orp

pytestmark = pytest.mark.gpu


def _gemm(prec, mode, M, N, K, relu, A, lda, B, ldb, bias, Cm, ldc, mask=None, ldm=0, bgrad=None):
    from rlmd_amd import _abi

    P = _abi.ptr
    _abi.check(_abi.lib().rlmd_gemm(prec, mode, M, N, K, relu, P(A), lda, P(B), ldb, P(bias), P(Cm), ldc,
                                    P(mask), ldm, P(bgrad), _abi.stream_ptr()))


SHAPES = [(512, 256, 6), (512, 256, 256), (200, 400, 7), (200, 300, 400), (37, 65, 129), (1, 256, 512)]


@pytest.mark.parametrize("prec", [0, 1])
@pytest.mark.parametrize("M,N,K", SHAPES)
def test_forward(dev, prec, M, N, K):
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N + K)
    x = torch.randn(M, K, generator=g).to(dev)
    w = torch.randn(N, K, generator=g).to(dev) / K**0.5
    b = torch.randn(N, generator=g).to(dev)
    y = torch.empty(M, N, device=dev)
    _gemm(prec, 0, M, N, K, 1, x, K, w, K, b, y, N)
    if prec == 1:
        x_, w_ = x.bfloat16().double(), w.bfloat16().double()
    else:
        x_, w_ = x.double(), w.double()
    ref = torch.relu(x_ @ w_.T + b.double())
    tol = 1e-5 if prec == 0 else 1e-4
    torch.testing.assert_close(y.double(), ref, rtol=tol, atol=tol)


@pytest.mark.parametrize("prec", [0, 1])
@pytest.mark.parametrize("M,N,K", SHAPES)
def test_backward(dev, prec, M, N, K):
    # layer y = relu(x W^T + b), x [M,K], W [N,K]; upstream g [M,N]
    g0 = torch.Generator(device="cpu").manual_seed(M + 3 * N + 5 * K)
    x = torch.randn(M, K, generator=g0).to(dev)
    w = torch.randn(N, K, generator=g0).to(dev)
    gy = torch.randn(M, N, generator=g0).to(dev)
    mask_src = torch.relu(torch.randn(M, K, generator=g0)).to(dev)
    dx = torch.empty(M, K, device=dev)
    _gemm(prec, 1, M, K, N, 0, gy, N, w, K, None, dx, K, mask_src, K)
    dw = torch.empty(N, K, device=dev)
    db = torch.empty(N, device=dev)
    _gemm(prec, 2, N, K, M, 0, gy, N, x, K, None, dw, K, None, 0, db)
    cast = (lambda t: t.bfloat16().double()) if prec == 1 else (lambda t: t.double())
    ref_dx = (cast(gy) @ cast(w)) * (mask_src > 0)
    ref_dw = cast(gy).T @ cast(x)
    ref_db = cast(gy).sum(0)
    tol = 1e-4 if prec == 0 else 1e-3
    scale_x = ref_dx.abs().max().item() + 1
    scale_w = ref_dw.abs().max().item() + 1
    torch.testing.assert_close(dx.double() / scale_x, ref_dx / scale_x, rtol=tol, atol=tol)
    torch.testing.assert_close(dw.double() / scale_w, ref_dw / scale_w, rtol=tol, atol=tol)
    torch.testing.assert_close(db.double(), ref_db, rtol=tol, atol=tol * (M ** 0.5))


def test_fp32_gemm_is_exact_fma_chain_on_integers(dev):
    """Small-integer operands: fp32 MFMA result must be exact."""
    M, N, K = 64, 64, 64
    x = torch.randint(-4, 5, (M, K), device=dev).float()
    w = torch.randint(-4, 5, (N, K), device=dev).float()
    y = torch.empty(M, N, device=dev)
    _gemm(0, 0, M, N, K, 0, x, K, w, K, None, y, N)
    assert torch.equal(y, x @ w.T)


@pytest.mark.parametrize("cap,inserts", [(5000, (1300, 2100, 3000)), (25000, (9000, 12000, 8000))])
def test_replay_ring_and_distinct_sampling(dev, cap, inserts):
    """Ring wrap-around + both sampling regimes (sort: M <= 8192, rounds: M > 8192)."""
    from rlmd_amd import _abi

    S, A = 5, 2
    h = C.c_void_p()
    _abi.check(_abi.lib().rlmd_replay_create(cap, S, A, C.byref(h)))
    rng = np.random.default_rng(0)
    store = {}
    mem = 0
    for n in inserts:  # wraps the ring
        s = torch.from_numpy(rng.random((n, S)).astype(np.float32)).to(dev)
        a = torch.from_numpy(rng.random((n, A)).astype(np.float32)).to(dev)
        r = torch.from_numpy(rng.random(n).astype(np.float32)).to(dev)
        s2 = torch.from_numpy(rng.random((n, S)).astype(np.float32)).to(dev)
        d = torch.from_numpy((rng.random(n) < 0.3).astype(np.uint8)).to(dev)
        P = _abi.ptr
        _abi.check(_abi.lib().rlmd_replay_insert(h, n, P(s), P(a), P(r), P(s2), P(d), _abi.stream_ptr()))
        for i, row in enumerate(orp.ring_rows(mem, n, cap)):
            store[int(row)] = (s[i].cpu(), a[i].cpu(), r[i].cpu(), s2[i].cpu(), d[i].cpu())
        mem += n
    m = C.c_int64()
    _abi.check(_abi.lib().rlmd_replay_mem_idx(h, C.byref(m)))
    assert m.value == mem
    for B, ctr in ((512, 3), (1024, 2**33 + 5), (200, 77)):
        idx = torch.empty(B, dtype=torch.int64, device=dev)
        s = torch.empty(B, S, device=dev)
        a = torch.empty(B, A, device=dev)
        r = torch.empty(B, device=dev)
        s2 = torch.empty(B, S, device=dev)
        d = torch.empty(B, dtype=torch.uint8, device=dev)
        P = _abi.ptr
        _abi.check(_abi.lib().rlmd_replay_sample(h, B, 42, ctr, P(idx), P(s), P(a), P(r), P(s2), P(d), None,
                                                 _abi.stream_ptr()))
        got = idx.cpu().numpy()
        assert len(set(got.tolist())) == B  # without replacement
        np.testing.assert_array_equal(got, orp.sample_indices(42, ctr, min(mem, cap), B).astype(np.int64))
        for i in range(B):
            ref = store[int(got[i])]
            assert torch.equal(s[i].cpu(), ref[0]) and torch.equal(a[i].cpu(), ref[1])
            assert torch.equal(r[i].cpu(), ref[2]) and torch.equal(s2[i].cpu(), ref[3])
            assert d[i].item() == ref[4].item()
    _abi.lib().rlmd_replay_destroy(h)


def test_replay_tiny_population_forces_duplicate_rounds(dev):
    """M = B + 3 (the sort regime): still a distinct subset, equal to the oracle's."""
    from rlmd_amd import _abi

    S, A, B = 3, 1, 300
    M = B + 3
    h = C.c_void_p()
    _abi.check(_abi.lib().rlmd_replay_create(M, S, A, C.byref(h)))
    z = torch.zeros(M, S, device=dev)
    za = torch.zeros(M, A, device=dev)
    zr = torch.arange(M, dtype=torch.float32, device=dev)
    zd = torch.zeros(M, dtype=torch.uint8, device=dev)
    P = _abi.ptr
    _abi.check(_abi.lib().rlmd_replay_insert(h, M, P(z), P(za), P(zr), P(z), P(zd), _abi.stream_ptr()))
    idx = torch.empty(B, dtype=torch.int64, device=dev)
    r = torch.empty(B, device=dev)
    _abi.check(_abi.lib().rlmd_replay_sample(h, B, 9, 1, P(idx), None, None, P(r), None, None, None, _abi.stream_ptr()))
    got = idx.cpu().numpy()
    ref = orp.sample_indices(9, 1, M, B)
    assert len(set(got.tolist())) == B
    np.testing.assert_array_equal(got, ref.astype(np.int64))
    np.testing.assert_array_equal(r.cpu().numpy(), got.astype(np.float32))
    _abi.lib().rlmd_replay_destroy(h)
