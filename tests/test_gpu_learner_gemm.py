"""Learner GEMMs (csrc/f110_gemm.hip, include/f110.h "learner GEMMs") against
a float64 torch reference of the same expression: forward layers with bias /
ReLU / action columns / masks, input gradients (nn), weight and bias
gradients; ragged M, K and N; grouped launches; run-to-run bit identity.
Tolerance: fp32 rounding of a length-K dot product, |err| <= 2e-6 * sum|a b|
(+1e-7) elementwise."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _lg():
    from f110_gymnasium_ros2_jazzy_amd import learner_gemm
    return learner_gemm


def _close(got, ref, absref):
    err = (got.double() - ref).abs()
    bound = 2e-6 * absref + 1e-7
    bad = err > bound
    assert not bool(bad.any()), f"{int(bad.sum())} of {bad.numel()} outside; max ratio {float((err / bound).max())}"


def _rand(g, *shape):
    return torch.randn(*shape, device="cuda", generator=g, dtype=torch.float32)


@pytest.mark.parametrize("M,K,N", [(4096, 1088, 128), (333, 12, 128), (200, 130, 200), (64, 64, 2), (1, 48, 40),
                                   (257, 1060, 72), (40, 36, 129)])
def test_forward_layers(gpu, M, K, N):
    lg = _lg()
    g = torch.Generator(device="cuda").manual_seed(M + K + N)
    X, W, b = _rand(g, M, K), _rand(g, N, K), _rand(g, N)
    y = torch.full((M, N), float("nan"), device="cuda")
    lg.gemm([lg.op(X, W, y, N, K, K, K, N, bias=b, relu=True)], M, X.device)
    ref = torch.relu(X.double() @ W.double().t() + b.double())
    _close(y, ref, X.double().abs() @ W.double().abs().t() + b.double().abs())


def test_grouped_forward_with_action_columns_and_masks(gpu):
    """The critic's fcs2 (K = 128 of a 130-wide weight, the 2 action columns
    from a separate tensor), a grouped launch of three ops with different A,
    and the output mask."""
    lg = _lg()
    g = torch.Generator(device="cuda").manual_seed(3)
    M = 1000
    z1, act, Ws2, bs2 = _rand(g, M, 128), _rand(g, M, 2), _rand(g, 128, 130), _rand(g, 128)
    X2, W2 = _rand(g, M, 1088), _rand(g, 128, 1088)
    om = _rand(g, M, 128)
    y1, y2, y3 = (torch.empty(M, 128, device="cuda") for _ in range(3))
    lg.gemm([lg.op(z1, Ws2, y1, 128, 128, 128, 130, 128, bias=bs2, x2=act, w2=(Ws2, 128), nx2=2, ldx2=2, ldw2=130,
                   relu=True),
             lg.op(X2, W2, y2, 128, 1088, 1088, 1088, 128, relu=False),
             lg.op(X2, W2, y3, 128, 1088, 1088, 1088, 128, bias=bs2, relu=True, omask=om)], M, z1.device)
    zc = torch.cat([z1, act], 1).double()
    _close(y1, torch.relu(zc @ Ws2.double().t() + bs2.double()), zc.abs() @ Ws2.double().abs().t() + bs2.double().abs())
    p = X2.double() @ W2.double().t()
    a = X2.double().abs() @ W2.double().abs().t()
    _close(y2, p, a)
    _close(y3, torch.where(om.double() > 0, torch.relu(p + bs2.double()), torch.zeros_like(p)), a + bs2.double().abs())


def test_grouped_lds_path_with_input_mask(gpu):
    """Rows of A and B 16-B aligned with K % 4 == 0 take the LDS-staged kernel
    (k_lgemm_lds): a grouped launch of two ops with an input mask (amask) on
    both, K with a partial last 32-k chunk, ragged M and N."""
    lg = _lg()
    g = torch.Generator(device="cuda").manual_seed(11)
    M, K = 301, 1092
    X1, X2, Am1, Am2 = _rand(g, M, K), _rand(g, M, K), _rand(g, M, K), _rand(g, M, K)
    W1, W2, b1 = _rand(g, 96, K), _rand(g, 128, K), _rand(g, 96)
    y1, y2 = torch.empty(M, 96, device="cuda"), torch.empty(M, 128, device="cuda")
    lg.gemm([lg.op(X1, W1, y1, 96, K, K, K, 96, bias=b1, relu=True, amask=Am1),
             lg.op(X2, W2, y2, 128, K, K, K, 128, amask=Am2)], M, X1.device)
    for X, Am, W, y, b, relu in ((X1, Am1, W1, y1, b1, True), (X2, Am2, W2, y2, None, False)):
        Xm = torch.where(Am > 0, X, torch.zeros_like(X)).double()
        ref = Xm @ W.double().t()
        absref = Xm.abs() @ W.double().abs().t()
        if b is not None:
            ref, absref = ref + b.double(), absref + b.double().abs()
        _close(y, torch.relu(ref) if relu else ref, absref)

@pytest.mark.parametrize("M,K,N,ldb,off", [(4096, 128, 128, 130, 0), (4096, 128, 2, 130, 128), (77, 128, 128, 128, 0),
                                           (50, 20, 33, 40, 3)])
def test_input_gradient_nn(gpu, M, K, N, ldb, off):
    """dX = (gy masked by y > 0) W[:, off:off+N] masked by the input's ReLU
    output (the fcs2 / fc2 backward and the critic's action gradient)."""
    lg = _lg()
    g = torch.Generator(device="cuda").manual_seed(M * 7 + N)
    G, Y, W, Z = _rand(g, M, K), _rand(g, M, K), _rand(g, K, ldb), _rand(g, M, N)
    out = torch.empty(M, N, device="cuda")
    lg.gemm([lg.op(G, (W, off), out, N, K, K, ldb, N, amask=Y, omask=Z, nn=True)], M, G.device)
    Gm = torch.where(Y > 0, G, torch.zeros_like(G)).double()
    Wd = W[:, off:off + N].double()
    ref = torch.where(Z > 0, Gm @ Wd, torch.zeros(M, N, dtype=torch.float64, device="cuda"))
    _close(out, ref, Gm.abs() @ Wd.abs())


@pytest.mark.parametrize("M", [4096, 333, 8])
def test_weight_gradients(gpu, M):
    """dW = G'^T X and db = sum G' for the critic-phase ops: fcs2's
    [128 x 128] + its 2 action columns (ldw 130) in one masked launch, fcs1's
    [128 x 1088] in an unmasked one (grouped with a second op); one op alone
    (a different slice count: same values); run twice: bit-identical."""
    lg = _lg()
    g = torch.Generator(device="cuda").manual_seed(M)
    G, Y, Z1, A, G1, S = _rand(g, M, 128), _rand(g, M, 128), _rand(g, M, 128), _rand(g, M, 2), _rand(g, M, 128), \
        _rand(g, M, 1088)
    outs = []
    for _ in range(2):
        dWs2, dbs2 = torch.full((128, 130), float("nan"), device="cuda"), torch.empty(128, device="cuda")
        dWs1, dbs1 = torch.empty(128, 1088, device="cuda"), torch.empty(128, device="cuda")
        lg.wgrad([lg.wop(G, Z1, dWs2, 128, 128, 128, 128, 130, db=dbs2, gmask=Y),
                  lg.wop(G, A, (dWs2, 128), 128, 2, 128, 2, 130, gmask=Y)], M, G.device)
        lg.wgrad([lg.wop(G1, S, dWs1, 128, 1088, 128, 1088, 1088, db=dbs1),
                  lg.wop(G1, Z1, dWs2, 128, 128, 128, 128, 130)], M, G.device)  # overwritten by the next line
        lg.wgrad([lg.wop(G, Z1, dWs2, 128, 128, 128, 128, 130, db=dbs2, gmask=Y)], M, G.device)
        outs.append((dWs2, dbs2, dWs1, dbs1))
    Gm = torch.where(Y > 0, G, torch.zeros_like(G)).double()
    zc = torch.cat([Z1, A], 1).double()
    dWs2, dbs2, dWs1, dbs1 = outs[0]
    _close(dWs2, Gm.t() @ zc, Gm.abs().t() @ zc.abs())
    _close(dbs2, Gm.sum(0), Gm.abs().sum(0))
    _close(dWs1, G1.double().t() @ S.double(), G1.double().abs().t() @ S.double().abs())
    _close(dbs1, G1.double().sum(0), G1.double().abs().sum(0))
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)


def test_rejects_bad_ops(gpu):
    from f110_gymnasium_ros2_jazzy_amd import _lib
    lg = _lg()
    x = torch.zeros(8, 16, device="cuda")
    y = torch.zeros(8, 4, device="cuda")
    with pytest.raises(RuntimeError):
        lg.gemm([lg.op(x, x, y, 4, 16, 8, 16, 4)], 8, x.device)  # lda < K
    with pytest.raises(RuntimeError):
        lg.gemm([lg.op(x, x, y, 4, 16, 16, 16, 4, nn=False), lg.op(x, x, y, 4, 16, 16, 16, 4, nn=True)], 8, x.device)
    with pytest.raises((RuntimeError, _lib.F110Error)):
        lg.wgrad([lg.wop(x, x, y, 4, 16, 2, 16, 16)], 8, x.device)  # ldg < N
    with pytest.raises((RuntimeError, _lib.F110Error)):  # gmask on one op of a launch only
        lg.wgrad([lg.wop(x, x, y, 4, 16, 16, 16, 16, gmask=x), lg.wop(x, x, y, 4, 16, 16, 16, 16)], 8, x.device)
    with pytest.raises(RuntimeError):  # amask on one op of a launch only
        lg.gemm([lg.op(x, x, y, 4, 16, 16, 16, 4, amask=x), lg.op(x, x, y, 4, 16, 16, 16, 4)], 8, x.device)


@pytest.mark.parametrize("M", [8, 4096])
def test_weight_gradients_with_loss(gpu, M):
    """f110_learner_wgrad_loss: the gradients as f110_learner_wgrad writes
    them, and *loss = sign * sum(partials) / M from the finishing launch --
    with S == 1 (M = 8: the finishing launch holds only the loss block) and
    S > 1 (M = 4096)."""
    lg = _lg()
    g = torch.Generator(device="cuda").manual_seed(21 + M)
    G, X = _rand(g, M, 128), _rand(g, M, 96)
    dW1, db1 = torch.empty(128, 96, device="cuda"), torch.empty(128, device="cuda")
    dW2, db2 = torch.empty(128, 96, device="cuda"), torch.empty(128, device="cuda")
    part = _rand(g, 37)
    loss = torch.full((), float("nan"), device="cuda")
    lg.wgrad([lg.wop(G, X, dW1, 128, 96, 128, 96, 96, db=db1)], M, G.device)
    lg.wgrad([lg.wop(G, X, dW2, 128, 96, 128, 96, 96, db=db2)], M, G.device, loss=(part, -1.0, loss))
    assert torch.equal(dW1, dW2) and torch.equal(db1, db2)
    ref = -float(part.double().sum()) / M
    assert abs(float(loss) - ref) <= 1e-6 * (float(part.double().abs().sum()) / M) + 1e-12
