"""Kernel-level parity: each libtmr entry point against a float64 CPU torch computation of
the same op (the reference's own ops: nn.Conv2d / BatchNorm2d / MaxPool2d / LSTM / Linear).
fp32 tolerances are stated per test, scaled by the magnitude of the result."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from tmrnet_amd import ops

pytestmark = pytest.mark.gpu


def rel_err(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return ((a - b).abs().max() / (b.abs().max() + 1e-30)).item()


CONV_CASES = [
    # n, h, w, cin, cout, r, stride, pad
    (2, 16, 16, 64, 64, 1, 1, 0),
    (2, 15, 13, 64, 128, 3, 1, 1),
    (3, 14, 14, 128, 128, 3, 2, 1),
    (2, 14, 14, 256, 512, 1, 2, 0),
    (2, 9, 9, 512, 2048, 1, 1, 0),
    (2, 7, 7, 2048, 512, 1, 1, 0),
    (1, 28, 28, 3, 64, 7, 2, 3),     # stem: 3 channels stored as 4
]


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd_dgrad_wgrad(dev, case):
    n, h, w, cin, cout, r, st, pad = case
    g = torch.Generator().manual_seed(hash(case) % 1000)
    x = torch.randn(n, cin, h, w, generator=g, dtype=torch.float64)
    wt = torch.randn(cout, cin, r, r, generator=g, dtype=torch.float64) / np.sqrt(cin * r * r)
    y_ref = F.conv2d(x, wt, stride=st, padding=pad)
    dy = torch.randn(y_ref.shape, generator=g, dtype=torch.float64)
    xr = x.clone().requires_grad_(True)
    wr = wt.clone().requires_grad_(True)
    F.conv2d(xr, wr, stride=st, padding=pad).backward(dy)
    cs = 4 if cin == 3 else cin
    x4 = ops.nchw_to_nhwc(x.float().to(dev), cpad=cs)
    wk = ops.weight_to_krsc(wt.float().to(dev).contiguous(), cpad=cs)
    y = ops.conv_fwd(x4, wk, st, pad)
    assert rel_err(y.permute(0, 3, 1, 2), y_ref) < 2e-6
    dyd = dy.float().permute(0, 2, 3, 1).contiguous().to(dev)
    if cin != 3:
        dx = ops.conv_dgrad(dyd, wk, (h, w), st, pad)
        assert rel_err(dx.permute(0, 3, 1, 2), xr.grad) < 2e-6
        # beta accumulate
        dx2 = ops.conv_dgrad(dyd, wk, (h, w), st, pad, out=dx.clone(), beta=1.0)
        assert rel_err(dx2, 2 * dx) < 1e-6
    dw = ops.conv_wgrad(x4, dyd, r, r, st, pad, c_real=cin)
    assert rel_err(dw, wr.grad) < 2e-6


@pytest.mark.parametrize("case", [c for c in CONV_CASES if c[3] != 3])
def test_conv_dgrad_fp32_transposed_weights(dev, case):
    """fp32 dgrad on the LDS-DMA engine (transposed fp32 weights, TMR_IO_WT_F32) against float64
    torch, and against the register-staged engine on the KRSC weights (same tolerance)."""
    n, h, w, cin, cout, r, st, pad = case
    g = torch.Generator().manual_seed(hash(case) % 997)
    wt = torch.randn(cout, cin, r, r, generator=g, dtype=torch.float64) / np.sqrt(cout * r * r)
    ho, wo = (h + 2 * pad - r) // st + 1, (w + 2 * pad - r) // st + 1
    dy = torch.randn(n, cout, ho, wo, generator=g, dtype=torch.float64)
    ref = torch.nn.grad.conv2d_input((n, cin, h, w), wt, dy, stride=st, padding=pad)
    wd = wt.float().to(dev).contiguous()
    wc = ops.weight_to_crsk(wd, bf16=False)
    assert wc.dtype == torch.float32 and wc.shape == (cin, r, r, cout)
    dyd = dy.float().permute(0, 2, 3, 1).contiguous().to(dev)
    dx = ops.conv_dgrad(dyd, wc, (h, w), st, pad, wt=True)
    assert rel_err(dx.permute(0, 3, 1, 2), ref) < 2e-6
    dxk = ops.conv_dgrad(dyd, ops.weight_to_krsc(wd), (h, w), st, pad)
    assert rel_err(dx, dxk) < 2e-6
    dx2 = ops.conv_dgrad(dyd, wc, (h, w), st, pad, out=dx.clone(), beta=1.0, wt=True)
    assert rel_err(dx2, 2 * dx) < 1e-6


def test_conv_fp32_transposed_weights_errors(dev):
    """fp32 transposed weights with a bf16 operand, or with bf16 math, are refused."""
    wc = ops.weight_to_crsk(torch.randn(64, 64, 1, 1, device=dev), bf16=False)
    dy = torch.randn(1, 4, 4, 64, device=dev)
    with pytest.raises(RuntimeError):
        ops.conv_dgrad(dy.to(torch.bfloat16), wc, (4, 4), 1, 0, wt=True, math="bf16")
    with pytest.raises(RuntimeError):
        ops.conv_dgrad(dy, wc, (4, 4), 1, 0, wt=True, math="bf16")


@pytest.mark.parametrize("M,N,K", [(64, 2048, 2048), (7, 512, 64), (64, 7, 512), (33, 65, 17),
                                   (640, 512, 1024)])
def test_gemms(dev, M, N, K):
    g = torch.Generator().manual_seed(M * 7 + N + K)
    a = torch.randn(M, K, generator=g, dtype=torch.float64)
    b = torch.randn(N, K, generator=g, dtype=torch.float64)
    bias = torch.randn(N, generator=g, dtype=torch.float64)
    ad, bd = a.float().to(dev), b.float().to(dev)
    out = ops.gemm_nt(ad, bd, bias=bias.float().to(dev))
    assert rel_err(out, a @ b.t() + bias) < 2e-6
    bkn = b.t().contiguous()
    out = ops.gemm_nn(ad, bkn.float().to(dev))
    assert rel_err(out, a @ bkn) < 2e-6
    # gemm_tn: out[K][N] = a^T @ c2 with a (M,K) read as [K'=M][M'=K]
    c2 = torch.randn(M, N, generator=g, dtype=torch.float64)
    out = ops.gemm_tn(ad, c2.float().to(dev))
    assert rel_err(out, a.t() @ c2) < 2e-6


@pytest.mark.parametrize("rows,c,relu,res", [(20000, 64, True, False), (3000, 256, True, True),
                                             (980, 2048, False, False), (4096, 128, True, True)])
def test_batchnorm(dev, rows, c, relu, res):
    g = torch.Generator().manual_seed(rows + c)
    y = (torch.randn(rows, c, generator=g, dtype=torch.float64) * 3 + 5)
    gamma = torch.rand(c, generator=g, dtype=torch.float64) + 0.5
    beta = torch.randn(c, generator=g, dtype=torch.float64)
    r = torch.randn(rows, c, generator=g, dtype=torch.float64) if res else None
    rm = torch.randn(c, generator=g, dtype=torch.float64)
    rv = torch.rand(c, generator=g, dtype=torch.float64) + 0.5
    # reference: torch batch_norm train mode (double)
    yr = y.clone().requires_grad_(True)
    gr = gamma.clone().requires_grad_(True)
    br = beta.clone().requires_grad_(True)
    rm_ref, rv_ref = rm.clone(), rv.clone()
    o = F.batch_norm(yr, rm_ref, rv_ref, gr, br, training=True, momentum=0.1, eps=1e-5)
    if res:
        o = o + r
    if relu:
        o = torch.relu(o)
    dz = torch.randn(rows, c, generator=g, dtype=torch.float64)
    o.backward(dz)
    yd = y.float().to(dev)
    rmd, rvd = rm.float().to(dev), rv.float().to(dev)
    mean, inv, scale, shift = ops.bn_fwd_train(yd, gamma.float().to(dev), beta.float().to(dev),
                                               rmd, rvd, 0.1, 1e-5)
    z = ops.bn_apply(yd, scale, shift, r.float().to(dev) if res else None, relu)
    assert rel_err(z, o) < 3e-6
    assert rel_err(rmd, rm_ref) < 1e-6 and rel_err(rvd, rv_ref) < 1e-6
    dy, dres, dgm, dbt = ops.bn_bwd(dz.float().to(dev), yd, z, mean, inv, gamma.float().to(dev),
                                    relu, want_dres=res)
    assert rel_err(dy, yr.grad) < 1e-5
    assert rel_err(dgm, gr.grad) < 1e-5
    assert rel_err(dbt, br.grad) < 1e-5
    if res:
        # dres aliasing dz: masked gradient written in place, same dy / dres / dgamma / dbeta
        dzi = dz.float().to(dev)
        dy3, dres3, dgm3, dbt3 = ops.bn_bwd(dzi, yd, z, mean, inv, gamma.float().to(dev), relu,
                                            want_dres=True, dres_out=dzi)
        assert dres3.data_ptr() == dzi.data_ptr()
        assert torch.equal(dres3, dres) and torch.equal(dy3, dy)
        assert torch.equal(dgm3, dgm) and torch.equal(dbt3, dbt)
    if relu and not res:
        # mask recomputed from y*scale+shift instead of reading z: bit-identical results
        dy2, _, dgm2, dbt2 = ops.bn_bwd(dz.float().to(dev), yd, None, mean, inv,
                                        gamma.float().to(dev), relu, scale=scale, shift=shift)
        assert torch.equal(dy2, dy) and torch.equal(dgm2, dgm) and torch.equal(dbt2, dbt)


def test_pools(dev):
    g = torch.Generator().manual_seed(3)
    x = torch.relu(torch.randn(2, 64, 112, 112, generator=g)).double()  # fp32-representable
    xr = x.clone().requires_grad_(True)
    yr = F.max_pool2d(xr, 3, 2, 1)
    dy = torch.randn(yr.shape, generator=g, dtype=torch.float64)
    yr.backward(dy)
    xd = x.float().permute(0, 2, 3, 1).contiguous().to(dev)
    y, am = ops.maxpool_fwd(xd)
    assert rel_err(y.permute(0, 3, 1, 2), yr) == 0.0
    dx = ops.maxpool_bwd(dy.float().permute(0, 2, 3, 1).contiguous().to(dev), am, (112, 112))
    assert rel_err(dx.permute(0, 3, 1, 2), xr.grad) < 1e-6
    x = torch.randn(3, 2048, 7, 7, generator=g, dtype=torch.float64)
    xd = x.float().permute(0, 2, 3, 1).contiguous().to(dev)
    y = ops.avgpool_fwd(xd)
    assert rel_err(y, x.mean((2, 3))) < 1e-6
    dx = ops.avgpool_bwd(y, (7, 7))
    assert rel_err(dx[:, 3, 4, :], x.mean((2, 3)) / 49) < 1e-6


def test_lstm_matches_torch(dev):
    from tmrnet_amd.lstm import LSTM
    torch.manual_seed(0)
    B, T, I, H = 3, 5, 64, 32
    ref = torch.nn.LSTM(I, H, batch_first=True).double()
    m = LSTM(I, H).to(dev)
    m.load_state_dict({k: v.float() for k, v in ref.state_dict().items()})
    x = torch.randn(B, T, I, dtype=torch.float64)
    dy = torch.randn(B, T, H, dtype=torch.float64)
    xr = x.clone().requires_grad_(True)
    yr, _ = ref(xr)
    yr.backward(dy)
    xd = x.float().to(dev).requires_grad_(True)
    y, (hn, cn) = m(xd)
    assert rel_err(y, yr) < 2e-6
    y.backward(dy.float().to(dev))
    assert rel_err(xd.grad, xr.grad) < 1e-5
    for (n1, p1), (n2, p2) in zip(m.named_parameters(), ref.named_parameters()):
        assert n1 == n2
        assert rel_err(p1.grad, p2.grad) < 1e-5, n1


def test_crop_normalize_matches_oracle(dev):
    from oracle.tmrnet_ref import crop_normalize_ref
    g = torch.Generator().manual_seed(1)
    fr = torch.randint(0, 256, (6, 250, 250, 3), generator=g, dtype=torch.uint8)
    off = torch.randint(0, 27, (2, 2), generator=g, dtype=torch.int32)
    ref = crop_normalize_ref(fr, off, 3)
    out = ops.crop_normalize(fr.to(dev), off.to(dev), 3)
    assert torch.equal(out[..., :3].permute(0, 3, 1, 2).cpu(), ref)   # bit-exact
    assert out[..., 3].abs().max().item() == 0.0


def test_ce_sum(dev):
    g = torch.Generator().manual_seed(5)
    x = torch.randn(64, 7, generator=g, dtype=torch.float64)
    y = torch.randint(0, 7, (64,), generator=g)
    w = torch.rand(7, generator=g, dtype=torch.float64) + 0.5
    for wt in (None, w):
        xr = x.clone().requires_grad_(True)
        lr = F.cross_entropy(xr, y, weight=wt, reduction="sum")
        lr.backward()
        loss, dl, preds = ops.ce_sum(x.float().to(dev), y.to(dev),
                                     wt.float().to(dev) if wt is not None else None)
        assert abs(loss.item() - lr.item()) / abs(lr.item()) < 1e-6
        assert rel_err(dl, xr.grad) < 1e-6
        assert torch.equal(preds.cpu(), x.float().argmax(1))


def test_sgd_matches_torch(dev):
    g = torch.Generator().manual_seed(9)
    p0 = torch.randn(1000, generator=g)
    grads = [torch.randn(1000, generator=g) for _ in range(3)]
    pr = p0.clone().requires_grad_(True)
    opt = torch.optim.SGD([pr], lr=0.1, momentum=0.9, weight_decay=5e-4)
    from tmrnet_amd.optim import SGD
    pd = p0.to(dev).requires_grad_(True)
    opt2 = SGD([pd], lr=0.1, momentum=0.9, weight_decay=5e-4)
    for gr in grads:
        pr.grad = gr.clone()
        opt.step()
        pd.grad = gr.to(dev)
        opt2.step()
    assert rel_err(pd, pr) < 1e-6


def test_lfb_index_and_gather_golden(dev):
    import os
    for name in ("tiny", "ragged", "c2", "c5"):
        z = np.load(os.path.join(os.path.dirname(__file__), "golden", "lfb_index_%s.npz" % name))
        starts = torch.from_numpy(z["starts"]).to(dev)
        q = torch.from_numpy(z["query"]).to(dev)
        rows = ops.lfb_index(starts, q, int(z["L"]))
        assert np.array_equal(rows.cpu().numpy(), z["table"]), name
    bank = torch.randn(50, 512, device=dev)
    rows = torch.randint(0, 50, (4, 7), device=dev, dtype=torch.int32)
    out = ops.lfb_gather(bank, rows)
    assert torch.equal(out, bank[rows.long()])


@pytest.mark.parametrize("case", [(2, 16, 16, 64, 64, 1, 1, 0), (3, 14, 14, 128, 256, 3, 2, 1),
                                  (1, 28, 28, 3, 64, 7, 2, 3), (5, 7, 7, 512, 2048, 1, 1, 0)])
def test_conv_fused_bn_stats(dev, case):
    """conv epilogue BN partials + tmr_bn_finalize == torch batch_norm statistics."""
    n, h, w, cin, cout, r, st, pad = case
    g = torch.Generator().manual_seed(11)
    x = torch.relu(torch.randn(n, cin, h, w, generator=g)) + 0.5   # non-zero-mean input
    wt = torch.randn(cout, cin, r, r, generator=g) / np.sqrt(cin * r * r)
    cs = 4 if cin == 3 else cin
    x4 = ops.nchw_to_nhwc(x.to(dev), cpad=cs)
    wk = ops.weight_to_krsc(wt.to(dev).contiguous(), cpad=cs)
    y, stats, nparts = ops.conv_fwd_bnstats(x4, wk, st, pad, c_real=cin)
    y_ref = ops.conv_fwd(x4, wk, st, pad)
    assert torch.equal(y, y_ref)
    yd = y_ref.double().view(-1, cout).cpu()
    gamma = torch.rand(cout, generator=g) + 0.5
    beta = torch.randn(cout, generator=g)
    rm, rv = torch.zeros(cout), torch.ones(cout)
    rmd, rvd = rm.to(dev), rv.to(dev)
    mean, inv, scale, shift = ops.bn_finalize(stats, nparts, gamma.to(dev), beta.to(dev), rmd, rvd,
                                              0.1, 1e-5)
    assert rel_err(mean, yd.mean(0)) < 1e-6
    var = yd.var(0, unbiased=False)
    assert rel_err(inv, 1 / torch.sqrt(var + 1e-5)) < 1e-5
    assert rel_err(rvd, 0.9 + 0.1 * yd.var(0, unbiased=True)) < 1e-6


@pytest.mark.parametrize("case", [(5, 14, 14, 64, 128, 3, 2, 1), (4, 9, 9, 256, 64, 1, 1, 0),
                                  (3, 28, 28, 3, 64, 7, 2, 3)])
def test_conv_frame_chunks(dev, case):
    """Batches whose operands exceed 2 GiB run as consecutive frame chunks
    (tmr_conv_desc.max_frames): forced here at 2 frames per launch, the results equal the
    single-launch ones (fwd, fused BN partials, dgrad bit-exact; wgrad to summation order)."""
    n, h, w, cin, cout, r, st, pad = case
    g = torch.Generator().manual_seed(sum(case))
    cs = 4 if cin == 3 else cin
    x = torch.randn(n, h, w, cs, generator=g)
    if cin == 3:
        x[..., 3] = 0
    x = x.to(dev)
    wk = torch.randn(cout, r, r, cs, generator=g).to(dev) / (cin * r * r) ** 0.5
    y1 = ops.conv_fwd(x, wk, st, pad)
    ys, stats, nparts = ops.conv_fwd_bnstats(x, wk, st, pad, c_real=cin)
    dy = torch.randn(y1.shape, generator=g).to(dev)
    dx1 = ops.conv_dgrad(dy, wk, (h, w), st, pad) if cin != 3 else None
    dw1 = ops.conv_wgrad(x, dy, r, r, st, pad, c_real=cin)
    old = ops.MAX_FRAMES
    try:
        ops.MAX_FRAMES = 2
        y2 = ops.conv_fwd(x, wk, st, pad)
        ys2, stats2, nparts2 = ops.conv_fwd_bnstats(x, wk, st, pad, c_real=cin)
        dx2 = ops.conv_dgrad(dy, wk, (h, w), st, pad) if cin != 3 else None
        dw2 = ops.conv_wgrad(x, dy, r, r, st, pad, c_real=cin)
    finally:
        ops.MAX_FRAMES = old
    assert torch.equal(y1, y2) and torch.equal(ys, ys2)
    assert nparts2 >= nparts
    if dx1 is not None:
        assert torch.equal(dx1, dx2)
    assert rel_err(dw2, dw1) < 1e-6
    # BN statistics from the chunked partials
    c = cout
    outs = []
    for st_, np_ in ((stats, nparts), (stats2, nparts2)):
        outs.append(ops.bn_finalize(st_, np_, torch.ones(c, device=dev), torch.zeros(c, device=dev),
                                    torch.zeros(c, device=dev), torch.ones(c, device=dev), 0.1, 1e-5))
    assert rel_err(outs[1][0], outs[0][0]) < 1e-5 and rel_err(outs[1][1], outs[0][1]) < 1e-5


@pytest.mark.parametrize("case", [(2, 16, 16, 64, 256, 1, 1, 0, True, True),
                                  (3, 14, 14, 128, 128, 3, 2, 1, False, True),
                                  (2, 9, 9, 256, 64, 1, 1, 0, False, False),
                                  (1, 28, 28, 3, 64, 7, 2, 3, False, True)])
def test_conv_fused_eval_bn(dev, case):
    """tmr_conv2d_fwd_fused (eval BN + residual + ReLU in the epilogue) is bit-identical to
    tmr_conv2d_fwd followed by tmr_bn_apply (the same fmaf/add/max sequence)."""
    n, h, w, cin, cout, r, st, pad, res, relu = case
    g = torch.Generator().manual_seed(7)
    cs = 4 if cin == 3 else cin
    x = torch.zeros(n, h, w, cs)
    x[..., :cin] = torch.randn(n, h, w, cin, generator=g)
    wt = torch.randn(cout, cin, r, r, generator=g) / np.sqrt(cin * r * r)
    x = x.to(dev)
    wk = ops.weight_to_krsc(wt.to(dev), cpad=cs)
    scale = (torch.rand(cout, generator=g) + 0.5).to(dev)
    shift = torch.randn(cout, generator=g).to(dev)
    y = ops.conv_fwd(x, wk, st, pad, c_real=cin)
    resid = torch.randn(y.shape, generator=g).to(dev) if res else None
    z_ref = ops.bn_apply(y, scale, shift, resid, relu)
    z = ops.conv_fwd_fused(x, wk, st, pad, scale, shift, resid, relu, c_real=cin)
    torch.cuda.synchronize()
    assert torch.equal(z, z_ref)
    # and against float64 torch: conv -> affine -> (+res) -> relu
    xd = x[..., :cin].permute(0, 3, 1, 2).double().cpu()
    yd = F.conv2d(xd, wt.double(), stride=st, padding=pad).permute(0, 2, 3, 1)
    zd = yd * scale.double().cpu() + shift.double().cpu()
    if res:
        zd = zd + resid.double().cpu()
    if relu:
        zd = zd.clamp_min(0)
    assert rel_err(z, zd) < 1e-5


def test_sgd_optimizer_multi_tensor_matches_torch(dev):
    """tmrnet_amd.SGD (one tmr_sgd_step_multi launch per step) vs torch.optim.SGD over three
    steps: groups with different lr / momentum / dampening / nesterov / weight decay, tensors
    straddling the 8192-element chunk, a parameter without grad, an lr change mid-run."""
    import tmrnet_amd
    g = torch.Generator().manual_seed(0)
    shapes = [(3,), (8192,), (8193,), (70, 300), (1,), (5, 7)]
    base = [torch.randn(s, generator=g) for s in shapes]
    ours = [torch.nn.Parameter(b.clone().to(dev)) for b in base]
    ref = [torch.nn.Parameter(b.clone().double()) for b in base]

    def groups(ps):
        return [{"params": ps[0:2]},
                {"params": ps[2:4], "lr": 0.05, "nesterov": True, "momentum": 0.8,
                 "dampening": 0.0},
                {"params": ps[4:5], "momentum": 0.0},
                {"params": ps[5:6], "dampening": 0.3, "weight_decay": 0.0}]
    o1 = tmrnet_amd.SGD(groups(ours), lr=0.01, momentum=0.9, weight_decay=5e-4)
    o2 = torch.optim.SGD(groups(ref), lr=0.01, momentum=0.9, weight_decay=5e-4)
    for step in range(3):
        if step == 2:
            for a, b in zip(o1.param_groups, o2.param_groups):
                a["lr"] *= 0.1; b["lr"] *= 0.1
        for i, (a, b) in enumerate(zip(ours, ref)):
            if i == 4 and step == 1:
                a.grad = None; b.grad = None        # no grad this step: untouched
                continue
            gr = torch.randn(a.shape, generator=g)
            a.grad = gr.to(dev) if i != 3 else gr.t().contiguous().t().to(dev)
            b.grad = gr.double()
        o1.step(); o2.step()
    torch.cuda.synchronize()
    for a, b in zip(ours, ref):
        assert rel_err(a, b) < 1e-6


def test_adam_optimizer_multi_tensor_matches_torch(dev):
    """tmrnet_amd.Adam (one tmr_adam_step_multi launch per step; the reference's -o 1 optimizer,
    train_only_non-local_pretrained.py:644-645) vs torch.optim.Adam in float64 over five steps:
    groups with different lr / betas / eps / weight decay, chunk-straddling tensors, a parameter
    without grad in one step, an lr change; state_dict keys interchange with torch's."""
    import tmrnet_amd
    g = torch.Generator().manual_seed(1)
    shapes = [(3,), (8192,), (8193,), (70, 300), (1,), (5, 7)]
    base = [torch.randn(s, generator=g) for s in shapes]
    ours = [torch.nn.Parameter(b.clone().to(dev)) for b in base]
    ref = [torch.nn.Parameter(b.clone().double()) for b in base]

    def groups(ps):
        return [{"params": ps[0:2]},
                {"params": ps[2:4], "lr": 3e-3, "betas": (0.8, 0.99)},
                {"params": ps[4:5], "weight_decay": 1e-2},
                {"params": ps[5:6], "eps": 1e-6}]
    o1 = tmrnet_amd.Adam(groups(ours), lr=1e-3)
    o2 = torch.optim.Adam(groups(ref), lr=1e-3)
    for step in range(5):
        if step == 3:
            for a, b in zip(o1.param_groups, o2.param_groups):
                a["lr"] *= 0.5; b["lr"] *= 0.5
        for i, (a, b) in enumerate(zip(ours, ref)):
            if i == 4 and step == 1:
                a.grad = None; b.grad = None
                continue
            gr = torch.randn(a.shape, generator=g)
            a.grad = gr.to(dev)
            b.grad = gr.double()
        o1.step(); o2.step()
    torch.cuda.synchronize()
    for a, b in zip(ours, ref):
        assert rel_err(a, b) < 2e-6
    sd = o1.state_dict()
    assert set(sd["state"][0]) == {"step", "exp_avg", "exp_avg_sq"}
    assert float(sd["state"][4]["step"]) == 4.0


@pytest.mark.parametrize("case", [
    # n, h, w, cin(dx channels), cout(dy channels), r, stride, pad, mask, beta
    (3, 14, 14, 64, 256, 1, 1, 0, 2, 0.0),     # conv3 dgrad -> conv2's BN (mask from y)
    (2, 14, 14, 128, 128, 3, 2, 1, 2, 0.0),    # strided 3x3: four parity-class launches
    (3, 12, 12, 256, 64, 1, 1, 0, 1, 1.0),     # conv1 dgrad += identity grad -> prev block (z)
    (2, 14, 14, 256, 512, 1, 2, 0, 1, 1.0),    # strided 1x1 downsample: tap-less classes
    (2, 9, 9, 64, 64, 3, 1, 1, 0, 0.0),        # no ReLU
])
@pytest.mark.parametrize("wtr", [False, True])
def test_conv_dgrad_fused_bn_backward(dev, case, wtr):
    """conv_dgrad_bnbwd + bn_bwd_parts == conv_dgrad followed by bn_bwd (the separate passes):
    the masked dx bit-exactly, dy / dgamma / dbeta to fp32 summation-order tolerance.  wtr: both
    on the fp32 LDS-DMA engine (transposed fp32 weights; its LDS-staged fused epilogue)."""
    n, h, w, cin, cout, r, st, pad, mask, beta = case
    g = torch.Generator().manual_seed(11)
    ho = (h + 2 * pad - r) // st + 1
    wo = (w + 2 * pad - r) // st + 1
    dy = torch.randn(n, ho, wo, cout, generator=g).to(dev)
    wt = (torch.randn(cout, cin, r, r, generator=g) / np.sqrt(cout * r * r)).to(dev)
    wk = ops.weight_to_crsk(wt, bf16=False) if wtr else ops.weight_to_krsc(wt)
    y = torch.randn(n, h, w, cin, generator=g).to(dev)
    mean = y.view(-1, cin).mean(0)
    inv = 1.0 / (y.view(-1, cin).var(0, unbiased=False) + 1e-5).sqrt()
    gamma = (torch.rand(cin, generator=g) + 0.5).to(dev)
    scale = gamma * inv
    shift = (torch.randn(cin, generator=g) * 0.1).to(dev) - mean * scale
    res = torch.randn(n, h, w, cin, generator=g).to(dev)
    z = torch.relu(y * scale + shift + res) if mask == 1 else None
    old = torch.randn(n, h, w, cin, generator=g).to(dev)
    # separate passes
    dz = ops.conv_dgrad(dy, wk, (h, w), st, pad, out=old.clone(), beta=beta, wt=wtr)
    dy_ref, dres_ref, dg_ref, db_ref = ops.bn_bwd(dz, y, z, mean, inv, gamma, mask != 0,
                                                  want_dres=True, scale=scale, shift=shift)
    # fused
    dzf, parts, npart = ops.conv_dgrad_bnbwd(dy, wk, (h, w), st, pad, y, mean, mask, z=z,
                                              scale=scale, shift=shift, out=old.clone(), beta=beta,
                                              wt=wtr)
    dyf, dgf, dbf = ops.bn_bwd_parts(dzf, y, parts, npart, mean, inv, gamma)
    if wtr and mask == 1:
        # the ReLU mask as bits (mask 3; bn_apply_bits): the same masked gradient and partials
        _, bits = ops.bn_apply_bits(y, scale, shift, res)
        dzb, partsb, npb = ops.conv_dgrad_bnbwd(dy, wk, (h, w), st, pad, y, mean, 3, z=bits,
                                                out=old.clone(), beta=beta, wt=True)
        torch.cuda.synchronize()
        assert torch.equal(dzb, dzf) and torch.equal(partsb, parts) and npb == npart
    torch.cuda.synchronize()
    assert torch.equal(dzf, dres_ref)          # the masked BN-output gradient
    assert rel_err(dyf, dy_ref) < 1e-5
    assert rel_err(dgf, dg_ref) < 1e-5 and rel_err(dbf, db_ref) < 1e-5


@pytest.mark.parametrize("wtr", [False, True])
def test_conv_dgrad_fused_bn_backward_frame_chunks(dev, wtr):
    """Partials stay in launch order across frame chunks (max_frames) and parity classes."""
    g = torch.Generator().manual_seed(12)
    n, h, w, cin, cout = 5, 14, 14, 128, 128
    dy = torch.randn(n, 7, 7, cout, generator=g).to(dev)
    w0 = (torch.randn(cout, cin, 3, 3, generator=g) * 0.05).to(dev)
    wk = ops.weight_to_crsk(w0, bf16=False) if wtr else ops.weight_to_krsc(w0)
    y = torch.randn(n, h, w, cin, generator=g).to(dev)
    mean = y.view(-1, cin).mean(0)
    inv = 1.0 / (y.view(-1, cin).var(0, unbiased=False) + 1e-5).sqrt()
    gamma = torch.ones(cin, device=dev)
    sc, sh = gamma * inv, -mean * inv
    a = ops.conv_dgrad_bnbwd(dy, wk, (h, w), 2, 1, y, mean, 2, scale=sc, shift=sh, wt=wtr)
    old = ops.MAX_FRAMES
    try:
        ops.MAX_FRAMES = 2
        b = ops.conv_dgrad_bnbwd(dy, wk, (h, w), 2, 1, y, mean, 2, scale=sc, shift=sh, wt=wtr)
    finally:
        ops.MAX_FRAMES = old
    ya = ops.bn_bwd_parts(a[0], y, a[1], a[2], mean, inv, gamma)[0]
    yb = ops.bn_bwd_parts(b[0], y, b[1], b[2], mean, inv, gamma)[0]
    torch.cuda.synchronize()
    assert b[2] > a[2]
    assert torch.equal(a[0], b[0]) and rel_err(yb, ya) < 1e-6


@pytest.mark.parametrize("case", [
    # n, h, w, cin (dx channels), cout (dy channels), r, pad
    (3, 14, 14, 128, 128, 3, 1),   # the layer3.0 conv2 geometry: classes of 1 / 2 / 2 / 4 taps
    (2, 7, 9, 64, 128, 3, 1),      # odd sizes: classes of unequal tile counts
    (2, 14, 14, 256, 512, 1, 0),   # 1x1 downsample: three tap-less (epilogue-only) classes
    (5, 13, 13, 64, 64, 3, 1),     # 64-channel dy (the 256x64 / 64x64 tiles)
])
@pytest.mark.parametrize("math", ["fp32", "bf16"])
def test_dgrad_parity_classes_one_launch(dev, case, math):
    """A stride-2 dgrad runs its four stride-parity classes as one launch (gemm16_par_kernel,
    round 5): bit-identical to one launch per class (TMR_IO_CLASSES) -- the plain dgrad, the fused
    BN-backward dgrad (masks 1 / 2 / 3; accumulating into an old dx) and its partial rows."""
    n, h, w, cin, cout, r, pad = case
    g = torch.Generator().manual_seed(31)
    ho = (h + 2 * pad - r) // 2 + 1
    wo = (w + 2 * pad - r) // 2 + 1
    b16 = math == "bf16"
    dt = torch.bfloat16 if b16 else torch.float32
    dy = torch.randn(n, ho, wo, cout, generator=g).to(dev).to(dt)
    w0 = (torch.randn(cout, cin, r, r, generator=g) / np.sqrt(cout * r * r)).to(dev)
    wct = ops.weight_to_crsk(w0, bf16=b16)
    y = torch.randn(n, h, w, cin, generator=g).to(dev).to(dt)
    ye = y.float()
    mean = ye.view(-1, cin).mean(0)
    inv = 1.0 / (ye.view(-1, cin).var(0, unbiased=False) + 1e-5).sqrt()
    sc = (torch.rand(cin, generator=g) + 0.5).to(dev) * inv
    sh = (torch.randn(cin, generator=g) * 0.1).to(dev) - mean * sc
    z = torch.relu(ye + torch.randn(n, h, w, cin, generator=g).to(dev) * 0.5).to(dt)
    bits = _pack_bits((z.float() > 0).cpu()).to(dev)
    old = torch.randn(n, h, w, cin, generator=g).to(dev)

    def run():
        out = [ops.conv_dgrad(dy, wct, (h, w), 2, pad, math=math, wt=True),
               ops.conv_dgrad(dy, wct, (h, w), 2, pad, out=old.clone(), beta=1.0, math=math, wt=True)]
        kw = dict(math=math, wt=True)
        out += ops.conv_dgrad_bnbwd(dy, wct, (h, w), 2, pad, y, mean, 2, scale=sc, shift=sh, **kw)[:2]
        out += ops.conv_dgrad_bnbwd(dy, wct, (h, w), 2, pad, y, mean, 1, z=z, out=old.clone(),
                                    beta=1.0, **kw)[:2]
        out += ops.conv_dgrad_bnbwd(dy, wct, (h, w), 2, pad, y, mean, 3, z=bits, out=old.clone(),
                                    beta=1.0, **kw)[:2]
        if b16:   # the bf16 step's g16 forms: non-residual (mask 2) and residual (old fp32 -> bf16)
            out += ops.conv_dgrad_bnbwd(dy, wct, (h, w), 2, pad, y, mean, 2, scale=sc, shift=sh,
                                        g16=True, **kw)[:2]
            out += ops.conv_dgrad_bnbwd(dy, wct, (h, w), 2, pad, y, mean, 1, z=z, beta=1.0, g16=True,
                                        old=old, **kw)[:2]
        return out

    one = run()
    with ops.dgrad_class_launches():
        per = run()
    torch.cuda.synchronize()
    for i, (u, v) in enumerate(zip(one, per)):
        assert u.shape == v.shape and torch.equal(u, v), i


def test_bn_apply_fused_consumers(dev):
    """The two BN applications folded into their consumers are bit-identical to the unfused
    sequence: bn_apply2 (Bottleneck bn3 + downsample-branch BN + ReLU, torchvision
    Bottleneck.forward) and maxpool_fwd_bn (share.bn1 -> relu -> maxpool, :205-207)."""
    g = torch.Generator().manual_seed(11)
    rows, c = 3 * 14 * 14, 256
    y = torch.randn(rows, c, generator=g).to(dev)
    yr = torch.randn(rows, c, generator=g).to(dev)
    sc, sh = torch.randn(c, generator=g).to(dev), torch.randn(c, generator=g).to(dev)
    rs, rf = torch.randn(c, generator=g).to(dev), torch.randn(c, generator=g).to(dev)
    for relu in (True, False):
        r = ops.bn_apply(yr, rs, rf, None, False)
        ref = ops.bn_apply(y, sc, sh, r, relu)
        assert torch.equal(ops.bn_apply2(y, sc, sh, yr, rs, rf, relu), ref)
    x = torch.randn(2, 37, 29, 64, generator=g).to(dev)        # odd sizes: padded windows
    s0, t0 = torch.randn(64, generator=g).to(dev), torch.randn(64, generator=g).to(dev)
    p_ref, am_ref = ops.maxpool_fwd(ops.bn_apply(x.view(-1, 64), s0, t0, None, True).view_as(x))
    p, am = ops.maxpool_fwd_bn(x, s0, t0)
    assert torch.equal(p, p_ref) and torch.equal(am, am_ref)


def test_stem_bwd_maxpool_fused(dev):
    """bn_bwd_maxpool (share.maxpool -> relu -> bn1 backward in two passes over y, dz gathered)
    against maxpool_bwd followed by bn_bwd with the mask recomputed from y: same arithmetic per
    element, partial sums in a different row order -> equal to fp32 rounding."""
    g = torch.Generator().manual_seed(12)
    n, h, w, c = 3, 37, 29, 64
    y = torch.randn(n, h, w, c, generator=g).to(dev)
    gamma = (torch.rand(c, generator=g) + 0.5).to(dev)
    beta = torch.randn(c, generator=g).to(dev)
    rm, rv = torch.zeros(c, device=dev), torch.ones(c, device=dev)
    mean, inv, scale, shift = ops.bn_fwd_train(y.view(-1, c), gamma, beta, rm, rv, 0.1, 1e-5)
    p, am = ops.maxpool_fwd_bn(y, scale, shift)
    dp = torch.randn(p.shape, generator=g).to(dev)
    dz = ops.maxpool_bwd(dp, am, (h, w))
    dy_ref, _, dg_ref, db_ref = ops.bn_bwd(dz.view(-1, c), y.view(-1, c), None, mean, inv, gamma,
                                           True, scale=scale, shift=shift)
    dy, dg, db = ops.bn_bwd_maxpool(dp, am, y, scale, shift, mean, inv, gamma)
    assert rel_err(dy.view(-1, c), dy_ref) < 1e-5
    assert rel_err(dg, dg_ref) < 1e-5 and rel_err(db, db_ref) < 1e-5


@pytest.mark.parametrize("engine", ["lds_dma", "register_staged"])
def test_bn_fold_bit_identical(dev, engine):
    """Train step with the BatchNorm folded into the conv loaders (tmr_conv_prologue: BN+ReLU of
    units 1-2 on the X operand, the BN backward on every dY operand) against the explicit passes
    (tmr_bn_apply / tmr_bn_bwd_parts / tmr_bn_bwd): same operand values by construction, same
    GEMM arithmetic -> logits, every gradient and the running statistics bit-identical.  Both
    sides on the fp32 LDS-DMA engine (prologues applied in LDS, gemm16_kernel PRO), or both on
    the register-staged engine (TMR_GEMM32=0, read per launch).  The prologues are a retired A/B
    experiment: this runs against the A/B build (make PROLOGUES=1; TMR_LIB_PATH=
    tmrnet_amd/libtmr_pro.so) and is skipped on the product library."""
    import os
    import tmrnet_amd
    from tmrnet_amd import trunk, _lib
    if not _lib.has_prologues():
        pytest.skip("operand prologues: A/B build only (make PROLOGUES=1, TMR_LIB_PATH)")
    B, T, L = 2, 5, 7
    g = torch.Generator().manual_seed(3)
    frames = torch.randint(0, 256, (B * T, 250, 250, 3), generator=g, dtype=torch.uint8).to(dev)
    off = torch.randint(0, 27, (B, 2), generator=g, dtype=torch.int32).to(dev)
    lt = (torch.rand(B, L, 512, generator=g) * 2 - 1).to(dev)
    labels = torch.randint(0, 7, (B,), generator=g).to(dev)
    res = {}
    saved = trunk.FOLD_BN
    saved_dma, saved_env = trunk.DMA32, os.environ.get("TMR_GEMM32")
    if engine == "register_staged":
        trunk.DMA32 = False
        os.environ["TMR_GEMM32"] = "0"
    try:
        for fold in (True, False):
            trunk.FOLD_BN = fold
            torch.manual_seed(0)
            m = tmrnet_amd.resnet_lstm(seq_len=T).to(dev).train()
            m.nl_block.forced_mask = torch.ones(B, 512, device=dev)
            m.forced_head_mask = torch.ones(B, 512, device=dev)
            x4 = ops.crop_normalize(frames, off, T)
            out = m(x4, lt)
            tmrnet_amd.CrossEntropyLoss(size_average=False)(out, labels).backward()
            torch.cuda.synchronize()
            res[fold] = (out.detach().clone(), {n: p.grad.clone() for n, p in m.named_parameters()},
                         {n: b.clone() for n, b in m.named_buffers()})
    finally:
        trunk.FOLD_BN = saved
        trunk.DMA32 = saved_dma
        if saved_env is None:
            os.environ.pop("TMR_GEMM32", None)
        else:
            os.environ["TMR_GEMM32"] = saved_env
    assert torch.equal(res[True][0], res[False][0])
    for n in res[True][1]:
        assert torch.equal(res[True][1][n], res[False][1][n]), n
    for n in res[True][2]:
        assert torch.equal(res[True][2][n], res[False][2][n]), n


@pytest.mark.parametrize("folds", [("FOLD16",), ("FOLD16DY",), ("FOLD16", "FOLD16DY")])
def test_bn_fold16_bit_identical(dev, folds):
    """The bf16 forms (round 5): under the bf16-activation step (FOLD16) the relu(bn1) /
    relu(bn2) outputs are never written -- conv2 / conv3 read the bf16 pre-BN y through the bf16
    X-operand prologue of the LDS-DMA engine, forward and wgrad views -- and (FOLD16DY) no
    BatchNorm backward writes dy -- every conv whose BN output gradient g is bf16 reads g and y
    through the bf16 dY-operand prologue, dgrad (fused BN-backward epilogues, the accumulating
    conv1 dgrads included) and wgrad views -- against the explicit bn_apply8_a16 /
    bn_bwd_apply8_a16 passes: the same rounded operand values by construction, so logits, every
    gradient and the running statistics bit-identical.  A/B build only (make PROLOGUES=1;
    TMR_LIB_PATH=tmrnet_amd/libtmr_pro.so), skipped on the product library."""
    import tmrnet_amd
    from tmrnet_amd import trunk, _lib
    if not _lib.has_prologues():
        pytest.skip("operand prologues: A/B build only (make PROLOGUES=1, TMR_LIB_PATH)")
    B, T, L = 2, 5, 7
    g = torch.Generator().manual_seed(4)
    frames = torch.randint(0, 256, (B * T, 250, 250, 3), generator=g, dtype=torch.uint8).to(dev)
    off = torch.randint(0, 27, (B, 2), generator=g, dtype=torch.int32).to(dev)
    lt = (torch.rand(B, L, 512, generator=g) * 2 - 1).to(dev)
    labels = torch.randint(0, 7, (B,), generator=g).to(dev)
    res = {}
    saved = {f: getattr(trunk, f) for f in folds}
    # the dY prologue really runs: count the coefficient-only BN backwards it takes
    ncoef = [0]
    wrapped = {n: getattr(ops, n) for n in ("bn_bwd_coefs", "bn_bwd_coefs_g16")}

    def counting(fn):
        def f(*a, **k):
            ncoef[0] += 1
            return fn(*a, **k)
        return f
    try:
        for n, fn in wrapped.items():
            setattr(ops, n, counting(fn))
        for fold in (True, False):
            for f in folds:
                setattr(trunk, f, fold)
            ncoef[0] = 0
            torch.manual_seed(0)
            m = tmrnet_amd.resnet_lstm(seq_len=T, precision="bf16").to(dev).train()
            m.nl_block.forced_mask = torch.ones(B, 512, device=dev)
            m.forced_head_mask = torch.ones(B, 512, device=dev)
            x4 = ops.crop_normalize(frames, off, T)
            out = m(x4, lt)
            tmrnet_amd.CrossEntropyLoss(size_average=False)(out, labels).backward()
            torch.cuda.synchronize()
            res[fold] = (out.detach().clone(), {n: p.grad.clone() for n, p in m.named_parameters()},
                         {n: b.clone() for n, b in m.named_buffers()})
            # ResNet-50: bn1 x 16, bn2 x 13 (layer1's conv2 runs direct), bn3 x 15 (not the last
            # block's: its gradient is fp32), downsample x 4
            assert ncoef[0] == (48 if fold and "FOLD16DY" in folds else 0), ncoef[0]
    finally:
        for f, v in saved.items():
            setattr(trunk, f, v)
        for n, fn in wrapped.items():
            setattr(ops, n, fn)
    assert torch.equal(res[True][0], res[False][0])
    for n in res[True][1]:
        assert torch.equal(res[True][1][n], res[False][1][n]), n
    for n in res[True][2]:
        assert torch.equal(res[True][2][n], res[False][2][n]), n


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("rows,c", [(3 * 56 * 56, 256), (1001, 8), (77, 2048)])
def test_bn_bwd_parts_ds_op(dev, dtype, rows, c):
    """tmr_bn_bwd_parts_ds against the two calls it replaces (bn_bwd_parts of bn3 from partials,
    bn_bwd of the downsample BN): dy, dy_ds, dgamma and dbeta of both bit-identical (fp32: the
    fp32 passes; bf16: the _g16 passes), ragged row counts and 8 / 2048 channels."""
    g = torch.Generator().manual_seed(rows + c)
    mk = lambda s=1.0: (torch.randn(rows, c, generator=g) * s).to(dtype).to(dev)
    gr, y, yd = mk(0.1), mk(), mk()
    mean, inv = [torch.randn(c, generator=g).to(dev) for _ in range(2)]
    md, invd = [torch.randn(c, generator=g).to(dev) for _ in range(2)]
    inv, invd = inv.abs() + 0.5, invd.abs() + 0.5
    gam, gamd = [(torch.rand(c, generator=g) + 0.5).to(dev) for _ in range(2)]
    nparts = 37
    parts = torch.randn(nparts, c, 2, generator=g).to(dev)
    dy, dg, db, dyd, dgd, dbd = ops.bn_bwd_parts_ds(gr, y, parts, nparts, mean, inv, gam, yd, md,
                                                    invd, gamd)
    dy2, dg2, db2 = ops.bn_bwd_parts(gr, y, parts, nparts, mean, inv, gam)
    dyd2, _, dgd2, dbd2 = ops.bn_bwd(gr, yd, None, md, invd, gamd, relu=False)
    for a, b in ((dy, dy2), (dg, dg2), (db, db2), (dyd, dyd2), (dgd, dgd2), (dbd, dbd2)):
        assert a.dtype == b.dtype and torch.equal(a, b)


@pytest.mark.parametrize("precision,backbone", [("fp32", "resnet50"), ("bf16", "resnet50"),
                                                ("bf16", "resnest50"), ("fp32", "resnest50")])
def test_bn_bwd_ds_dual_bit_identical(dev, precision, backbone):
    """trunk.DS_DUAL (tmr_bn_bwd_parts_ds): the BatchNorm backward of each downsample block's bn3
    and downsample BN with one apply pass that reads the shared gradient once, against the two
    separate passes (tmr_bn_bwd_parts_x / _g16 and tmr_bn_bwd_x / tmr_bn_bwd_g16): logits, every
    gradient and the running statistics bit-identical, fp32 and bf16 steps of both trunks
    (ResNet-50 / ResNeSt-50: all four downsample blocks take it -- each one's g comes from the
    next block's fused dgrad)."""
    import tmrnet_amd
    from tmrnet_amd import trunk
    B, T, L = 2, 5, 7
    g = torch.Generator().manual_seed(5)
    frames = torch.randint(0, 256, (B * T, 250, 250, 3), generator=g, dtype=torch.uint8).to(dev)
    off = torch.randint(0, 27, (B, 2), generator=g, dtype=torch.int32).to(dev)
    lt = (torch.rand(B, L, 512, generator=g) * 2 - 1).to(dev)
    labels = torch.randint(0, 7, (B,), generator=g).to(dev)
    res, calls = {}, [0]
    saved, fn = trunk.DS_DUAL, ops.bn_bwd_parts_ds

    def counting(*a, **k):
        calls[0] += 1
        return fn(*a, **k)
    try:
        ops.bn_bwd_parts_ds = counting
        for dual in (True, False):
            trunk.DS_DUAL = dual
            calls[0] = 0
            torch.manual_seed(0)
            kw = {} if backbone == "resnet50" else {"time_conv": True, "backbone": backbone}
            m = tmrnet_amd.resnet_lstm(seq_len=T, precision=precision, **kw).to(dev).train()
            m.nl_block.forced_mask = torch.ones(B, 512, device=dev)
            m.forced_head_mask = torch.ones(B, 512, device=dev)
            x4 = ops.crop_normalize(frames, off, T)
            out = m(x4, lt)
            tmrnet_amd.CrossEntropyLoss(size_average=False)(out, labels).backward()
            torch.cuda.synchronize()
            res[dual] = (out.detach().clone(), {n: p.grad.clone() for n, p in m.named_parameters()},
                         {n: b.clone() for n, b in m.named_buffers()})
            assert calls[0] == (4 if dual else 0), calls[0]
    finally:
        trunk.DS_DUAL = saved
        ops.bn_bwd_parts_ds = fn
    assert torch.equal(res[True][0], res[False][0])
    for n in res[True][1]:
        assert torch.equal(res[True][1][n], res[False][1][n]), n
    for n in res[True][2]:
        assert torch.equal(res[True][2][n], res[False][2][n]), n


@pytest.mark.parametrize("precision,backbone", [("fp32", "resnet50"), ("bf16", "resnet50"),
                                                ("bf16", "resnest50")])
def test_weight_layout_sessions(dev, precision, backbone):
    """ops.layout_session: the trunk's weight layouts (KRSC / CRSK, fp32 / bf16, grouped) recorded
    on the first step and refreshed by one tmr_weight_layouts_multi launch on later steps --
    three SGD steps with sessions give bit-identical logits, gradients, weights and running
    statistics to three steps with per-conv conversions (the refresh must see every update)."""
    import tmrnet_amd
    B, T, L = 2, 5, 7
    g = torch.Generator().manual_seed(9)
    frames = torch.randint(0, 256, (B * T, 250, 250, 3), generator=g, dtype=torch.uint8).to(dev)
    off = torch.randint(0, 27, (B, 2), generator=g, dtype=torch.int32).to(dev)
    lt = (torch.rand(B, L, 512, generator=g) * 2 - 1).to(dev)
    labels = torch.randint(0, 7, (B,), generator=g).to(dev)
    res = {}
    saved = ops.LAYOUT_SESSIONS
    try:
        for on in (True, False):
            ops.LAYOUT_SESSIONS = on
            torch.manual_seed(0)
            kw = {} if backbone == "resnet50" else {"time_conv": True, "backbone": backbone}
            m = tmrnet_amd.resnet_lstm(seq_len=T, precision=precision, **kw).to(dev).train()
            m.nl_block.forced_mask = torch.ones(B, 512, device=dev)
            m.forced_head_mask = torch.ones(B, 512, device=dev)
            opt = tmrnet_amd.SGD(m.parameters(), lr=1e-3, momentum=0.9)
            outs = []
            for _ in range(3):
                opt.zero_grad(set_to_none=True)
                out = m(ops.crop_normalize(frames, off, T), lt)
                tmrnet_amd.CrossEntropyLoss(size_average=False)(out, labels).backward()
                opt.step()
                outs.append(out.detach().clone())
            torch.cuda.synchronize()
            res[on] = (outs, {n: p.detach().clone() for n, p in m.named_parameters()},
                       {n: b.clone() for n, b in m.named_buffers()})
    finally:
        ops.LAYOUT_SESSIONS = saved
    for a, b in zip(res[True][0], res[False][0]):
        assert torch.equal(a, b)
    for n in res[True][1]:
        assert torch.equal(res[True][1][n], res[False][1][n]), n
    for n in res[True][2]:
        assert torch.equal(res[True][2][n], res[False][2][n]), n


def _pack_bits(m):
    """(numel,) bool -> int32 words, element e = bit e % 32 of word e // 32."""
    m = m.reshape(-1).to(torch.int64)
    m = torch.cat([m, torch.zeros((-m.numel()) % 32, dtype=torch.int64)]).view(-1, 32)
    w = (m << torch.arange(32, dtype=torch.int64)).sum(1)
    return torch.where(w >= 2 ** 31, w - 2 ** 32, w).to(torch.int32)


@pytest.mark.parametrize("rows,c", [(1000, 256), (77, 64), (3, 8), (101, 12), (5001, 512)])
def test_bn_apply_relu_bits(dev, rows, c):
    """bn_apply_bits / bn_apply2_bits: z bit-identical to bn_apply / bn_apply2 (ReLU) and the
    bits are exactly (z > 0) packed 32 per word (ragged tails included)."""
    g = torch.Generator().manual_seed(rows + c)
    y = torch.randn(rows, c, generator=g).to(dev)
    res = torch.randn(rows, c, generator=g).to(dev)
    yr = torch.randn(rows, c, generator=g).to(dev)
    sc, sh = (torch.rand(c, generator=g) + 0.5).to(dev), torch.randn(c, generator=g).to(dev)
    rs, rf = (torch.rand(c, generator=g) + 0.5).to(dev), torch.randn(c, generator=g).to(dev)
    for resid in (res, None):
        z, bits = ops.bn_apply_bits(y, sc, sh, resid)
        zr = ops.bn_apply(y, sc, sh, resid, True)
        torch.cuda.synchronize()
        assert torch.equal(z, zr)
        assert torch.equal(bits.cpu(), _pack_bits((zr > 0).cpu()))
    z2, bits2 = ops.bn_apply2_bits(y, sc, sh, yr, rs, rf)
    z2r = ops.bn_apply2(y, sc, sh, yr, rs, rf, True)
    torch.cuda.synchronize()
    assert torch.equal(z2, z2r) and torch.equal(bits2.cpu(), _pack_bits((z2r > 0).cpu()))
    # the 8-wide forms (round 6; c % 8 == 0, 16-B aligned) against the 4-wide ones, which the
    # library takes for operands 8 bytes off a 16-B boundary: identical z and bits
    from tests.test_stem_pool8_gpu import _off8
    for resid in (res, None):
        z8, b8 = ops.bn_apply_bits(y, sc, sh, resid)
        z4, b4 = ops.bn_apply_bits(_off8(y), sc, sh, _off8(resid) if resid is not None else None)
        torch.cuda.synchronize()
        assert torch.equal(z8, z4) and torch.equal(b8, b4)
    z8, b8 = ops.bn_apply2_bits(y, sc, sh, yr, rs, rf)
    z4, b4 = ops.bn_apply2_bits(_off8(y), sc, sh, _off8(yr), rs, rf)
    torch.cuda.synchronize()
    assert torch.equal(z8, z4) and torch.equal(b8, b4)
    with pytest.raises(RuntimeError):
        ops.conv_dgrad_bnbwd(torch.randn(1, 4, 4, 64, device=dev),
                             ops.weight_to_krsc(torch.randn(64, 64, 1, 1, device=dev)), (4, 4), 1, 0,
                             torch.randn(1, 4, 4, 64, device=dev), torch.zeros(64, device=dev), 3,
                             z=ops.relu_bits_empty(torch.empty(1, 4, 4, 64, device=dev)))


@pytest.mark.parametrize("rows,c", [(1000, 256), (77, 64), (3, 8)])
def test_bn_apply_relu_bits_bf16(dev, rows, c):
    """The bf16-activation forms (tmr_bn_apply_bits_a16 / _apply2_bits_a16): z bit-identical to
    bn_apply / bn_apply2 on bf16 tensors, bits exactly (z > 0) of the stored bf16 z -- the test
    the mask-1 dgrads apply to z -- and the bf16 LDS-DMA dgrad with mask 3 bit-identical to
    mask 1 on the same z."""
    g = torch.Generator().manual_seed(rows * 3 + c)
    b16 = torch.bfloat16
    y = torch.randn(rows, c, generator=g).to(dev).to(b16)
    res = torch.randn(rows, c, generator=g).to(dev).to(b16)
    yr = torch.randn(rows, c, generator=g).to(dev).to(b16)
    sc, sh = (torch.rand(c, generator=g) + 0.5).to(dev), torch.randn(c, generator=g).to(dev)
    rs, rf = (torch.rand(c, generator=g) + 0.5).to(dev), torch.randn(c, generator=g).to(dev)
    for resid in (res, None):
        z, bits = ops.bn_apply_bits(y, sc, sh, resid)
        zr = ops.bn_apply(y, sc, sh, resid, True)
        torch.cuda.synchronize()
        assert z.dtype == b16 and torch.equal(z, zr)
        assert torch.equal(bits.cpu(), _pack_bits((zr > 0).cpu()))
    z2, bits2 = ops.bn_apply2_bits(y, sc, sh, yr, rs, rf)
    z2r = ops.bn_apply2(y, sc, sh, yr, rs, rf, True)
    torch.cuda.synchronize()
    assert torch.equal(z2, z2r) and torch.equal(bits2.cpu(), _pack_bits((z2r > 0).cpu()))
    if rows == 1000:   # a residual-gradient 1x1 dgrad over these rows as (10, 10, 10) pixels
        n, hw = 10, 10
        yv, zv, bv = y.view(n, hw, hw, c), z2.view(n, hw, hw, c), bits2
        k = 64
        dy = torch.randn(n, hw, hw, k, generator=g).to(dev).to(b16)
        w = torch.randn(k, c, 1, 1, generator=g).to(dev) / c ** 0.5
        wt = ops.weight_to_crsk(w)
        mu = torch.randn(c, generator=g).to(dev) * 0.1
        old = torch.randn(n, hw, hw, c, generator=g).to(dev)
        d1, p1, n1 = ops.conv_dgrad_bnbwd(dy, wt, (hw, hw), 1, 0, yv, mu, 1, z=zv,
                                          out=old.clone(), beta=1.0, math="bf16", wt=True)
        d3, p3, n3 = ops.conv_dgrad_bnbwd(dy, wt, (hw, hw), 1, 0, yv, mu, 3, z=bv,
                                          out=old.clone(), beta=1.0, math="bf16", wt=True)
        torch.cuda.synchronize()
        assert n1 == n3 and torch.equal(d1, d3) and torch.equal(p1[:n1], p3[:n3])


def test_stem_direct_fwd_bnstats(dev, monkeypatch, engine):
    """The fp32 7x7/2 stem with BatchNorm statistics as a direct convolution over its 147 real
    (tap, channel) pairs (stem.hip, the train step's 224x224 geometry) against float64: the
    output, and the BN statistics from its per-output-row partials; the implicit-GEMM engine
    (ops.engine_only, TMR_IO_ENGINE) agrees to fp32 summation order.  Six frames: 672 output rows, more than
    the persistent grid's 512 workgroups, so workgroups run the prefetched second row."""
    n = 6
    g = torch.Generator().manual_seed(12)
    x = torch.relu(torch.randn(n, 3, 224, 224, generator=g)) + 0.5
    wt = torch.randn(64, 3, 7, 7, generator=g) / np.sqrt(147)
    x4 = ops.nchw_to_nhwc(x.to(dev), cpad=4)
    wk = ops.weight_to_krsc(wt.to(dev).contiguous(), cpad=4)
    engine.use(False)
    y, stats, nparts = ops.conv_fwd_bnstats(x4, wk, 2, 3, c_real=3)
    engine.use(True)
    y0, stats0, nparts0 = ops.conv_fwd_bnstats(x4, wk, 2, 3, c_real=3)
    torch.cuda.synchronize()
    assert nparts == 4 * 512 and tuple(y.shape) == (n, 112, 112, 64)   # merged per workgroup
    ref = F.conv2d(x.double(), wt.double(), stride=2, padding=3).permute(0, 2, 3, 1)
    assert rel_err(y, ref) < 1e-6 and rel_err(y0, ref) < 1e-6
    yd = ref.reshape(-1, 64)
    for st_, np_ in ((stats, nparts), (stats0, nparts0)):
        ones, zeros = torch.ones(64, device=dev), torch.zeros(64, device=dev)
        rm, rv = zeros.clone(), ones.clone()
        mean, inv, _, _ = ops.bn_finalize(st_, np_, ones, zeros, rm, rv, 0.1, 1e-5)
        assert rel_err(mean, yd.mean(0)) < 1e-6
        assert rel_err(inv, 1 / torch.sqrt(yd.var(0, unbiased=False) + 1e-5)) < 1e-5


def test_stem16_direct_fwd_bnstats(dev, monkeypatch, engine):
    """The bf16-activation step's 7x7/2 stem as a direct convolution (stem16.hip: the NHWC4 fp32
    input rounded to bf16 in LDS, 147 real of 176 reduction rows on v_mfma_f32_32x32x16_bf16, y
    stored bf16, BatchNorm partials merged per workgroup) against float64 of the bf16-rounded
    operands (y within one bf16 rounding: the fp32 accumulation order decides ties), its
    statistics against float64 statistics of its own stored y, and the LDS-DMA engine on the
    NHWC8 copy (ops.engine_only, TMR_IO_ENGINE) within one bf16 ulp.  Sixteen frames: 1792 output rows over the
    768 persistent workgroups, each a contiguous range of 2-3 rows (the input-row ring reused across
    a range, ranges crossing frame boundaries, statistics merged over a range)."""
    n = 16
    g = torch.Generator().manual_seed(14)
    x = torch.relu(torch.randn(n, 3, 224, 224, generator=g)) + 0.5
    wt = torch.randn(64, 3, 7, 7, generator=g) / np.sqrt(147)
    x4 = ops.nchw_to_nhwc(x.to(dev), cpad=4)
    wk4 = ops.weight_to_krsc(wt.to(dev).contiguous(), cpad=4, bf16=True)
    engine.use(False)
    y, stats, nparts = ops.conv_fwd_bnstats(x4, wk4, 2, 3, c_real=3, math="bf16", y16=True)
    engine.use(True)
    x8 = ops.nhwc4_to_bf16x8(x4)
    wk8 = ops.weight_to_krsc(wt.to(dev).contiguous(), cpad=8, bf16=True)
    y0, _, _ = ops.conv_fwd_bnstats(x8, wk8, 2, 3, c_real=3, math="bf16", y16=True)
    torch.cuda.synchronize()
    assert y.dtype == torch.bfloat16 and tuple(y.shape) == (n, 112, 112, 64)
    assert nparts == 4 * 768
    ref = F.conv2d(x.to(torch.bfloat16).double(), wt.to(torch.bfloat16).double(), stride=2,
                   padding=3).permute(0, 2, 3, 1)
    yf = y.double().cpu()
    # one bf16 ulp of the exact value, plus the fp32 accumulation's absolute error (a result
    # that cancels to ~1e-6 of the row's magnitude rounds at a finer ulp than that error)
    ulp = 2.0 ** (torch.floor(torch.log2(ref.abs().clamp_min(1e-30))) - 7)
    floor = 1e-6 * ref.abs().max().item()
    assert ((yf - ref).abs() <= ulp * 1.0001 + floor).all()
    assert ((yf - y0.double().cpu()).abs() <= 2 * ulp * 1.0001 + 2 * floor).all()
    yd = yf.reshape(-1, 64)
    ones, zeros = torch.ones(64, device=dev), torch.zeros(64, device=dev)
    rm, rv = zeros.clone(), ones.clone()
    mean, inv, _, _ = ops.bn_finalize(stats, nparts, ones, zeros, rm, rv, 0.1, 1e-5)
    assert rel_err(mean, yd.mean(0)) < 1e-6
    assert rel_err(inv, 1 / torch.sqrt(yd.var(0, unbiased=False) + 1e-5)) < 1e-5


def test_stem16_direct_wgrad(dev, monkeypatch, engine):
    """The bf16 stem's weight gradient as a direct convolution (stem16.hip: per-row im2col and
    transposed dy in LDS, bf16 MFMA, per-workgroup slabs summed by the tap reduction) against
    float64 of the bf16 operands, with beta accumulation, and against the engine
    (ops.engine_only, TMR_IO_ENGINE).  Sixteen frames: 1792 output rows over the 768 persistent workgroups
    (contiguous ranges of 2-3 rows: the input-row ring reused, ranges crossing frames)."""
    n = 16
    g = torch.Generator().manual_seed(15)
    x = torch.relu(torch.randn(n, 3, 224, 224, generator=g)) + 0.5
    dy = torch.randn(n, 64, 112, 112, generator=g).to(torch.bfloat16)
    x4 = ops.nchw_to_nhwc(x.to(dev), cpad=4)
    dyn = dy.to(dev).permute(0, 2, 3, 1).contiguous()
    ref = torch.nn.grad.conv2d_weight(x.to(torch.bfloat16).double(), (64, 3, 7, 7), dy.double(),
                                      stride=2, padding=3)
    engine.use(False)
    dw = ops.conv_wgrad(x4, dyn, 7, 7, 2, 3, c_real=3, math="bf16")
    prev = torch.randn(64, 3, 7, 7, generator=g).to(dev)
    acc = ops.conv_wgrad(x4, dyn, 7, 7, 2, 3, c_real=3, math="bf16", out=prev.clone(), beta=0.5)
    engine.use(True)
    dw0 = ops.conv_wgrad(x4, dyn, 7, 7, 2, 3, c_real=3, math="bf16")
    torch.cuda.synchronize()
    assert rel_err(dw, ref) < 2e-6 and rel_err(dw0, ref) < 2e-6
    assert rel_err(acc, 0.5 * prev.double().cpu() + ref) < 2e-6


@pytest.mark.gpu
def test_stem_direct_wgrad(dev, monkeypatch, engine):
    """The fp32 stem's weight gradient as a direct convolution (stem.hip: per-workgroup partial
    slabs over the 147 real (tap, channel) pairs, summed by the engine's tap reduction) against
    float64, with beta accumulation, and against the implicit-GEMM engine (ops.engine_only, TMR_IO_ENGINE).
    Six frames: 672 output rows over the 512 persistent workgroups."""
    n = 6
    g = torch.Generator().manual_seed(13)
    x = torch.relu(torch.randn(n, 3, 224, 224, generator=g)) + 0.5
    dy = torch.randn(n, 64, 112, 112, generator=g)
    x4 = ops.nchw_to_nhwc(x.to(dev), cpad=4)
    dyn = dy.to(dev).permute(0, 2, 3, 1).contiguous()
    ref = torch.nn.grad.conv2d_weight(x.double(), (64, 3, 7, 7), dy.double(), stride=2, padding=3)
    engine.use(False)
    dw = ops.conv_wgrad(x4, dyn, 7, 7, 2, 3, c_real=3)
    prev = torch.randn(64, 3, 7, 7, generator=g).to(dev)
    acc = ops.conv_wgrad(x4, dyn, 7, 7, 2, 3, c_real=3, out=prev.clone(), beta=0.5)
    engine.use(True)
    dw0 = ops.conv_wgrad(x4, dyn, 7, 7, 2, 3, c_real=3)
    torch.cuda.synchronize()
    assert tuple(dw.shape) == (64, 3, 7, 7)
    # fp32 sums of 75,264 products per weight (random-sign dy): ~1e-6 of the largest weight
    assert rel_err(dw, ref) < 4e-6 and rel_err(dw0, ref) < 4e-6
    assert rel_err(acc, ref + 0.5 * prev.double().cpu()) < 4e-6


def test_layout_sessions_model_lifetime(dev):
    """a layout record belongs to its trunk module.  Build a model and step it, delete
    it and release its memory (empty_cache), then build a second model -- which may reuse the
    first one's id() and addresses -- and step it: its logits and gradients must be bit-identical
    to the same model run without layout sessions, and the first model's records (and the
    converted weight copies they hold) must be gone.  A parameter replaced in place of its
    storage (p.data = ...) forces a re-record instead of a refresh from the old address."""
    import gc
    import tmrnet_amd
    B, T, L = 2, 3, 5
    g = torch.Generator().manual_seed(19)
    frames = torch.randint(0, 256, (B * T, 250, 250, 3), generator=g, dtype=torch.uint8).to(dev)
    off = torch.randint(0, 27, (B, 2), generator=g, dtype=torch.int32).to(dev)
    lt = (torch.rand(B, L, 512, generator=g) * 2 - 1).to(dev)
    labels = torch.randint(0, 7, (B,), generator=g).to(dev)

    def model(seed):
        torch.manual_seed(seed)
        m = tmrnet_amd.resnet_lstm(seq_len=T, precision="bf16").to(dev).train()
        m.nl_block.forced_mask = torch.ones(B, 512, device=dev)
        m.forced_head_mask = torch.ones(B, 512, device=dev)
        return m

    def step(m):
        m.zero_grad(set_to_none=True)
        out = m(ops.crop_normalize(frames, off, T), lt)
        tmrnet_amd.CrossEntropyLoss(size_average=False)(out, labels).backward()
        torch.cuda.synchronize()
        return out.detach().clone(), {n: p.grad.clone() for n, p in m.named_parameters()}

    saved = ops.LAYOUT_SESSIONS
    try:
        ops.LAYOUT_SESSIONS = False
        ref = step(model(2))
        ops.LAYOUT_SESSIONS = True
        ops.clear_layout_sessions()
        m1 = model(1)
        step(m1); step(m1)
        assert ops.layout_session_count() == 1
        del m1
        gc.collect()
        torch.cuda.empty_cache()
        assert ops.layout_session_count() == 0        # freed with its model
        m2 = model(2)
        for _ in range(2):                            # record, then refresh
            out, grads = step(m2)
            assert torch.equal(out, ref[0])
            for n in grads:
                assert torch.equal(grads[n], ref[1][n]), n
        # new storage for one conv weight: the refresh must not read the old address
        w = m2.share.layer1[0].conv2.weight
        w.data = w.data.clone()
        torch.cuda.empty_cache()
        out, grads = step(m2)
        assert torch.equal(out, ref[0])
    finally:
        ops.LAYOUT_SESSIONS = saved
        ops.clear_layout_sessions()
