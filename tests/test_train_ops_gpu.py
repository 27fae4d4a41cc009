"""Fused training kernels (ops/csrc/train_kernels.hip via models/train_ops.py) against
plain PyTorch fp32 references of the same ops, forward and backward, and the fused
training forward against reference_forward (loss and gradients)."""
import dataclasses

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

dev = "cuda"


def _rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


def test_rms_norm_forward_backward():
    from smsgate_amd.models import train_ops

    torch.manual_seed(0)
    R, H, eps = 1000, 576, 1e-5
    x = torch.randn(R, H, device=dev) * 3
    w = torch.rand(H, device=dev) + 0.5
    dy = torch.randn(R, H, device=dev).to(torch.bfloat16)
    xa, wa = x.clone().requires_grad_(), w.clone().requires_grad_()
    y = train_ops.rms_norm(xa, wa, eps)
    y.backward(dy)
    xr, wr = x.clone().requires_grad_(), w.clone().requires_grad_()
    yr = xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + eps) * wr
    yr.backward(dy.float())
    assert y.dtype == torch.bfloat16
    assert _rel(y, yr) < 5e-3
    assert _rel(xa.grad, xr.grad) < 1e-4
    assert _rel(wa.grad, wr.grad) < 1e-4


@pytest.mark.parametrize("rep", [1, 3])
def test_rope_split_forward_backward(rep):
    """rep = 3: k / v expanded to the 9 query heads (repeat_interleave order), the
    adjoint summing the copies' gradients."""
    from smsgate_amd.models import train_ops
    from smsgate_amd.models.extractor import _rope, _rope_tables

    torch.manual_seed(1)
    B, T, nh, nkv, D = 3, 37, 9, 3, 64
    qkv = torch.randn(B, T, (nh + 2 * nkv) * D, device=dev).to(torch.bfloat16)
    cos, sin = _rope_tables(T, D, 100000.0, dev)
    c2, s2 = cos.reshape(T, D // 2).contiguous(), sin.reshape(T, D // 2).contiguous()
    qa = qkv.clone().requires_grad_()
    q, k, v = train_ops.rope_split(qa, c2, s2, nh, nkv, rep)
    gq, gk, gv = (torch.randn_like(t) for t in (q, k, v))
    (q.float() * gq.float()).sum().add((k.float() * gk.float()).sum()).add((v.float() * gv.float()).sum()).backward()
    qr_in = qkv.float().clone().requires_grad_()
    a, b, c = qr_in.split([nh * D, nkv * D, nkv * D], -1)
    qr = _rope(a.reshape(B, T, nh, D), cos, sin).transpose(1, 2)
    kr = _rope(b.reshape(B, T, nkv, D), cos, sin).transpose(1, 2)
    vr = c.reshape(B, T, nkv, D).transpose(1, 2)
    kr, vr = kr.repeat_interleave(rep, dim=1), vr.repeat_interleave(rep, dim=1)
    (qr * gq.float()).sum().add((kr * gk.float()).sum()).add((vr * gv.float()).sum()).backward()
    for got, want in ((q, qr), (k, kr), (v, vr)):
        assert got.shape == want.shape and _rel(got, want) < 5e-3
    assert _rel(qa.grad, qr_in.grad) < 5e-3


def test_swiglu_forward_backward():
    from smsgate_amd.models import train_ops

    torch.manual_seed(2)
    R, I = 777, 1536
    gu = (torch.randn(R, 2 * I, device=dev) * 2).to(torch.bfloat16)
    da = torch.randn(R, I, device=dev).to(torch.bfloat16)
    ga = gu.clone().requires_grad_()
    a = train_ops.swiglu(ga)
    a.backward(da)
    gr = gu.float().clone().requires_grad_()
    g, u = gr.chunk(2, dim=-1)
    ar = F.silu(g) * u
    ar.backward(da.float())
    assert _rel(a, ar) < 5e-3
    assert _rel(ga.grad, gr.grad) < 5e-3


@pytest.mark.parametrize("T", [37, 150, 192])
def test_attention_forward_backward(T):
    """The training attention kernels vs an fp32 causal GQA reference (9 query heads on 3
    kv heads), forward and every input gradient."""
    from smsgate_amd.models import train_ops

    torch.manual_seed(4)
    B, nh, nkv, D = 3, 9, 3, 64
    scale = 1.0 / 8.0
    q = torch.randn(B, nh, T, D, device=dev).to(torch.bfloat16)
    k = torch.randn(B, nkv, T, D, device=dev).to(torch.bfloat16)
    v = torch.randn(B, nkv, T, D, device=dev).to(torch.bfloat16)
    g = torch.randn(B, T, nh * D, device=dev).to(torch.bfloat16)
    qa, ka, va = (t.clone().requires_grad_() for t in (q, k, v))
    out = train_ops.attention(qa, ka, va, scale)
    out.backward(g)
    qr, kr, vr = (t.float().clone().requires_grad_() for t in (q, k, v))
    ke, ve = kr.repeat_interleave(nh // nkv, 1), vr.repeat_interleave(nh // nkv, 1)
    s = (qr @ ke.transpose(-1, -2)) * scale
    s = s.masked_fill(torch.ones(T, T, dtype=torch.bool, device=dev).triu(1), float("-inf"))
    ref = (s.softmax(-1) @ ve).transpose(1, 2).reshape(B, T, nh * D)
    ref.backward(g.float())
    assert out.shape == ref.shape and _rel(out, ref) < 1e-2
    for got, want in ((qa.grad, qr.grad), (ka.grad, kr.grad), (va.grad, vr.grad)):
        assert _rel(got, want) < 2e-2


@pytest.mark.parametrize("sdpa", ["", "efficient", "own"])
def test_fused_forward_matches_reference_forward(sdpa, monkeypatch):
    """Loss and every gradient of the fused training forward agree with
    reference_forward's (both bf16 autocast over fp32 master weights); also with the
    efficient SDPA backend on expanded k / v."""
    monkeypatch.setenv("SMSGATE_TRAIN_SDPA", sdpa)
    from smsgate_amd.models import train_ops
    from smsgate_amd.models.extractor import CONFIGS, ExtractorWeights, reference_forward

    cfg = dataclasses.replace(CONFIGS["smollm-135m"], layers=3, vocab=1024)
    torch.manual_seed(3)
    ids = torch.randint(0, cfg.vocab, (4, 45), device=dev)
    add = torch.where(torch.rand(4, 45, device=dev) < 0.5, torch.randint(0, cfg.vocab, (4, 45), device=dev),
                      torch.full((4, 45), -1, device=dev))
    tgt = torch.randn(4, 45, cfg.hidden, device=dev)
    res = []
    for fused in (True, False):
        w = ExtractorWeights(cfg, device=dev, dtype=torch.float32, seed=5)
        with torch.autocast(device_type="cuda", dtype=torch.bfloat16):
            if fused:
                h = train_ops.fused_forward(w, ids, add)
            else:
                h = reference_forward(w, ids, compute_dtype=torch.float32, return_hidden=True, add_ids=add)
            loss = (h.float() * tgt).mean()
        loss.backward()
        res.append((float(loss), h.detach().float(), {n: p.grad.detach().clone() for n, p in w.named_parameters()}))
    (lf, hf, gf), (lr, hr, gr) = res
    assert abs(lf - lr) <= 2e-2 * abs(lr) + 1e-4
    assert _rel(hf, hr) < 2e-2
    for n in gr:
        assert _rel(gf[n], gr[n]) < 5e-2, n
